"""Config C5 probe: 3M Gaussians (density-matched), 1920x1080, fwd+bwd of a few of the 100 orbit views
with the fit loop's losses; prints per-stage device time (HIP events) and Mpx/s of the render op."""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

pkg = importlib.import_module("3dgaussian_amd")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 3_000_000
W, H, V = 1920, 1080, 100
dev = torch.device("cuda:0")
params = bench.synthetic_params(N, dev)
cams = fm.orbit_cameras(V, W, H, dev)
g = torch.Generator(device=dev).manual_seed(1)
views = list(range(0, V, 25))
targets = [torch.rand((H, W, 3), generator=g, device=dev) for _ in views]
masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
fitter = fm.ViewShardedFitter(params, [cams[i] for i in views], targets, W, H, masks=masks)
fitter.step()
torch.cuda.synchronize()
pkg._native.profile_begin()
t0 = time.perf_counter()
reps = 3
for _ in range(reps):
    fitter.step()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
p = pkg._native.profile_end()
nv = reps * len(views)
print(f"C5 {N} Gaussians {W}x{H}: {1e3 * dt / nv:.2f} ms/view fwd+bwd+loss+Adam(share) -> {W * H * nv / dt / 1e6:.1f} Mpx/s;",
      "  ".join(f"{k} {1e3 * v[0] / max(v[1], 1):.1f}us" for k, v in p.items()))
