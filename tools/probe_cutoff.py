"""Dev probe: dense-sample error of the HIP gradients vs the tail cutoff, with an upstream depth gradient
(tests/test_scale_gpu.py's dense check) at config C4 / C5 size.  Usage: python tools/probe_cutoff.py C5 7 8 9"""
import importlib, sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import numpy as np, torch
sys.path.insert(0, "tests")
from oracle import oracle as orc
import test_scale_gpu as tsg

pkg = importlib.import_module("3dgaussian_amd")
tr = pkg.torch_renderer
cfg = sys.argv[1]
n, W, H, V = tsg.CONFIGS[cfg]
sc = tsg._scene(n)
view, proj = orc.orbit_cameras(V, W, H)[0]
rng = np.random.default_rng(7)
g_rgb = rng.standard_normal((H, W, 3)).astype(np.float32)
g_a = rng.standard_normal((H, W)).astype(np.float32)
g_d = rng.standard_normal((H, W)).astype(np.float32)
sel = np.sort(rng.choice(n, 1000, replace=False)).astype(np.int32)
dev = torch.device("cuda:0")
dense = None
for c in [float(x) for x in sys.argv[2:]]:
    t = [torch.from_numpy(a).to(dev).requires_grad_(True) for a in sc.arrays()]
    out, alpha, depth = tr.rasterize(*t, view, proj, W, H, cutoff=c)
    ((out * torch.from_numpy(g_rgb).to(dev)).sum() + (alpha * torch.from_numpy(g_a).to(dev)).sum()
     + (depth * torch.from_numpy(g_d).to(dev)).sum()).backward()
    hip = [x.grad.cpu().numpy()[sel] for x in t]
    v = orc.make_view(view, proj, W, H, None, cutoff=c, core_cutoff=tr.DEFAULT_CORE_CUTOFF)
    if dense is None:
        dense = orc.dense_grads_sel(v, sc, sel, g_rgb, g_a, g_d)
    errs = [orc.rel_l2(a, b) for a, b in zip(hip, dense)]
    st = tr.forward_native(*[x.detach() for x in t], tr.make_view(view, proj, W, H, None, c))[3]
    print(f"{cfg} cutoff {c}: pairs {st.num_pairs} core {int(st.plan.num_core_pairs)} dense-sample relL2 "
          f"means {errs[0]:.2e} scales {errs[1]:.2e} colors {errs[2]:.2e} opac {errs[3]:.2e}", flush=True)
