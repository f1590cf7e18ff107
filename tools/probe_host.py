"""Host-side cost of the fit step at a small config (C2 by default): wall time per step with the device
synchronised, time until the host has enqueued the step (no sync), and a cProfile of the enqueue.
    python tools/probe_host.py [C2|C3] [steps]"""
import cProfile, importlib, os, pstats, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

cfgs = importlib.import_module("tools.bench_configs") if False else None
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
bc = importlib.import_module("bench_configs")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
name = sys.argv[1] if len(sys.argv) > 1 else "C2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
c = bc.CONFIGS[name]
dev = torch.device("cuda:0")
params = bc.params_for(c["n"], c["sh"], dev)
cams = fm.orbit_cameras(c["views"], c["w"], c["h"], dev)
g = torch.Generator(device=dev).manual_seed(1)
targets = [torch.rand((c["h"], c["w"], 3), generator=g, device=dev) for _ in range(c["views"])]
masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
depths = [torch.rand((c["h"], c["w"]), generator=g, device=dev) for _ in range(c["views"])] if c["depth"] else None
f = fm.ViewShardedFitter(params, cams, targets, c["w"], c["h"], lr=0.02, masks=masks, depths=depths)
for _ in range(3):
    f.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
enq = 0.0
for _ in range(steps):
    a = time.perf_counter()
    f.step()
    enq += time.perf_counter() - a
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / steps
print(f"{name}: wall {1e3 * wall:.3f} ms/step, host enqueue {1e3 * enq / steps:.3f} ms/step")
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    f.step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
