"""Dev probe: time fwd / bwd of one view at a given config with HIP events (not the bench)."""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from oracle import oracle as orc

pkg = importlib.import_module("3dgaussian_amd")
tr = pkg.torch_renderer
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 800
dev = torch.device("cuda:0")
scene = orc.synthetic_scene(N, seed=0)
view, proj = orc.orbit_cameras(50, R, R)[0]
t = [torch.from_numpy(a).to(dev).requires_grad_(True) for a in scene.arrays()]
g = torch.randn(R, R, 3, device=dev)
for it in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, a, d = tr.rasterize(*t, view, proj, R, R)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    (out * g).sum().backward()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"N={N} {R}x{R}: fwd {1e3*(t1-t0):.2f} ms  bwd {1e3*(t2-t1):.2f} ms  total {1e3*(t2-t0):.2f} ms  -> {R*R/(t2-t0)/1e6:.1f} Mpx/s", flush=True)
