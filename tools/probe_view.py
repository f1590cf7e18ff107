"""Dev probe: fwd+bwd of one C4 view, repeated (for rocprofv3 counter runs)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import oracle as orc
pkg = importlib.import_module("3dgaussian_amd")
tr = pkg.torch_renderer
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 800
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda:0")
scene = orc.synthetic_scene(N, seed=0)
view, proj = orc.orbit_cameras(50, R, R)[0]
t = [torch.from_numpy(a).to(dev) for a in scene.arrays()]
if os.environ.get("PROBE_RANDOM_ORDER") != "1":  # the trainer's layout (fit_multiview.morton_order)
    perm = importlib.import_module("3dgaussian_amd.fit_multiview").morton_order(t[0])
    t = [x[perm].contiguous() for x in t]
t = [x.requires_grad_(True) for x in t]
g = torch.randn(R, R, 3, device=dev)
for _ in range(reps):
    out, a, d = tr.rasterize(*t, view, proj, R, R)
    (out * g).sum().backward()
torch.cuda.synchronize()
print("ok")
