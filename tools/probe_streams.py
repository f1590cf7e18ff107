"""Dev probe: do two views rendered (fwd+bwd) on two HIP streams overlap?  Times V views on one stream
and alternating over two streams (same work), C4 scene in the trainer's Morton order."""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import oracle as orc

pkg = importlib.import_module("3dgaussian_amd")
tr = pkg.torch_renderer
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 800
V = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
scene = orc.synthetic_scene(N, seed=0)
t = [torch.from_numpy(a).to(dev) for a in scene.arrays()]
perm = fm.morton_order(t[0])
t = [x[perm].contiguous().requires_grad_(True) for x in t]
views = orc.orbit_cameras(50, R, R)
g = torch.randn(R, R, 3, device=dev)
streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]


def run(nstreams):
    for x in t:
        x.grad = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(V):
        s = streams[i % nstreams]
        with torch.cuda.stream(s):
            out, a, d = tr.rasterize(*t, *views[i], R, R)
            (out * g).sum().backward()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


for rep in range(3):
    t1 = run(1)
    t2 = run(2)
    print(f"{V} views fwd+bwd: one stream {1e3*t1/V:.3f} ms/view, two streams {1e3*t2/V:.3f} ms/view", flush=True)
