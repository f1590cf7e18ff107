"""A/B helper: average raster fwd/bwd kernel time (HIP events) for the library in $GR_HIP_LIB."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import oracle as orc
pkg = importlib.import_module("3dgaussian_amd")
tr = pkg.torch_renderer
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 800
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
dev = torch.device("cuda:0")
scene = orc.synthetic_scene(N, seed=0)
views = orc.orbit_cameras(50, R, R)
t = [torch.from_numpy(a).to(dev) for a in scene.arrays()]
if os.environ.get("AB_RANDOM_ORDER") != "1":  # the trainer's layout (fit_multiview.morton_order)
    perm = importlib.import_module("3dgaussian_amd.fit_multiview").morton_order(t[0])
    t = [x[perm].contiguous() for x in t]
t = [x.requires_grad_(True) for x in t]
g = torch.randn(R, R, 3, device=dev)
gd = torch.randn(R, R, device=dev) if os.environ.get("AB_DEPTH") == "1" else None
CORE = float(os.environ.get("AB_CORE", tr.DEFAULT_CORE_CUTOFF))  # 0: one zone
DEPTH_GRAD = gd is not None or os.environ.get("AB_PRECISE") == "1"  # no depth loss -> no_depth_grad mode


FIT = os.environ.get("AB_FIT", "1") == "1"  # the fused fit path's settings (one 5.5-sigma zone, no depth)


def fit_view(i):
    gv = tr.make_view(*views[i], R, R, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, depth_grad=False)
    m, s, c, o = (x.detach() for x in t)
    out, a, _, st = tr.forward_native(m, s, c, o, gv, want_depth=False)
    tr.backward_native(m, s, c, o, st, g, a, None)


def loss_of(out, d):
    l = (out * g).sum()
    return l + (d * gd).sum() if gd is not None else l


for i in range(2):
    if FIT:
        fit_view(i)
        continue
    out, a, d = tr.rasterize(*t, *views[i], R, R, core_cutoff=CORE, depth_grad=DEPTH_GRAD)
    loss_of(out, d).backward()
torch.cuda.synchronize()
pkg._native.profile_begin()
for i in range(reps):
    if FIT:
        fit_view(i % 10)
        continue
    out, a, d = tr.rasterize(*t, *views[i % 10], R, R, core_cutoff=CORE, depth_grad=DEPTH_GRAD)
    loss_of(out, d).backward()
torch.cuda.synchronize()
p = pkg._native.profile_end()
lib = os.path.basename(os.environ.get("GR_HIP_LIB", "libgr_hip.so"))
print(f"{lib:20s} fit={int(FIT)} depth={int(gd is not None)} core={CORE} " + "  ".join(f"{k} {1e3*v[0]/max(v[1],1):7.1f}us" for k, v in p.items()))
