"""Digest of the fused fit path's outputs on one seeded view (k_fwd32_l1 + k_bwd32 + gather + chain rule): run it in two
tree copies to check that a kernel variant is bit-identical (tools/ab_variant.sh).   python tools/bitcheck.py [n] [res]"""
import hashlib
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import oracle as orc  # noqa: E402  (scene and cameras only)
from test_tile32_gpu import _fused_view  # noqa: E402

tr = importlib.import_module("3dgaussian_amd.torch_renderer")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 800
cuda = torch.device("cuda:0")
sc = orc.synthetic_scene(n, seed=0)
t = [torch.from_numpy(a).to(cuda).contiguous() for a in sc.arrays()]
view, proj = orc.orbit_cameras(8, R, R)[1]
g = torch.Generator(device=cuda).manual_seed(3)
target = torch.rand((R, R, 3), generator=g, device=cuda)
mask = (target.mean(dim=2) > 0.5).float().contiguous()
loss, out, alpha, grads, _ = _fused_view(tr, t, view, proj, R, R, 32, target, mask, 0.2, 0.02, cuda)
h = hashlib.sha256()
for x in (out, alpha) + tuple(grads):
    h.update(x.cpu().numpy().tobytes())
print(f"bitcheck n={n} res={R} loss={loss!r} sha256={h.hexdigest()[:16]}")
