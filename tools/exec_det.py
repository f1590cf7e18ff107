"""Determinism probe (round 6): the fused fit step at C4 size (1M Gaussians, 13 views 800x800, 2 steps) run twice
through the Python schedule and twice through the native executor; prints which runs agree bit for bit."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")
cuda = torch.device("cuda", 0)
R, V = 800, 13
cams = fm.orbit_cameras(V, R, R, cuda)
g = torch.Generator(device=cuda).manual_seed(4)
targets = [torch.rand((R, R, 3), generator=g, device=cuda) for _ in range(V)]
masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
res = []
for native in (False, False, True, True):
    fm.NATIVE_EXEC, fm.REDUCE_BATCH = ("1" if native else "0"), 2
    f = fm.ViewShardedFitter(bench.synthetic_params(1_000_000, cuda), cams, targets, R, R, masks=masks)
    out = []
    for _ in range(2):
        l = float(f.step())
        torch.cuda.synchronize()
        out.append((l, {k: v.detach().clone() for k, v in f.params.items()}))
    res.append((native, out))
    del f
    torch.cuda.empty_cache()
names = ["py1", "py2", "ex1", "ex2"]
for a in range(4):
    for b in range(a + 1, 4):
        for s in range(2):
            la, pa = res[a][1][s]
            lb, pb = res[b][1][s]
            diff = {k: float((pa[k] - pb[k]).abs().max()) for k in pa if not torch.equal(pa[k], pb[k])}
            print(names[a], names[b], "step", s + 1, "loss", la == lb, "params differ:", diff or "none", flush=True)
