"""Diagnostic: fused parameter step vs autograd + torch Adam, one and three steps (grads, state, params)."""
import importlib
import sys

import torch

sys.path.insert(0, ".")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")
cuda = torch.device("cuda:0")
W, H = 128, 96
cams = fm.orbit_cameras(4, W, H, cuda)
g = torch.Generator(device=cuda).manual_seed(9)
targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
masks = [(t.mean(dim=2) > 0.5).float() for t in targets]


def run(fused, steps):
    fm.FUSED_STEP = fused
    f = fm.ViewShardedFitter(bench.synthetic_params(20_000, cuda), cams, targets, W, H, masks=masks)
    losses = [float(f.step()) for _ in range(steps)]
    out = {}
    for k, p in f.params.items():
        st = f.opt.state[p]
        out[k] = (p.detach().clone(), p.grad.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(),
                  float(st["step"]))
    return losses, out


for steps in (1, 3):
    ref = run(False, steps)
    ref2 = run(False, steps)
    fus = run(True, steps)
    print("steps", steps, "losses", ref[0], ref2[0], fus[0])
    for k in ref[1]:
        for nm, i in (("param", 0), ("grad", 1), ("m", 2), ("v", 3)):
            a, b, c = ref[1][k][i], ref2[1][k][i], fus[1][k][i]
            d_rr = (a - b).abs()
            d_rf = (a - c).abs()
            print(f"  {k:14s} {nm:5s} rerun max {float(d_rr.max()):.3e} n {int((d_rr > 0).sum())}  "
                  f"fused max {float(d_rf.max()):.3e} n {int((d_rf > 0).sum())} of {a.numel()}  "
                  f"scale {float(a.abs().max()):.3e}")
        print("  step", ref[1][k][4], fus[1][k][4])
