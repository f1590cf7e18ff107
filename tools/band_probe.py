"""Per-band cost of the fused path at C4 (one GPU): a leftover view rendered whole and in bands of tile rows, each band's
pair count and the single-stream time of its preparation + binning + forward + backward + gather (HIP events,
median of reps).   python tools/band_probe.py [view] [reps]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
tr = importlib.import_module("3dgaussian_amd.torch_renderer")
bench = importlib.import_module("bench")
vi = int(sys.argv[1]) if len(sys.argv) > 1 else 48
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
R, V, N = 800, 50, 1_000_000
params = bench.synthetic_params(N, dev)
cams = fm.orbit_cameras(V, R, R, dev)
g = torch.Generator(device=dev).manual_seed(1)
targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(V)]
masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
f = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
with torch.no_grad():
    acts = [a.detach().float().contiguous() for a in fm.activations(f.params)]
base = f._fit_view(vi, dev)
ty = -(-R // 32)


def run(row0, rows):
    gv = tr._native.GrView.from_buffer_copy(base)
    gv.row0, gv.rows = row0, rows
    ts, pairs = [], 0
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        prep = tr.prepare_native(*acts, gv)
        loss = torch.zeros(1, device=dev)
        st, ws = tr.forward_l1_native(*acts, gv, prep, targets[vi], masks[vi], 0.2, 1.0 / V, loss)
        tr.backward_splat_native(st, ws)
        tr.gather_view_native(st, ws)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
        pairs = int(st.plan.num_pairs)
    return pairs, float(np.median(ts))


p_all, t_all = run(0, ty)
print(f"view {vi} whole ({ty} tile rows): {p_all} pairs, {t_all * 1e3:.1f} us")
for g_ in (2, 4, 8):
    cuts = [ty * k // g_ for k in range(g_ + 1)]
    line = []
    for k in range(g_):
        p, t = run(cuts[k], cuts[k + 1] - cuts[k])
        line.append(f"rows {cuts[k]}-{cuts[k + 1]}: {p} pairs ({p / p_all:.2f}) {t * 1e3:.1f} us")
    print(f"{g_} bands: " + "; ".join(line))
