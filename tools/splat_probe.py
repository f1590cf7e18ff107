"""Kernel-level timing probe of the fit path's two 32-pixel splats on fixed inputs (round 6).

Builds the bench's C4 scene (bench.synthetic_params, orbit views 800x800), runs a few fit steps so the state is a
fitted one, then for each of K views: prepares and bins it once, and times gr_fwd_render_l1 and gr_bwd_splat R times
each on the same inputs with HIP events on one stream (the kernels are idempotent on their inputs: the forward's tickets
are left zero, the backward only writes its pair rows).  Prints one JSON line: mean us per launch of each kernel.
Run from a tree (or an ab/<variant> copy of it) so that its libgr_hip.so is the one timed.
   python tools/splat_probe.py [--views K] [--reps R] [--steps S]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

fm, tr = bench.fm, bench.tr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--res", type=int, default=800)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    V, R = 50, a.res
    params = bench.synthetic_params(a.gaussians, dev)
    cams = fm.orbit_cameras(V, R, R, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
    fitter = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
    for _ in range(a.steps):
        fitter.step()
    torch.cuda.synchronize()
    L = tr._native.lib()
    nat = tr._native
    with torch.no_grad():
        acts = [x.detach().float().contiguous() for x in fm.activations(fitter.params)]
    n = int(acts[0].shape[0])
    cur = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(cur.cuda_stream)
    res = {"fwd_us": [], "bwd_us": [], "pairs": []}
    for i in range(a.views):
        gv = fitter._fit_view(i, dev)
        prep = tr.prepare_native(*acts, gv)
        torch.cuda.synchronize()
        plan = prep.plan()
        bins, scratch, bgv, done = tr._bin_launch(L, gv, n, plan, prep, cur, dev)
        ws = torch.empty((tr._ws_round(L.gr_bwd_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),), dtype=torch.uint8,
                         device=dev)
        loss = torch.zeros(1, device=dev)
        mask = fitter.masks[fitter._vi(i)]

        def fwd():
            nat.check(L.gr_fwd_render_l1(ctypes.byref(bgv), n, ctypes.byref(plan), nat.ptr(prep.geom), nat.ptr(bins),
                                         bins.numel(), nat.ptr(scratch), scratch.numel(),
                                         nat.ptr(fitter.targets[fitter._vi(i)]), nat.ptr(mask),
                                         ctypes.c_float(fitter.w_sil), ctypes.c_float(1.0 / V), nat.ptr(loss), None, None,
                                         nat.ptr(ws), ws.numel(), sp), "gr_fwd_render_l1")

        def bwd():
            nat.check(L.gr_bwd_splat(ctypes.byref(gv), n, ctypes.byref(plan), nat.ptr(prep.geom), nat.ptr(bins),
                                     nat.ptr(ws), ws.numel(), sp), "gr_bwd_splat")

        fwd()
        bwd()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * a.reps + 1)]
        ev[0].record(cur)
        for r in range(a.reps):
            fwd()
            ev[3 * r + 1].record(cur)
            bwd()
            ev[3 * r + 2].record(cur)
            ev[3 * r + 3].record(cur)  # an empty pair: the markers' own cost
        torch.cuda.synchronize()
        mk = sum(ev[3 * r + 2].elapsed_time(ev[3 * r + 3]) for r in range(a.reps)) / a.reps
        f = sum(ev[3 * r].elapsed_time(ev[3 * r + 1]) for r in range(a.reps)) / a.reps
        b = sum(ev[3 * r + 1].elapsed_time(ev[3 * r + 2]) for r in range(a.reps)) / a.reps
        res["fwd_us"].append(1e3 * (f - mk))
        res["bwd_us"].append(1e3 * (b - mk))
        res["pairs"].append(int(plan.num_pairs))
        del bins, scratch, ws, prep
    out = {k: round(sum(v) / len(v), 2) for k, v in res.items()}
    out["tree"] = os.path.basename(ROOT)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
