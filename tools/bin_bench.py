"""Binning alone (gr_fwd_bin: emission, column scan, placement) of one C4 bench view, repeated on one stream:
prints the mean microseconds per binning (HIP events).  Run under rocprofv3 --kernel-trace --stats for the
per-kernel split; GR_TUNE_PLACE_WAVES / GR_TUNE_COL_TARGET select the placement variant.
    python tools/bin_bench.py [reps] [n] [res]"""
import ctypes
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
bench = importlib.import_module("bench")
tr = importlib.import_module("3dgaussian_amd.torch_renderer")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
sp = importlib.import_module("3dgaussian_amd.spatial")
nat = importlib.import_module("3dgaussian_amd._native")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    res = int(sys.argv[3]) if len(sys.argv) > 3 else 800
    dev = torch.device("cuda", 0)
    L = nat.lib()
    params = bench.synthetic_params(n, dev)
    with torch.no_grad():
        order = sp.morton_order(params["means"])
        params = {k: v[order].contiguous() for k, v in params.items()}
        m, s, c, o = (t.contiguous() for t in fm.activations(params))
        cam = fm.orbit_cameras(50, res, res, dev)[0]
        gv = tr.make_view(cam.view, cam.proj, res, res, None, 5.0, 5.0)
        gv.no_depth_grad = 1
        p = tr.prepare_native(m, s, c, o, gv)
        torch.cuda.synchronize()
        plan = p.plan()
        bins = torch.empty((tr._ws_round(L.gr_bins_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),), dtype=torch.uint8,
                           device=dev)
        scratch = torch.empty((tr._ws_round(L.gr_fwd_scratch_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),),
                              dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream(dev)

        def once():
            nat.check(L.gr_fwd_bin(ctypes.byref(gv), n, ctypes.byref(plan), nat.ptr(p.geom), nat.ptr(bins), bins.numel(),
                                   nat.ptr(scratch), scratch.numel(), ctypes.c_void_p(st.cuda_stream)), "gr_fwd_bin")

        for _ in range(3):
            once()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            once()
        b.record(st)
        torch.cuda.synchronize()
    print(json.dumps({"us_per_binning": 1000.0 * a.elapsed_time(b) / reps, "pairs": int(plan.num_pairs), "reps": reps,
                      "place_waves": os.environ.get("GR_TUNE_PLACE_WAVES"), "col_target": os.environ.get("GR_TUNE_COL_TARGET")}))


if __name__ == "__main__":
    main()
