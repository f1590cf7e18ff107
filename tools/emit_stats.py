"""Pair-emission balance of the C4 bench view (diagnostic for k_emit_cols): per Gaussian its tile rectangle's
cells and its pairs, and per wave of 64 consecutive (Morton-ordered) Gaussians the largest rectangle, i.e. the
serial loop a one-Gaussian-per-lane emission runs.  Prints one JSON line.
    python tools/emit_stats.py [n] [res]"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
bench = importlib.import_module("bench")
tr = importlib.import_module("3dgaussian_amd.torch_renderer")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
sp = importlib.import_module("3dgaussian_amd.spatial")
nat = importlib.import_module("3dgaussian_amd._native")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    res = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    dev = torch.device("cuda", 0)
    params = bench.synthetic_params(n, dev)
    with torch.no_grad():
        order = sp.morton_order(params["means"])
        params = {k: v[order].contiguous() for k, v in params.items()}
        m, s, c, o = (t.contiguous() for t in fm.activations(params))
        cams = fm.orbit_cameras(50, res, res, dev)
        out = {}
        for vi in (0, 25):
            gv = tr.make_view(cams[vi].view, cams[vi].proj, res, res, None, 5.0, 5.0)
            p = tr.prepare_native(m, s, c, o, gv)
            torch.cuda.synchronize()
            off = nat.geom_layout(n)
            geom = p.geom.cpu().numpy()
            rect = geom[off[1]: off[1] + 16 * n].view(np.int32).reshape(n, 4).astype(np.int64)
            cnt = geom[off[2]: off[2] + 8 * n].view(np.uint64)
            pairs = (cnt & 0xFFFFFFFF).astype(np.int64) + (cnt >> 32).astype(np.int64)
            cells = np.where(pairs > 0, (rect[:, 2] - rect[:, 0] + 1) * (rect[:, 3] - rect[:, 1] + 1), 0)
            w = n // 64
            wmax = cells[: w * 64].reshape(w, 64).max(1)
            pb = pairs[: (n // 256) * 256].reshape(-1, 256).sum(1)
            out[f"view{vi}"] = {
                "pairs": int(pairs.sum()), "cells": int(cells.sum()),
                "mean_cells": float(cells.mean()), "mean_wave_max_cells": float(wmax.mean()),
                "lane_efficiency": float(cells[: w * 64].mean() / max(wmax.mean(), 1e-9)),
                "pairs_per_256_block": {"mean": float(pb.mean()), "p99": float(np.percentile(pb, 99)), "max": int(pb.max())},
            }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
