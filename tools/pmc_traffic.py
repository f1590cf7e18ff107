"""Summarise rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE in separate runs) into per-launch HBM
bytes per kernel, corrected as MI355X_MICROARCH.md §HBM prescribes: counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so read bytes = 2 x FETCH_SIZE
(the kernels below read with 16-B-per-lane loads).  Writes profiles/pmc_traffic.json.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json]
"""
import collections
import csv
import glob
import json
import sys

KERNELS = ("k_raster_bwd_bf16", "k_raster_bwd_mfma", "k_raster_fwd_mfma", "k_reduce_bwd", "k_reduce_views", "k_emit_zones",
           "k_tile_place", "k_tile_count", "k_tile_colscan", "k_pixel_grads", "k_fwd_finalize", "k_preprocess")


def per_launch(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            for k in KERNELS:
                if k in name:
                    vals[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items() if v}, {k: len(v) for k, v in vals.items()}


def main():
    fetch, nf = per_launch(sys.argv[1], "FETCH_SIZE")
    write, nw = per_launch(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in KERNELS:
        if k in fetch or k in write:
            fb = fetch.get(k, 0.0) * 1024.0
            wb = write.get(k, 0.0) * 1024.0
            out[k] = {"fetch_size_kib_raw": fetch.get(k), "write_size_kib_raw": write.get(k),
                      "hbm_bytes_per_launch": 2.0 * fb + wb, "read_bytes_corrected": 2.0 * fb, "write_bytes": wb,
                      "launches_fetch": nf.get(k, 0), "launches_write": nw.get(k, 0),
                      "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 wide-read halving), write = WRITE_SIZE x 1024"}
    path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
