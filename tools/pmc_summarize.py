"""Summarise the PMC passes of tools/pmc_profile.sh into per-launch figures per kernel, written to
<dir>/pmc.json (copy it to profiles/pmc_traffic.json for bench.py) and printed.

Corrections as MI355X_MICROARCH.md §HBM/rocprofv3 prescribes: FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B per lane) coalesced reads, so read bytes = 2 x FETCH_SIZE.
SQ_* busy counters count quad-cycles per SIMD and are summed over the chip; GRBM_GUI_ACTIVE is summed
over the 8 XCDs, so a launch spans GRBM_GUI_ACTIVE / 8 cycles on each of the 1024 SIMDs:
  valu_frac = 4 SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 x 1024)   (VALU issue share of SIMD cycles)
  mfma_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024)
  wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES                            (waves parked on memory / barriers)
usage: python tools/pmc_summarize.py <dir>
"""
import collections
import csv
import glob
import hashlib
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024


def source_sha256() -> str:
    with open(os.path.join(REPO, "3dgaussian_amd", "csrc", "gr_hip.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def collect(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)(<[^>]*>)?", r.get("Kernel_Name", ""))
            if not m:
                continue
            vals[m.group(1) + (m.group(2) or "").replace(" ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}, \
        {k: {c: len(v) for c, v in cs.items()} for k, cs in vals.items()}


def main():
    d = sys.argv[1]
    avg, cnt = collect(d)
    out = {"source_sha256": source_sha256(), "dir": d, "kernels": {}}
    for k, c in sorted(avg.items()):
        e = {"counters": c, "launches": cnt[k]}
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            rb, wb = 2.0 * 1024.0 * c.get("FETCH_SIZE", 0.0), 1024.0 * c.get("WRITE_SIZE", 0.0)
            e.update(hbm_bytes_per_launch=rb + wb, read_bytes_corrected=rb, write_bytes=wb)
        g = c.get("GRBM_GUI_ACTIVE")
        if g:
            simd_cycles = g / 8.0 * SIMDS
            if "SQ_ACTIVE_INST_VALU" in c:
                e["valu_frac"] = round(4.0 * c["SQ_ACTIVE_INST_VALU"] / simd_cycles, 4)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                e["mfma_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles, 4)
        if c.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
        if c.get("SQ_INSTS_MFMA"):
            # the splats issue 12 MFMA per 32-pair step (bench.py's FLOP model): VALU instructions per step
            e["valu_per_12_mfma"] = round(12.0 * c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"], 1)
        out["kernels"][k] = e
    json.dump(out, open(os.path.join(d, "pmc.json"), "w"), indent=1)
    for k, e in out["kernels"].items():
        keep = {x: e[x] for x in ("hbm_bytes_per_launch", "valu_frac", "mfma_frac", "wait_frac", "valu_per_12_mfma") if x in e}
        print(k, json.dumps(keep))


if __name__ == "__main__":
    main()
