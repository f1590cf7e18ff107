"""Where a multi-stream step's time goes, from a rocprofv3 --kernel-trace CSV run: per kernel class the
union of its intervals, and how much of it overlaps a splat kernel (middle third of the run, steady state).
    python tools/overlap.py <dir>"""
import csv
import glob
import re
import sys

CLASSES = [("splat", r"k_raster_(fwd|bwd)"), ("gather", r"k_gather_view"), ("reduce", r"k_reduce_(views|sums|bwd)"),
           ("binning", r"k_(emit|tile_|work_items|pos_of|ranges|pair_values|fwd_finalize|tile_loss)"),
           ("prepare", r"k_(preprocess|plan|offsets)"), ("step", r"k_(fit_param_step|adam)")]


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    i = j = tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        tot += max(0, e - s)
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: r[1])
    n = len(rows)
    rows = rows[n // 3: 2 * n // 3]
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    span = t1 - t0
    cls = {c: union([(s, e) for k, s, e in rows if re.search(p, k)]) for c, p in CLASSES}
    alli = union([(s, e) for _, s, e in rows])
    busy = sum(e - s for s, e in alli)
    print(f"window {span / 1e6:.2f} ms, GPU busy {100 * busy / span:.1f}%")
    sp = cls["splat"]
    for c, iv in cls.items():
        t = sum(e - s for s, e in iv)
        ov = overlap(iv, sp) if c != "splat" else t
        print(f"  {c:8s} union {100 * t / span:5.1f}% of the window, beside a splat {100 * ov / max(t, 1):5.1f}% of its time,"
              f" alone {100 * (t - ov) / span:5.1f}% of the window")
    print(f"  no splat running: {100 * (span - sum(e - s for s, e in sp)) / span:.1f}% of the window")


if __name__ == "__main__":
    main()
