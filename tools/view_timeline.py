"""Kernel timeline around the k-th-from-last launch of a kernel in a rocprofv3 --kernel-trace CSV run:
    python tools/view_timeline.py <dir> [kernel substring, default k_raster_fwd] [k, default 30] [launches shown, default 40]"""
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:50]


def main():
    f = sorted(glob.glob(sys.argv[1] + "/**/*k*t*.csv", recursive=True))[0]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_raster_fwd"
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    cnt = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: r[1])
    hits = [i for i, r in enumerate(rows) if pat in r[0]]
    i0 = hits[-k]
    t0 = rows[i0][1]
    busy = rows[i0 - 4][1]
    for n, s, e, q in rows[i0 - 4:i0 - 4 + cnt]:
        if s - busy > 2000:
            print(f"   -- idle {(s - busy) / 1e3:.1f} us")
        busy = max(busy, e)
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{q} {short(n)}")


if __name__ == "__main__":
    main()
