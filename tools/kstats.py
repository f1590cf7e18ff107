"""Per-kernel stats of a rocprofv3 --kernel-trace run: python tools/kstats.py <dir> [--last N].

Reads *kernel_stats.csv (csv output) or the rocpd *_results.db (default output of rocprofv3 7.x).
"""
import csv
import glob
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    agg = defaultdict(list)
    for name, ns in rows:
        agg[name].append(ns)
    total = sum(sum(v) for v in agg.values()) or 1
    out = []
    for name, v in agg.items():
        out.append((name, len(v), sum(v) / len(v) / 1e3, 100.0 * sum(v) / total))
    return sorted(out, key=lambda r: -r[3])


def main():
    root = sys.argv[1]
    for f in sorted(glob.glob(root + "/**/*kernel_stats.csv", recursive=True)):
        print("==", f)
        for r in csv.DictReader(open(f)):
            print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f} "
                  f"pct={float(r['Percentage']):5.1f}")
    for f in sorted(glob.glob(root + "/**/*results.db", recursive=True)):
        print("==", f)
        for name, n, avg, pct in from_db(f):
            print(f"{name[:70]:70s} calls={n:5d} avg_us={avg:9.1f} pct={pct:5.1f}")


if __name__ == "__main__":
    main()
