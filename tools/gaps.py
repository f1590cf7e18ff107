"""GPU idle gaps between kernels in a rocprofv3 kernel trace (rocpd db): python tools/gaps.py <dir> [min_us].

Prints busy / idle time over the last complete optimizer step (between the last two groups of Adam
kernels) and the largest gaps with the kernels on either side, to find host synchronisation points.
"""
import glob
import sqlite3
import sys
from collections import Counter


def main():
    root = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    f = sorted(glob.glob(root + "/**/*results.db", recursive=True))[0]
    c = sqlite3.connect(f)
    rows = c.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    # the last full optimizer step: between the last two groups of Adam (multi_tensor_apply) kernels
    adam = [k for k, r in enumerate(rows) if "multi_tensor_apply" in r[0]]
    ends = [k for k, nxt in zip(adam, adam[1:] + [None]) if nxt is None or nxt != k + 1]
    if len(ends) >= 2:
        rows = rows[ends[-2] + 1: ends[-1] + 1]
    else:
        rows = rows[len(rows) // 2:]
    busy = sum(e - s for _, s, e in rows)
    span = rows[-1][2] - rows[0][1]
    gaps = []
    for (n0, s0, e0), (n1, s1, e1) in zip(rows, rows[1:]):
        g = s1 - e0
        if g > min_us * 1e3:
            gaps.append((g, n0[:40], n1[:40]))
    print(f"span {span/1e6:.2f} ms  busy {busy/1e6:.2f} ms  idle {(span-busy)/1e6:.2f} ms  kernels {len(rows)}")
    tot = Counter()
    cnt = Counter()
    for g, a, b in gaps:
        tot[(a, b)] += g
        cnt[(a, b)] += 1
    for (a, b), g in tot.most_common(15):
        print(f"{g/1e3:9.1f} us over {cnt[(a, b)]:4d} gaps  after {a:40s} before {b}")


if __name__ == "__main__":
    main()
