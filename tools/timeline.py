"""Busy/idle summary of a rocprofv3 kernel trace (rocpd db):
python tools/timeline.py <dir> [top] [first_kernel_substring occurrence last_kernel_substring occurrence]
(the optional window starts at the given occurrence of one kernel and ends at that of another)."""
import glob, sqlite3, sys
from collections import defaultdict

db = sorted(glob.glob(sys.argv[1] + "/**/*results.db", recursive=True))[0]
c = sqlite3.connect(db)
rows = c.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                 "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
if len(sys.argv) > 6:
    def nth(sub, k):
        hits = [r for r in rows if sub in r[0]]
        return hits[k]
    a, b = nth(sys.argv[3], int(sys.argv[4])), nth(sys.argv[5], int(sys.argv[6]))
    rows = [r for r in rows if r[1] >= a[1] and r[2] <= b[2]]
t0, t1 = rows[0][1], rows[-1][2]
busy, last_end, gaps = 0, t0, []
agg = defaultdict(lambda: [0, 0])
for name, s, e in rows:
    if s > last_end:
        gaps.append((s - last_end, name))
    busy += max(0, e - max(s, last_end))
    last_end = max(last_end, e)
    agg[name[:60]][0] += e - s
    agg[name[:60]][1] += 1
span = t1 - t0
print(f"span {span/1e6:.2f} ms, busy {busy/1e6:.2f} ms ({100*busy/span:.1f}%), idle {(span-busy)/1e6:.2f} ms in {len(gaps)} gaps")
gaps.sort(reverse=True)
for g, n in gaps[: int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"  gap {g/1e3:8.1f} us before {n[:70]}")
agg = defaultdict(lambda: [0, 0])
for name, s, e in rows:
    agg[name[:70]][0] += e - s
    agg[name[:70]][1] += 1
print("per kernel in the window (total ms, calls, avg us):")
for name, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
    print(f"  {t/1e6:8.3f} ms {n:5d} {t/n/1e3:9.1f} us  {name}")
