"""Memory copies of a rocprofv3 --memory-copy-trace run, by direction and size: count per step of the
drop-in loop (tools/dropin_run.py), to show which copies remain per view.   python tools/copy_summary.py <dir> [views*steps]"""
import collections
import csv
import glob
import sys

f = sorted(glob.glob(sys.argv[1] + "/**/*memory_copy_trace.csv", recursive=True))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if not f:
    print("no memory copy trace under", sys.argv[1])
    sys.exit(0)
rows = list(csv.DictReader(open(f[0])))
c = collections.Counter()
for r in rows:
    d = r.get("Direction", r.get("Kind", "?"))
    size = int(r.get("Bytes", r.get("Size", 0)) or 0)
    c[(d, "<=64B" if size <= 64 else ("<=4KiB" if size <= 4096 else ">4KiB"))] += 1
print(f"{len(rows)} copies in {f[0]}")
for (d, s), n in sorted(c.items()):
    print(f"  {d:28s} {s:8s} {n:6d}" + (f"  ({n / per:.2f} per rendered view)" if per else ""))
