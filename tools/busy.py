"""GPU busy fraction (union of kernel intervals, overlapping streams counted once) over the middle
of a rocprofv3 --kernel-trace CSV run:  python tools/busy.py <dir>"""
import csv, glob, sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f)))
n = len(iv)
iv = iv[n // 3: 2 * n // 3]  # steady state
t0, t1 = iv[0][0], max(e for _, e in iv)
busy, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
conc = sum(e - s for s, e in iv)
print(f"window {1e-6 * (t1 - t0):.2f} ms: union busy {100.0 * busy / (t1 - t0):.1f}%, mean concurrency {conc / max(busy, 1):.2f}")
