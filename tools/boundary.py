"""Timeline of the fit step boundary from a rocprofv3 --kernel-trace CSV: every kernel from `before` us
ahead of the second-to-last parameter-step launch to `after` us past it (start, duration, stream, name).
    python tools/boundary.py <dir> [before_us] [after_us]"""
import csv, glob, re, sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
before = float(sys.argv[2]) if len(sys.argv) > 2 else 1500.0
after = float(sys.argv[3]) if len(sys.argv) > 3 else 2500.0
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
              for r in csv.DictReader(open(f)))
steps = [k for k, r in enumerate(rows) if any(m in r[2] for m in ("k_fit_param_step", "multi_tensor_apply"))]
groups = [k for k, nxt in zip(steps, steps[1:] + [None]) if nxt is None or nxt != k + 1]
t0 = rows[groups[-2]][0]


def fam(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else "torch/" + name.split("(")[0].split("<")[0].split("::")[-1][:30]


for s, e, n, st in rows:
    if t0 - before * 1e3 <= s <= t0 + after * 1e3:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  s{st:>3s}  {fam(n)}")
