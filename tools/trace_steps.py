"""Per-step view of a rocprofv3 --kernel-trace CSV (bench.py run): for the last complete fit step (between
the last two groups of Adam kernels), wall time, union-busy time, idle gaps, and per kernel family the
summed duration and the time it ran alone (no other kernel in flight).
    python tools/trace_steps.py <dir>"""
import csv, glob, re, sys
from collections import defaultdict

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in csv.DictReader(open(f)))
adam = [k for k, r in enumerate(rows) if any(m in r[2] for m in ("multi_tensor_apply", "k_fit_param_step", "k_adam_step"))]
ends = [k for k, nxt in zip(adam, adam[1:] + [None]) if nxt is None or nxt != k + 1]
lo, hi = ends[-3] + 1, ends[-2] + 1
rows = rows[lo:hi]
t0, t1 = rows[0][0], max(e for _, e, _, _ in rows)


def fam(name):
    m = re.search(r"(k_\w+)", name)
    if m:
        return m.group(1)
    return "torch/" + name.split("(")[0].split("<")[0].split("::")[-1][:30]


# sweep: union busy, alone time per family
ev = []
for s, e, n, st in rows:
    ev.append((s, 1, fam(n)))
    ev.append((e, -1, fam(n)))
ev.sort()
active = defaultdict(int)
alone = defaultdict(float)
busy = 0.0
last = ev[0][0]
for t, d, fm in ev:
    tot = sum(active.values())
    if tot > 0:
        busy += t - last
        if tot == 1:
            (only,) = [k for k, v in active.items() if v]
            alone[only] += t - last
    active[fm] += d
    if active[fm] == 0:
        del active[fm]
    last = t
dur = defaultdict(float)
cnt = defaultdict(int)
for s, e, n, st in rows:
    dur[fam(n)] += e - s
    cnt[fam(n)] += 1
wall = t1 - t0
print(f"step wall {wall/1e3:.0f} us, union busy {busy/1e3:.0f} us ({100*busy/wall:.1f}%), idle {(wall-busy)/1e3:.0f} us")
print(f"{'family':40s} {'calls':>5s} {'sum_us':>9s} {'avg_us':>8s} {'alone_us':>9s}")
for k in sorted(dur, key=lambda k: -dur[k])[:25]:
    print(f"{k:40s} {cnt[k]:5d} {dur[k]/1e3:9.0f} {dur[k]/1e3/cnt[k]:8.1f} {alone[k]/1e3:9.0f}")
# idle gaps
gaps = []
cur_end = rows[0][1]
prev = rows[0]
for r in rows[1:]:
    if r[0] > cur_end:
        gaps.append((r[0] - cur_end, fam(prev[2]), fam(r[2])))
    if r[1] > cur_end:
        cur_end, prev = r[1], r
gaps.sort(reverse=True)
print("largest idle gaps:")
for g, a, b in gaps[:10]:
    print(f"  {g/1e3:8.1f} us after {a} before {b}")
