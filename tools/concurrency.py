"""Concurrency profile of the overlapped fit step from a rocprofv3 --kernel-trace CSV run: over the last
`steps` whole steps (between parameter-update launches), how long the GPU ran 0, 1, 2, 3, 4+ kernels at once,
and per kernel its total time, the time it ran alone and its time-share (each instant split evenly over the
kernels running then): the share sums to the step's busy time, so it is the kernel's claim on the step.
    python tools/concurrency.py <dir> [steps, default 5] [views per step, default 50]"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "").replace(" ", "")) if m else re.sub(r"\W+", "_", name)[:40]


def main():
    f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    views = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    rows = sorted(((short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                   for r in csv.DictReader(open(f))), key=lambda r: r[1])
    upd = [i for i, r in enumerate(rows) if r[0].startswith(("k_fit_param_step", "k_adam_step"))]
    ends = [a for a, b in zip(upd, upd[1:]) if b - a > 20] + upd[-1:]
    if len(ends) < steps + 2:
        sys.exit("too few steps in the trace")
    t0, t1 = rows[ends[-steps - 2]][2], rows[ends[-2]][2]
    ev = []
    for name, s, e in rows:
        s, e = max(s, t0), min(e, t1)
        if e > s:
            ev += [(s, 1, name), (e, -1, name)]
    ev.sort(key=lambda x: (x[0], x[1]))
    live = collections.Counter()
    conc = collections.Counter()
    total, alone, share = collections.Counter(), collections.Counter(), collections.Counter()
    prev = t0
    for t, d, name in ev:
        dt = t - prev
        if dt > 0:
            k = sum(live.values())
            conc[min(k, 4)] += dt
            for n, c in live.items():
                total[n] += dt * c
                share[n] += dt * c / k
                if k == 1:
                    alone[n] += dt
        live[name] += d
        if live[name] == 0:
            del live[name]
        prev = t
    span = (t1 - t0) / 1e3
    per = steps * views
    print(f"{steps} steps, {span / steps:.1f} us per step, {span / per:.1f} us per view")
    print("kernels running at once (us per view): " + "  ".join(f"{k}{'+' if k == 4 else ''}: {conc[k] / 1e3 / per:.1f}"
                                                          for k in range(5)))
    print(f"{'kernel':44s} {'total':>8s} {'alone':>8s} {'share':>8s}   (us per view)")
    for n, v in sorted(share.items(), key=lambda x: -x[1]):
        if v / 1e3 / per < 0.2:
            continue
        print(f"{n[:44]:44s} {total[n] / 1e3 / per:8.1f} {alone[n] / 1e3 / per:8.1f} {v / 1e3 / per:8.1f}")


if __name__ == "__main__":
    main()
