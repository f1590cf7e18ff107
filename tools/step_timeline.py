"""One steady-state fit step's kernel timeline from a rocprofv3 --kernel-trace CSV run: every kernel's
start / end (us from the step's first kernel), its queue, and the idle gaps of the whole GPU; the step is
the span between two consecutive parameter-update launches (k_adam_step, or k_fit_param_step at world size 1) in the middle of the run.
    python tools/step_timeline.py <dir> [step index from the end, default 3]"""
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main():
    f = sorted(glob.glob(sys.argv[1] + "/**/*k*t*.csv", recursive=True))[0]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")))
            for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: r[1])
    adam = [i for i, r in enumerate(rows) if ("k_adam_step" in r[0] or "k_fit_param_step" in r[0])]
    # the last Adam launch of each step: a gap of > 20 launches to the next Adam launch
    ends = [a for a, b in zip(adam, adam[1:]) if b - a > 20] + adam[-1:]
    if len(ends) < back + 1:
        sys.exit("too few steps in the trace")
    i0, i1 = ends[-back - 1] + 1, ends[-back]
    step = rows[i0:i1 + 1]
    t0 = step[0][1]
    print(f"step of {len(step)} kernels, {(step[-1][2] - t0) / 1e3:.1f} us (first start -> last end); "
          f"{(t0 - max(r[2] for r in rows[:i0])) / 1e3:.1f} us idle before it; "
          f"previous step {(rows[i0 - 1][2] - rows[ends[-back - 2] + 1][1]) / 1e3:.1f} us" if back + 2 <= len(ends) else "")
    busy_end = t0
    idle = 0
    for name, s, e, q in step:
        gap = s - busy_end
        if gap > 2000:
            print(f"   -- GPU idle {gap / 1e3:7.1f} us")
        if gap > 0:
            idle += gap
        busy_end = max(busy_end, e)
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:<4} {short(name)}")
    print(f"GPU idle inside the step: {idle / 1e3:.1f} us")


if __name__ == "__main__":
    main()
