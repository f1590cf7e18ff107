"""Per-kernel averages of the SQ counter passes (tools/pmc_sq_bench.sh): python tools/pmc_summary_sq.py <dir>"""
import collections, csv, glob, re, sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)(<[^>]*>)?", r.get("Kernel_Name", ""))
        if not m:
            continue
        vals[m.group(1) + (m.group(2) or "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    d = {c: sum(v) / len(v) for c, v in vals[k].items()}
    print(k)
    print("   " + "  ".join(f"{c}={d[c]:.4g}" for c in sorted(d)))
