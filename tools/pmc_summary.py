"""Per-kernel mean of every PMC counter in rocprofv3 counter_collection CSVs: python tools/pmc_summary.py <dir>..."""
import collections, csv, glob, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            m = re.search(r"(k_\w+|\w*kernel\w*)", name)
            short = m.group(1) if m else name[:40]
            acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print("==", k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v)/len(v):16.1f}  (n={len(v)})")
