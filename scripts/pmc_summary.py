"""Average PMC counters per scan-kernel dispatch from rocprofv3 CSV passes."""
import collections, csv, glob, sys
d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "scan_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in sorted(tot.items()):
    vals = list(v.values())
    print(f"{c:24s} {sum(vals) / len(vals):16.0f}")
