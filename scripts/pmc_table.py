"""Per-record PMC table from scripts/pmc_detail.sh output: python scripts/pmc_table.py DIR RECORDS"""
import collections, csv, glob, sys
d, recs = sys.argv[1], float(sys.argv[2])
rows = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{d}/*/run_counter_collection.csv")):
    v = f.split("/")[-2].rsplit("_", 1)[0]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "scan_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, x in tot.items():
        vals = list(x.values())
        rows[c][v] = sum(vals) / len(vals) / recs
vs = sorted({v for r in rows.values() for v in r})
print(f"{'counter':26s}" + "".join(f"{v:>12s}" for v in vs))
for c in sorted(rows):
    print(f"{c:26s}" + "".join(f"{rows[c].get(v, float('nan')):12.2f}" for v in vs))
