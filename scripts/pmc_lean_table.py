"""Per-window PMC table of lean_kernel stage builds: python scripts/pmc_lean_table.py DIR [BYTES]"""
import collections, csv, glob, os, sys
d = sys.argv[1]
nbytes = float(sys.argv[2]) if len(sys.argv) > 2 else 389_000_000.0
wins = nbytes / 3968.0
rows = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{d}/*/run_counter_collection.csv")):
    v = f.split("/")[-2]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "lean_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, x in tot.items():
        vals = list(x.values())
        rows[c][v] = sum(vals) / len(vals) / wins
vs = sorted({v for r in rows.values() for v in r})
print("per 3968-byte window")
print(f"{'counter':26s}" + "".join(f"{v:>10s}" for v in vs))
for c in sorted(rows):
    print(f"{c:26s}" + "".join(f"{rows[c].get(v, float('nan')):10.1f}" for v in vs))
