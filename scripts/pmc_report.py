"""Per-window PMC summary of lean_kernel from a prof_pmc.sh output directory:
    python scripts/pmc_report.py gpurun_out/<tag> [file_bytes] [window_bytes]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
nbytes = float(sys.argv[2]) if len(sys.argv) > 2 else 389_108_980.0
wbytes = float(sys.argv[3]) if len(sys.argv) > 3 else 1952.0
wins = nbytes / wbytes
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lean_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
avg = {c: sum(v.values()) / len(v) for c, v in tot.items()}
print(f"per {wbytes:.0f}-byte window ({wins:.0f} windows per launch)")
for c in sorted(avg):
    print(f"  {c:24s} {avg[c] / wins:12.1f}   total {avg[c]:.4g}")
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in avg:
            print(f"  {c} / SQ_WAVE_CYCLES = {avg[c] / wc:.3f}")
if "FETCH_SIZE" in avg:
    print(f"  HBM read (FETCH_SIZE KiB x 1024 x 2, gfx950 correction) = {avg['FETCH_SIZE'] * 2048:.4g} B per launch")
