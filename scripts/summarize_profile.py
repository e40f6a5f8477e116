"""Summarise a scripts/round_profile.sh output directory into profiles/.

    python scripts/summarize_profile.py gpurun_out/r1 profiles/r1 --rows 100000000

Writes <prefix>_kernel_stats.csv (rocprofv3 --stats, verbatim), <prefix>_pmc.json
(per-dispatch averages of the scan kernel's counters) and profiles/hbm_traffic.json
(FETCH_SIZE x 2 + WRITE_SIZE in bytes per scan launch, the gfx950 correction of
MI355X_MICROARCH.md 'HBM'), which bench.py reports as roofline.traffic.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil


def pmc(d, kernel="lean_kernel"):
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for c, v in per.items():
            out[c].extend(v.values())
    return {c: sum(v) / len(v) for c, v in out.items() if v}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("prefix")
    ap.add_argument("--rows", type=int, default=100_000_000)
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.prefix), exist_ok=True)
    stats = glob.glob(os.path.join(a.src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], a.prefix + "_kernel_stats.csv")
    # counters per kernel class: config 3's and config 2's fast_kernel, config 5's jx kernels
    classes = {"config3": "fast_kernel<true", "config2": "fast_kernel<false",
               # config 5's rank step (the typed exchange): the sender's count / emit window
               # walks, the receiver's STAR build, partition pass, partitioned probe, first pairs
               "config5_count_build": "jx_extract_kernel<true, true, 1, false, false, 3, false, 1>",
               "config5_count_probe": "jx_extract_kernel<false, true, 1, false, false, 3, false, 1>",
               "config5_emit_build": "jx_extract_kernel<true, true, 2, false, false, 3, false, 2>",
               "config5_emit_probe": "jx_extract_kernel<false, true, 2, false, false, 3, false, 2>",
               "config5_ent_build": "jx_ent_build_kernel", "config5_ent_part": "jx_ent_part_kernel",
               "config5_part_probe": "jx_part_probe_kernel", "config5_star_first": "jx_star_first_kernel"}
    out = {}
    for name, pat in classes.items():
        counters = {}
        for sub in ("fetch", "write", "sq", "sq2"):
            counters.update(pmc(os.path.join(a.src, sub), pat))
        if counters:
            if "FETCH_SIZE" in counters:
                counters["hbm_bytes_per_launch"] = counters["FETCH_SIZE"] * 1024 * 2 + counters.get("WRITE_SIZE", 0.0) * 1024
            out[name] = counters
    json.dump(out, open(a.prefix + "_pmc.json", "w"), indent=1, sort_keys=True)
    c3 = out.get("config3", {})
    if "FETCH_SIZE" in c3:
        fetch = c3["FETCH_SIZE"] * 1024 * 2          # KiB, half-counted on gfx950
        write = c3.get("WRITE_SIZE", 0.0) * 1024
        traffic = {"rows": a.rows, "hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch,
                   "write_bytes": write, "source": a.prefix + "_pmc.json",
                   "correction": "FETCH_SIZE(KiB)*1024*2 + WRITE_SIZE(KiB)*1024 (MI355X_MICROARCH.md HBM)"}
        json.dump(traffic, open(os.path.join(os.path.dirname(a.prefix), "hbm_traffic.json"), "w"), indent=1)
    counters = out
    stats2 = glob.glob(os.path.join(a.src, "kt2", "**", "*kernel_stats.csv"), recursive=True)
    if stats2:
        shutil.copy(stats2[0], a.prefix + "_config2_kernel_stats.csv")
    for f in ("bench.json", "bench2.json", "pytest_gpu.log"):
        p = os.path.join(a.src, f)
        if os.path.exists(p):
            shutil.copy(p, a.prefix + "_" + f)
    print(json.dumps(counters, indent=1))


if __name__ == "__main__":
    main()
