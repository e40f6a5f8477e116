"""Per-kernel PMC averages of the config-5 rank share (scripts/r5_join_ab.py under
rocprofv3 --pmc, one pass per counter group) and the HBM traffic of one step:
    python scripts/r5_config5_pmc.py gpurun_out/<tag> profiles/r5_config5_pmc.json [--traffic profiles/config5_traffic.json]
Traffic per launch = FETCH_SIZE (KiB, half-counted on gfx950 for wide streaming
reads) x 1024 x 2 + WRITE_SIZE (KiB) x 1024 (MI355X_MICROARCH.md 'HBM'); the step's
traffic is the sum over its jx_* kernels."""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("out")
ap.add_argument("--traffic", default=None)
ap.add_argument("--rows-total", type=int, default=500_000_000)
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--rank-bytes", type=int, default=None, help="rank 0's routed bytes (bench config5 rank_bytes)")
a = ap.parse_args()
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(a.src, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "jx_" not in k:
            continue
        name = k.split("(")[0].replace("void ", "").replace("cq::fast::", "")
        per[(name, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for (n, c), v in per.items():
        res[n][c].extend(v.values())
out = {}
step = 0.0
for n, cs in res.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in d:
        d["hbm_bytes_per_launch"] = d["FETCH_SIZE"] * 1024 * 2 + d.get("WRITE_SIZE", 0.0) * 1024
        step += d["hbm_bytes_per_launch"]
    if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
        d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
    out[n] = d
doc = {"source": a.src, "kernels": out, "hbm_bytes_per_step": step,
       "correction": "FETCH_SIZE(KiB)*1024*2 + WRITE_SIZE(KiB)*1024 per launch, summed over the step's jx_* kernels"}
json.dump(doc, open(a.out, "w"), indent=1)
print(json.dumps({k: round(v.get("hbm_bytes_per_launch", 0) / 1e9, 3) for k, v in out.items()}), "step GB", step / 1e9)
if a.traffic:
    json.dump({"rows_total": a.rows_total, "ranks": a.ranks, "rank_bytes": a.rank_bytes,
               "hbm_bytes_per_step": step, "source": a.out}, open(a.traffic, "w"), indent=1)
