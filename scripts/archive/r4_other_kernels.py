"""Roofline of the non-specialised scans on config 3's file (1e8 rows, 3.89 GB):
lean_kernel (config 3 with WHERE gender = 'f'), scan_kernel (config 3 + MIN(height))
and fast_kernel (config 3 itself), each a median of --steps launches (GPU box):
    python scripts/r4_other_kernels.py [--rows N] [--steps K]"""
import argparse
import json
import os
import sys

import torch  # noqa: F401  (HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cq_amd  # noqa: E402
from cq_amd import datagen  # noqa: E402
import bench  # noqa: E402
import cqtest  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--only", default="", help="run the plans whose name holds this text")
args = ap.parse_args()
data = datagen.header_of(True) + bench.gen_rows(42, 0, args.rows, True, 8)
nb = len(data)
path = "/tmp/r4_other.csv"
with open(path, "wb") as fh:
    fh.write(data)
t = cq_amd.Table.from_bytes(data)
del data
Q = {
    "fast_kernel (config 3)": "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role",
    "lean_kernel (WHERE gender = 'f')": "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE gender = 'f' GROUP BY role",
    "scan_kernel (+ MIN(height))": "SELECT role, COUNT(*), SUM(height), MIN(height) FROM '{p}' WHERE age > 30 GROUP BY role",
    "scan_kernel (config 3 forced)": "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role",
    "scan_kernel (MIN(height) only)": "SELECT role, MIN(height) FROM '{p}' GROUP BY role",
}
FORCE = {"scan_kernel (config 3 forced)": 1}
KIND = {0: "scan_kernel", 1: "lean_kernel", 2: "fast_kernel"}
out = {}
for name, sql in Q.items():
    if args.only not in name:
        continue
    q = sql.format(p=path)
    ms = []
    old = cq_amd.set_scan_kernel(FORCE.get(name, 0))
    with cqtest.Parsed(q) as ast:
        for i in range(args.steps + 2):
            got = cq_amd.query(ast, [t])
            st = cq_amd.stats()
            if i >= 2:
                ms.append(st["scan_ms"])
    cq_amd.set_scan_kernel(old)
    ms.sort()
    k = ms[len(ms) // 2]
    out[name] = {"kernel": KIND.get(st["scan_kernel"], st["scan_kernel"]), "kernel_ms": round(k, 4),
                 "GB_per_s": round(nb / k / 1e6, 1), "frac": round(nb / k / 1e6 / 8000.0, 4),
                 "groups": st["groups"], "slow_records": st["slow_records"]}
    print(name, json.dumps(out[name]), flush=True)
print(json.dumps({"bytes": nb, "rows": args.rows, "results": out}))
t.close()
os.unlink(path)
