"""Roofline of the scans of other plan shapes over config 3's file (1e8 rows of Shape
A+role, 3.89 GB), each the median of --steps launches (GPU box).  Entries are named by
PLAN; "kernel" is the kernel that actually ran (stats scan_kernel), so a label never
claims a kernel the plan did not take:
    python scripts/r6_other_kernels.py [--rows N] [--steps K] [--only TEXT]"""
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
path = "/tmp/r6_other.csv"
with open(path, "wb") as fh:
    fh.write(data)
t = cq_amd.Table.from_bytes(data)
del data
G = "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE %s GROUP BY role"
Q = {   # name -> (sql, forced kernel mode: 0 auto, 1 scan_kernel)
    "config 3": (G % "age > 30", 0),
    "config 3, general scan_kernel forced": (G % "age > 30", 1),
    "WHERE gender = 'f'": (G % "gender = 'f'", 0),
    "WHERE age BETWEEN 20 AND 40": (G % "age BETWEEN 20 AND 40", 0),
    "WHERE age BETWEEN 20 AND 40, general scan_kernel forced": (G % "age BETWEEN 20 AND 40", 1),
    "WHERE age > 30 AND gender = 'f'": (G % "age > 30 AND gender = 'f'", 0),
    "WHERE age > 30 AND gender = 'f', general scan_kernel forced": (G % "age > 30 AND gender = 'f'", 1),
    # (7 items: the WHERE program's stack holds the left side and at most 7 literals)
    "WHERE role IN (7 roles)": (G % ("role IN ('role_001', 'role_100', 'role_200', 'role_300', 'role_400', "
                                     "'role_500', 'role_999')"), 0),
    "WHERE role IN (7 roles), general scan_kernel forced": (G % ("role IN ('role_001', 'role_100', 'role_200', "
                                                                 "'role_300', 'role_400', 'role_500', "
                                                                 "'role_999')"), 1),
    "WHERE age < 20 OR gender != 'm'": (G % "age < 20 OR gender != 'm'", 0),
    "config 3 + MIN(height)": ("SELECT role, COUNT(*), SUM(height), MIN(height) FROM '{p}' WHERE age > 30 GROUP BY role", 0),
    "SELECT role, MIN(height) GROUP BY role": ("SELECT role, MIN(height) FROM '{p}' GROUP BY role", 0),
}
KIND = {0: "scan_kernel", 1: "lean_kernel", 2: "fast_kernel"}
out = {}
for name, (sql, force) in Q.items():
    if args.only not in name:
        continue
    q = sql.format(p=path)
    ms = []
    old = cq_amd.set_scan_kernel(force)
    with cqtest.Parsed(q) as ast:
        for i in range(args.steps + 2):
            got = cq_amd.query(ast, [t])
            st = cq_amd.stats()
            if i >= 2:
                ms.append(st["scan_ms"])
    cq_amd.set_scan_kernel(old)
    ms.sort()
    if not got or not ms or ms[len(ms) // 2] <= 0:
        out[name] = {"sql": sql.replace("'{p}'", "'big.csv'"), "error": cq_amd.last_error() or cq_amd.last_ineligible()}
        print(name, json.dumps(out[name]), flush=True)
        continue
    k = ms[len(ms) // 2]
    out[name] = {"sql": sql.replace("'{p}'", "'big.csv'"), "kernel": KIND.get(st["scan_kernel"], st["scan_kernel"]),
                 "kernel_ms": round(k, 4), "GB_per_s": round(nb / k / 1e6, 1), "frac": round(nb / k / 1e6 / 8000.0, 4),
                 "groups": st["groups"], "passed": st.get("passed"), "slow_records": st["slow_records"]}
    print(name, json.dumps(out[name]), flush=True)
print(json.dumps({"bytes": nb, "rows": args.rows, "results": out}))
t.close()
os.unlink(path)
