"""Host-side cost of one config-3 step (GPU box): per-call wall time of
cqgpu_query + result_free with and without the stats read, and the library's
own phase clock (CQ_AMD_TIMING=1, on stderr).
    CQ_AMD_TIMING=1 python scripts/r4_host_phases.py [--rows N] [--steps K]"""
import argparse
import ctypes as C
import os
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cq_amd  # noqa: E402
from cq_amd import datagen  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
data = datagen.header_of(True) + bench.gen_rows(42, 0, args.rows, True, 8)
t = cq_amd.Table.from_bytes(data)
del data
L = cq_amd.lib()
P, q = bench.build_plan("big.csv", 3)
ast = C.pointer(q)
arr = (C.c_void_p * 1)(t.handle.value)
for mode in ("plain", "stats", "plain"):
    ts = []
    last = None
    for i in range(args.steps + 3):
        t0 = time.perf_counter()
        tp = L.cqgpu_query(ast, arr, 1)
        if mode == "stats":
            cq_amd.stats()
        if last:
            cq_amd.result_free(last)
        last = tp
        ts.append((time.perf_counter() - t0) * 1e3)
    cq_amd.result_free(last)
    ts = sorted(ts[3:])
    print(f"{mode:6s} ms per call: median {ts[len(ts) // 2]:.4f} min {ts[0]:.4f} max {ts[-1]:.4f}", flush=True)
t.close()
