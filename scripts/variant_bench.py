"""Kernel time of several builds of libcqgpu.so in ONE process on the same generated
data (config 3: 1e8 Shape A+role rows, or --config 2), interleaved rounds:
    python scripts/variant_bench.py base f1 a0 ...   (base = cq_amd/lib/libcqgpu.so,
                                                       v = cq_amd/lib/libcqgpu_<v>.so)
Each library is loaded privately (RTLD_LOCAL) and uploads its own copy of the table."""
import argparse
import ctypes as C
import json
import os
import sys

import torch  # noqa: F401  (HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cq_amd import abi, datagen  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--config", type=int, default=3)
args = ap.parse_args()

role = args.config == 3
data = datagen.header_of(role) + bench.gen_rows(42, 0, args.rows, role, 8)
torch.zeros(1, device="cuda")


class Stats(C.Structure):
    _fields_ = [("scan_ms", C.c_double), ("total_ms", C.c_double), ("scan_bytes", C.c_uint64),
                ("records", C.c_uint64), ("groups", C.c_uint64), ("lds_spills", C.c_uint64),
                ("grid", C.c_int), ("path", C.c_int), ("retries", C.c_int),
                ("slow_records", C.c_uint64), ("passed", C.c_uint64), ("scan_kernel", C.c_int), ("wide", C.c_int)]


libs = {}
for v in args.variants:
    path = os.path.join(ROOT, "cq_amd", "lib", "libcqgpu.so" if v == "base" else f"libcqgpu_{v}.so")
    L = C.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
    L.cqgpu_table_from_bytes.restype = C.c_void_p
    L.cqgpu_table_from_bytes.argtypes = [C.c_void_p, C.c_size_t, abi.CsvConfig, C.c_uint64, C.c_char_p, C.c_size_t]
    L.cqgpu_query.restype = C.c_void_p
    L.cqgpu_query.argtypes = [C.POINTER(abi.Node), C.POINTER(C.c_void_p), C.c_int]
    L.cqgpu_result_free.argtypes = [C.c_void_p]
    L.cqgpu_last_stats.argtypes = [C.POINTER(Stats)]
    L.cqgpu_table_free.argtypes = [C.c_void_p]
    libs[v] = L
P, q = bench.build_plan("big.csv", args.config)
ast = C.pointer(q)
res = {v: [] for v in args.variants}
for r in range(args.rounds):
    for v, L in libs.items():
        t = L.cqgpu_table_from_bytes(C.cast(C.c_char_p(data), C.c_void_p), len(data), abi.csv_config(), 0, None, 0)
        arr = (C.c_void_p * 1)(t)
        ms = []
        st = Stats()
        for i in range(args.steps + 2):
            tp = L.cqgpu_query(ast, arr, 1)
            L.cqgpu_last_stats(C.byref(st))
            if i >= 2:
                ms.append(st.scan_ms)
            L.cqgpu_result_free(tp)
        L.cqgpu_table_free(t)
        torch.cuda.synchronize()
        m = sorted(ms)[len(ms) // 2]
        res[v].append(m)
        print(f"{v:8s} round {r}: kernel median {m:.4f} ms  (kernel kind {st.scan_kernel}, slow {st.slow_records}, "
              f"spills {st.lds_spills}, groups {st.groups})", flush=True)
print(json.dumps({v: min(x) for v, x in res.items()}))
