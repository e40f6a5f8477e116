"""Config-5 join (users x orders, --rows each) through several builds of libcqgpu.so in
ONE process, interleaved rounds; prints the scan time (extraction .. merge) per build:
    python scripts/join_variant_bench.py base v1 v2 ...  (v = cq_amd/lib/libcqgpu_<v>.so)"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cq_amd import abi  # noqa: E402
import bench_join as bj  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--rows", type=int, default=62_500_000)
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--rounds", type=int, default=2)
args = ap.parse_args()
torch.zeros(1, device="cuda")
n = args.rows
rng = np.random.default_rng([42, 0])
ub = b"id,name,age,role\n" + bj.users_shard(n, 0, rng)
ob = b"id,price,quantity,customer_id\n" + bj.orders_shard(n, 0, n, rng)


class Stats(C.Structure):
    _fields_ = [("scan_ms", C.c_double), ("total_ms", C.c_double), ("scan_bytes", C.c_uint64),
                ("records", C.c_uint64), ("groups", C.c_uint64), ("lds_spills", C.c_uint64),
                ("grid", C.c_int), ("path", C.c_int), ("retries", C.c_int),
                ("slow_records", C.c_uint64), ("passed", C.c_uint64), ("scan_kernel", C.c_int), ("wide", C.c_int)]


P = abi.Plan()
q = P.query([P.ident("u.role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("o.price"))],
            "users.csv", alias="u", group_by=["u.role"],
            joins=[("orders.csv", "o", P.cond("=", P.ident("u.id"), P.ident("o.customer_id")), abi.JOIN_INNER)])
ast = C.pointer(q)
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
res = {v: [] for v in args.variants}
for r in range(args.rounds):
    for v, L in libs.items():
        ut = L.cqgpu_table_from_bytes(C.cast(C.c_char_p(ub), C.c_void_p), len(ub), abi.csv_config(), 0, None, 0)
        ot = L.cqgpu_table_from_bytes(C.cast(C.c_char_p(ob), C.c_void_p), len(ob), abi.csv_config(), 0, None, 0)
        arr = (C.c_void_p * 2)(ut, ot)
        st = Stats()
        ms = []
        for i in range(args.steps + 2):
            tp = L.cqgpu_query(ast, arr, 2)
            L.cqgpu_last_stats(C.byref(st))
            if tp:
                L.cqgpu_result_free(tp)
            if i >= 2:
                ms.append(st.scan_ms)
        res[v].append(sorted(ms)[len(ms) // 2])
        print(v, "round", r, "scan_ms", round(res[v][-1], 4), "kernel", st.scan_kernel, flush=True)
        L.cqgpu_table_free(ut)
        L.cqgpu_table_free(ot)
print(json.dumps({v: round(min(x), 4) for v, x in res.items()}))
