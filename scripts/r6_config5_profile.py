"""Config 5's whole rank step (bench_join.typed_rank_step_leg) alone, for profiling:
    CQ_AMD_TIMING=1 rocprofv3 --kernel-trace --stats -d OUT -- python scripts/r6_config5_profile.py
(--rows: rows per side in total, --ranks)"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench_join as bj  # noqa: E402
from cq_amd import abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=500_000_000)
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--steps", type=int, default=5)
args = ap.parse_args()
P = abi.Plan()
q = P.query([P.ident("u.role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("o.price"))],
            "users.csv", alias="u", group_by=["u.role"],
            joins=[("orders.csv", "o", P.cond("=", P.ident("u.id"), P.ident("o.customer_id")), abi.JOIN_INNER)])
r = bj.typed_rank_step_leg(args.rows, args.ranks, args.steps, 1, 42, torch.device("cuda"), C.pointer(q))
print(json.dumps({k: v for k, v in r.items()}), flush=True)
