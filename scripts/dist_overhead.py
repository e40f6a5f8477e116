"""Where the N > 1 step's time goes beside the scan, at world size 1 over RCCL:
    torchrun --nproc-per-node 1 scripts/dist_overhead.py [rows]
wraps the library calls, collectives and synchronisations of
cq_amd.dist.scan_partitioned_dense with wall-clock timers and prints per-step totals."""
import collections
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
import cq_amd  # noqa: E402
from cq_amd import abi, datagen  # noqa: E402
import cq_amd.dist as D  # noqa: E402
import bench  # noqa: E402

data = datagen.header_of(True) + bench.gen_rows(42, 0, rows, True, 8)
table = cq_amd.Table.from_bytes(data, abi.csv_config())
P, q = bench.build_plan("big.csv", 3)
import ctypes as C  # noqa: E402
ast = C.pointer(q)
T = collections.defaultdict(float)
N = collections.Counter()


def wrap(obj, name, key):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[key] += time.perf_counter() - t0
            N[key] += 1
    setattr(obj, name, g)


for nm in ("__init__", "next", "put", "result"):
    wrap(D.DensePartial, nm, "lib." + nm)
wrap(D, "agree", "agree")
wrap(D, "_sync", "_sync")
wrap(D, "allgather_var", "allgather_var")
wrap(D.dist, "all_reduce", "dist.all_reduce")
wrap(D.dist, "reduce", "dist.reduce")
for i in range(3):
    tp = D.scan_partitioned_dense(ast, table)
    cq_amd.result_free(tp)
T.clear()
N.clear()
steps = 10
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(steps):
    tp = D.scan_partitioned_dense(ast, table)
    cq_amd.result_free(tp)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / steps
print(f"rows {rows}: step {el * 1e3:.3f} ms, scan kernel {cq_amd.stats()['scan_ms']:.3f} ms")
for k, v in sorted(T.items(), key=lambda kv: -kv[1]):
    print(f"  {k:20s} {v / steps * 1e3:8.3f} ms/step  ({N[k] / steps:.0f} calls)")
dist.destroy_process_group()
