"""Host-side cost of one config-3 query step (cqgpu_query) beside its scan kernel:
    CQ_AMD_TIMING=1 python scripts/host_overhead.py [rows]
prints the library's phase times (stderr) and the Python-side step wall time."""
import ctypes as C
import os
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cq_amd  # noqa: E402
from cq_amd import abi, datagen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
data = datagen.shape_a_bytes(rows, seed=42, with_role=True)
t = cq_amd.Table.from_bytes(data)
P = abi.Plan()
q = P.query([P.ident("role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("height")),
             P.func("AVG", P.ident("height"))], "x", where=P.cond(">", P.ident("age"), P.lit("30")), group_by=["role"])
L = cq_amd.lib()
arr = (C.c_void_p * 1)(t.handle.value)
for it in range(8):
    t0 = time.perf_counter()
    tp = L.cqgpu_query(C.pointer(q), arr, 1)
    t1 = time.perf_counter()
    cq_amd.result_free(tp)
    t2 = time.perf_counter()
    st = cq_amd.stats()
    print(f"step {(t1 - t0) * 1e3:.3f} ms  free {(t2 - t1) * 1e3:.3f}  lib total {st['total_ms']:.3f}  scan {st['scan_ms']:.3f}",
          file=sys.stderr, flush=True)
