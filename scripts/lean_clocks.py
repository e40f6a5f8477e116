"""Per-phase shader cycles of lean_kernel (profiling build -DLEAN_CLK).

    CQ_AMD_LIB=cq_amd/lib/libcqgpu_clk.so python scripts/lean_clocks.py [rows]
"""
import ctypes as C
import os
import sys

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cq_amd
from cq_amd import abi, datagen

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
data = datagen.shape_a_bytes(rows, seed=42, with_role=True)
t = cq_amd.Table.from_bytes(data)
P = abi.Plan()
q = P.query([P.ident("role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("height")),
             P.func("AVG", P.ident("height"))], "x", where=P.cond(">", P.ident("age"), P.lit("30")), group_by=["role"])
L = cq_amd.lib()
L.cqgpu_debug_clocks.argtypes = [C.POINTER(C.c_ulonglong)]
names = ["wait data", "stage+classify", "walk+loads", "typing", "slow/stats", "aggregate", "window end", "-"]
for it in range(3):
    res = cq_amd.query(C.pointer(q), [t])
    st = cq_amd.stats()
    clk = (C.c_ulonglong * 8)()
    L.cqgpu_debug_clocks(clk)
windows = (len(data) + 3967) // 3968
tot = sum(clk)
print(f"rows {rows} scan_ms {st['scan_ms']:.3f} grid {st['grid']} windows {windows}")
for i, n in enumerate(names[:7]):
    print(f"{n:16s} {clk[i] / windows:10.0f} cyc/window/wave  {100 * clk[i] / tot:5.1f}%")
