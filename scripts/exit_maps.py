"""Which HIP / HSA / RCCL runtime files a process maps after loading libcqgpu then
torch (ORDER=lib) or torch then libcqgpu (ORDER=torch) (GPU box)"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
order = os.environ.get("ORDER", "lib")
if order == "torch":
    import torch
    torch.empty(1, device="cuda")
import cq_amd
cq_amd.lib()
cq_amd.lib().cqgpu_cache_clear()
if order == "lib":
    import torch
    torch.empty(1, device="cuda")
    import torch.distributed  # noqa: F401
seen = set()
for ln in open("/proc/self/maps"):
    p = ln.split()[-1]
    if any(k in p for k in ("amdhip", "hsa-runtime", "rccl", "rocprofiler-register")) and p not in seen:
        seen.add(p)
        print(order, p)
