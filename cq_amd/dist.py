"""Multi-GPU plumbing for range-partitioned scans (one process per GPU).

Each rank scans its own byte range of the file with cqgpu_query_partial; the
partial group states (opaque blobs, a few KB per thousand groups) are exchanged
with one all_gather over RCCL (torch.distributed "nccl") -- or gloo on CPU in
the tests -- and merged on rank 0 by cqgpu_merge_partials.  There is no
collective on the data path: the CSV bytes never leave their GPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def gather_blobs(blob: bytes, device: torch.device | str = "cpu") -> list[bytes]:
    """all_gather of variable-size byte strings; every rank gets every rank's blob."""
    world = dist.get_world_size()
    n = torch.tensor([len(blob)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)
    lens = [int(s.item()) for s in sizes]
    mx = max(max(lens), 1)
    buf = torch.zeros(mx, dtype=torch.uint8, device=device)
    if blob:
        buf[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device)
    outs = [torch.empty(mx, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(outs, buf)
    return [bytes(o[:k].cpu().numpy()) for o, k in zip(outs, lens)]


def shard_bounds(sizes: list[int], rank: int) -> tuple[int, int]:
    """whole-file byte offset of rank's shard given every rank's shard size"""
    base = sum(sizes[:rank])
    return base, base + sizes[rank]
