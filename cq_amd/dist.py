"""Multi-GPU plumbing for range-partitioned scans and joins (one process per GPU).

Each rank scans its own byte range of the file with cqgpu_query_partial; the
partial group states (opaque blobs, a few KB per thousand groups) are exchanged
with one all_gather over RCCL (torch.distributed "nccl") -- or gloo on CPU in
the tests -- and merged on rank 0 by cqgpu_merge_partials.  There is no
collective on the data path: the CSV bytes never leave their GPU.

The INNER JOIN has a real exchange step: each rank routes
its records of both inputs by join-key hash (cqgpu_route_plan / route_fill on the
device), one all_to_all_single of record bytes and one of global record ids move
them over xGMI, and each rank joins what it received (cqgpu_table_from_routed +
cqgpu_query_partial) before the same blob gather and merge.
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


def exchange(send: torch.Tensor, send_counts: list[int]) -> tuple[torch.Tensor, list[int]]:
    """all_to_all of variable-size slices of a 1-D tensor: rank r's slice d goes
    to rank d; the result is the received slices concatenated in source-rank order."""
    world = dist.get_world_size()
    dev = send.device
    sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc)
    recv_counts = [int(x) for x in rc.cpu().tolist()]
    recv = torch.empty(sum(recv_counts), dtype=send.dtype, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=recv_counts, input_split_sizes=list(send_counts))
    return recv, recv_counts


def exclusive_base(count: int, device: torch.device | str = "cpu") -> int:
    """sum of `count` over lower ranks (global record id of this rank's first record)"""
    world = dist.get_world_size()
    t = torch.tensor([count], dtype=torch.int64, device=device)
    allc = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(allc, t)
    return sum(int(x.item()) for x in allc[: dist.get_rank()])


def scan_partitioned(ast, table, comm_device: torch.device | str | None = None):
    """One range-partitioned query step (config 4): this rank's partial over its
    shard (cqgpu_query_partial), the blobs gathered (RCCL all_gather on a device
    group, gloo with comm_device="cpu"), merged on rank 0 (cqgpu_merge_partials).
    Returns the result pointer on rank 0 (free with cq_amd.result_free), None on
    the other ranks.  Every rank must call it (collectives inside)."""
    import cq_amd
    comm = torch.device(comm_device) if comm_device is not None else torch.device("cuda", torch.cuda.current_device())
    blob = cq_amd.query_partial(ast, [table])
    blobs = gather_blobs(blob, comm)
    if dist.get_rank() != 0:
        return None
    tp = cq_amd.merge_partials(ast, blobs)
    if not tp:
        raise RuntimeError(cq_amd.last_error() or "cqgpu_merge_partials failed")
    return tp


def join_partitioned(ast, lshard, rshard, lheader: bytes, rheader: bytes, device: torch.device | str,
                     comm_device: torch.device | str | None = None):
    """Repartitioned INNER JOIN over this rank's shards of both inputs.

    Returns the merged result pointer on rank 0 (free with cq_amd.result_free)
    and None elsewhere.  Every rank must call it (collectives inside).
    comm_device: where the collectives run -- `device` for RCCL (default); "cpu"
    stages the exchange through host memory for a gloo group (tests)."""
    import cq_amd
    world, rank = dist.get_world_size(), dist.get_rank()
    comm = torch.device(comm_device) if comm_device is not None else torch.device(device)
    routed = []
    for side, (tab, header) in enumerate(((lshard, lheader), (rshard, rheader))):
        nbytes, nrecs = cq_amd.route_plan(ast, [lshard, rshard], side, world)
        base = exclusive_base(sum(nrecs), comm)
        sb = torch.empty(max(sum(nbytes), 1), dtype=torch.uint8, device=device)
        sg = torch.empty(max(sum(nrecs), 1), dtype=torch.int64, device=device)
        cq_amd.route_fill(tab, base, sb.data_ptr(), sg.data_ptr())
        torch.cuda.synchronize(device)
        rb, _ = exchange(sb[: sum(nbytes)].to(comm), nbytes)
        rg, _ = exchange(sg[: sum(nrecs)].to(comm), nrecs)
        rb, rg = rb.to(device), rg.to(device)
        torch.cuda.synchronize(device)
        routed.append(cq_amd.table_from_routed(rb.data_ptr(), rb.numel(), rg.data_ptr(), rg.numel(), header))
    blob = cq_amd.query_partial(ast, routed)
    blobs = gather_blobs(blob, comm)
    if rank != 0:
        return None
    return cq_amd.merge_partials(ast, blobs)
