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


class PeerFailure(RuntimeError):
    """A rank-local step failed on this rank or on a peer; every rank raises it
    together, after the same collectives, so no rank is left waiting in one."""


def agree(err, comm) -> None:
    """One MAX all-reduce of "this rank failed": raises PeerFailure on every rank
    when any rank's local step raised (err: that exception, or None)."""
    flag = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=comm)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if int(flag.item()):
        msg = f"rank {dist.get_rank()}: {err}" if err is not None else f"rank {dist.get_rank()}: a peer rank failed"
        raise PeerFailure(msg) from err


def _local(fn, *a):
    """(result, None) or (None, exception) of a rank-local step"""
    try:
        return fn(*a), None
    except Exception as e:  # reported to every rank by agree()
        return None, e


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
    blob, err = _local(cq_amd.query_partial, ast, [table])
    agree(err, comm)
    blobs = gather_blobs(blob, comm)
    if dist.get_rank() != 0:
        return None
    tp = cq_amd.merge_partials(ast, blobs)
    if not tp:
        raise RuntimeError(cq_amd.last_error() or "cqgpu_merge_partials failed")
    return tp


class DensePartial:
    """This rank's device-resident partial groups (cqgpu_partial_*): the library
    side of scan_partitioned_dense, kept behind four calls so the collective
    choreography can be exercised on CPU with a stand-in (tests/test_dist_gloo.py)."""

    KEYREC = 32

    def __init__(self, ast, table):
        import ctypes as C
        import cq_amd
        self.C, self.L, self.ast = C, cq_amd.lib(), ast
        arr = (C.c_void_p * 1)(table.handle.value)
        self.p = self.L.cqgpu_partial_new(ast, arr, 1)
        w = C.c_uint32(0)
        self.m = self.L.cqgpu_partial_keys(self.p, None, C.byref(w)) if self.p else 0
        self.W = w.value

    @property
    def ok(self) -> bool:
        return bool(self.p)

    def keys(self, device) -> torch.Tensor:
        t = torch.empty(max(self.m * self.KEYREC, 1), dtype=torch.uint8, device=device)
        if self.m:
            self.L.cqgpu_partial_keys(self.p, t.data_ptr(), None)
        return t[: self.m * self.KEYREC]

    def dict(self, all_keys: torch.Tensor, nall: int, mine: int) -> int:
        g = self.L.cqgpu_partial_dict(self.p, all_keys.data_ptr() if nall else None, nall, mine)
        if g < 0:
            import cq_amd
            raise RuntimeError(cq_amd.last_error())
        return int(g)

    def scatter(self, dsum, dfirst, drep):
        if self.L.cqgpu_partial_scatter(self.p, dsum.data_ptr(), dfirst.data_ptr(), drep.data_ptr()) != 0:
            import cq_amd
            raise RuntimeError(cq_amd.last_error())

    def mask_reps(self, dfirst, drep):
        if self.L.cqgpu_partial_mask_reps(self.p, dfirst.data_ptr(), drep.data_ptr()) != 0:
            import cq_amd
            raise RuntimeError(cq_amd.last_error())

    def finish(self, dsum, dfirst, drep):
        return self.L.cqgpu_partial_finish(self.p, self.ast, dsum.data_ptr(), dfirst.data_ptr(), drep.data_ptr())

    def free(self):
        if self.p:
            self.L.cqgpu_partial_free(self.p)
            self.p = None


def _sync(device):
    """order torch's stream (collectives, copies) before the library's own stream"""
    d = torch.device(device)
    if d.type == "cuda":
        torch.cuda.synchronize(d)


def dense_merge(part, device, comm_device=None):
    """The collective part of the device-side merge: one
    all_gather of the key records (sizes first), the dictionary and dense arrays
    on every rank, MIN all-reduce of first positions, SUM reduce of the dense sums
    and representative cells to rank 0, where `part.finish` builds the result.
    Returns that on rank 0, None elsewhere.  comm_device: where the collectives run
    (the device for RCCL; "cpu" stages through host memory for a gloo group)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    comm = torch.device(comm_device) if comm_device is not None else torch.device(device)
    mine, err = _local(part.keys, device)
    agree(err, comm)
    n = torch.tensor([part.m], dtype=torch.int64, device=comm)
    sizes = [torch.zeros(1, dtype=torch.int64, device=comm) for _ in range(world)]
    dist.all_gather(sizes, n)
    counts = [int(x.item()) for x in sizes]                  # a few integers, not the blobs
    if sum(counts) >= DICT_MAX_KEYS:
        return NOT_DENSE                                     # every rank sees the same total
    kb = part.KEYREC
    mx = max(max(counts), 1) * kb
    buf = torch.zeros(mx, dtype=torch.uint8, device=comm)
    buf[: mine.numel()] = mine.to(comm)
    outs = [torch.empty(mx, dtype=torch.uint8, device=comm) for _ in range(world)]
    dist.all_gather(outs, buf)
    all_keys = torch.cat([o[: c * kb] for o, c in zip(outs, counts)]).to(device)
    nall, off = sum(counts), sum(counts[:rank])
    _sync(device)          # the library's stream reads what torch's stream wrote

    def local_dense():
        g = part.dict(all_keys, nall, off)
        ds = torch.empty(max(g * part.W, 1), dtype=torch.float64, device=device)
        df = torch.empty(max(g, 1), dtype=torch.int64, device=device)
        dr = torch.empty(max(2 * g, 1), dtype=torch.int64, device=device)
        part.scatter(ds, df, dr)
        return ds, df, dr
    out, err = _local(local_dense)
    agree(err, comm)
    dsum, dfirst, drep = out
    f = dfirst.to(comm)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    dfirst.copy_(f)
    _sync(device)
    _, err = _local(part.mask_reps, dfirst, drep)
    agree(err, comm)
    s, r = dsum.to(comm), drep.to(comm)
    dist.reduce(s, 0, op=dist.ReduceOp.SUM)
    dist.reduce(r, 0, op=dist.ReduceOp.SUM)
    if rank != 0:
        return None
    dsum.copy_(s)
    drep.copy_(r)
    _sync(device)
    return part.finish(dsum, dfirst, drep)


DICT_MAX_KEYS = 1 << 29      # cqgpu_partial_dict's limit: more keys take the blob path
NOT_DENSE = object()


def scan_partitioned_dense(ast, table, comm_device=None):
    """One range-partitioned query step with the merge on the devices (config 4):
    this rank's scan keeps its groups in HBM (cqgpu_partial_new), the ranks agree
    on the path (a MIN all-reduce of "eligible"), and dense_merge reduces the
    groups over RCCL.  Plans outside the dense path (MIN/MAX, plain columns other
    than the group key, long text keys) take scan_partitioned's blobs."""
    import cq_amd
    device = torch.device("cuda", torch.cuda.current_device())
    comm = torch.device(comm_device) if comm_device is not None else device
    part, err = _local(DensePartial, ast, table)
    agree(err, comm)
    try:
        ok = torch.tensor([1 if part.ok else 0], dtype=torch.int32, device=comm)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            part.free()
            return scan_partitioned(ast, table, comm_device)
        tp = dense_merge(part, device, comm_device)
        if tp is NOT_DENSE:
            part.free()
            return scan_partitioned(ast, table, comm_device)
        if dist.get_rank() == 0 and not tp:
            raise RuntimeError(cq_amd.last_error() or "cqgpu_partial_finish failed")
        return tp
    finally:
        part.free()


def join_partitioned(ast, lshard, rshard, lheader: bytes, rheader: bytes, device: torch.device | str,
                     comm_device: torch.device | str | None = None):
    """Repartitioned INNER JOIN over this rank's shards of both inputs.

    Returns the merged result pointer on rank 0 (free with cq_amd.result_free)
    and None elsewhere.  Every rank must call it (collectives inside).
    comm_device: where the collectives run -- `device` for RCCL (default); "cpu"
    stages the exchange through host memory for a gloo group (tests)."""
    import cq_amd
    world, rank = dist.get_world_size(), dist.get_rank()
    if world == 1:
        # one rank: every record routes to itself in its own order (the stable sort by
        # destination is the identity), so the shards are already the routed tables
        # and their record ids the local row indexes
        return cq_amd.merge_partials(ast, [cq_amd.query_partial(ast, [lshard, rshard])])
    comm = torch.device(comm_device) if comm_device is not None else torch.device(device)
    routed = []
    for side, (tab, header) in enumerate(((lshard, lheader), (rshard, rheader))):
        plan, err = _local(cq_amd.route_plan, ast, [lshard, rshard], side, world)
        agree(err, comm)
        nbytes, nrecs = plan
        base = exclusive_base(sum(nrecs), comm)

        def fill():
            b = torch.empty(max(sum(nbytes), 1), dtype=torch.uint8, device=device)
            g = torch.empty(max(sum(nrecs), 1), dtype=torch.int64, device=device)
            cq_amd.route_fill(tab, base, b.data_ptr(), g.data_ptr())
            torch.cuda.synchronize(device)
            return b, g
        out, err = _local(fill)
        agree(err, comm)
        sb, sg = out
        rb, _ = exchange(sb[: sum(nbytes)].to(comm), nbytes)
        rg, _ = exchange(sg[: sum(nrecs)].to(comm), nrecs)
        rb, rg = rb.to(device), rg.to(device)
        torch.cuda.synchronize(device)
        t, err = _local(cq_amd.table_from_routed, rb.data_ptr(), rb.numel(), rg.data_ptr(), rg.numel(), header)
        agree(err, comm)
        routed.append(t)
    blob, err = _local(cq_amd.query_partial, ast, routed)
    agree(err, comm)
    blobs = gather_blobs(blob, comm)
    if rank != 0:
        return None
    return cq_amd.merge_partials(ast, blobs)
