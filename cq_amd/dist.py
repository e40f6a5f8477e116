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


def base_and_total(count: int, device: torch.device | str = "cpu") -> tuple[int, int]:
    """(sum of `count` over lower ranks, sum over all ranks): the global record id of
    this rank's first record and the whole input's record count"""
    world = dist.get_world_size()
    t = torch.tensor([count], dtype=torch.int64, device=device)
    allc = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(allc, t)
    counts = [int(x) for x in torch.cat(allc).cpu().tolist()]
    return sum(counts[: dist.get_rank()]), sum(counts)


def exclusive_base(count: int, device: torch.device | str = "cpu") -> int:
    """sum of `count` over lower ranks (global record id of this rank's first record)"""
    return base_and_total(count, device)[0]


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


# cqgpu_coll ops (cqgpu.h)
DONE, ALLGATHER, ALLREDUCE_MIN_I64, ALLREDUCE_SUM_F64, REDUCE_SUM_I64, REDUCE_SUM_F64, DECLINE = range(7)
NOT_DENSE = object()


class DensePartial:
    """This rank's device-resident partial groups (cqgpu_partial_*): the library
    asks for one collective at a time (next), fills its payload (put) and takes
    the result on the following next; kept behind these calls so the collective
    loop can be exercised on CPU with a stand-in (tests/test_dist_gloo.py)."""

    def __init__(self, ast, table):
        import ctypes as C
        import cq_amd
        self.C, self.L, self.ast, self.cq = C, cq_amd.lib(), ast, cq_amd
        arr = (C.c_void_p * 1)(table.handle.value)
        self.p = self.L.cqgpu_partial_new(ast, arr, 1)

    @property
    def ok(self) -> bool:
        return bool(self.p)

    def next(self, result, sizes, rank, world):
        """(op, count) of the next collective, after taking `result` (a device
        tensor, or None) of the last one; `sizes`: per-rank byte counts of an ALLGATHER"""
        C = self.C
        c = self.cq.Coll()
        arr = (C.c_uint64 * world)(*sizes) if sizes is not None else None
        ptr = result.data_ptr() if result is not None and result.numel() else None
        if self.L.cqgpu_partial_next(self.p, ptr, arr, rank, world, C.byref(c)) != 0:
            raise RuntimeError(self.cq.last_error() or "cqgpu_partial_next failed")
        return c.op, c.count

    def put(self, buf):
        if self.L.cqgpu_partial_put(self.p, buf.data_ptr() if buf.numel() else None) != 0:
            raise RuntimeError(self.cq.last_error() or "cqgpu_partial_put failed")

    def result(self):
        return self.L.cqgpu_partial_result(self.p, self.ast)

    def free(self):
        if self.p:
            self.L.cqgpu_partial_free(self.p)
            self.p = None


def _sync(device):
    """order torch's stream (collectives, copies) before the library's own stream"""
    d = torch.device(device)
    if d.type == "cuda":
        torch.cuda.synchronize(d)


def allgather_var(buf: torch.Tensor, comm) -> tuple[torch.Tensor, list[int]]:
    """all_gather of a variable-length uint8 tensor: the ranks' payloads
    concatenated in rank order, and their lengths"""
    world = dist.get_world_size()
    n = torch.tensor([buf.numel()], dtype=torch.int64, device=comm)
    sizes = torch.empty(world, dtype=torch.int64, device=comm)
    dist.all_gather_into_tensor(sizes, n)
    lens = sizes.tolist()                     # one device-to-host transfer
    mx = max(max(lens), 1)
    pad = torch.empty(mx, dtype=torch.uint8, device=comm)
    pad[: buf.numel()] = buf.to(comm)         # (bytes past a rank's length are never read)
    out = torch.empty(world * mx, dtype=torch.uint8, device=comm)
    dist.all_gather_into_tensor(out, pad)
    if all(k == mx for k in lens):
        return out, lens
    return torch.cat([out[r * mx:r * mx + k] for r, k in enumerate(lens)]), lens


_DTYPES = {ALLGATHER: torch.uint8, ALLREDUCE_MIN_I64: torch.int64, ALLREDUCE_SUM_F64: torch.float64,
           REDUCE_SUM_I64: torch.int64, REDUCE_SUM_F64: torch.float64}


def dense_merge(part, device, comm_device=None):
    """Run the collectives the library asks for: the key
    all_gather, MIN all-reduces of positions and order keys, SUM reduces of the
    dense planes and the owners' cells, over RCCL on device tensors (or gloo
    through host memory with comm_device="cpu").  Returns cqgpu_partial_result on
    rank 0, None elsewhere, NOT_DENSE when the library declines (every rank
    declines together: the decision depends on the gathered keys only)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    comm = torch.device(comm_device) if comm_device is not None else torch.device(device)
    result, sizes = None, None

    def step(result, sizes):
        """take the last result, learn the next collective and fill its payload (one
        rank-local step, so one agreement per collective; cqgpu_partial_put returns
        after its copy has completed, so the payload is ready for torch's stream)"""
        op, count = part.next(result, sizes, rank, world)
        if op in (DONE, DECLINE):
            return op, count, None
        buf = torch.empty(max(count, 1), dtype=_DTYPES[op], device=device)[:count]
        part.put(buf)
        return op, count, buf

    while True:
        out, err = _local(step, result, sizes)
        agree(err, comm)
        op, count, buf = out
        if op == DONE:
            break
        if op == DECLINE:
            return NOT_DENSE
        sizes = None
        if op == ALLGATHER:
            result, sizes = allgather_var(buf, comm)
        elif count == 0:                     # every rank has the same G: skip together
            result = buf
        else:
            x = buf.to(comm)
            if op == ALLREDUCE_MIN_I64:
                dist.all_reduce(x, op=dist.ReduceOp.MIN)
            elif op == ALLREDUCE_SUM_F64:
                dist.all_reduce(x, op=dist.ReduceOp.SUM)
            else:
                dist.reduce(x, 0, op=dist.ReduceOp.SUM)
            result = x
        result = result.to(device)
        _sync(device)
    if rank != 0:
        return None
    return part.result()


def scan_partitioned_dense(ast, table, comm_device=None):
    """One range-partitioned query step with the merge on the devices (config 4):
    this rank's scan keeps its groups in HBM (cqgpu_partial_new), the ranks agree
    on the path (a MIN all-reduce of "eligible"), and dense_merge reduces the
    groups over RCCL.  Plans outside the dense path (MEDIAN, MIN/MAX over long
    text, too many keys) take scan_partitioned's blobs."""
    import cq_amd
    device = torch.device("cuda", torch.cuda.current_device())
    comm = torch.device(comm_device) if comm_device is not None else device
    part, err = _local(DensePartial, ast, table)
    # one MAX all-reduce for both questions: did any rank fail, is any rank off the dense path
    flags = torch.tensor([0 if err is None else 1, 0 if (err is None and part.ok) else 1], dtype=torch.int32,
                         device=comm)
    dist.all_reduce(flags, op=dist.ReduceOp.MAX)
    failed, declined = flags.tolist()
    if failed:
        if part is not None:
            part.free()
        msg = f"rank {dist.get_rank()}: {err}" if err is not None else f"rank {dist.get_rank()}: a peer rank failed"
        raise PeerFailure(msg) from err
    try:
        if declined:
            part.free()
            return scan_partitioned(ast, table, comm_device)
        tp = dense_merge(part, device, comm_device)
        if tp is NOT_DENSE:
            part.free()
            return scan_partitioned(ast, table, comm_device)
        if dist.get_rank() == 0 and not tp:
            raise RuntimeError(cq_amd.last_error() or "cqgpu_partial_result failed")
        return tp
    finally:
        part.free()


def init_library_comm(device: torch.device | str | None = None) -> None:
    """Create the library's own RCCL communicator on this rank's device (once per
    process, before the first scan_partitioned_rccl): rank 0's unique id reaches
    the other ranks through the torch.distributed group (any backend)."""
    import cq_amd
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    comm = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    uid = cq_amd.comm_unique_id() if rank == 0 else bytes(cq_amd.COMM_ID_BYTES)
    t = torch.frombuffer(bytearray(uid), dtype=torch.uint8).to(comm)
    dist.broadcast(t, 0)
    cq_amd.comm_init(bytes(t.cpu().numpy()), rank, world)


_HOST_COMM = {}      # device -> the ctypes callback (kept alive while the library holds it)

_GLOO_DT = {0: torch.uint8, 1: torch.int32, 2: torch.int64, 3: torch.int64, 4: torch.float64}
_ELEM = {0: 1, 1: 4, 2: 8, 3: 8, 4: 8}


def init_host_comm() -> None:
    """TEST backend of the library's N > 1 step (cqgpu_comm_init_host): the library
    stages each collective's device buffers through host memory and calls back here,
    where torch.distributed (gloo) runs it.  The library's own protocol code --
    cqgpu_dist_query's gather-merge / dense / blob merges and cqgpu_dist_join's
    exchange, outer sets and status agreements -- then runs unchanged at world size
    > 1 on a one-GPU box (several ranks sharing the device, which RCCL refuses).
    u32 / u64 travel as int32 / int64 (their reductions here are MAX over small
    values and SUM of counts); byte movements are dtype-blind."""
    import ctypes as C
    import sys
    import numpy as np
    import cq_amd
    rank, world = dist.get_rank(), dist.get_world_size()
    pending, own_send, own_recv = [], [], []
    ops = {0: dist.ReduceOp.SUM, 1: dist.ReduceOp.MIN, 2: dist.ReduceOp.MAX}

    def raw(ptr, nbytes):
        if nbytes == 0:
            return torch.zeros(0, dtype=torch.uint8)
        return torch.from_numpy(np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(ptr)))

    def view(ptr, count, dtype):
        return raw(ptr, count * _ELEM[dtype]).view(_GLOO_DT[dtype])

    def fn(user, op, dtype, redop, peer, send, recv, count):
        try:
            nb = count * _ELEM[dtype]
            if op == 1:                                   # ALLREDUCE (in place)
                if count:
                    dist.all_reduce(view(send, count, dtype), op=ops[redop])
            elif op == 2:                                 # ALLGATHER
                if nb:
                    tmp = [torch.empty(nb, dtype=torch.uint8) for _ in range(world)]
                    dist.all_gather(tmp, raw(send, nb).clone())
                    raw(recv, nb * world).copy_(torch.cat(tmp))
            elif op == 3:                                 # REDUCE to `peer` (in place)
                if count:
                    dist.reduce(view(send, count, dtype), dst=peer, op=ops[redop])
            elif op == 4:                                 # BROADCAST from `peer` (in place)
                if count:
                    dist.broadcast(view(send, count, dtype), src=peer)
            elif op == 5:                                 # SEND (posted until GROUP_END)
                if nb and peer == rank:                   # (gloo has no self transfer: matched in order below)
                    own_send.append(raw(send, nb).clone())
                elif nb:
                    pending.append(dist.isend(raw(send, nb), dst=peer))
            elif op == 6:                                 # RECV (posted until GROUP_END)
                if nb and peer == rank:
                    own_recv.append(raw(recv, nb))
                elif nb:
                    pending.append(dist.irecv(raw(recv, nb), src=peer))
            elif op == 7:                                 # GROUP_END
                for w in pending:
                    w.wait()
                pending.clear()
                if len(own_send) != len(own_recv):
                    raise RuntimeError("unmatched transfers to self")
                for a, b in zip(own_send, own_recv):
                    b.copy_(a)
                own_send.clear()
                own_recv.clear()
            else:
                return 1
            return 0
        except Exception as e:                            # (the library fails the step)
            print(f"cq_amd host collective op {op} on rank {rank}: {e!r}", file=sys.stderr, flush=True)
            return 1

    cb = cq_amd.COLL_FN(fn)
    _HOST_COMM[torch.cuda.current_device() if torch.cuda.is_available() else 0] = cb
    if cq_amd.lib().cqgpu_comm_init_host(rank, world, cb, None) != 0:
        raise RuntimeError(cq_amd.last_error() or "cqgpu_comm_init_host failed")


def scan_partitioned_rccl(ast, table):
    """One range-partitioned query step with the whole merge inside the library
    (cqgpu_dist_query over its own RCCL communicator, init_library_comm): no
    Python collective, no per-stage host agreement.  Returns (result pointer on
    rank 0 / None elsewhere, path name); raises PeerFailure on EVERY rank when any
    rank failed.  Every rank must call it."""
    import cq_amd
    tp, status, path = cq_amd.dist_query_raw(ast, table)
    if status != 0:
        raise PeerFailure(f"rank {dist.get_rank()}: {cq_amd.last_error()}")
    if dist.get_rank() == 0 and tp is None:
        raise RuntimeError(cq_amd.last_error() or cq_amd.last_ineligible() or "cqgpu_dist_query failed")
    return tp, cq_amd.DIST_PATHS.get(path, str(path))


def join_partitioned_rccl(ast, lshard, rshard, rest=()):
    """The repartitioned JOIN step with the whole exchange inside the library
    (cqgpu_dist_join over its own RCCL communicator, init_library_comm): device
    routing, one grouped send / recv per side, rebuilt sides, local join, partials
    merged on rank 0.  Returns the result pointer on rank 0 (None elsewhere); raises
    PeerFailure on EVERY rank when any rank failed.  Every rank must call it."""
    import cq_amd
    tp, status = cq_amd.dist_join_raw(ast, [lshard, rshard, *rest])
    if status != 0:
        raise PeerFailure(cq_amd.last_error() or "cqgpu_dist_join failed")
    return tp


def outer_sets(ast, tables, nlevels: int, comm) -> None:
    """A chain's later RIGHT / FULL levels (cqgpu_join_outer_* in include/cqgpu.h): per
    level, every rank's matched flags over the level's whole table, OR-ed by a MAX
    all-reduce over bytes; rank 0's partial carries the records no rank matched.
    Every rank must call it, before query_partial."""
    import cq_amd
    cq_amd.join_outer_clear()
    for j in range(1, nlevels + 1):
        flags, err = _local(cq_amd.join_outer_matched, ast, tables, j)
        agree(err, comm)
        if flags is None:                  # (decided by the plan alone: the same on every rank)
            continue
        # the level's table is whole on every rank: the same record count, checked
        # before the byte all-reduce (mismatched sizes would not reduce)
        n = torch.tensor([len(flags), -len(flags)], dtype=torch.int64, device=comm)
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
        if int(n[0]) != -int(n[1]):
            raise PeerFailure(f"rank {dist.get_rank()}: a chain table's record count differs between ranks")
        t = torch.frombuffer(bytearray(flags), dtype=torch.uint8).to(comm) if flags else \
            torch.zeros(0, dtype=torch.uint8, device=comm)
        if t.numel():
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        _, err = _local(cq_amd.join_outer_set, j, bytes(t.cpu().numpy()), dist.get_rank() == 0)
        agree(err, comm)


def first_join_cross(ast) -> bool:
    """the plan's first JOIN has no ON (a cross join: side 1 goes to every rank)"""
    q = ast.contents.u.q
    return q.join_count > 0 and not q.joins[0].contents.u.join.on


def join_partitioned(ast, lshard, rshard, lheader: bytes, rheader: bytes, device: torch.device | str,
                     comm_device: torch.device | str | None = None, rest=()):
    """Repartitioned JOIN over this rank's shards of both inputs of the first JOIN.

    rest: a chain's later JOIN tables, each whole on every rank (the joined rows of
    the first level are spread over the ranks by its key; each rank joins its own
    with the whole next table).
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
        comm = torch.device(comm_device) if comm_device is not None else torch.device(device)
        try:
            outer_sets(ast, [lshard, rshard, *rest], len(rest), comm)
            return cq_amd.merge_partials(ast, [cq_amd.query_partial(ast, [lshard, rshard, *rest])])
        finally:
            cq_amd.join_outer_clear()
    comm = torch.device(comm_device) if comm_device is not None else torch.device(device)
    cross = first_join_cross(ast)
    mode = 0
    if not cross:
        # the routing mode (cqgpu_route_plan2): keys of several value classes route the
        # majority class by key and replicate the others -- agreed from every rank's
        # class counts of both sides before anything moves
        counts, err = _local(lambda: [cq_amd.route_plan2(ast, [lshard, rshard], s, world, rank)[3]
                                      for s in (0, 1)])
        agree(err, comm)
        t = torch.tensor(counts[0] + counts[1], dtype=torch.int64, device=comm)
        dist.all_reduce(t)
        tot = [int(x) for x in t.cpu()]
        mode = cq_amd.route_major(tot[:4], tot[4:])
    routed = []
    for side, (tab, header) in enumerate(((lshard, lheader), (rshard, rheader))):
        plan, err = _local(cq_amd.route_plan2, ast, [lshard, rshard], side, world, rank, mode)
        agree(err, comm)
        nbytes, nrecs, nown, _ = plan
        base, total = base_and_total(nown, comm)

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
        if t is not None:
            _, e2 = _local(cq_amd.table_set_record_total, t, total)
            _, e3 = _local(cq_amd.table_set_key_stride, t, world)   # whole keys routed by key mod N
            _, e4 = _local(cq_amd.table_set_replicated, t, (4 if side == 1 else 0) if cross else mode, rank == 0)
            err = err or e2 or e3 or e4
        agree(err, comm)
        routed.append(t)
    try:
        outer_sets(ast, routed + list(rest), len(rest), comm)
        blob, err = _local(cq_amd.query_partial, ast, routed + list(rest))
    finally:
        cq_amd.join_outer_clear()
    agree(err, comm)
    blobs = gather_blobs(blob, comm)
    if rank != 0:
        return None
    return cq_amd.merge_partials(ast, blobs)


def typed_join_local(ast, lshards, rshards, stats: dict | None = None):
    """The typed exchange (include/cqgpu.h cqgpu_typed_*) over N simulated ranks held
    by this one process on one GPU, in cqgpu_dist_join's order: every rank's count
    passes, the global ids' bases and qbase, every rank's emit passes, the regions
    gathered per destination (a device copy standing in for the xGMI transfer), every
    destination's STAR partial.  Returns the N blobs for cq_amd.merge_partials, or None
    when the plan or the data leave the typed exchange (the caller takes the CSV
    exchange).  stats (optional) receives the entry counts per rank."""
    import cq_amd
    n = len(lshards)
    pair = lambda r: [lshards[r], rshards[r]]  # noqa: E731
    if not cq_amd.typed_plan(ast, pair(0)):
        return None
    smin = min(cq_amd.typed_sample_kmin(ast, pair(r)) for r in range(n))
    qbase = 0 if smin == (1 << 64) - 1 else smin // n
    for attempt in range(2):
        flags, kmin, kmax, cu, co, nrec = 0, (1 << 64) - 1, 0, [], [], []
        for r in range(n):
            nu, c1, kr, f1 = cq_amd.typed_count(ast, pair(r), 0, n, qbase)
            _, c2, _, f2 = cq_amd.typed_count(ast, pair(r), 1, n, qbase)
            flags |= f1 | f2
            kmin, kmax = min(kmin, kr[0]), max(kmax, kr[1])
            cu.append(c1)
            co.append(c2)
            nrec.append(nu)
        if flags & (1 | 8) or (flags & 16 and attempt == 1):
            return None
        if flags & 16:
            qbase = kmin // n
            continue
        break
    if sum(nrec) >= 1 << 32:
        return None
    if kmin > kmax:                                # no build keys at all
        kmin = kmax = qbase * n
    qoff = kmin // n - qbase
    rng = kmax // n - kmin // n + 1
    recv_u = [sum(cu[s][d] for s in range(n)) for d in range(n)]
    recv_o = [sum(co[s][d] for s in range(n)) for d in range(n)]
    if rng > 4 * min(recv_u) + 1024:               # not a dense key range on every rank
        return None
    ef = 0
    for r in range(n):
        ef |= cq_amd.typed_send(ast, pair(r), 0, sum(nrec[:r]))
        ef |= cq_amd.typed_send(ast, pair(r), 1, 0)
    if ef:
        return None
    blobs = []
    for d in range(n):
        bu = torch.empty(max(recv_u[d], 1) * 16, dtype=torch.uint8, device="cuda")
        bo = torch.empty(max(recv_o[d], 1) * 8, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        nu = cq_amd.typed_gather(lshards, d, bu.data_ptr(), recv_u[d])
        no = cq_amd.typed_gather(rshards, d, bo.data_ptr(), recv_o[d])
        blob = cq_amd.typed_partial(ast, pair(d), bu.data_ptr(), nu, bo.data_ptr(), no, qoff, rng)
        if blob is None:
            return None
        blobs.append(blob)
    if stats is not None:
        stats.update({"sent_entries_u": [sum(x) for x in cu], "sent_entries_o": [sum(x) for x in co],
                      "recv_entries_u": recv_u, "recv_entries_o": recv_o, "qoff": qoff, "range": rng,
                      "qbase": qbase, "attempts": attempt + 1})
    return blobs
