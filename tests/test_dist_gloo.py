"""Multi-rank exchange of partial group states, world_size 2 over gloo on CPU.

The GPU path (bench.py --gpus N) uses the same cq_amd.dist.gather_blobs over
RCCL; here the blobs are synthetic byte strings of different sizes.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from cq_amd.dist import gather_blobs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = bytes([rank + 1]) * (1000 * (rank + 1) + rank) + b"end%d" % rank
        got = gather_blobs(mine, "cpu")
        empty = gather_blobs(b"" if rank == 0 else b"x", "cpu")
        q.put((rank, got, empty))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_blobs_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [bytes([r + 1]) * (1000 * (r + 1) + r) + b"end%d" % r for r in range(world)]
    for rank, got, empty in res:
        assert got == want, rank
        assert empty == [b"", b"x"]


def test_shard_bounds():
    from cq_amd.dist import shard_bounds
    assert shard_bounds([10, 20, 5], 0) == (0, 10)
    assert shard_bounds([10, 20, 5], 1) == (10, 30)
    assert shard_bounds([10, 20, 5], 2) == (30, 35)


def _xworker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from cq_amd.dist import exchange, exclusive_base
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r sends (r*10 + d) repeated d + r + 1 times to rank d (rank 0 sends nothing to 1)
        counts = [0 if (rank == 0 and d == 1) else d + rank + 1 for d in range(world)]
        send = torch.cat([torch.full((c,), rank * 10 + d, dtype=torch.uint8) for d, c in enumerate(counts)])
        recv, rc = exchange(send, counts)
        ids = torch.arange(sum(counts), dtype=torch.int64) + 1000 * rank
        rids, _ = exchange(ids, counts)
        q.put((rank, recv.tolist(), rc, rids.tolist(), exclusive_base(rank + 5)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_gloo(world):
    """the join repartition's all_to_all: slices land on their destination, in source-rank order"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xworker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, recv, rc, rids, base in res:
        want, wids = [], []
        for s in range(world):
            counts = [0 if (s == 0 and d == 1) else d + s + 1 for d in range(world)]
            want += [s * 10 + rank] * counts[rank]
            off = sum(counts[:rank])
            wids += [1000 * s + off + i for i in range(counts[rank])]
        assert recv == want, rank
        assert rids == wids, rank
        assert rc == [0 if (s == 0 and rank == 1) else rank + s + 1 for s in range(world)]
        assert base == sum(r + 5 for r in range(rank))


# ---------------------------------------------------------------- dense merge choreography
class _StandInPartial:
    """numpy stand-in for cq_amd.dist.DensePartial with the library's contract
    (cqgpu.h, cqgpu_partial_next): it asks for the key all_gather (8-byte count,
    then 8-byte keys), numbers distinct keys by first occurrence in the
    concatenation, asks for a MIN all-reduce of first positions, a SUM reduce of
    the representative cells masked to the rank holding the first row, a SUM
    reduce of the dense sums, and an all_gather of an (empty) side blob"""
    STAGES = ["keys", "min", "cell", "sumr", "side"]
    ABS = 0x7FFFFFFFFFFFFFFF

    def __init__(self, groups):
        import numpy as np
        self.np = np
        self.groups = groups                      # [(key int, cnt, sum, first, rep)]
        self.at = 0
        self.payload = None

    def next(self, result, sizes, rank, world):
        np = self.np
        if self.at > 0:
            done = self.STAGES[self.at - 1]
            r = result.cpu().numpy() if result is not None else None
            if done == "keys":
                assert sizes is not None and sum(sizes) == r.size
                keys, o = [], 0
                for sz in sizes:
                    m = int(r[o:o + 8].view(np.int64)[0])
                    keys += [int(x) for x in r[o + 8:o + 8 + 8 * m].view(np.int64)]
                    o += sz
                self.dense = {}
                for k in keys:
                    self.dense.setdefault(k, len(self.dense))
                self.order = list(self.dense)
                G = len(self.order)
                self.sum = np.zeros(3 * G)
                self.first = np.full(G, self.ABS, dtype=np.int64)
                self.rep = np.zeros(G, dtype=np.int64)
                for k, cnt, sm, first, rep in self.groups:
                    d = self.dense[k]
                    self.sum[3 * d:3 * d + 3] = (cnt, sm, cnt)
                    self.first[d], self.rep[d] = first, rep
                self.my_first = self.first.copy()
            elif done == "min":
                self.first = r.copy()
            elif done == "cell":
                self.rep = r.copy()
            elif done == "sumr":
                self.sum = r.copy()
        if self.at == len(self.STAGES):
            return 0, 0
        st = self.STAGES[self.at]
        self.at += 1
        if st == "keys":
            self.payload = np.array([len(self.groups)] + [g[0] for g in self.groups], dtype=np.int64).view(np.uint8)
            return 1, self.payload.size
        if st == "min":
            self.payload = self.first
            return 2, self.payload.size
        if st == "cell":
            self.payload = np.where(self.my_first == self.first, self.rep, 0)
            return 4, self.payload.size
        if st == "sumr":
            self.payload = self.sum
            return 5, self.payload.size
        self.payload = np.zeros(0, dtype=np.uint8)
        return 1, 0

    def put(self, buf):
        import torch
        buf.copy_(torch.from_numpy(self.payload.copy()))

    def result(self):
        rows = [(k, int(self.sum[3 * d]), float(self.sum[3 * d + 1]), int(self.first[d]), int(self.rep[d]))
                for d, k in enumerate(self.order)]
        return sorted(rows, key=lambda r: r[3])

    def free(self):
        pass


def _rank_groups(rank):
    # keys 0..9 spread unevenly; rank r holds positions [1000r, 1000r + 1000)
    import random
    rng = random.Random(rank)
    out = []
    for k in rng.sample(range(10), 3 + 2 * rank):
        out.append((k * 0x1000003 + 7, rng.randint(1, 50), rng.randint(-100, 100),
                    1000 * rank + rng.randint(0, 999), 10_000 * rank + k))
    return out


def _dworker(rank, world, port, q):
    import torch.distributed as dist
    from cq_amd.dist import dense_merge
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, dense_merge(_StandInPartial(_rank_groups(rank)), "cpu", "cpu")))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_dense_merge_choreography_gloo(world):
    """cq_amd.dist.dense_merge's collective loop (variable-size all_gathers, MIN
    all_reduce, SUM reduces to rank 0, as the library asks for them) over gloo"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dworker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res[r] is None for r in range(1, world))
    want = {}
    for r in range(world):
        for k, cnt, sm, first, rep in _rank_groups(r):
            w = want.setdefault(k, [k, 0, 0.0, 1 << 62, 0])
            w[1] += cnt
            w[2] += sm
            if first < w[3]:
                w[3], w[4] = first, rep
    assert res[0] == sorted((tuple(w) for w in want.values()), key=lambda r: r[3])


class _FailingPartial(_StandInPartial):
    """the stand-in, but this rank's payload step for the cell reduce raises (a
    rank-local failure such as a HIP out-of-memory on that rank only)"""

    def put(self, buf):
        if self.STAGES[self.at - 1] == "cell":
            raise RuntimeError("injected rank-local failure")
        super().put(buf)


def _fworker(rank, world, port, q, bad):
    import torch.distributed as dist
    from cq_amd.dist import PeerFailure, dense_merge
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cls = _FailingPartial if rank == bad else _StandInPartial
        try:
            dense_merge(cls(_rank_groups(rank)), "cpu", "cpu")
            q.put((rank, "returned"))
        except PeerFailure as e:
            q.put((rank, "peer-failure: " + str(e)))
        # every rank still reaches the same next collective (nobody was left inside one)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad", [(2, 1), (3, 0)])
def test_dense_merge_rank_local_failure_raises_everywhere(world, bad):
    """a rank-local failure inside the merge loop must not leave the other
    ranks blocked in a collective -- every rank raises PeerFailure after the same
    agreement, the failing rank naming its own error"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fworker, args=(r, world, port, q, bad)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r].startswith("peer-failure"), res
    assert "injected rank-local failure" in res[bad]


def _oworker(rank, world, port, q):
    """dist.outer_sets over gloo with the library's three calls replaced by fakes:
    level 1 (RIGHT / FULL) flags differ per rank, level 2 needs no set"""
    import torch.distributed as dist
    import cq_amd
    from cq_amd import dist as cd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    try:
        def matched(ast, tables, level):
            calls.append(("matched", level))
            if level == 2:
                return None
            return bytes(1 if i % (rank + 2) == 0 else 0 for i in range(23))
        cq_amd.join_outer_matched = matched
        cq_amd.join_outer_set = lambda level, flags, emit: calls.append(("set", level, bytes(flags), emit))
        cq_amd.join_outer_clear = lambda: calls.append(("clear",))
        cd.outer_sets(None, [], 2, "cpu")
        q.put((rank, calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_outer_sets_gloo(world):
    """a chain's later RIGHT / FULL level (cq_amd.dist.outer_sets): every rank gets the
    OR of the ranks' matched flags, rank 0 alone emits, a level that needs no set is
    skipped on every rank"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oworker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = bytes(1 if any(i % (r + 2) == 0 for r in range(world)) else 0 for i in range(23))
    for rank, calls in res.items():
        assert calls == [("clear",), ("matched", 1), ("set", 1, want, rank == 0), ("matched", 2)], (rank, calls)


def _omworker(rank, world, port, q):
    """dist.outer_sets where rank 1's level table holds fewer records"""
    import torch.distributed as dist
    import cq_amd
    from cq_amd import dist as cd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cq_amd.join_outer_matched = lambda ast, tables, level: bytes(23 if rank != 1 else 20)
        cq_amd.join_outer_set = lambda level, flags, emit: None
        cq_amd.join_outer_clear = lambda: None
        try:
            cd.outer_sets(None, [], 1, "cpu")
            q.put((rank, "no error"))
        except cd.PeerFailure as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_outer_sets_size_mismatch_gloo():
    """flags of different lengths (a chain table that differs between ranks) are a
    PeerFailure on every rank, never a mismatched all-reduce"""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_omworker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, msg in res.items():
        assert "record count differs" in msg, (rank, msg)


def _jworker(rank, world, port, q, kind):
    """cq_amd.dist.join_partitioned's sequence with the library's device calls faked:
    the routing mode agreed from every rank's class counts, global-id bases from each
    rank's own record count, both rebuilt sides marked replicated alike"""
    import ctypes as C
    import torch
    import torch.distributed as dist
    import cq_amd
    from cq_amd import abi
    from cq_amd import dist as cd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.synchronize = lambda *a, **k: None
        calls = []
        # ON keys per value class (NULL, number, string, date) on this rank, per side
        counts = {0: [1, 5 + rank, 0, 0], 1: [0, 3, 2 if kind == "mixed" and rank == 1 else 0, 0]}

        def plan2(ast, tables, side, n, r, mode=0):
            assert r == rank
            calls.append(("plan", side, mode))
            nown = 10 + 3 * rank + side
            nr = [nown // n + (1 if d < nown % n else 0) for d in range(n)]
            return [4 * x for x in nr], nr, nown, counts[side]
        cq_amd.route_plan2 = plan2
        cq_amd.route_fill = lambda tab, base, b, g: calls.append(("fill", base))
        cq_amd.table_from_routed = lambda *a: object()
        cq_amd.table_set_record_total = lambda t, total: calls.append(("total", total))
        cq_amd.table_set_key_stride = lambda t, s: None
        cq_amd.table_set_replicated = lambda t, mode, owner: calls.append(("rep", mode, owner))
        cq_amd.query_partial = lambda ast, tabs: b"blob%d" % rank
        cq_amd.merge_partials = lambda ast, blobs: list(blobs)
        cq_amd.join_outer_clear = lambda: None
        P = abi.Plan()
        on = None if kind == "cross" else P.cond("=", P.ident("a.k"), P.ident("b.k"))
        qn = P.query([P.func("COUNT", P.lit("*"))], "l.csv", alias="a", joins=[("r.csv", "b", on, abi.JOIN_INNER)])
        res = cd.join_partitioned(C.pointer(qn), "L", "R", b"k\n", b"k\n", "cpu", "cpu")
        q.put((rank, calls, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["plain", "mixed", "cross"])
@pytest.mark.parametrize("world", [2, 3])
def test_join_partitioned_routing_mode_gloo(world, kind):
    """every rank takes the same routing mode (cqgpu_route_major over the summed class
    counts: numbers vs a rank's STRING keys -> replicate, majority class 1), bases its
    global ids on the lower ranks' own record counts and marks its rebuilt sides alike,
    rank 0 the owner; a JOIN without ON skips the class agreement and marks side 1 whole"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_jworker, args=(r, world, port, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (c, m) for r, c, m in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mode = {"plain": 0, "mixed": 1, "cross": 0}[kind]
    for rank, (calls, merged) in res.items():
        plans = [c for c in calls if c[0] == "plan"]
        want_plans = ([] if kind == "cross" else [("plan", 0, 0), ("plan", 1, 0)]) + [("plan", 0, mode),
                                                                                     ("plan", 1, mode)]
        assert plans == want_plans, (rank, plans)
        for side in (0, 1):
            own = [10 + 3 * r + side for r in range(world)]
            fills = [c for c in calls if c[0] == "fill"]
            assert fills[side] == ("fill", sum(own[:rank])), (rank, fills)
            totals = [c for c in calls if c[0] == "total"]
            assert totals[side] == ("total", sum(own)), (rank, totals)
        reps = [c for c in calls if c[0] == "rep"]
        want = [("rep", 0, rank == 0), ("rep", 4, rank == 0)] if kind == "cross" else \
               [("rep", mode, rank == 0), ("rep", mode, rank == 0)]
        assert reps == want, (rank, reps)
        if rank == 0:
            assert merged == [b"blob%d" % r for r in range(world)]
