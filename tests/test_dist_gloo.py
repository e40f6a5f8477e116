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
