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
