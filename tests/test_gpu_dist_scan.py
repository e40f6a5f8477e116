"""bench.py's N > 1 step in real processes: two ranks on one GPU.

Each rank opens its newline-snapped range of one file (cqgpu_table_open_range),
runs cq_amd.dist.scan_partitioned -- the function bench.py times at N > 1
(cqgpu_query_partial, gather_blobs, cqgpu_merge_partials on rank 0) -- over a
gloo group (RCCL needs one GPU per rank), and rank 0's result must equal the
oracle on the whole file for the config-3 query.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

import cqtest
from cq_amd import datagen

pytestmark = pytest.mark.gpu

SQL = "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, q, sql=SQL, dense=False):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        import cqtest as ct
        import cq_amd
        from cq_amd import abi
        from cq_amd.dist import scan_partitioned, scan_partitioned_dense
        fn = scan_partitioned_dense if dense else scan_partitioned
        t = cq_amd.Table.open_range(path, rank, world)
        with ct.Parsed(sql.format(p=path)) as ast:
            tp = None
            for _ in range(2):                 # a warm-up step, then the checked one
                if tp:
                    cq_amd.result_free(tp)
                tp = fn(ast, t, "cpu")
        t.close()
        if rank == 0:
            res = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            q.put((rank, res, None))
        else:
            q.put((rank, tp is None, None))
    except Exception as e:   # reported to the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(path, world, sql, dense):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, q, sql, dense)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=110)
        assert err is None, f"rank {rank}: {err}"
        out[rank] = res
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(out[r] is True for r in range(1, world))
    return out[0]


@pytest.mark.parametrize("dense", [False, True])
def test_bench_step_two_processes(tmp_path, dense):
    """bench.py's N > 1 step: blobs + host merge, and the device-side dense merge"""
    path = str(tmp_path / "big.csv")
    datagen.write_logical(path, 400_000, seed=42, with_role=True)
    got = _run(path, 2, SQL, dense)
    want, unsup = cqtest.oracle_query(SQL.format(p=path))
    assert not unsup
    from test_gpu_parity import compare
    compare(got, want, {2, 3}, f"2-process config-3 step (dense={dense})")
    assert len(want["rows"]) == 1000


def test_dense_step_falls_back_together(tmp_path):
    """a key over 16 bytes on ONE rank only: every rank must leave the dense path
    (the agreement all-reduce), or the ranks would wait in different collectives"""
    rows = ["k,v"] + [f"k{i % 7},{i}" for i in range(3000)] + [f"a_key_longer_than_sixteen,{i}" for i in range(40)]
    path = str(tmp_path / "mixed.csv")
    with open(path, "w") as fh:
        fh.write("\n".join(rows) + "\n")
    sql = "SELECT k, COUNT(*), SUM(v) FROM '{p}' GROUP BY k"
    got = _run(path, 3, sql, True)
    want, _ = cqtest.oracle_query(sql.format(p=path))
    from test_gpu_parity import compare
    compare(got, want, {2}, "dense fallback")


@pytest.mark.parametrize("sql", [
    "SELECT name, age, height FROM '{p}' WHERE height > 198 AND age > 60",
    "SELECT * FROM '{p}' WHERE role = 'role_042' ORDER BY height DESC LIMIT 30 OFFSET 2",
    "SELECT role, MEDIAN(height), STDDEV(height) FROM '{p}' WHERE age < 20 GROUP BY role",
])
def test_rows_and_median_two_processes(tmp_path, sql):
    """row-returning SELECTs and MEDIAN over real ranks: each rank's rows / values
    travel in its blob, rank 0 orders them by whole-file position"""
    path = str(tmp_path / "rows.csv")
    datagen.write_logical(path, 200_000, seed=7, with_role=True)
    for dense in (False, True):          # the dense path must decline them on every rank
        got = _run(path, 2, sql, dense)
        want, unsup = cqtest.oracle_query(sql.format(p=path))
        assert not unsup
        from test_gpu_parity import compare
        compare(got, want, {2} if "STDDEV" in sql else set(), f"2-process: {sql} (dense={dense})")
