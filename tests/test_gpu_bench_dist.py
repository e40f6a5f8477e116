"""The bench's N > 1 step on one GPU: torchrun with one rank, the nccl (RCCL) backend
and CQ_BENCH_FORCE_DIST=1, so the range partial + dense merge runs its collectives
on device tensors through RCCL (bench.py, cq_amd/dist.py dense_merge) -- the path
the driver's 2/4/8-GPU runs take.  The step's answer is verified by bench.py itself
against the rows' expected COUNT/SUM per role (exit code 3 on a mismatch)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_dense_merge_over_rccl_one_rank():
    env = dict(os.environ, CQ_BENCH_FORCE_DIST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1",
           "--steps", "3", "--warmup", "1", "--rows", "3000000", "--no-cpu", "--no-e2e", "--no-config2",
           "--no-config5", "--gen-workers", "4"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout[-2000:]          # one JSON line on stdout (no RCCL banner)
    d = json.loads(lines[0])
    assert d["verified"] is True
    assert d["config"]["rows_total"] == 3_000_000
