"""The drop-in: the reference's unchanged main.c + parser front end linked against
libcqgpu.so (oracle/_ref/cq_amd_cli, built by oracle/ref.mk) must print exactly
what the reference CLI (oracle/_ref/cq_ref) prints -- config 1 of BASELINE.json
and a few more GPU-eligible queries.  Both binaries are prebuilt; nothing here
reads /root/reference.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "cq_ref")
GPU = os.path.join(ROOT, "oracle", "_ref", "cq_amd_cli")
D = "tests/golden/data"

QUERIES = [
    f"SELECT COUNT(*) FROM '{D}/test_data.csv' WHERE age > 30",            # BASELINE config 1
    f"SELECT role, COUNT(*), AVG(age) FROM '{D}/test_data.csv' GROUP BY role",
    f"SELECT COUNT(*), SUM(price), MIN(price), MAX(quantity) FROM '{D}/orders.csv'",
    f"SELECT city, COUNT(*) FROM '{D}/users.csv' GROUP BY city ORDER BY COUNT(*) DESC",
]


@pytest.mark.skipif(not (os.path.exists(REF) and os.path.exists(GPU)), reason="oracle/ref.mk not built")
@pytest.mark.parametrize("sql", QUERIES)
def test_cli_output_identical(sql):
    env = dict(os.environ)
    want = subprocess.run([REF, "-q", sql, "-p"], cwd=ROOT, capture_output=True, timeout=120)
    got = subprocess.run([GPU, "-q", sql, "-p"], cwd=ROOT, capture_output=True, timeout=300, env=env)
    assert got.returncode == want.returncode, got.stderr.decode(errors="replace")
    assert got.stdout == want.stdout, (got.stdout.decode(errors="replace"), want.stdout.decode(errors="replace"))
