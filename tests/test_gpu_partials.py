"""Range-partitioned aggregation: per-shard cqgpu_query_partial + cqgpu_merge_partials
must give exactly the whole-table answer (SUM/AVG within 1e-6 relative).

The shards split one synthetic file at record boundaries; each is uploaded with
its whole-file base offset and the header bytes, as bench.py does per rank.
"""
import pytest

import cqtest
import cq_amd
from cq_amd import abi, datagen
from test_gpu_parity import compare, tolerant_columns

pytestmark = pytest.mark.gpu

QUERIES = [
    "SELECT role, COUNT(*), SUM(height), AVG(height) FROM 'x' WHERE age > 30 GROUP BY role",
    "SELECT COUNT(*), SUM(height), MIN(height), MAX(age) FROM 'x' WHERE gender = 'f'",
    "SELECT name, COUNT(*), MIN(role), MAX(role) FROM 'x' GROUP BY name",
    "SELECT age, COUNT(*) FROM 'x' GROUP BY age HAVING COUNT(*) > 1900 ORDER BY COUNT(*) DESC LIMIT 5",
    "SELECT gender, AVG(age) FROM 'x' WHERE role LIKE 'role_0%' GROUP BY gender",
]


@pytest.fixture(scope="module")
def shards():
    data = datagen.shape_a_bytes(120_000, seed=11, with_role=True)
    header, body = data.split(b"\n", 1)
    header += b"\n"
    cuts = [0]
    for frac in (0.31, 0.64):
        i = body.index(b"\n", int(len(body) * frac)) + 1
        cuts.append(i)
    cuts.append(len(body))
    pieces = [body[a:b] for a, b in zip(cuts, cuts[1:])]
    whole = cq_amd.Table.from_bytes(data)
    parts = []
    base = 0
    for i, pc in enumerate(pieces):
        if i == 0:
            parts.append(cq_amd.Table.from_bytes(header + pc))
            base = len(header) + len(pc)
        else:
            parts.append(cq_amd.Table.from_bytes(pc, base_offset=base, header=header))
            base += len(pc)
    yield whole, parts
    whole.close()
    for p in parts:
        p.close()


@pytest.mark.parametrize("sql", QUERIES)
def test_merge_equals_whole(shards, sql):
    whole, parts = shards
    with cqtest.Parsed(sql) as ast:
        want = cq_amd.query(ast, [whole])
        assert want is not None, cq_amd.last_error()
        blobs = [cq_amd.query_partial(ast, [p]) for p in parts]
        tp = cq_amd.merge_partials(ast, blobs)
        assert tp, cq_amd.last_error()
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql)
