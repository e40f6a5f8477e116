"""STDDEV / MEDIAN on the GPU (executor.hip compute_vla, scan.hip vla_* kernels)
against the oracle's evaluate_aggregate (reference evaluator_aggregates.c:328-411).

Population STDDEV (two passes: mean, squared deviations) within 1e-6 relative;
MEDIAN bit-exact (middle value, or the mean of the two middle values); groups
without a numeric value give NULL; strings, dates and NULLs are skipped; WHERE
filters first.
"""
import numpy as np
import pytest

import cqtest
import cq_amd
from cq_amd import abi, datagen

pytestmark = pytest.mark.gpu
REL = 1e-6


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("stats")
    rng = np.random.default_rng(23)
    lines = ["g,x,y,s"]
    for i in range(40_000):
        g = "g%02d" % rng.integers(0, 60)
        k = rng.integers(0, 30)
        x = "" if k == 0 else ("abc" if k == 1 else ("%d" % rng.integers(-500, 500) if k < 15
                                                    else "%.3f" % rng.normal(10.0, 3.0)))
        y = "%d" % rng.integers(0, 7)
        lines.append(f"{g},{x},{y},{'t' if i % 3 else 'f'}")
    lines.append("gnull,abc,1,t")                  # a group with no numeric x
    f = {"mix": d / "mix.csv"}
    f["mix"].write_text("\n".join(lines) + "\n")
    f["role"] = d / "role.csv"
    datagen.write_shape_a(str(f["role"]), 200_000, seed=5, with_role=True)
    f["users"] = d / "users.csv"
    f["users"].write_bytes(datagen.users_bytes(4_000, seed=31))
    f["orders"] = d / "orders.csv"
    f["orders"].write_bytes(datagen.orders_bytes(15_000, 4_800, seed=32))
    return f


def _check(sql):
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        inel = cq_amd.last_ineligible()
    assert not inel, (sql, inel)
    assert cq_amd.stats()["path"] == 1
    sel = sql.split(" FROM ")[0][len("SELECT "):]
    tol = {i for i, t in enumerate(s.strip().upper() for s in sel.split(",")) if t.startswith(("STDDEV", "SUM", "AVG"))}
    assert got["columns"] == want["columns"], sql
    assert len(got["rows"]) == len(want["rows"]), sql
    for i, (g, w) in enumerate(zip(got["rows"], want["rows"])):
        for j, (x, y) in enumerate(zip(g, w)):
            assert cqtest.cell_equal(x, y, REL if j in tol else 0.0), f"{sql}: row {i} col {j}: {x} vs {y}"


QUERIES = [
    "SELECT STDDEV(x), MEDIAN(x), COUNT(*) FROM '{M}'",
    "SELECT g, STDDEV(x), MEDIAN(x), AVG(x) FROM '{M}' GROUP BY g",
    "SELECT g, MEDIAN(y), STDDEV_POP(y) FROM '{M}' WHERE s = 't' GROUP BY g",
    "SELECT y, MEDIAN(x), COUNT(*) FROM '{M}' WHERE x > 0 GROUP BY y ORDER BY y",
    "SELECT s, STDDEV(x) FROM '{M}' WHERE g = 'gnull' GROUP BY s",
    "SELECT role, STDDEV(height), MEDIAN(age) FROM '{R}' WHERE age > 30 GROUP BY role",
    "SELECT MEDIAN(height), STDDEV(age) FROM '{R}'",
    # composite and expression keys (cells path, compute_vla_pairs over identity pairs)
    "SELECT gender, role, STDDEV(height), MEDIAN(age) FROM '{R}' WHERE age > 50 GROUP BY gender, role",
    "SELECT g, y, MEDIAN(x), STDDEV(x) FROM '{M}' GROUP BY g, y",
    "SELECT age / 7 AS b, MEDIAN(height), COUNT(*) FROM '{R}' GROUP BY b",
    # MIN/MAX over a column mixing classes beside STDDEV / MEDIAN
    "SELECT g, MIN(x), MEDIAN(x), STDDEV(x) FROM '{M}' GROUP BY g",
    # joins (pairs of parsed cells)
    "SELECT u.role, STDDEV(o.price), MEDIAN(o.quantity), COUNT(*) FROM '{U}' AS u JOIN '{O}' AS o ON u.id = o.customer_id GROUP BY u.role",
    "SELECT MEDIAN(o.price), STDDEV(u.age) FROM '{U}' AS u JOIN '{O}' AS o ON u.id = o.customer_id WHERE o.quantity > 3",
    "SELECT u.age, MEDIAN(o.price), STDDEV(o.price) FROM '{U}' AS u LEFT JOIN '{O}' AS o ON u.id = o.customer_id GROUP BY u.age",
    "SELECT o.quantity, u.role, MEDIAN(u.age) FROM '{U}' AS u JOIN '{O}' AS o ON u.id = o.customer_id GROUP BY o.quantity, u.role",
]


@pytest.mark.parametrize("tmpl", QUERIES)
def test_stddev_median(files, tmpl):
    _check(tmpl.replace("{M}", str(files["mix"])).replace("{R}", str(files["role"]))
           .replace("{U}", str(files["users"])).replace("{O}", str(files["orders"])))


PARTIAL_STDDEV = [
    "SELECT role, STDDEV(height), COUNT(*) FROM '{R}' WHERE age > 30 GROUP BY role",
    "SELECT STDDEV(age), STDDEV(height), AVG(age) FROM '{R}'",
    "SELECT g, STDDEV(x), STDDEV_POP(y) FROM '{M}' GROUP BY g",
    "SELECT gender, role, STDDEV(age) FROM '{R}' GROUP BY gender, role",
    "SELECT g, MIN(y), MAX(y), STDDEV(x) FROM '{M}' GROUP BY g",
    # MEDIAN: every rank ships its groups' numeric values, the merge sorts them
    "SELECT role, MEDIAN(age) FROM '{R}' GROUP BY role",
    "SELECT g, MEDIAN(x), STDDEV(x), MIN(x) FROM '{M}' GROUP BY g",
    "SELECT gender, role, MEDIAN(height), MEDIAN(age) FROM '{R}' WHERE age > 50 GROUP BY gender, role",
    "SELECT MEDIAN(height) FROM '{R}' WHERE age > 200",
]


@pytest.mark.parametrize("nranks", [1, 3, 8])
@pytest.mark.parametrize("tmpl", PARTIAL_STDDEV)
def test_stddev_across_partials(files, tmpl, nranks):
    """per range: (sum, squared deviations, count) per group, merged by the
    parallel-variance rule; population STDDEV within 1e-6 of the oracle; MEDIAN
    from every rank's values, exact"""
    path = str(files["mix"]) if "{M}" in tmpl else str(files["role"])
    sql = tmpl.replace("{M}", path).replace("{R}", path)
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    with cqtest.Parsed(sql) as ast:
        tabs = [cq_amd.Table.open_range(path, r, nranks) for r in range(nranks)]
        try:
            blobs = [cq_amd.query_partial(ast, [t]) for t in tabs]
        finally:
            for t in tabs:
                t.close()
        tp = cq_amd.merge_partials(ast, blobs)
        assert tp, cq_amd.last_error()
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
    sel = sql.split(" FROM ")[0][len("SELECT "):]
    tol = {i for i, t in enumerate(x.strip().upper() for x in sel.split(",")) if t.startswith(("STDDEV", "SUM", "AVG"))}
    assert got["columns"] == want["columns"]
    assert len(got["rows"]) == len(want["rows"])
    for i, (g, w) in enumerate(zip(got["rows"], want["rows"])):
        for j, (x, y) in enumerate(zip(g, w)):
            assert cqtest.cell_equal(x, y, REL if j in tol else 0.0), f"{sql} @ {nranks}: row {i} col {j}: {x} vs {y}"
