"""Plans over more than 8 columns, GROUP BY of more than 8 parts, and the
no-role COUNT(*) at 1e6 rows.

The fused scans parse at most 8 need slots into registers; a plan over more
distinct columns ("wide") runs on the cells path: the needed columns of every
record parsed into a cell table (cells_kernel), then the WHERE / GROUP BY /
aggregates read the cells in place (scan.hip PairView).  The reference evaluates
any condition tree and copies every column into a joined row
(evaluator_joins.c:30-37, :110-120; `*` over all of them, evaluator_utils.c:272-417;
GROUP BY parts without bound, evaluator.c:113-212).  Checked against the
reference's own vectors (tests/golden/queries.json, mid.json) and the oracle on
larger synthetic files, single GPU and range partials at 1/3/8 ranks, blob and
dense merge.  Counts, groups, order, cells bit-exact; SUM/AVG/STDDEV 1e-6 relative.
"""
import os

import numpy as np
import pytest

import cqtest
import cq_amd
from cq_amd import datagen
from test_gpu_parity import compare, tolerant_columns
from test_gpu_partials import _dense, _merged

pytestmark = pytest.mark.gpu

QUERIES = cqtest.golden("queries.json")
WIDE_GOLDEN = [i for i, q in enumerate(QUERIES) if "synth_wide" in q["sql"] or q["sql"].startswith("SELECT * FROM '{D}/users")
               or "u.age + u.height + u.active" in q["sql"]]


def _run(sql):
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        st = cq_amd.stats()
        inel = cq_amd.last_ineligible()
        tol = tolerant_columns(ast)
    return got, st, inel, tol


@pytest.mark.skipif(not cqtest.front_available(), reason="reference front end not built")
@pytest.mark.parametrize("idx", WIDE_GOLDEN)
def test_wide_golden(idx):
    q = QUERIES[idx]
    sql = cqtest.sql_for(q["sql"])
    got, st, inel, tol = _run(sql)
    assert not inel, (sql, inel)
    assert st["path"] == 1, sql
    want = cqtest.table_from_json(q["result"])
    compare(got, want, tol, sql)
    if "synth_wide" in sql and "c4 > 0.5 AND c5" in sql:
        assert st["wide"] == 1, (sql, st)                 # the 9-column WHERE: the cells path


def test_group_by_parts_beyond_eight():
    assert any("GROUP BY c0, c1, c2, c3, c4, c5, c6, c7, c8, c9" in q["sql"] for q in QUERIES)


# ---------------------------------------------------------------- 1e6 rows, no role (fast_kernel NR = 0)
@pytest.fixture(scope="module")
def mid(tmp_path_factory):
    g = cqtest.golden("mid.json")
    p = os.path.join(str(tmp_path_factory.mktemp("mid")), "mid.csv")
    size = datagen.write_logical(p, g["rows"], g["seed"], with_role=g["with_role"])
    assert size == g["bytes"]
    return p, g


def test_mid_golden(mid):
    path, g = mid
    for q in g["queries"]:
        sql = q["sql"].format(p=path)
        got, st, inel, tol = _run(sql)
        assert not inel, (sql, inel)
        compare(got, cqtest.table_from_json(q["result"]), tol, sql)
        if "GROUP BY" not in sql:
            assert st["scan_kernel"] == 2, (sql, "fast_kernel did not run", st)
            assert st["slow_records"] == 0 and st["records"] == g["rows"], st


# ---------------------------------------------------------------- larger synthetic wide files vs the oracle
def _wide_rows(n, seed, ncols=14):
    rng = np.random.default_rng(seed)
    hdr = ",".join("c%d" % i for i in range(ncols))
    cols = []
    for j in range(ncols):
        if j % 5 == 4:
            cols.append(np.array(["%d.%02d" % (a, b) for a, b in zip(rng.integers(0, 20, n), rng.integers(0, 100, n))]))
        elif j % 5 == 3:
            cols.append(np.array(["s%d" % a for a in rng.integers(0, 9, n)]))
        else:
            v = rng.integers(-100, 1000, n).astype(str)
            blank = rng.integers(0, 50, n) == 0
            v[blank] = ""
            cols.append(v)
    cols[-1] = rng.integers(0, 100, n).astype(str)      # the last field never empty (parse_line drops it)
    lines = [",".join(r) for r in zip(*cols)]
    return (hdr + "\n" + "\n".join(lines) + "\n").encode()


@pytest.fixture(scope="module")
def wide(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("wide"))
    p = os.path.join(d, "wide.csv")
    with open(p, "wb") as fh:
        fh.write(_wide_rows(60_000, 21))
    a = os.path.join(d, "a.csv")
    b = os.path.join(d, "b.csv")
    rng = np.random.default_rng(5)
    with open(a, "wb") as fh:
        fh.write(("k,a1,a2,a3,a4,a5,a6,a7,a8,a9\n" + "\n".join(
            "%d,%d,%d.%d,x%d,%d,%d,%d,y%d,%d,%d" % (i, i % 7, i % 13, i % 10, i % 5, i % 11, i % 17, i % 19, i % 3,
                                                   i % 23, i % 29)
            for i in range(2_000)) + "\n").encode())
    with open(b, "wb") as fh:
        fh.write(("id,k,b1,b2,b3,b4,b5\n" + "\n".join(
            "%d,%d,%d,%d.%d,z%d,%d,%d" % (i, rng.integers(0, 2_500), i % 31, i % 9, i % 10, i % 4, i % 37, i % 41)
            for i in range(3_000)) + "\n").encode())
    return {"wide": p, "a": a, "b": b}


W9 = "c0 > -50 AND c1 < 900 AND c2 != 7 AND c3 != 's4' AND c4 > 1.5 AND c5 < 990 AND c6 > -90 AND c7 != 5 AND c8 != 's2'"
SYN = [
    "SELECT COUNT(*), SUM(c13), AVG(c9) FROM '{w}' WHERE " + W9,
    "SELECT c3, COUNT(*), SUM(c12), AVG(c4) FROM '{w}' WHERE " + W9 + " GROUP BY c3",
    "SELECT c8, MIN(c10), MAX(c11), MIN(c3) FROM '{w}' WHERE " + W9 + " GROUP BY c8",
    "SELECT c3, STDDEV(c10), MEDIAN(c11) FROM '{w}' WHERE " + W9 + " GROUP BY c3",
    "SELECT c0, c13, c3 FROM '{w}' WHERE " + W9 + " AND c13 > 90",
    "SELECT * FROM '{w}' WHERE " + W9 + " AND c12 > 950 LIMIT 50 OFFSET 3",
    "SELECT c3, COUNT(*) FROM '{w}' GROUP BY c3, c8, c0 % 2, c1 % 2, c2 % 2, c5 % 2, c3, c8, c3, c6 % 2",
]
JOINS = [
    "SELECT * FROM '{a}' AS a JOIN '{b}' AS b ON a.k = b.k WHERE b.b1 < 3",
    "SELECT * FROM '{a}' AS a LEFT JOIN '{b}' AS b ON a.k = b.k WHERE a.a1 = 2 LIMIT 300",
    "SELECT a.a3, COUNT(*), SUM(b.b2), AVG(a.a2) FROM '{a}' AS a JOIN '{b}' AS b ON a.k = b.k "
    "WHERE a.a1 + a.a4 + a.a5 + a.a6 > 10 AND b.b1 + b.b4 + b.b5 > 5 AND a.a7 != 'y1' GROUP BY a.a3",
    "SELECT COUNT(*), MIN(a.a9), MAX(b.b3) FROM '{a}' AS a JOIN '{b}' AS b ON a.k = b.k "
    "WHERE a.a1 + a.a2 + a.a4 + a.a5 + a.a6 + a.a8 + a.a9 + b.b1 + b.b5 > 40",
]


@pytest.mark.parametrize("sql", SYN + JOINS)
def test_wide_synthetic_vs_oracle(wide, sql):
    q = sql.format(w=wide["wide"], a=wide["a"], b=wide["b"])
    want, unsup = cqtest.oracle_query(q)
    assert not unsup, q
    got, st, inel, tol = _run(q)
    assert not inel, (q, inel)
    assert st["path"] == 1
    compare(got, want, tol, q)
    if "WHERE" in q and "JOIN" not in q:
        assert st["wide"] == 1, (q, st)


@pytest.mark.parametrize("sql", SYN)
@pytest.mark.parametrize("nranks", [1, 3, 8])
def test_wide_across_ranges(wide, sql, nranks):
    q = sql.format(w=wide["wide"])
    want, unsup = cqtest.oracle_query(q)
    assert not unsup
    with cqtest.Parsed(q) as ast:
        got = _merged(ast, wide["wide"], nranks)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{nranks} ranks: {q}")


@pytest.mark.parametrize("sql", [s for s in SYN[:3] + SYN[6:]])
@pytest.mark.parametrize("nranks", [1, 3])
def test_wide_dense_merge(wide, sql, nranks):
    q = sql.format(w=wide["wide"])
    want, unsup = cqtest.oracle_query(q)
    assert not unsup
    with cqtest.Parsed(q) as ast:
        got = _dense(ast, wide["wide"], nranks)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"dense {nranks} ranks: {q}")
