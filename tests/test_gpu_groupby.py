"""Composite and expression GROUP BY on the GPU vs the oracle.

Reference: evaluator.c:71-98 (a GROUP BY name matching a SELECT alias groups by
that item's expression), :113-212 (several parts: key texts joined with '\\t',
columns looked up WITHOUT the table-prefix fallback, a missing column is the
part "NULL") and evaluator_aggregates.c:179-250 (create_groups_by_expression).
(At most 4 SELECT items: the reference parser crashes on more, SURVEY Appendix
A Q13.)  Counts, group sets, first-appearance order, MIN/MAX and representative cells
exact; SUM/AVG within 1e-6 relative.
"""
import os

import pytest

import cqtest
import cq_amd
from cq_amd import datagen
from test_gpu_parity import compare, tolerant_columns

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def synth(tmp_path_factory):
    p = tmp_path_factory.mktemp("gb") / "role.csv"
    datagen.write_shape_a(str(p), 240_000, seed=21, with_role=True)
    return str(p)


QUERIES = [
    "SELECT role, gender, COUNT(*), SUM(height) FROM '{P}' GROUP BY role, gender",
    "SELECT role, gender, AVG(height) FROM '{P}' GROUP BY role, gender",
    "SELECT gender, age, COUNT(*), AVG(height) FROM '{P}' WHERE age > 40 GROUP BY gender, age",
    "SELECT gender, age, MIN(name), MAX(role) FROM '{P}' WHERE age > 40 GROUP BY gender, age",
    "SELECT name, surname, gender, COUNT(*) FROM '{P}' GROUP BY name, surname, gender",
    "SELECT height, role, COUNT(*), SUM(age) FROM '{P}' WHERE role < 'role_050' GROUP BY height, age, gender, role",
    "SELECT age / 10 AS decade, COUNT(*), AVG(height) FROM '{P}' GROUP BY decade",
    "SELECT height * 100 AS cm, COUNT(*) FROM '{P}' GROUP BY cm ORDER BY cm DESC LIMIT 7",
    "SELECT gender, age * 2 AS a2, COUNT(*), MIN(height) FROM '{P}' GROUP BY gender, a2",
    "SELECT role AS r, COUNT(*) FROM '{P}' WHERE age < 20 GROUP BY r",
    "SELECT gender, COUNT(*) FROM '{P}' GROUP BY gender, nosuch",
    "SELECT gender, role, COUNT(*) FROM '{P}' GROUP BY gender, role HAVING COUNT(*) > 130 ORDER BY COUNT(*) DESC LIMIT 12",
    "SELECT age - age AS z, gender, COUNT(*) FROM '{P}' GROUP BY z, gender",
]


@pytest.mark.parametrize("tmpl", QUERIES)
def test_composite_vs_oracle(synth, tmpl):
    sql = tmpl.replace("{P}", synth)
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        tol = tolerant_columns(ast)
    assert not cq_amd.last_ineligible(), (sql, cq_amd.last_ineligible())
    assert cq_amd.stats()["path"] == 1
    compare(got, want, tol, sql)


def test_composite_typed_parts(tmp_path):
    """parts of every value class: NULL / "NULL" text, dates vs date-shaped text,
    1 vs 1.0 vs 1.000000, long strings (> 16 bytes), negative zero"""
    rows = ["a,b,c"]
    vals_a = ["", "NULL", "2024-01-05", " 2024-01-05 ", "1", "1.0", "1.0000001", "-0.0", "0",
              "a_rather_long_text_value_1", "a_rather_long_text_value_2", "x"]
    vals_b = ["1", "1.00", "01", "", "z", "2023-12-31", "12/31/2023"]
    for i in range(6000):
        rows.append("%s,%s,%d" % (vals_a[i % len(vals_a)], vals_b[(i * 7) % len(vals_b)], i % 5))
    p = tmp_path / "typed.csv"
    p.write_text("\n".join(rows) + "\n")
    for sql in (f"SELECT a, b, COUNT(*), SUM(c) FROM '{p}' GROUP BY a, b",
                f"SELECT b, a, c, COUNT(*) FROM '{p}' GROUP BY b, a, c",
                f"SELECT c + 0.5 AS h, COUNT(*) FROM '{p}' GROUP BY h"):
        want, unsup = cqtest.oracle_query(sql)
        assert not unsup
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
            tol = tolerant_columns(ast)
        assert not cq_amd.last_ineligible(), (sql, cq_amd.last_ineligible())
        compare(got, want, tol, sql)


def test_tab_in_composite_parts(tmp_path):
    """text parts holding a tab key on the joined text (evaluator.c:124): ("x\ty", 1)
    and ("x", "y\t1") are one group; numbers, dates, NULL and expressions render as
    the reference renders them (%lld, %.6f, %04d-%02d-%02d, "NULL"); also across
    range partials"""
    import random
    rng = random.Random(5)
    a_vals = ["x\ty", "x", "1\t2", "1", "", "2024-01-05\tz", "2024-01-05", "p\tq\tr", "p", "0.5\t1"]
    b_vals = ["1", "y\t1", "2", "2\t3", "", "z", "q\tr", "1.5", "2024-01-05", "1\t0.500000"]
    rows = ["a,b,c"] + ["%s,%s,%d" % (rng.choice(a_vals), rng.choice(b_vals), rng.randrange(9))
                        for _ in range(4000)]
    p = tmp_path / "tabs.csv"
    p.write_text("\n".join(rows) + "\n")
    sqls = (f"SELECT a, b, COUNT(*), SUM(c) FROM '{p}' GROUP BY a, b",
            f"SELECT b, COUNT(*) FROM '{p}' GROUP BY b, a, c",
            f"SELECT a, c / 2 AS h, COUNT(*) FROM '{p}' WHERE c > 2 GROUP BY a, h",
            f"SELECT a, COUNT(*) FROM '{p}' GROUP BY a, b, nosuch")
    for sql in sqls:
        want, unsup = cqtest.oracle_query(sql)
        assert not unsup
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
            tol = tolerant_columns(ast)
            assert not cq_amd.last_ineligible(), (sql, cq_amd.last_ineligible())
            compare(got, want, tol, sql)
            tabs = [cq_amd.Table.open_range(str(p), r, 3) for r in range(3)]
            blobs = [cq_amd.query_partial(ast, [t]) for t in tabs]
            for t in tabs:
                t.close()
            from cq_amd import abi
            tp = cq_amd.merge_partials(ast, blobs)
            assert tp, cq_amd.last_error()
            merged = abi.table_to_py(tp)
            cq_amd.result_free(tp)
        compare(merged, want, tol, sql + " (3 partials)")


def test_many_parts_across_partials(synth):
    """GROUP BY of 6 parts (the reference's list grows without bound,
    parser_clauses.c:241-246) on one GPU and over 4 range partials"""
    sql = (f"SELECT role, COUNT(*), SUM(height) FROM '{synth}' WHERE age > 70 "
           f"GROUP BY gender, role, age, name, height, surname")
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        tol = tolerant_columns(ast)
        assert not cq_amd.last_ineligible(), cq_amd.last_ineligible()
        compare(got, want, tol, sql)
        tabs = [cq_amd.Table.open_range(synth, r, 4) for r in range(4)]
        blobs = [cq_amd.query_partial(ast, [t]) for t in tabs]
        for t in tabs:
            t.close()
        from cq_amd import abi
        tp = cq_amd.merge_partials(ast, blobs)
        assert tp, cq_amd.last_error()
        merged = abi.table_to_py(tp)
        cq_amd.result_free(tp)
    compare(merged, want, tol, sql + " (4 partials)")


def test_composite_across_partials(synth):
    sql = QUERIES[1].replace("{P}", synth)
    want, _ = cqtest.oracle_query(sql)
    with cqtest.Parsed(sql) as ast:
        tabs = [cq_amd.Table.open_range(synth, r, 4) for r in range(4)]
        blobs = [cq_amd.query_partial(ast, [t]) for t in tabs]
        for t in tabs:
            t.close()
        from cq_amd import abi
        tp = cq_amd.merge_partials(ast, blobs)
        assert tp, cq_amd.last_error()
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql)


# ---------------------------------------------------------------- mixed-class MIN/MAX
def test_mixed_class_min_max(tmp_path):
    """MIN/MAX over columns mixing numbers, strings and dates: the reference's
    row-order fold keeps the class of each group's first non-NULL cell
    (evaluator_aggregates.c:311-326, value_compare calls other classes equal)."""
    import numpy as np
    rng = np.random.default_rng(5)
    shapes = ["12", "-3", "7.5", "abc", "Zed", "2024-02-03", "1999-12-31", "", "0", "b", "10.25", "2001-01-01"]
    rows = ["g,v,w"]
    for i in range(30000):
        rows.append("%d,%s,%s" % (rng.integers(0, 40), shapes[rng.integers(0, len(shapes))],
                                  shapes[rng.integers(0, len(shapes))]))
    p = tmp_path / "mixed.csv"
    p.write_text("\n".join(rows) + "\n")
    for sql in (f"SELECT g, MIN(v), MAX(v), COUNT(*) FROM '{p}' GROUP BY g",
                f"SELECT MIN(v), MAX(w), MIN(w), MAX(v) FROM '{p}'",
                f"SELECT g, MIN(w), MAX(w) FROM '{p}' WHERE v > 5 GROUP BY g",
                f"SELECT g, v, MIN(w), COUNT(*) FROM '{p}' GROUP BY g, v"):
        want, unsup = cqtest.oracle_query(sql)
        assert not unsup
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
        assert not cq_amd.last_ineligible(), (sql, cq_amd.last_ineligible())
        compare(got, want, set(), sql)


def test_composite_digest_collision_fails_loudly(synth, monkeypatch):
    """Composite keys are grouped by a 128-bit digest of the parts; every passing
    row's parts are then checked against its group's first row's parts
    (evaluator.c:113-212 groups by the exact joined key text).  The test knob
    CQGPU_TEST_DIGEST_BITS cuts the digest to 2 bits, so different part lists must
    collide: the query has to fail with the collision named, never merge them.
    Full digests on the same query: exact against the oracle."""
    sql = f"SELECT role, gender, COUNT(*) FROM '{synth}' GROUP BY role, gender"
    monkeypatch.setenv("CQGPU_TEST_DIGEST_BITS", "2")
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
    assert got is None
    assert "digest" in cq_amd.last_error(), cq_amd.last_error()
    monkeypatch.delenv("CQGPU_TEST_DIGEST_BITS")
    want, _ = cqtest.oracle_query(sql)
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql)


def test_joined_text_collision_fails_loudly(tmp_path, monkeypatch):
    """Composite keys with a tab inside a text part key on the reference's joined
    text (evaluator.c:113-212); a hit is re-checked by comparing the two joined
    texts byte for byte.  CQGPU_TEST_DIGEST_BITS cuts their hash to 2 bits: the
    query must fail with the collision named; full hashes: exact vs the oracle."""
    rows = ["a\tb,c,%d" % i for i in range(50)] + ["a,b\tc,%d" % i for i in range(50)] + \
           ["x\ty,z%d,%d" % (i % 9, i) for i in range(400)]
    p = tmp_path / "tabs.csv"
    p.write_text("t1,t2,n\n" + "\n".join(rows) + "\n")
    sql = f"SELECT t1, t2, COUNT(*), SUM(n) FROM '{p}' GROUP BY t1, t2"
    monkeypatch.setenv("CQGPU_TEST_DIGEST_BITS", "2")
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
    assert got is None
    assert "digest" in cq_amd.last_error(), cq_amd.last_error()
    monkeypatch.delenv("CQGPU_TEST_DIGEST_BITS")
    want, _ = cqtest.oracle_query(sql)
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql)
    assert len(want["rows"]) == 10        # 'a\tb'+'c' and 'a'+'b\tc' join to one text


def test_tab_parts_with_large_doubles(tmp_path):
    """A composite key whose text part holds a tab next to a DOUBLE part of 2^43 or
    more: the joined text renders the double's full "%.6f" (the exact binary value,
    integer digits up to the key_part[256] cut, evaluator.c:113-212), so
    ("x\\t9007199254740993.000000", ...) style collisions of the reference's texts
    are reproduced; one GPU and 3 range partials against the oracle"""
    import random
    rng = random.Random(11)
    a_vals = ["x\ty", "x", "p\tq", "p"]
    d_vals = ["8796093022208.5", "9007199254740993", "123456789012345.125", "1e20", "1.5e300", "-2.5e17",
              "17592186044416.0078125", "8796093022208.00048828125", "3", "0.5"]
    rows = ["a,d,c"] + ["%s,%s,%d" % (rng.choice(a_vals), rng.choice(d_vals), rng.randrange(9)) for _ in range(3000)]
    p = tmp_path / "bigd.csv"
    p.write_text("\n".join(rows) + "\n")
    from cq_amd import abi
    for sql in (f"SELECT a, d, COUNT(*), SUM(c) FROM '{p}' GROUP BY a, d",
                f"SELECT d, COUNT(*) FROM '{p}' GROUP BY d, a"):
        want, unsup = cqtest.oracle_query(sql)
        assert not unsup
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
            tol = tolerant_columns(ast)
            assert not cq_amd.last_ineligible(), (sql, cq_amd.last_ineligible())
            compare(got, want, tol, sql)
            tabs = [cq_amd.Table.open_range(str(p), r, 3) for r in range(3)]
            blobs = [cq_amd.query_partial(ast, [t]) for t in tabs]
            for t in tabs:
                t.close()
            assert all(blobs), cq_amd.last_error() or cq_amd.last_ineligible()
            tp = cq_amd.merge_partials(ast, blobs)
            assert tp, cq_amd.last_error()
            merged = abi.table_to_py(tp)
            cq_amd.result_free(tp)
        compare(merged, want, tol, sql + " (3 partials)")
