"""Row-returning SELECT on the GPU vs the oracle.

filter_rows + build_result (reference evaluator_utils.c:986-1006, :249-549):
the scan emits the offsets of matching records, a device radix sort puts them
in file order, and project_kernel parses the referenced columns and evaluates
each SELECT item.  Results must match the oracle cell for cell (bit-exact:
projection copies cells or applies the same double arithmetic).
"""
import os

import pytest

import cqtest
import cq_amd
from cq_amd import datagen
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def synth(tmp_path_factory):
    p = tmp_path_factory.mktemp("rows") / "role.csv"
    datagen.write_shape_a(str(p), 120_000, seed=5, with_role=True)
    return str(p)


ROW_QUERIES = [
    "SELECT name, age FROM '{P}' WHERE age > 30",
    "SELECT * FROM '{P}' WHERE role = 'role_007'",
    "SELECT name, age * 2, age + height, -height FROM '{P}' WHERE height < 1.5",
    "SELECT name, age % 7 FROM '{P}' WHERE height < 1.5",
    "SELECT role AS r, age AS years FROM '{P}' WHERE age BETWEEN 20 AND 22",
    "SELECT main.name, surname FROM '{P}' WHERE gender = 'f' AND age < 19",
    "SELECT name, missing_col, 'lit', 42 FROM '{P}' WHERE age = 55",
    "SELECT age, *, height FROM '{P}' WHERE age = 60 AND role LIKE 'role_00%'",
    "SELECT name, age FROM '{P}' ORDER BY age DESC LIMIT 50",
    "SELECT DISTINCT gender FROM '{P}'",
    "SELECT name FROM '{P}' LIMIT 7 OFFSET 1000",
    "SELECT name FROM '{P}' WHERE age > 200",
    "SELECT name FROM '{P}' LIMIT 0",
    "SELECT age FROM '{P}' WHERE age > 90 LIMIT 5 OFFSET 1000000",
    "SELECT height / (age - 40), age & 6, age | 1 FROM '{P}' WHERE age > 35 AND age < 45",
    "SELECT r2 FROM (SELECT role AS r2 FROM '{P}') AS s",
]


def _check(sql, expect_eligible=True):
    want, unsup = cqtest.oracle_query(sql)
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
    inel = cq_amd.last_ineligible()
    if not expect_eligible:
        assert inel, sql
        return
    assert not unsup, sql
    assert not inel, (sql, inel)
    assert cq_amd.stats()["path"] == 1
    compare(got, want, set(), sql)


@pytest.mark.parametrize("tmpl", ROW_QUERIES)
def test_rows_vs_oracle(synth, tmpl):
    sql = tmpl.replace("{P}", synth)
    _check(sql, expect_eligible="(SELECT" not in sql)


def test_rows_small_capacity_and_batches(synth, monkeypatch):
    """first-pass offset buffer too small (exact-size rescan) and many projection batches"""
    monkeypatch.setenv("CQGPU_ROW_CAP0", "1000")
    monkeypatch.setenv("CQGPU_ROW_BATCH", "1024")
    _check(f"SELECT name, age, height * 2 FROM '{synth}' WHERE age > 30")
    _check(f"SELECT * FROM '{synth}'")


def test_rows_ragged_and_quoted(tmp_path):
    """short rows, quoted fields with delimiters, blank and CRLF lines"""
    p = tmp_path / "ragged.csv"
    p.write_bytes(b"a,b,c,d\r\n1,2,3,4\r\n5,6\r\n\r\n"
                  b"\"x,y\",\"q\"\"q\",7, 8 \n  9 ,10,,\n11,12,13\n\"unterminated,14\n15")
    for sql in (f"SELECT * FROM '{p}'", f"SELECT d, c, b, a FROM '{p}'",
                f"SELECT a, b + c FROM '{p}' WHERE b > 1"):
        want, unsup = cqtest.oracle_query(sql)
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
        assert not cq_amd.last_ineligible(), sql
        assert not unsup
        compare(got, want, set(), sql)


def test_rows_header_only(tmp_path):
    p = tmp_path / "h.csv"
    p.write_bytes(b"a,b\n")
    _check(f"SELECT * FROM '{p}'")
    _check(f"SELECT b FROM '{p}' WHERE a > 1")


def test_rows_wide_star(tmp_path):
    """more columns than one aggregate plan may reference (the projection has no 8-column cap)"""
    ncol = 40
    lines = [",".join(f"c{j}" for j in range(ncol))]
    for i in range(3000):
        lines.append(",".join(str((i * 31 + j * 7) % 1000 - (j % 3)) for j in range(ncol)))
    p = tmp_path / "wide.csv"
    p.write_text("\n".join(lines) + "\n")
    _check(f"SELECT * FROM '{p}' WHERE c3 > 500")
    _check(f"SELECT c39, c0 * c1, c20 FROM '{p}' WHERE c5 < 100 ORDER BY c39")
