"""cells_kernel's mask-based fast path (scan.hip) against the oracle.

Every JOIN, composite / expression GROUP BY and STDDEV/MEDIAN plan reads its
columns through cells_kernel.  Its fast path types short numerals and plain
strings in registers and hands every other field to parse_cell; the records it
cannot bound (quotes, leading blanks, no terminator in 64 bytes) take the byte
walk.  This fuzz puts each shape at each field position: numerals of 1-20 bytes
with and without a dot (8-10 bytes: parse_date's lengths, e.g. compact dates),
signs, leading zeros, blanks before / after, quotes, tabs, long strings, empty
fields, short rows, CR / CRLF terminators, records longer than 64 bytes.  The
composite GROUP BY over the typed cells must match the oracle exactly (group
set, first-appearance order, first-row cells, MIN/MAX).
"""
import random

import pytest

import cqtest
import cq_amd
from test_gpu_parity import compare, tolerant_columns

pytestmark = pytest.mark.gpu


def _field(rng):
    k = rng.randrange(16)
    if k < 4:                                   # numerals of every length
        n = rng.randrange(1, 21)
        s = "".join(rng.choice("0123456789") for _ in range(n))
        if rng.random() < 0.4 and n > 1:
            p = rng.randrange(0, n)
            s = s[:p] + "." + s[p:]
        return s
    if k == 4:
        return rng.choice(["20240105", "2024-01-05", "01/05/2024", "05.01.2024", "19991231", "12345678"])
    if k == 5:
        return rng.choice(["+5", "-7", "-0", "-0.0", "+1.5", ".5", "5.", "00012", "0", "0.000"])
    if k == 6:
        return rng.choice(["", " ", "  x", "y  ", " 12", "12 ", "\t3", "a b"])
    if k == 7:
        return rng.choice(['"q"', '"a,b"', 'x"y', '""', '"12"'])
    if k == 8:
        return "".join(rng.choice("abcdefghij") for _ in range(rng.randrange(17, 40)))
    if k == 9:
        return rng.choice(["NULL", "null", "inf", "nan", "1e5", "0x1A", "1,5"]).replace(",", ";")
    return "".join(rng.choice("abcXYZ_") for _ in range(rng.randrange(1, 16)))


@pytest.fixture(scope="module")
def fuzz(tmp_path_factory):
    rng = random.Random(77)
    lines = ["a,b,c,d,e"]
    for i in range(30_000):
        nf = rng.choice([5, 5, 5, 5, 4, 3, 6])
        fields = [_field(rng) for _ in range(nf)]
        if rng.random() < 0.02:
            fields[0] = "w" * 70                # longer than the 64-byte view
        lines.append(",".join(fields))
    data = ""
    for ln in lines:
        data += ln + rng.choice(["\n", "\n", "\n", "\r\n", "\r"])
    p = tmp_path_factory.mktemp("cf") / "fuzz.csv"
    p.write_text(data)
    return str(p)


QUERIES = [
    "SELECT a, b, COUNT(*) FROM '{F}' GROUP BY a, b",
    "SELECT c, d, MIN(e), MAX(a) FROM '{F}' GROUP BY c, d",
    "SELECT e, b, COUNT(*), SUM(c) FROM '{F}' GROUP BY e, b",
    "SELECT d, MEDIAN(c), STDDEV(b) FROM '{F}' GROUP BY d",
]


@pytest.mark.parametrize("tmpl", QUERIES)
def test_cells_fast_path_vs_oracle(fuzz, tmpl):
    sql = tmpl.format(F=fuzz)
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        assert not cq_amd.last_ineligible(), cq_amd.last_ineligible()
        assert cq_amd.stats()["path"] == 1
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql)
