"""Parity of fast_kernel (cq_amd/csrc/fast.hip) with the oracle, lean_kernel and the
general scan_kernel on inputs aimed at its own edges.

fast_kernel covers WHERE `col op numeric-literal` (or none), COUNT / SUM / AVG over
at most two columns, and GROUP BY one column of <= 8-byte keys, with the roles'
columns ascending.  Its own edges, on top of lean_kernel's (test_gpu_lean.py):
  * the ',' / '"' classifier flags '&' bytes as possible quotes (whole windows then
    take the exact quote-bitmap path) and must never miss a real quote;
  * the LDS table is seeded from the first 256 KiB: keys that first appear later
    are inserted by the kernel, and beyond the table's room they spill to HBM;
  * SUM addends of <= 4 bytes are summed as exact 10^-3 fixed point, wider
    numerals as doubles, in the same group;
  * records the straight path cannot type (blanks, signs, short rows, 9+ byte
    keys, long records) go whole to slow_kernel.
Counts, group sets / order bit-exact; SUM / AVG 1e-6 relative (north_star)."""
import numpy as np
import pytest

import cqtest
import cq_amd

pytestmark = pytest.mark.gpu
REL = 1e-6


def _run(sql, mode):
    old = cq_amd.set_scan_kernel(mode)
    try:
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
        return got, cq_amd.stats(), cq_amd.last_ineligible()
    finally:
        cq_amd.set_scan_kernel(old)


def _tol(sql):
    sel = sql.split(" FROM ")[0]
    items = [s.strip() for s in sel[len("SELECT "):].split(",")]
    return {i for i, s in enumerate(items) if s.upper().startswith(("SUM(", "AVG("))}


def _cmp(got, want, tol, ctx):
    assert (got is None) == (want is None), ctx
    if want is None:
        return
    assert got["columns"] == want["columns"], ctx
    assert len(got["rows"]) == len(want["rows"]), (ctx, len(got["rows"]), len(want["rows"]))
    for i, (g, w) in enumerate(zip(got["rows"], want["rows"])):
        for j, (x, y) in enumerate(zip(g, w)):
            assert cqtest.cell_equal(x, y, REL if j in tol else 0.0), f"{ctx}: row {i} col {j}: {x} vs {y}"


def check(sql, fast=True):
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    tol = _tol(sql)
    got, st, inel = _run(sql, 0)
    assert not inel, (sql, inel)
    if fast:
        assert st["scan_kernel"] == 2, (sql, "fast_kernel did not run", st)
    _cmp(got, want, tol, "auto: " + sql)
    lean, _, _ = _run(sql, 2)
    _cmp(lean, want, tol, "lean: " + sql)
    return st


def _write(path, header, rows, term="\n"):
    path.write_text(header + term + term.join(rows) + term)
    return str(path)


@pytest.fixture(scope="module")
def d(tmp_path_factory):
    return tmp_path_factory.mktemp("fast")


def test_fast_bench_shape(d):
    rng = np.random.default_rng(1)
    rows = ["n%d,s,%d,%s,%d.%02d,role_%03d" % (i % 7, rng.integers(10, 81), "fm"[i % 2], rng.integers(1, 3),
                                                rng.integers(0, 100), rng.integers(0, 1000)) for i in range(200_000)]
    p = _write(d / "bench.csv", "name,surname,age,gender,height,role", rows)
    st = check(f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role")
    assert st["slow_records"] == 0 and st["lds_spills"] == 0, st
    check(f"SELECT COUNT(*) FROM '{p}' WHERE age > 30")
    check(f"SELECT COUNT(*), SUM(age), AVG(height) FROM '{p}' WHERE age <= 45.5")
    check(f"SELECT role, COUNT(*) FROM '{p}' GROUP BY role")
    check(f"SELECT role, SUM(age), SUM(height), AVG(age) FROM '{p}' WHERE age != 50 GROUP BY role")


def test_fast_late_keys_and_spill(d):
    """keys absent from the sample (first 256 KiB) and more keys than the table holds"""
    rows = ["k%05d,%d,%d" % (i % 40, i % 13, i % 100) for i in range(60_000)]          # 40 keys seeded
    rows += ["L%06d,%d,%d" % (i % 5000, i % 7, i % 9) for i in range(120_000)]         # 5000 late keys
    p = _write(d / "late.csv", "a,b,c", rows)
    st = check(f"SELECT c, COUNT(*) FROM '{p}' WHERE b >= 3 GROUP BY c")
    st = check(f"SELECT a, COUNT(*), SUM(c) FROM '{p}' GROUP BY a")
    assert st["lds_spills"] > 0, st


def test_fast_quotes_and_ampersands(d):
    """'&' looks like a quote to the ',' classifier; real quotes in front of needed fields"""
    rng = np.random.default_rng(3)
    rows = []
    for i in range(50_000):
        a = ["a&b", "plain", '"q,uoted"', "x+y", "&", '"'][rng.integers(0, 6)]
        rows.append("%s,%d,g%d,%d.%d" % (a, rng.integers(0, 99), rng.integers(0, 30), rng.integers(0, 9),
                                         rng.integers(0, 9)))
    p = _write(d / "quotes.csv", "a,b,c,e", rows)
    check(f"SELECT c, COUNT(*), SUM(e) FROM '{p}' WHERE b > 40 GROUP BY c")
    check(f"SELECT COUNT(*), SUM(e) FROM '{p}' WHERE b < 10")


def test_fast_numeral_shapes(d):
    """wide and odd numerals in WHERE / SUM fields: 5-7 byte numerals, doubles, signs,
    blanks, exponents, empty fields, dates -- typed in place or sent to slow_kernel"""
    rng = np.random.default_rng(4)
    shapes = ["%d" % rng.integers(0, 99), "%d.%d" % (rng.integers(0, 99), rng.integers(0, 9)), "123456",
              "12.3456", "-5", "+7", " 8", "1e3", "", "2024-01-15", "0.001", ".5", "5.", "abc"]
    rows = []
    for i in range(80_000):
        b = shapes[rng.integers(0, len(shapes))] if rng.integers(0, 4) == 0 else str(rng.integers(0, 60))
        c = shapes[rng.integers(0, len(shapes))] if rng.integers(0, 4) == 0 else "%d.%02d" % (rng.integers(0, 9),
                                                                                            rng.integers(0, 99))
        rows.append("x%d,%s,%s,k%d" % (i % 3, b, c, rng.integers(0, 50)))
    p = _write(d / "shapes.csv", "a,b,c,d", rows)
    check(f"SELECT d, COUNT(*), SUM(c), AVG(c) FROM '{p}' WHERE b > 20 GROUP BY d")
    check(f"SELECT COUNT(*), SUM(b), SUM(c) FROM '{p}' WHERE b <= 30.5")
    check(f"SELECT d, COUNT(*), AVG(b) FROM '{p}' GROUP BY d")


def test_fast_keys(d):
    """empty keys, 8-byte keys, keys with blanks (slow), numerals as keys, CRLF; and
    9-byte keys that appear only after the sampled bytes (the plan chose 8-byte tags:
    those records go to slow_kernel)"""
    rng = np.random.default_rng(5)
    keys = ["", "abcdefgh", "k 1", "z", "12345678", "1.5", "1.50", "NULL", " z"]
    rows = ["%d,%d,%s" % (rng.integers(0, 50), rng.integers(0, 9), keys[rng.integers(0, len(keys))])
            for _ in range(40_000)]
    p = _write(d / "keys.csv", "v,w,k", rows, term="\r\n")
    check(f"SELECT k, COUNT(*), SUM(w) FROM '{p}' WHERE v > 10 GROUP BY k")
    late = rows + ["%d,%d,%s" % (rng.integers(0, 50), rng.integers(0, 9), ["abcdefghi", "z", "toolongkey1"][i % 3])
                   for i in range(30_000)]
    p2 = _write(d / "latelong.csv", "v,w,k", late)
    st = check(f"SELECT k, COUNT(*), SUM(w) FROM '{p2}' WHERE v > 10 GROUP BY k")
    assert st["slow_records"] > 0, st
    rows3 = ["%d,%s" % (i % 50, ["abcdefghi", "x"][i % 2]) for i in range(5000)]
    p3 = _write(d / "long.csv", "v,k", rows3)
    st = check(f"SELECT k, COUNT(*) FROM '{p3}' WHERE v > 10 GROUP BY k", fast=False)   # 16-byte tags: lean_kernel
    assert st["scan_kernel"] == 1, st


def test_fast_role_orders(d):
    """roles in any column order and sharing columns (runtime ranks, skip 0)"""
    rng = np.random.default_rng(6)
    rows = ["k%d,%d,%d.%d,%d" % (rng.integers(0, 90), rng.integers(0, 99), rng.integers(0, 9), rng.integers(0, 9),
                                 rng.integers(0, 5)) for _ in range(60_000)]
    p = _write(d / "orders.csv", "a,b,c,e", rows)
    check(f"SELECT a, COUNT(*), SUM(c) FROM '{p}' WHERE e > 1 GROUP BY a")       # GROUP first
    check(f"SELECT e, COUNT(*), SUM(b), AVG(b) FROM '{p}' WHERE b > 20 GROUP BY e")   # WHERE = SUM column
    check(f"SELECT b, SUM(c), SUM(b) FROM '{p}' WHERE c < 4.5 GROUP BY b")         # GROUP = SUM column
    check(f"SELECT COUNT(*), SUM(e), SUM(b) FROM '{p}' WHERE c >= 2")                # SUM columns reversed


def test_fast_not_for_other_shapes(d):
    rows = ["%d,%d,k%d" % (i % 9, i % 4, i % 3) for i in range(1000)]
    p = _write(d / "other.csv", "a,b,c", rows)
    # a STRING literal over 8 bytes and row-returning SELECTs are lean_kernel's shapes
    st = check(f"SELECT c, COUNT(*) FROM '{p}' WHERE c != 'x12345678' GROUP BY c", fast=False)
    assert st["scan_kernel"] != 2, st
    st = check(f"SELECT a, b FROM '{p}' WHERE b > 1", fast=False)
    assert st["scan_kernel"] != 2, st


def test_plan_sample_misses(d):
    """The plan (tag width, window stride, seeded keys) comes from the first 256 KiB.
    A file whose keys grow past 16 bytes and whose records grow 10x only after that
    must still give the oracle's answer: the records the chosen plan cannot take go
    to slow_kernel (counted in stats), nothing is dropped."""
    rng = np.random.default_rng(8)
    rows = ["%d,k%d,%d.%d" % (rng.integers(0, 99), rng.integers(0, 20), rng.integers(0, 9), rng.integers(0, 9))
            for _ in range(40_000)]                                   # ~0.5 MB of short records
    rows += ["%d,%s,%d.%d" % (rng.integers(0, 99), "a_key_of_more_than_sixteen_bytes_%d" % (i % 30),
                              rng.integers(0, 9), rng.integers(0, 9)) + ",pad" + "x" * int(rng.integers(100, 400))
             for i in range(20_000)]                                  # late long keys, long records
    p = _write(d / "drift.csv", "v,k,h", rows)
    for sql in (f"SELECT k, COUNT(*), SUM(h), AVG(h) FROM '{p}' WHERE v > 30 GROUP BY k",
                f"SELECT COUNT(*), SUM(h) FROM '{p}' WHERE v < 50"):
        want, unsup = cqtest.oracle_query(sql)
        assert not unsup
        got, st, inel = _run(sql, 0)
        assert not inel, inel
        _cmp(got, want, _tol(sql), "drift: " + sql)
    assert st["records"] == 60_000, st


def test_slow_list_overflow_rescan(d, monkeypatch):
    """more slow records than the slow list holds (CQGPU_SLOW_CAP shrinks it from
    2^20 to 512): the scan reruns in byte-range chunks and still equals the oracle"""
    rng = np.random.default_rng(9)
    rows = []
    for i in range(30_000):
        a = '"q,%d"' % (i % 11) if i % 3 == 0 else "p%d" % (i % 11)      # a third quoted: slow records
        rows.append("%s,%d,%d.%d" % (a, rng.integers(0, 99), rng.integers(0, 9), rng.integers(0, 9)))
    p = _write(d / "slowcap.csv", "a,b,c", rows)
    monkeypatch.setenv("CQGPU_SLOW_CAP", "512")
    for sql in (f"SELECT a, COUNT(*), SUM(c) FROM '{p}' WHERE b > 20 GROUP BY a",
                f"SELECT COUNT(*), AVG(c) FROM '{p}'"):
        want, unsup = cqtest.oracle_query(sql)
        assert not unsup
        got, st, inel = _run(sql, 0)
        assert not inel, inel
        _cmp(got, want, _tol(sql), "slow cap: " + sql)
        assert st["slow_records"] > 512, st


@pytest.mark.parametrize("rp2", [False, True])
def test_fast_three_record_pass(d, monkeypatch, rp2):
    """ungrouped plans over records shorter than ~33 bytes take the three-records-per-
    lane pass over windows of the largest stride (config 2's Shape A is 29.9 B/row);
    CQGPU_FAST_RP2 keeps the two-record pass: both must match the oracle, including
    lanes with four record starts (18-byte records), mixed with long records and a
    window whose records a chunk cut splits"""
    from cq_amd import datagen
    if rp2:
        monkeypatch.setenv("CQGPU_FAST_RP2", "1")
    p = d / "shape_a.csv"
    p.write_bytes(datagen.shape_a_bytes(150_000, seed=5, with_role=False))
    for sql in (f"SELECT COUNT(*) FROM '{p}' WHERE age > 30",
                f"SELECT COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age <= 44",
                f"SELECT COUNT(*), SUM(age) FROM '{p}'"):
        check(sql)
    rng = np.random.default_rng(9)
    rows = []
    for i in range(120_000):
        if i % 97 == 0:
            rows.append("x" * int(rng.integers(40, 90)) + ",%d,1.5" % rng.integers(0, 99))
        else:
            rows.append("%s,%d,%d.%d" % ("ab"[i % 2] * int(rng.integers(1, 6)), rng.integers(0, 99),
                                         rng.integers(0, 9), rng.integers(0, 9)))
    q = _write(d / "tiny.csv", "name,age,height", rows)
    check(f"SELECT COUNT(*), SUM(height), AVG(height) FROM '{q}' WHERE age > 50")
    check(f"SELECT COUNT(*) FROM '{q}'")


def test_fast_count_star_no_roles(d):
    """`SELECT COUNT(*) FROM f` with no WHERE has no role at all (NR = 0): every
    record counts as it is -- quotes, records longer than the 64-byte view, short
    and ragged rows, blank lines, CR / CRLF runs -- and none goes to slow_kernel"""
    rng = np.random.default_rng(12)
    rows = []
    for i in range(200_000):
        r = int(rng.integers(0, 8))
        rows.append(['a,1', '"q,x",2', 'x' * int(rng.integers(70, 200)) + ',3', 'z', '"', ',,', ' ', 'k,"y"'][r])
    body = "h1,h2\n" + "\n".join(rows[:100_000]) + "\r\n\r\n" + "\r".join(rows[100_000:]) + "\n\n"
    p = d / "nroles.csv"
    p.write_text(body)
    st = check(f"SELECT COUNT(*) FROM '{p}'")
    assert st["slow_records"] == 0, st


@pytest.mark.parametrize("wn", [False, True])
def test_fast_narrow_numerals_late_wide(d, monkeypatch, wn):
    """When the sampled WHERE / SUM fields (first 256 KiB) are all <= 4 bytes the plan
    takes the narrow-numeral kernel (no 5-7 byte / double side path): numerals wider
    than that which appear only later go whole to slow_kernel.  CQGPU_FAST_WN keeps
    the side path (typed in place, no slow record).  Both equal the oracle."""
    if wn:
        monkeypatch.setenv("CQGPU_FAST_WN", "1")
    rng = np.random.default_rng(13)
    rows = ["%d,%d.%d,k%d" % (rng.integers(0, 99), rng.integers(0, 9), rng.integers(0, 9), i % 37)
            for i in range(60_000)]
    rows += ["%s,%s,k%d" % (["12345", "7", "12.50", "3"][i % 4], ["1.2345", "99999", "2.5", "0.125"][i % 4], i % 37)
             for i in range(40_000)]
    # (the roles in canonical column order: WHERE, SUM, GROUP BY)
    p = _write(d / "latewide.csv", "v,h,k", rows)
    for sql in (f"SELECT k, COUNT(*), SUM(h), AVG(h) FROM '{p}' WHERE v > 30 GROUP BY k",
                f"SELECT COUNT(*), SUM(h), AVG(h) FROM '{p}' WHERE v < 50"):
        st = check(sql)
        if wn:
            assert st["slow_records"] == 0, st
        else:
            assert st["slow_records"] > 0, st


def test_fast_min_max(d):
    """MIN / MAX of narrow numerals in fast_kernel (EXT builds): (10^-3 fixed-point
    value, first-row code) in one 64-bit LDS atomic; the blocks' extremes merged as
    (value, record offset) keys by one global atomicMin and the winner's cell typed
    once from its record by raw_merge_kernel (evaluate_aggregate keeps the first cell that compares
    strictly better, evaluator_aggregates.c:311-326): ties between spellings of one
    value ("1.5" / "1.50" / INTEGER vs DOUBLE) keep the first record's cell; NULLs
    skipped; groups whose every value is NULL keep NULL"""
    rng = np.random.default_rng(31)
    heights = ["1.5", "1.50", "2", "2.0", "0.75", "3", "", "9.99", "0.5"]
    rows = ["n%d,s,%d,%s,%s,role_%03d" % (i % 7, rng.integers(10, 81), "fm"[i % 2],
                                           heights[int(rng.integers(0, len(heights)))] if i % 97 else "",
                                           int(rng.integers(0, 300))) for i in range(150_000)]
    rows += ["n0,s,40,f,,role_999"] * 5                               # a group of NULLs only
    p = _write(d / "ext.csv", "name,surname,age,gender,height,role", rows)
    for q in (f"SELECT role, COUNT(*), SUM(height), AVG(height), MIN(height) FROM '{p}' WHERE age > 30 GROUP BY role",
              f"SELECT role, MAX(height) FROM '{p}' GROUP BY role",
              f"SELECT role, MIN(height), COUNT(*) FROM '{p}' WHERE age <= 40 GROUP BY role",
              f"SELECT MIN(height) FROM '{p}'",
              f"SELECT COUNT(*), MAX(height), SUM(height) FROM '{p}' WHERE age > 70",
              f"SELECT gender, MAX(age) FROM '{p}' GROUP BY gender"):
        check(q)


def test_fast_min_max_declined_and_mixed(d):
    """shapes the EXT builds leave to the general scan: two extremes, an extreme over
    a second numeric column; and a column that mixes numbers with text (the slow
    path's STRING cells: value_compare's cross-class "equal" makes the result order-
    dependent, which the class-split passes reproduce)"""
    rows = ["%d,%s,%d" % (i % 50, ("x%d" % i) if i % 1009 == 0 else "%d.%d" % (i % 9, i % 10), i % 77)
            for i in range(80_000)]
    p = _write(d / "mixed_ext.csv", "g,v,w", rows)
    check(f"SELECT g, MIN(v), COUNT(*) FROM '{p}' GROUP BY g", fast=False)
    check(f"SELECT g, MIN(w), MAX(w) FROM '{p}' GROUP BY g", fast=False)
    check(f"SELECT g, SUM(v), MAX(w) FROM '{p}' GROUP BY g", fast=False)
    check(f"SELECT g, MAX(w), COUNT(*) FROM '{p}' WHERE w > 5 GROUP BY g")


def test_fast_string_literal_where(d):
    """WHERE `column op 'literal'` (1-8 byte STRING literal) in fast_kernel: a field of
    1-8 bytes with no leading digit / sign / dot and no byte <= ' ' is a STRING
    (infer_type, csv_reader.c:133-240) compared by strcmp order (evaluate_expression
    -> value_compare); numeral- or date-shaped fields, 9+ byte fields and fields with
    blanks go whole to slow_kernel, which types them exactly (value_compare across
    classes); empty fields are NULL"""
    rng = np.random.default_rng(77)
    words = ["f", "m", "fe", "ff", "e", "g", "role_001", "role_0010", "12", "1990-01-01", "-x", ".5", "f ",
             "zz", "F", "", "a&b"]
    rows = ["%s,%d,%s,%d.%d,role_%03d" % ("n%d" % (i % 5), i % 90, words[int(rng.integers(0, len(words)))],
                                         i % 3, i % 10, int(rng.integers(0, 200))) for i in range(120_000)]
    p = _write(d / "wstr.csv", "name,age,gender,height,role", rows)
    for lit, op in (("f", "="), ("m", "!="), ("f", "<"), ("fe", ">"), ("role_001", ">="), ("g", "<="), ("F", "=")):
        check(f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE gender {op} '{lit}' GROUP BY role")
    check(f"SELECT COUNT(*), SUM(height) FROM '{p}' WHERE gender = 'f'")
    check(f"SELECT COUNT(*) FROM '{p}' WHERE gender > 'e'")
    check(f"SELECT role, COUNT(*) FROM '{p}' WHERE gender = 'f' GROUP BY role")
    # the literal itself numeral-shaped (a STRING literal all the same) and a 9-byte literal
    check(f"SELECT role, COUNT(*) FROM '{p}' WHERE gender = '12' GROUP BY role")
    check(f"SELECT role, COUNT(*) FROM '{p}' WHERE gender = 'role_0010' GROUP BY role", fast=False)


def test_fast_compound_where(d):
    """compound WHEREs on fast_kernel (the WX builds): NOT / AND / OR trees of up to 4
    leaves over up to 2 columns -- comparisons either way round, BETWEEN (AND of >= and
    <=, parser_expressions.c:481-523), [NOT] IN lists of up to 8 literals -- evaluated
    as the parsed tree with every leaf evaluated (evaluator_conditions.c:62-164;
    right-associative, no precedence).  NUMBER columns: 1-4 byte numerals typed as exact
    10^-3 fixed point compared with the reference's double semantics (dotted fields,
    literals such as 1.1 that no double equals exactly, negative literals); STRING
    columns: 1-8 byte words.  Fields of other shapes (wide numerals, dates, blanks,
    signs, 9+ bytes) and empty ones (NULL) exercise slow_kernel and the NULL outcomes."""
    rng = np.random.default_rng(91)
    words = ["f", "m", "fe", "ff", "e", "g", "role_001", "role_0010", "12", "1990-01-01", "-x", ".5", "f ",
             "zz", "F", ""]
    # the plan sample (the first 256 KiB) sees 1-4 byte numerals only: the compound builds
    # type <= 4-byte numerals; the wider / other shapes come later and go to slow_kernel
    ages = [str(x) for x in range(0, 100)] + ["", "-3", "1.5", "7.25", " 8", "abc", "30.0"]
    late_ages = ages + ["12345", "2024-01-05", "1234567"]
    hts = ["1.1", "1.10", "2.25", "1.5", ".001", "1.", ".5", "2", "", "9999", "1.0"]
    late_hts = hts + ["1.1234", "0.001", "12345.5"]
    rows = []
    for i in range(150_000):
        a, h = (late_ages, late_hts) if i >= 20_000 else (ages, hts)
        rows.append("%s,%s,%s,%s,role_%03d" % ("n%d" % (i % 5), a[int(rng.integers(0, len(a)))] if i % 13 else str(i % 90),
                                              words[int(rng.integers(0, len(words)))], h[int(rng.integers(0, len(h)))],
                                              int(rng.integers(0, 40))))
    p = _write(d / "wx.csv", "name,age,gender,height,role", rows)
    G = "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE {w} GROUP BY role"
    for w in ("age BETWEEN 20 AND 40",
              "age > 30 AND gender = 'f'",
              "age < 20 OR gender != 'm'",
              "gender = 'f' AND age > 30 OR age < 10",          # AND(=, OR(>, <)): no precedence
              "NOT age > 30",
              "30 < age AND 50 >= age",
              "age > -5 AND height < 2",
              "height = 1.1 OR height >= 2.25",
              "height BETWEEN 1.1 AND 1.5",
              "age IN (10, 20, 30.0, 45)",
              "age NOT IN (10, 20, 30, 45) AND gender IN ('f', 'm', 'fe')",
              "role IN ('role_001', 'role_002', 'role_010', 'role_039')",
              "gender NOT IN ('f', 'm') OR age = 7",
              "height IN (1.1, 2.25, 0.001, 2)",
              "age != 50 AND age != 60 AND age != 70 AND gender > 'e'"):
        check(G.format(p=p, w=w))
    # ungrouped, two SUM columns, the WHERE column also summed
    check(f"SELECT COUNT(*), SUM(height) FROM '{p}' WHERE age BETWEEN 25 AND 35")
    check(f"SELECT COUNT(*) FROM '{p}' WHERE gender = 'f' OR gender = 'm'")
    check(f"SELECT role, SUM(age), AVG(height) FROM '{p}' WHERE age > 20 AND height > 1.2 GROUP BY role")
    # (GROUP BY gender: its sampled keys exceed 8 bytes -- lean_kernel's 16-byte tags)
    check(f"SELECT gender, COUNT(*), SUM(age) FROM '{p}' WHERE age BETWEEN 10 AND 60 GROUP BY gender", fast=False)
    # outside the compound builds (5 leaves; a column compared with both classes;
    # 3 WHERE columns): the general kernels, same answers
    check(G.format(p=p, w="age = 1 OR age = 2 OR age = 3 OR age = 4 OR age = 5"), fast=False)
    check(G.format(p=p, w="age > 30 OR age = 'abc'"), fast=False)
    check(G.format(p=p, w="age > 30 AND gender = 'f' AND height > 1.2"), fast=False)


def test_fast_compound_where_declines_wide_numerals(d):
    """a NUMBER WHERE column whose sampled fields exceed 4 bytes keeps the general
    kernels (the compound builds type <= 4-byte numerals only)"""
    rows = ["%d,%d.%03d,g%d" % (i % 100, 1000 + i % 9000, i % 1000, i % 7) for i in range(30_000)]
    p = _write(d / "wxwide.csv", "a,b,g", rows)
    st = check(f"SELECT g, COUNT(*) FROM '{p}' WHERE b BETWEEN 2000 AND 3000 AND a > 10 GROUP BY g", fast=False)
    assert st["scan_kernel"] != 2, st
