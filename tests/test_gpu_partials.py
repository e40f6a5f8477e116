"""Range-partitioned aggregation and row SELECTs (SURVEY.md section 8e, config 4 on one GPU).

Every "rank" opens its own newline-snapped byte range of one file with the
product entry point (cqgpu_table_open_range), runs cqgpu_query_partial on it,
and cqgpu_merge_partials over all ranks' blobs must equal the ORACLE's answer on
the whole file (oracle/cq_oracle.c, pinned to the reference): counts, group set,
first-appearance order, MIN/MAX and representative cells exact, SUM/AVG within
1e-6 relative.  Files carry CR, CRLF and blank-line runs, so cuts land on them.
"""
import os
import random

import pytest

import cqtest
import cq_amd
from cq_amd import abi, datagen
from test_gpu_parity import compare, tolerant_columns

pytestmark = pytest.mark.gpu

QUERIES = [
    "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role",
    "SELECT COUNT(*), SUM(height), MIN(height), MAX(age) FROM '{p}' WHERE gender = 'f'",
    "SELECT name, COUNT(*), MIN(role), MAX(role) FROM '{p}' GROUP BY name",
    "SELECT age, COUNT(*) FROM '{p}' GROUP BY age HAVING COUNT(*) > 1900 ORDER BY COUNT(*) DESC LIMIT 5",
    "SELECT gender, AVG(age) FROM '{p}' WHERE role LIKE 'role_0%' GROUP BY gender",
    "SELECT COUNT(*) FROM '{p}' WHERE age > 30",
]


def _mixed_terminators(data: bytes, seed: int) -> bytes:
    """the same records with every terminator replaced by a random run"""
    rng = random.Random(seed)
    runs = [b"\n", b"\r\n", b"\r", b"\n\n", b"\r\n\r\n", b"\n\r"]
    lines = data.split(b"\n")
    out = []
    for i, ln in enumerate(lines):
        out.append(ln)
        if i + 1 < len(lines):
            out.append(rng.choice(runs) if i > 0 else b"\n")
    return b"\r\n\n" + b"".join(out)


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("ranges")
    plain = datagen.shape_a_bytes(120_000, seed=11, with_role=True)
    paths = {}
    for name, data in (("plain", plain), ("mixed", _mixed_terminators(datagen.shape_a_bytes(30_000, seed=12,
                                                                                              with_role=True), 3))):
        p = os.path.join(str(d), name + ".csv")
        with open(p, "wb") as fh:
            fh.write(data)
        paths[name] = p
    return paths


def _merged(ast, path, nranks):
    tabs = [cq_amd.Table.open_range(path, r, nranks) for r in range(nranks)]
    try:
        sizes = [t.nbytes for t in tabs]
        assert sum(sizes) == os.path.getsize(path)
        blobs = [cq_amd.query_partial(ast, [t]) for t in tabs]
    finally:
        for t in tabs:
            t.close()
    tp = cq_amd.merge_partials(ast, blobs)
    assert tp, cq_amd.last_error()
    got = abi.table_to_py(tp)
    cq_amd.result_free(tp)
    return got


@pytest.mark.parametrize("sql", QUERIES)
@pytest.mark.parametrize("nranks", [1, 3, 8])
def test_merge_equals_oracle(files, sql, nranks):
    path = files["plain"]
    q = sql.format(p=path)
    want, unsup = cqtest.oracle_query(q)
    assert not unsup and want is not None
    with cqtest.Parsed(q) as ast:
        got = _merged(ast, path, nranks)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{nranks} ranks: {q}")


@pytest.mark.parametrize("nranks", [2, 5, 7, 16])
def test_mixed_terminator_cuts(files, nranks):
    path = files["mixed"]
    for sql in QUERIES[:3]:
        q = sql.format(p=path)
        want, unsup = cqtest.oracle_query(q)
        assert not unsup and want is not None
        with cqtest.Parsed(q) as ast:
            got = _merged(ast, path, nranks)
            tol = tolerant_columns(ast)
        compare(got, want, tol, f"{nranks} ranks: {q}")


def test_range_bases_are_record_starts(files):
    path = files["mixed"]
    data = open(path, "rb").read()
    for n in (2, 5, 16):
        for r in range(n):
            t = cq_amd.Table.open_range(path, r, n)
            lo, hi, _, _ = cq_amd.range_bounds(data, r, n)
            assert t.base_offset == lo and t.nbytes == hi - lo
            t.close()


def test_more_ranks_than_records(tmp_path):
    p = tmp_path / "tiny.csv"
    p.write_bytes(b"a,b\n1,x\n2,y\n")
    q = f"SELECT b, COUNT(*), SUM(a) FROM '{p}' GROUP BY b"
    want, _ = cqtest.oracle_query(q)
    with cqtest.Parsed(q) as ast:
        got = _merged(ast, str(p), 9)
        tol = tolerant_columns(ast)
    compare(got, want, tol, q)


# ---------------------------------------------------------------- device-side dense merge
# (queries keep at most 4 SELECT items: the reference parser corrupts its heap on more,
# SURVEY appendix A Q13 -- the parse itself, before any evaluation)
def _collectives_by_hand(parts):
    """cqgpu_partial_next / put over simulated ranks in one process: an all_gather
    is a concatenation, the reduces are torch reductions over the ranks' buffers
    (a reduce to rank 0 leaves the other ranks' buffers as they were)"""
    import torch
    from cq_amd import dist as D
    n = len(parts)
    results, sizes = [None] * n, None
    while True:
        colls = [p.next(results[r], sizes, r, n) for r, p in enumerate(parts)]
        ops = {op for op, _ in colls}
        assert len(ops) == 1, colls                 # every rank asks for the same collective
        op = ops.pop()
        if op == D.DONE:
            return parts[0].result()
        if op == D.DECLINE:
            return None
        bufs = []
        for (o, cnt), p in zip(colls, parts):
            b = torch.empty(max(cnt, 1), dtype=D._DTYPES[op], device="cuda")[:cnt]
            p.put(b)
            bufs.append(b)
        torch.cuda.synchronize()
        sizes = None
        if op == D.ALLGATHER:
            cat = torch.cat(bufs)
            sizes = [b.numel() for b in bufs]
            results = [cat] * n
        else:
            assert len({b.numel() for b in bufs}) == 1
            st = torch.stack(bufs)
            red = st.min(0).values if op == D.ALLREDUCE_MIN_I64 else st.sum(0)
            if op in (D.ALLREDUCE_MIN_I64, D.ALLREDUCE_SUM_F64):
                results = [red] * n
            else:
                results = [red] + bufs[1:]
        torch.cuda.synchronize()


def _dense_merge_by_hand(ast, tabs):
    from cq_amd.dist import DensePartial
    parts = [DensePartial(ast, t) for t in tabs]
    try:
        if not all(p.ok for p in parts):
            return None
        return _collectives_by_hand(parts)
    finally:
        for p in parts:
            p.free()


def _dense(ast, path, nranks):
    tabs = [cq_amd.Table.open_range(path, r, nranks) for r in range(nranks)]
    try:
        tp = _dense_merge_by_hand(ast, tabs)
    finally:
        for t in tabs:
            t.close()
    assert tp, cq_amd.last_error() or cq_amd.last_ineligible()
    got = abi.table_to_py(tp)
    cq_amd.result_free(tp)
    return got


DENSE = QUERIES + [
    "SELECT role, MIN(height), MAX(age), STDDEV(height) FROM '{p}' WHERE age > 30 GROUP BY role",
    "SELECT gender, role, COUNT(*), AVG(age) FROM '{p}' WHERE height > 1.8 GROUP BY gender, role",
    "SELECT name, surname, COUNT(*), MAX(height) FROM '{p}' WHERE age < 22 GROUP BY role",
    "SELECT age / 10 AS decade, COUNT(*), MIN(surname), MAX(role) FROM '{p}' GROUP BY decade",
    "SELECT role, height * 100 AS hc, COUNT(*) FROM '{p}' GROUP BY role HAVING COUNT(*) > 100 "
    "ORDER BY role DESC LIMIT 7",
    "SELECT role, age + 1 AS a1, name, COUNT(*) FROM '{p}' WHERE age > 50 GROUP BY role",
    "SELECT STDDEV(age), STDDEV(height), MIN(gender), MAX(surname) FROM '{p}'",
    "SELECT role, MIN(name), MAX(name), COUNT(*) FROM '{p}' WHERE age > 60 GROUP BY role",
]


@pytest.mark.parametrize("sql", DENSE)
@pytest.mark.parametrize("nranks", [1, 3, 8])
def test_dense_merge_equals_oracle(files, sql, nranks):
    path = files["plain"]
    q = sql.format(p=path)
    want, unsup = cqtest.oracle_query(q)
    assert not unsup and want is not None
    with cqtest.Parsed(q) as ast:
        got = _dense(ast, path, nranks)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"dense {nranks} ranks: {q}")


def test_dense_merge_mixed_terminators(files):
    path = files["mixed"]
    for sql in DENSE[:3] + DENSE[6:9]:
        q = sql.format(p=path)
        want, unsup = cqtest.oracle_query(q)
        assert not unsup and want is not None
        for n in (2, 5):
            with cqtest.Parsed(q) as ast:
                got = _dense(ast, path, n)
                tol = tolerant_columns(ast)
            compare(got, want, tol, f"dense {n} ranks: {q}")


def test_dense_merge_typed_keys(tmp_path):
    """group keys of every class across ranks; a representative cell that is a DATE
    on one rank and the same text as a STRING on another keeps the first row's kind"""
    rows = ["k,v"]
    vals = ["2024-01-05", " 2024-01-05 ", "NULL", "", "7", "7.0", "-0.5", "x", "2024-1-5"]
    for i in range(9000):
        rows.append(f"{vals[(i * 5) % len(vals)]},{i % 13}")
    p = tmp_path / "typed.csv"
    p.write_text("\n".join(rows) + "\n")
    for q in (f"SELECT k, COUNT(*), SUM(v), AVG(v) FROM '{p}' GROUP BY k",
              f"SELECT k, MIN(v), MAX(k) FROM '{p}' GROUP BY k"):
        want, _ = cqtest.oracle_query(q)
        for n in (2, 5):
            with cqtest.Parsed(q) as ast:
                got = _dense(ast, str(p), n)
                tol = tolerant_columns(ast)
            compare(got, want, tol, f"dense typed keys, {n} ranks: {q}")


def test_dense_merge_long_text(tmp_path):
    """group keys over 16 bytes (gathered with their bytes, compared exactly) and
    representative / extreme texts over 8 bytes (the owners' side gather)"""
    rng = random.Random(9)
    rows = ["k,name,v"]
    keys = [f"a_group_key_longer_than_sixteen_{i:03d}" for i in range(40)] + ["short", "mid_len_key_1234"]
    for i in range(12000):
        k = keys[rng.randrange(len(keys))]
        rows.append(f"{k},person_{rng.randrange(10**6)}_{'x' * rng.randrange(0, 12)},{rng.randrange(-50, 50)}")
    p = tmp_path / "long.csv"
    p.write_text("\n".join(rows) + "\n")
    for sql in (f"SELECT k, name, COUNT(*), SUM(v) FROM '{p}' GROUP BY k",
                f"SELECT k, MIN(v), MAX(v) FROM '{p}' WHERE v < 40 GROUP BY k",
                f"SELECT k, COUNT(*), STDDEV(v) FROM '{p}' WHERE v > 0 GROUP BY k ORDER BY k"):
        want, _ = cqtest.oracle_query(sql)
        for n in (1, 3, 8):
            with cqtest.Parsed(sql) as ast:
                got = _dense(ast, str(p), n)
                tol = tolerant_columns(ast)
            compare(got, want, tol, f"dense long text, {n} ranks: {sql}")


def test_dense_merge_mixed_classes(mixed_classes):
    for sql in ("SELECT g, MIN(v), MAX(v), COUNT(*) FROM '{p}' GROUP BY g",
                "SELECT MIN(v), MAX(v) FROM '{p}'"):
        q = sql.format(p=mixed_classes)
        want, _ = cqtest.oracle_query(q)
        for n in (1, 2, 3, 5, 8):
            with cqtest.Parsed(q) as ast:
                got = _dense(ast, mixed_classes, n)
                tol = tolerant_columns(ast)
            compare(got, want, tol, f"dense mixed classes, {n} ranks: {q}")


def test_dict_build_high_contention(tmp_path):
    """dict_build_kernel's relaxed publish (memory model) under
    contention: 64 simulated ranks holding the same 1,000 keys (64,000 inserts of
    the same keys from every CU, lanes of a wave racing for one slot) must build
    exactly the 1,000-entry dictionary: COUNT and SUM come out 64 times the oracle's,
    AVG equal, groups in the same order"""
    p = tmp_path / "role.csv"
    datagen.write_shape_a(str(p), 60_000, seed=31, with_role=True)
    q = f"SELECT COUNT(*), SUM(height), AVG(height) FROM '{p}' GROUP BY role"
    want, unsup = cqtest.oracle_query(q)
    assert not unsup and len(want["rows"]) == 1000
    from cq_amd.dist import DensePartial
    with cqtest.Parsed(q) as ast:
        t = cq_amd.Table.open_range(str(p), 0, 1)
        parts = [DensePartial(ast, t) for _ in range(64)]
        try:
            assert all(x.ok for x in parts), cq_amd.last_ineligible()
            tp = _collectives_by_hand(parts)
            assert tp, cq_amd.last_error()
            got = abi.table_to_py(tp)
            cq_amd.result_free(tp)
        finally:
            for x in parts:
                x.free()
            t.close()
    assert len(got["rows"]) == 1000
    for g, w in zip(got["rows"], want["rows"]):
        assert g[0] == ("I", 64 * w[0][1])
        assert cqtest.cell_equal(g[1], ("D", 64 * w[1][1]), 1e-9)
        assert cqtest.cell_equal(g[2], w[2], 1e-9)


def test_dense_merge_refusals(files):
    """MEDIAN needs every value: it leaves the dense path (the blob merge takes it)"""
    from cq_amd.dist import DensePartial
    for sql, why in (("SELECT role, MEDIAN(age) FROM '{p}' GROUP BY role", "MEDIAN"),):
        q = sql.format(p=files["plain"])
        with cqtest.Parsed(q) as ast:
            t = cq_amd.Table.open_range(files["plain"], 0, 2)
            part = DensePartial(ast, t)
            ok = part.ok
            part.free()
            t.close()
        assert not ok and why in cq_amd.last_ineligible(), (sql, cq_amd.last_ineligible())


# ---------------------------------------------------------------- row-returning SELECT across ranges
# Every rank projects its shard's matching rows, each keyed by its record's whole-file
# byte position ("CQR1"); the merge orders all ranks' rows by position -- build_result's
# row order over the whole file -- before ORDER BY / DISTINCT / LIMIT / OFFSET.
ROW_QUERIES = [
    "SELECT name, age FROM '{p}' WHERE age > 62 AND height < 150",
    "SELECT * FROM '{p}' WHERE height > 195 LIMIT 40 OFFSET 17",
    "SELECT name, age * 2 AS a2, height FROM '{p}' WHERE role = 'role_003' ORDER BY age DESC LIMIT 25",
    "SELECT DISTINCT gender, role FROM '{p}' WHERE age < 19 AND role LIKE 'role_00%'",
    "SELECT surname FROM '{p}' LIMIT 9 OFFSET 3000",
    "SELECT name, height FROM '{p}' WHERE name LIKE 'Zz%'",          # no row anywhere
]


@pytest.mark.parametrize("sql", ROW_QUERIES)
@pytest.mark.parametrize("nranks", [1, 3, 8])
def test_row_select_across_ranges(files, sql, nranks):
    path = files["plain"]
    q = sql.format(p=path)
    want, unsup = cqtest.oracle_query(q)
    assert not unsup and want is not None
    with cqtest.Parsed(q) as ast:
        got = _merged(ast, path, nranks)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{nranks} ranks: {q}")


@pytest.mark.parametrize("nranks", [2, 5, 16])
def test_row_select_mixed_terminator_cuts(files, nranks):
    """CR / CRLF / blank-line runs at the cuts: no record lost, none twice, file order"""
    path = files["mixed"]
    for sql in ROW_QUERIES[:3] + ["SELECT * FROM '{p}' WHERE age > 70"]:
        q = sql.format(p=path)
        want, unsup = cqtest.oracle_query(q)
        assert not unsup and want is not None
        with cqtest.Parsed(q) as ast:
            got = _merged(ast, path, nranks)
            tol = tolerant_columns(ast)
        compare(got, want, tol, f"{nranks} ranks: {q}")


# ---------------------------------------------------------------- MEDIAN / mixed-class MIN/MAX across ranges
VLA_QUERIES = [
    "SELECT role, MEDIAN(height), STDDEV(age), COUNT(*) FROM '{p}' WHERE age > 40 GROUP BY role",
    "SELECT MEDIAN(age), MEDIAN(height) FROM '{p}'",
    "SELECT gender, MEDIAN(age) FROM '{p}' WHERE role LIKE 'role_01%' GROUP BY gender",
]


@pytest.mark.parametrize("sql", VLA_QUERIES)
@pytest.mark.parametrize("nranks", [1, 3, 8])
def test_median_across_ranges(files, sql, nranks):
    path = files["plain"]
    q = sql.format(p=path)
    want, unsup = cqtest.oracle_query(q)
    assert not unsup and want is not None
    with cqtest.Parsed(q) as ast:
        got = _merged(ast, path, nranks)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{nranks} ranks: {q}")


@pytest.fixture(scope="module")
def mixed_classes(tmp_path_factory):
    """a column whose cells mix numbers, strings and dates, with groups whose first
    non-NULL cell is of each class, and shards that see only one class of a group"""
    rng = random.Random(5)
    vals = {"num": ["7", "-3.5", "12", "0", "100", "2.25"],
            "str": ["pear", "apple", "zeta", "Apple", "m"],
            "date": ["2024-01-05", "1999-12-31", "2030-06-01", "2001-02-03"]}
    rows = ["g,v"]
    for i in range(6000):
        g = f"g{i % 23}"
        # each group's first cells come from a group-dependent class, later ones from any
        if i < 23 * 3:
            cls = ("num", "str", "date")[(i % 23) % 3]
        elif i % 23 == 5 and i < 3000:
            cls = "str"
        else:
            cls = rng.choice(("num", "str", "date", "null"))
        rows.append(f"{g}," + ("" if cls == "null" else rng.choice(vals[cls])))
    p = tmp_path_factory.mktemp("mixed_cls") / "mixed.csv"
    p.write_text("\n".join(rows) + "\n")
    return str(p)


@pytest.mark.parametrize("nranks", [1, 2, 3, 5, 8])
def test_mixed_class_minmax_across_ranges(mixed_classes, nranks):
    for sql in ("SELECT g, MIN(v), MAX(v), COUNT(*) FROM '{p}' GROUP BY g",
                "SELECT MIN(v), MAX(v) FROM '{p}'",
                "SELECT g, MAX(v), MEDIAN(v) FROM '{p}' WHERE g = 'g5' OR g = 'g7' GROUP BY g"):
        q = sql.format(p=mixed_classes)
        want, unsup = cqtest.oracle_query(q)
        assert not unsup and want is not None
        with cqtest.Parsed(q) as ast:
            got = _merged(ast, mixed_classes, nranks)
            tol = tolerant_columns(ast)
        compare(got, want, tol, f"{nranks} ranks: {q}")


def _very_long_file(tmp_path):
    p = tmp_path / "verylong.csv"
    p.write_text("k,v\n" + "\n".join("%s,%d" % ("x" * 60 + str(i % 5), i % 7) for i in range(20_000)) + "\n")
    return str(p)


def _many_groups_file(tmp_path):
    p = tmp_path / "many.csv"
    p.write_text("k,v\n" + "\n".join("%d,%d" % (i % 9000, i % 7) for i in range(40_000)) + "\n")
    return str(p)


@pytest.mark.parametrize("kind", ["verylong", "many"])
def test_single_gpu_keys_past_gather_merge(tmp_path, kind):
    """the data the gather-merge declines (group keys over 48 bytes, more than 4096
    groups) on one GPU, through cqgpu_query: the oracle's answer"""
    path = _very_long_file(tmp_path) if kind == "verylong" else _many_groups_file(tmp_path)
    q = f"SELECT k, COUNT(*), SUM(v) FROM '{path}' GROUP BY k"
    want, _ = cqtest.oracle_query(q)
    with cqtest.Parsed(q) as ast:
        got = cq_amd.evaluate(ast)
        tol = tolerant_columns(ast)
    assert got is not None, cq_amd.last_error()
    compare(got, want, tol, q)


@pytest.mark.parametrize("kind", ["verylong", "many"])
@pytest.mark.parametrize("nranks", [1, 3])
def test_dense_merge_keys_past_gather_merge(tmp_path, kind, nranks):
    """the same data through the dense merge (where cqgpu_dist_query sends it when
    the gather-merge declines)"""
    path = _very_long_file(tmp_path) if kind == "verylong" else _many_groups_file(tmp_path)
    q = f"SELECT k, COUNT(*), SUM(v) FROM '{path}' GROUP BY k"
    want, _ = cqtest.oracle_query(q)
    with cqtest.Parsed(q) as ast:
        got = _dense(ast, path, nranks)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"dense {nranks} ranks: {q}")


@pytest.mark.parametrize("merge", ["dense", "blobs"])
def test_composite_keys_exact_across_ranks(tmp_path, monkeypatch, merge):
    """composite GROUP BY keys cross the ranks as their joined key texts (executor.hip
    comp_key_texts: create_groups' identity, evaluator.c:113-212), not as the 128-bit
    part digest: with the digest cut to 2 bits (CQGPU_TEST_DIGEST_BITS) six ranks
    holding one key each must collide somewhere, and both merges must still keep the
    six groups apart (VERDICT r4 missing 2)"""
    monkeypatch.setenv("CQGPU_TEST_DIGEST_BITS", "2")
    header = b"a,b,v\n"
    blocks = [b"".join(b"%d,k%d,%d\n" % (r, r * 7, i) for i in range(300)) for r in range(6)]
    data = header + b"".join(blocks)
    p = tmp_path / "comp.csv"
    p.write_bytes(data)
    q = f"SELECT a, b, COUNT(*), SUM(v) FROM '{p}' GROUP BY a, b"
    want, unsup = cqtest.oracle_query(q)
    assert not unsup and want
    tabs, at = [], len(header)
    for r, blk in enumerate(blocks):
        tabs.append(cq_amd.Table.from_bytes(header + blk) if r == 0 else
                    cq_amd.Table.from_bytes(blk, base_offset=at, header=header))
        at += len(blk)
    try:
        with cqtest.Parsed(q) as ast:
            if merge == "dense":
                tp = _dense_merge_by_hand(ast, tabs)
            else:
                tp = cq_amd.merge_partials(ast, [cq_amd.query_partial(ast, [t]) for t in tabs])
            assert tp, cq_amd.last_error()
            got = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            tol = tolerant_columns(ast)
    finally:
        for t in tabs:
            t.close()
    assert len(got["rows"]) == 6
    compare(got, want, tol, f"{merge}: {q}")
