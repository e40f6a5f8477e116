"""Parity of the wave-autonomous scans -- fast_kernel (cq_amd/csrc/fast.hip) where the
plan has its shape, lean_kernel (lean.hip) forced, and the general scan_kernel --
with the oracle on inputs aimed at their edges.

lean_kernel splits the file into 2 KiB windows, one wave each, and sees only the
first 64 bytes of a record through its separator bitmaps; records it cannot type
exactly go whole to slow_kernel.  The files below put records across window
boundaries, make records longer than 64 bytes, put quotes, CR/LF runs, empty
lines, short rows, trailing delimiters and blank fields in front of needed
columns, and pack > 64 records into one window (several passes), so every branch
of the window walk is compared with the reference semantics (oracle).

Counts, group sets / order and row sets bit-exact; SUM / AVG 1e-6 relative
(north_star tolerance).
"""
import ctypes as C

import numpy as np
import pytest

import cqtest
import cq_amd
from cq_amd import datagen

pytestmark = pytest.mark.gpu
REL = 1e-6


def _messy_lines(n, seed):
    rng = np.random.default_rng(seed)
    words = ["x", "y", "zz", "role_007", "averyveryverylongkey", "", " pad", "k9"]
    out = ["a,b,c,d,e"]
    for i in range(n):
        a = words[rng.integers(0, len(words))]
        b = str(int(rng.integers(-5, 60)))
        c = "%d.%02d" % (rng.integers(0, 3), rng.integers(0, 100))
        d = "g%d" % rng.integers(0, 40)
        e = "x" if rng.integers(0, 2) else "y"
        k = rng.integers(0, 40)
        if k == 0:
            a = "q" * int(rng.integers(60, 140))            # needed fields past the first 64 bytes
        elif k == 1:
            a = '"' + "u,v" + '"'                           # quoted delimiter before needed fields
        elif k == 2:
            c = '"' + c + '"'
        elif k == 3:
            b = " " + b                                      # blank in a needed field
        elif k == 4:
            out.append("")                                   # empty line
        elif k == 5:
            out.append(f"{a},{b}")                           # short row
            continue
        elif k == 6:
            out.append(f"{a},{b},{c},{d},")                  # trailing delimiter: e dropped
            continue
        elif k == 7:
            out.append(f"{a},{b},{c},{d}, ")                 # blank trailing field: dropped
            continue
        elif k == 8:
            c = "1e2"                                        # strtod-only numeral shape
        elif k == 9:
            b = "+%d" % rng.integers(0, 9)
        elif k == 10:
            c = ""
        out.append(f"{a},{b},{c},{d},{e}")
    return out


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("lean")
    f = {}
    lines = _messy_lines(60_000, 5)
    f["messy_lf"] = d / "messy_lf.csv"
    f["messy_lf"].write_text("\n".join(lines) + "\n")
    f["messy_crlf"] = d / "messy_crlf.csv"
    f["messy_crlf"].write_text("\r\n".join(lines))                     # no final terminator
    rng = np.random.default_rng(9)
    tiny = ["a,b,c,d,e"] + ["%d" % rng.integers(0, 4) for _ in range(40_000)]   # 2-byte records
    f["tiny"] = d / "tiny.csv"
    f["tiny"].write_text("\n".join(tiny) + "\n")
    runs = ["a,b,c,d,e"]
    for i in range(30_000):
        runs.append("%s,%d,%d.5,g%d,x" % ("w" if i % 3 else "v", i % 17, i % 5, i % 7))
        if i % 11 == 0:
            runs.append("\r\n\n\r")
    f["runs"] = d / "runs.csv"
    f["runs"].write_text("\n".join(runs))
    f["role"] = d / "role.csv"
    datagen.write_shape_a(str(f["role"]), 300_000, seed=21, with_role=True)
    return f


GENERIC = [
    "SELECT COUNT(*) FROM '{P}'",
    "SELECT COUNT(*), SUM(c), AVG(c) FROM '{P}' WHERE b > 10",
    "SELECT a, COUNT(*), SUM(c) FROM '{P}' GROUP BY a",
    "SELECT d, COUNT(*), AVG(b), SUM(c) FROM '{P}' WHERE e = 'x' GROUP BY d",
    "SELECT b, COUNT(*) FROM '{P}' WHERE c <= 1.5 GROUP BY b",
    "SELECT e, COUNT(*), SUM(b) FROM '{P}' GROUP BY e",
    "SELECT c, COUNT(*) FROM '{P}' WHERE d != 'g3' GROUP BY c",
    "SELECT a, c FROM '{P}' WHERE b > 50",
]
ROLE = [
    "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{P}' WHERE age > 30 GROUP BY role",
    "SELECT COUNT(*) FROM '{P}' WHERE age > 30",
    "SELECT name, COUNT(*), AVG(age) FROM '{P}' GROUP BY name",
    "SELECT height, COUNT(*), SUM(age) FROM '{P}' WHERE gender = 'm' GROUP BY height",
    "SELECT age, COUNT(*) FROM '{P}' GROUP BY age",
    "SELECT surname, age FROM '{P}' WHERE height >= 1.99",
]


def _tol(sql):
    sel = sql.split(" FROM ")[0]
    items = [s.strip() for s in sel[len("SELECT "):].split(",")]
    return {i for i, s in enumerate(items) if s.upper().startswith(("SUM(", "AVG("))}


def _run(sql, mode):
    old = cq_amd.set_scan_kernel(mode)
    try:
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
        return got, cq_amd.stats(), cq_amd.last_ineligible()
    finally:
        cq_amd.set_scan_kernel(old)


def _check(sql):
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    tol = _tol(sql)
    auto, st, inel = _run(sql, 0)                 # fast_kernel where the plan has its shape
    assert not inel, (sql, inel)
    assert st["scan_kernel"] in (1, 2), (sql, "neither fast_kernel nor lean_kernel ran")
    _cmp(auto, want, tol, "auto: " + sql)
    lean, st1, _ = _run(sql, 2)                   # lean_kernel forced
    assert st1["scan_kernel"] == 1, (sql, "lean_kernel did not run")
    _cmp(lean, want, tol, "lean: " + sql)
    general, st2, _ = _run(sql, 1)
    assert st2["scan_kernel"] == 0
    _cmp(general, want, tol, "general: " + sql)
    return st


def _cmp(got, want, tol, ctx):
    assert (got is None) == (want is None), ctx
    if want is None:
        return
    assert got["columns"] == want["columns"], ctx
    assert len(got["rows"]) == len(want["rows"]), (ctx, len(got["rows"]), len(want["rows"]))
    for i, (g, w) in enumerate(zip(got["rows"], want["rows"])):
        for j, (x, y) in enumerate(zip(g, w)):
            assert cqtest.cell_equal(x, y, REL if j in tol else 0.0), f"{ctx}: row {i} col {j}: {x} vs {y}"


@pytest.mark.parametrize("name", ["messy_lf", "messy_crlf", "tiny", "runs"])
@pytest.mark.parametrize("tmpl", GENERIC)
def test_lean_generic(files, name, tmpl):
    _check(tmpl.replace("{P}", str(files[name])))


@pytest.mark.parametrize("tmpl", ROLE)
def test_lean_role(files, tmpl):
    st = _check(tmpl.replace("{P}", str(files["role"])))
    assert st["slow_records"] == 0, st      # clean data: every record on the fast path


def test_lean_declines_messy_records(files):
    """the messy file sends its odd records to slow_kernel, and only those"""
    st = _check("SELECT d, COUNT(*), SUM(c) FROM '%s' GROUP BY d" % files["messy_lf"])
    assert 0 < st["slow_records"] < st["records"] // 4, st


def test_lean_many_groups_spill(tmp_path):
    """more distinct keys than the LDS table holds: the HBM table takes the rest"""
    lines = [b"k,v\n"] + [b"key%06d,%d\n" % (i % 70000, i) for i in range(200_000)]
    p = tmp_path / "many.csv"
    p.write_bytes(b"".join(lines))
    _check(f"SELECT k, COUNT(*), SUM(v) FROM '{p}' GROUP BY k")


def test_lean_resident_rescans(files):
    """the same resident table, lean and general kernels, several times"""
    sql = ROLE[0].replace("{P}", str(files["role"]))
    t = cq_amd.Table.open(str(files["role"]))
    try:
        with cqtest.Parsed(sql) as ast:
            ref = cq_amd.query(ast, [t])
            for mode in (0, 1, 2, 0):
                old = cq_amd.set_scan_kernel(mode)
                got = cq_amd.query(ast, [t])
                cq_amd.set_scan_kernel(old)
                _cmp(got, ref, {2, 3}, sql)
    finally:
        t.close()
