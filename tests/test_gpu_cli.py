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


# `-o FILE` (main.c:133 -> write_csv_file, utils.c:220-289): cq_amd_cli binds the
# call to libcqgpu's GPU writer (cqgpu_write_csv); the files must be byte-identical
OUT_QUERIES = [
    (f"SELECT * FROM '{D}/test_data.csv' WHERE age > 30", ","),
    (f"SELECT name, age * 1.005, age / 7 FROM '{D}/test_data.csv'", ","),
    (f"SELECT q1, q2, q3 FROM '{D}/edge_quotes.csv'", ","),
    (f"SELECT q1, q2, q3 FROM '{D}/edge_quotes.csv'", ";"),
    (f"SELECT * FROM '{D}/edge_dates.csv'", ","),
    (f"SELECT * FROM '{D}/edge_numbers.csv'", "|"),
    (f"SELECT a, COUNT(*), MIN(b), MAX(c) FROM '{D}/edge_numbers.csv' GROUP BY a", ","),
    # integer SUM / AVG: exact in any order (double SUM / AVG are compared at 1e-6
    # relative elsewhere: a different addition order can move a %.2f tie)
    (f"SELECT role, COUNT(*), SUM(age), AVG(age) FROM '{D}/synth_role.csv' WHERE height > 1.5 GROUP BY role", ","),
    (f"SELECT * FROM '{D}/events.csv'", ","),
    (f"SELECT * FROM '{D}/test_data.csv' WHERE age > 1000", ","),
]


@pytest.mark.skipif(not (os.path.exists(REF) and os.path.exists(GPU)), reason="oracle/ref.mk not built")
@pytest.mark.parametrize("sql,delim", OUT_QUERIES)
def test_cli_output_file_identical(tmp_path, sql, delim):
    fw, fg = tmp_path / "want.csv", tmp_path / "got.csv"
    want = subprocess.run([REF, "-q", sql, "-o", str(fw), "-d", delim], cwd=ROOT, capture_output=True, timeout=120)
    got = subprocess.run([GPU, "-q", sql, "-o", str(fg), "-d", delim], cwd=ROOT, capture_output=True, timeout=300)
    assert got.returncode == want.returncode, got.stderr.decode(errors="replace")
    assert got.stdout.replace(str(fg).encode(), b"F") == want.stdout.replace(str(fw).encode(), b"F")
    assert fg.read_bytes() == fw.read_bytes()


def test_writer_double_formats(tmp_path):
    """%.2f edge cases through cqgpu_write_csv vs the reference's write_csv_file
    (libcqfront.so) on the same result table: ties at the second decimal, values
    just below / above ties, -0.0, tiny negatives, 2^53 + 1 neighbours, huge
    values (every digit), subnormals, inf / nan, extreme integers, dates."""
    import ctypes as C
    import math
    import cqtest
    import cq_amd
    from cq_amd import abi
    doubles = [0.125, 0.135, 0.145, 2.675, 1.005, -0.001, -0.0, 0.0, 0.005, 0.015, 0.025, 1e-300, 5e-324,
               -5e-324, 9007199254740993.0, 2.0 ** 60 + 0.5, 1e22, 1.7976931348623157e308, -1e300, 123456.785,
               math.inf, -math.inf, math.nan, -1234.5, 99.995, 0.995, 4503599627370495.5]
    ints = [0, -1, 2 ** 63 - 1, -2 ** 63, 42]
    front = cqtest.front()
    front.write_csv_file.argtypes = [C.c_char_p, C.c_void_p, C.c_char]
    # a result table built by hand in the reference's layout (cq_abi.h)
    n = max(len(doubles), len(ints))
    strs = [b"plain", b"a,b", b'q"x', b"line\nbreak", b"", b"cr\r", b"semi;colon", None]
    cols = (abi.Column * 4)()
    for i, nm in enumerate([b"d", b"i", b"dt", b"s"]):
        cols[i].name = nm
    rows = (abi.Row * n)()
    keep = []
    for r in range(n):
        vals = (abi.Value * 4)()
        keep.append(vals)
        if r < len(doubles):
            vals[0].kind = abi.V_DOUBLE
            vals[0].u.f = doubles[r]
        if r < len(ints):
            vals[1].kind = abi.V_INT
            vals[1].u.i = ints[r]
        vals[2].kind = abi.V_DATE
        vals[2].u.date.y, vals[2].u.date.m, vals[2].u.date.d = 1999 + r, 1 + r % 12, 1 + r % 28
        sv = strs[r % len(strs)]
        if sv is not None:
            buf = C.create_string_buffer(sv)
            keep.append(buf)
            vals[3].kind = abi.V_STRING
            vals[3].u.s = C.cast(buf, C.c_void_p)
        rows[r].values = vals
        rows[r].ncols = 4
    t = abi.Table()
    t.ncols = 4
    t.columns = cols
    t.nrows = n
    t.rows = rows
    fw, fg = tmp_path / "want.csv", tmp_path / "got.csv"
    L = cq_amd.lib()
    L.cqgpu_write_csv.argtypes = [C.c_char_p, C.c_void_p, C.c_char]
    L.cqgpu_write_csv.restype = C.c_int
    for delim in (b",", b";"):
        front.write_csv_file(str(fw).encode(), C.addressof(t), delim)
        assert L.cqgpu_write_csv(str(fg).encode(), C.addressof(t), delim) == 0
        assert fg.read_bytes() == fw.read_bytes(), (fg.read_bytes(), fw.read_bytes())

