"""Record starts of a whole table (the join's and the key routing's row list):
the two-pass record-start kernels (route.hip rs_count / rs_write) against a
host restatement of csv_load's line split (reference csv_reader.c:403-427: any
'\\n' / '\\r' ends a record, runs of them are skipped, the first non-empty line
is the header) and against the general scan path; bit-exact offsets.
"""
import ctypes as C

import numpy as np
import pytest

import cq_amd
from cq_amd import abi, datagen

pytestmark = pytest.mark.gpu


def _starts(data: bytes, has_header: bool = True):
    """host restatement: start offsets of the non-empty lines after the header"""
    out, p, n, first = [], 0, len(data), True
    while p < n:
        s = p
        while p < n and data[p] not in (10, 13):
            p += 1
        if p > s:
            if first and has_header:
                first = False
            else:
                first = False
                out.append(s)
        while p < n and data[p] in (10, 13):
            p += 1
    return out


def _gpu(table, method):
    L = cq_amd.lib()
    L.cqgpu_debug_all_records.restype = C.c_size_t
    L.cqgpu_debug_all_records.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_ulonglong), C.c_size_t]
    n = L.cqgpu_debug_all_records(table.handle, method, None, 0)
    assert n != 2**64 - 1, cq_amd.last_error()
    buf = (C.c_ulonglong * max(n, 1))()
    assert L.cqgpu_debug_all_records(table.handle, method, buf, n) == n
    return list(buf)[:n]


def _cases():
    rng = np.random.default_rng(3)
    yield "shape_a", datagen.shape_a_bytes(50_000, seed=4, with_role=True)
    yield "crlf", b"a,b\r\n1,2\r\n\r\n3,4\r\r\n5,6"
    yield "blank_lines", b"\n\n\na,b\n\n1,2\n   \n,\n\n\n7,8\n\n"
    yield "no_trailing_newline", b"x\n1\n2\n3"
    yield "header_only", b"a,b,c\n"
    yield "empty", b""
    # random bytes with many terminators, across block (4 KiB) boundaries
    raw = rng.choice(np.frombuffer(b"ab,1\n\r \"", dtype=np.uint8), size=200_003).tobytes()
    yield "random", raw
    # long records straddling block boundaries
    yield "long", b"h\n" + b"".join(b"z" * int(k) + b"\n" for k in rng.integers(1, 9000, 300))


@pytest.mark.parametrize("name,data", list(_cases()), ids=[c[0] for c in _cases()])
def test_record_starts(name, data):
    t = cq_amd.Table.from_bytes(data)
    try:
        want = _starts(data)
        got = _gpu(t, 0)
        assert got == want, name
        assert _gpu(t, 1) == want, name
    finally:
        t.close()


def test_record_starts_shard_with_header():
    """a shard uploaded with a separate header: every byte is data"""
    body = b"1,2\n\n3,4\r\n5,6\n"
    t = cq_amd.Table.from_bytes(body, base_offset=100, header=b"a,b\n")
    try:
        assert _gpu(t, 0) == [0, 5, 10]
    finally:
        t.close()


def test_record_starts_no_header():
    data = b"1,2\n3,4\n"
    t = cq_amd.Table.from_bytes(data, abi.csv_config(has_header=False))
    try:
        assert _gpu(t, 0) == _starts(data, has_header=False)
    finally:
        t.close()
