"""HIP tokenizer + typing vs the reference's own csv_load output (tests/golden/cells.json).

Record splitting (csv_load, reference csv_reader.c:404-427), field splitting
(parse_line :278-338) and cell typing (infer_type/parse_value :133-240) on the
GPU must reproduce every typed cell the reference produced, bit for bit.
"""
import ctypes as C
import os

import pytest

import cqtest
import cq_amd
from cq_amd import abi

pytestmark = pytest.mark.gpu
CELLS = cqtest.golden("cells.json")


def _lib():
    L = cq_amd.lib()
    L.cqgpu_debug_records.restype = C.c_size_t
    L.cqgpu_debug_records.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_size_t]
    L.cqgpu_debug_cells.restype = C.POINTER(abi.Table)
    L.cqgpu_debug_cells.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_ulonglong),
                                    C.c_size_t]
    return L


def gpu_cells(table: cq_amd.Table, ncols: int):
    L = _lib()
    cap = 1 << 20
    buf = (C.c_ulonglong * cap)()
    n = L.cqgpu_debug_records(table.handle, buf, cap)
    assert n <= cap
    rows = [[] for _ in range(n)]
    for c0 in range(0, ncols, 8):
        cols = list(range(c0, min(ncols, c0 + 8)))
        carr = (C.c_int * len(cols))(*cols)
        tp = L.cqgpu_debug_cells(table.handle, carr, len(cols), buf, n)
        assert tp, cq_amd.last_error()
        t = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        for i, r in enumerate(t["rows"]):
            rows[i].extend(r)
    return n, [buf[i] for i in range(n)], rows


def _cfg_for(key):
    if key.endswith("#noheader"):
        return key.split("#")[0], abi.csv_config(has_header=False)
    if key.endswith("#semicolon"):
        return key.split("#")[0], abi.csv_config(delimiter=";")
    return key, abi.csv_config()


@pytest.mark.parametrize("key", sorted(CELLS))
def test_cells_match_reference(key):
    fname, cfg = _cfg_for(key)
    with open(os.path.join(cqtest.GOLDEN_DATA, fname), "rb") as fh:
        data = fh.read()
    want = cqtest.table_from_json(CELLS[key])
    if cfg.delimiter in (b" ", b"\t"):
        pytest.skip("whitespace delimiters are outside the GPU subset")
    t = cq_amd.Table.from_bytes(data, cfg)
    ncols = len(want["columns"])
    n, offs, rows = gpu_cells(t, ncols)
    t.close()
    assert n == len(want["rows"]), f"{key}: {n} records vs {len(want['rows'])}"
    for i, (g, w) in enumerate(zip(rows, want["rows"])):
        w = list(w[:ncols]) + [("N",)] * max(0, ncols - len(w))   # short rows: UB in the reference
        for j in range(ncols):
            assert cqtest.cell_equal(g[j], w[j]), f"{key} row {i} (offset {offs[i]}) col {j}: got {g[j]} want {w[j]}"


@pytest.mark.parametrize("key", sorted(k for k in CELLS if "#" not in k))
def test_scan_kernel_cells_match_reference(key):
    """the fused scan kernel parses fields from its LDS window: same cells required"""
    with open(os.path.join(cqtest.GOLDEN_DATA, key), "rb") as fh:
        data = fh.read()
    want = cqtest.table_from_json(CELLS[key])
    ncols = min(len(want["columns"]), 8)
    if ncols == 0:
        pytest.skip("no columns")
    L = _lib()
    L.cqgpu_debug_scan_cells.restype = C.POINTER(abi.Table)
    L.cqgpu_debug_scan_cells.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int,
                                         C.POINTER(C.c_ulonglong), C.c_size_t]
    t = cq_amd.Table.from_bytes(data)
    cap = 1 << 20
    recs = (C.c_ulonglong * cap)()
    carr = (C.c_int * ncols)(*range(ncols))
    tp = L.cqgpu_debug_scan_cells(t.handle, carr, ncols, recs, cap)
    assert tp, cq_amd.last_error()
    got = abi.table_to_py(tp)
    cq_amd.result_free(tp)
    t.close()
    order = sorted(range(len(got["rows"])), key=lambda i: recs[i])
    rows = [got["rows"][i] for i in order]
    assert len(rows) == len(want["rows"])
    for i, (g, w) in enumerate(zip(rows, want["rows"])):
        w = list(w[:ncols]) + [("N",)] * max(0, ncols - len(w))
        for j in range(ncols):
            assert cqtest.cell_equal(g[j], w[j]), f"{key} row {i} (offset {recs[order[i]]}) col {j}: got {g[j]} want {w[j]}"
