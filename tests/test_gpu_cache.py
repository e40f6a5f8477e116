"""Device-resident table cache of the drop-in evaluate_query.

The reference re-reads the file on every query (csv_load per evaluate_query);
the cache must be invisible to results: a hit returns the same answer as a fresh
load, a rewritten file is re-read, and a zero budget disables caching.  Each
result is checked against the oracle.
"""
import ctypes as C
import os
import time

import pytest

import cqtest
import cq_amd
from test_gpu_parity import compare, tolerant_columns

pytestmark = pytest.mark.gpu


def _lib():
    L = cq_amd.lib()
    L.cqgpu_cache_info.argtypes = [C.POINTER(C.c_uint64)] * 3
    L.cqgpu_set_cache_limit.restype = C.c_longlong
    L.cqgpu_set_cache_limit.argtypes = [C.c_longlong]
    return L


def _info():
    e, b, h = C.c_uint64(), C.c_uint64(), C.c_uint64()
    _lib().cqgpu_cache_info(C.byref(e), C.byref(b), C.byref(h))
    return e.value, b.value, h.value


def _check(sql):
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        assert cq_amd.stats()["path"] == 1, sql
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql)
    return got


def test_cache_hit_and_invalidation(tmp_path):
    L = _lib()
    L.cqgpu_cache_clear()
    prev = L.cqgpu_set_cache_limit(1 << 30)
    try:
        p = tmp_path / "c.csv"
        p.write_text("a,b\n1,x\n2,y\n3,x\n")
        sql = f"SELECT b, COUNT(*), SUM(a) FROM '{p}' GROUP BY b"
        r1 = _check(sql)
        e, nbytes, h0 = _info()
        assert e == 1 and nbytes == os.path.getsize(p)
        r2 = _check(sql)
        assert r2 == r1
        assert _info()[2] == h0 + 1                 # served from HBM
        # rewrite: new size and mtime -> re-read, new answer
        time.sleep(0.01)
        p.write_text("a,b\n1,x\n2,y\n3,x\n40,z\n")
        r3 = _check(sql)
        assert r3 != r1 and len(r3["rows"]) == 3
        e, nbytes, _ = _info()
        assert e == 1 and nbytes == os.path.getsize(p)
        # same size, new content and mtime -> re-read
        time.sleep(0.01)
        p.write_text("a,b\n9,x\n2,y\n3,x\n40,z\n")
        r4 = _check(sql)
        assert r4 != r3
        # self-join through the cache: one entry serves both sides
        _check(f"SELECT COUNT(*) FROM '{p}' AS l JOIN '{p}' AS r ON l.b = r.b")
        assert _info()[0] == 1
    finally:
        L.cqgpu_set_cache_limit(prev)
        L.cqgpu_cache_clear()


def test_cache_budget_and_disable(tmp_path):
    L = _lib()
    L.cqgpu_cache_clear()
    prev = L.cqgpu_set_cache_limit(100)
    try:
        paths = []
        for k in range(3):
            p = tmp_path / f"f{k}.csv"
            p.write_text("v\n" + "".join(f"{k * 10 + i}\n" for i in range(10)))   # 32-33 bytes
            paths.append(p)
            _check(f"SELECT COUNT(*), SUM(v) FROM '{p}'")
        e, nbytes, _ = _info()
        assert nbytes <= 100 and e >= 2                     # LRU within the budget
        L.cqgpu_set_cache_limit(0)                          # disable: empties the cache
        assert _info()[0] == 0
        _check(f"SELECT COUNT(*), SUM(v) FROM '{paths[0]}'")
        assert _info()[0] == 0
    finally:
        L.cqgpu_set_cache_limit(prev)
        L.cqgpu_cache_clear()
