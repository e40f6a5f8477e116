"""Shared test helpers: library loading, golden vectors, result comparison.

Test infrastructure may load the oracle (oracle/liboracle.so, our CPU
restatement) and the reference front end built from /root/reference by
oracle/ref.mk (oracle/_ref/libcqfront.so: tokenizer + parser, used only to turn
SQL text into the plan the reference parser would hand to evaluate_query).
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from cq_amd import abi  # noqa: E402

GOLDEN = os.path.join(HERE, "golden")
GOLDEN_DATA = os.path.join(GOLDEN, "data")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
FRONT_SO = os.path.join(REPO, "oracle", "_ref", "libcqfront.so")

_libs = {}


def _ensure_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)


def oracle():
    if "oracle" not in _libs:
        _ensure_oracle()
        lib = C.CDLL(ORACLE_SO)
        lib.orc_load.restype = C.POINTER(abi.Table)
        lib.orc_load.argtypes = [C.c_char_p, C.c_size_t, abi.CsvConfig]
        lib.orc_evaluate.restype = C.POINTER(abi.Table)
        lib.orc_evaluate.argtypes = [C.POINTER(abi.Node), abi.CsvConfig, C.POINTER(C.c_int)]
        lib.orc_free.argtypes = [C.POINTER(abi.Table)]
        lib.orc_parse_cell.restype = abi.Value
        lib.orc_parse_cell.argtypes = [C.c_char_p, C.c_size_t]
        _libs["oracle"] = lib
    return _libs["oracle"]


def front_available() -> bool:
    return os.path.exists(FRONT_SO)


def front():
    """The reference parser (unchanged front end) as a ctypes library."""
    if "front" not in _libs:
        lib = C.CDLL(FRONT_SO)
        lib.parse.restype = C.POINTER(abi.Node)
        lib.parse.argtypes = [C.c_char_p]
        lib.releaseNode.argtypes = [C.POINTER(abi.Node)]
        _libs["front"] = lib
    return _libs["front"]


class Parsed:
    """Context manager: SQL text -> reference plan pointer (released on exit)."""

    def __init__(self, sql: str):
        self.sql = sql

    def __enter__(self):
        self.ast = front().parse(self.sql.encode("latin-1"))
        if not self.ast:
            raise ValueError(f"reference parser rejected: {self.sql}")
        return self.ast

    def __exit__(self, *a):
        front().releaseNode(self.ast)


def oracle_query(sql: str, cfg=None):
    """Evaluate with the oracle; returns (python table | None, unsupported flag)."""
    cfg = cfg or abi.csv_config()
    lib = oracle()
    unsup = C.c_int(0)
    with Parsed(sql) as ast:
        tp = lib.orc_evaluate(ast, cfg, C.byref(unsup))
    if not tp:
        return None, unsup.value
    res = abi.table_to_py(tp)
    lib.orc_free(tp)
    return res, unsup.value


# ---------------------------------------------------------------- golden data
def golden(name: str):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def cell_from_json(c):
    t = c["t"]
    if t == "N":
        return ("N",)
    if t == "I":
        return ("I", int(c["v"]))
    if t == "D":
        return ("D", float(c["v"]))
    if t == "S":
        return ("S", c["v"].encode("latin-1"))
    if t == "T":
        return ("T", tuple(c["v"]))
    return ("?",)


def table_from_json(j):
    if j.get("error"):
        return None
    return {"columns": [c.encode("latin-1") for c in j["columns"]],
            "rows": [[cell_from_json(c) for c in r] for r in j["rows"]]}


def sql_for(q: str, data_dir: str = GOLDEN_DATA) -> str:
    return q.replace("{D}", data_dir)


# ---------------------------------------------------------------- comparison
def cell_equal(a, b, rel: float = 0.0) -> bool:
    if a[0] != b[0]:
        return False
    if a[0] == "D":
        x, y = a[1], b[1]
        if math.isnan(x) or math.isnan(y):
            return math.isnan(x) and math.isnan(y)
        if rel == 0.0:
            return x == y and math.copysign(1, x) == math.copysign(1, y)
        return x == y or abs(x - y) <= rel * max(abs(x), abs(y))
    return a == b


def assert_tables_equal(got, want, rel: float = 0.0, ctx: str = ""):
    """Exact for every cell except doubles, which may differ by `rel` relative."""
    assert (got is None) == (want is None), f"{ctx}: error mismatch got={got is None} want={want is None}"
    if want is None:
        return
    assert got["columns"] == want["columns"], f"{ctx}: columns {got['columns']} != {want['columns']}"
    assert len(got["rows"]) == len(want["rows"]), f"{ctx}: {len(got['rows'])} rows != {len(want['rows'])}"
    for i, (gr, wr) in enumerate(zip(got["rows"], want["rows"])):
        assert len(gr) == len(wr), f"{ctx}: row {i} width"
        for j, (g, w) in enumerate(zip(gr, wr)):
            assert cell_equal(g, w, rel), f"{ctx}: row {i} col {j}: got {g} want {w}"
