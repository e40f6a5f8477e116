"""The oracle (oracle/cq_oracle.c) against the reference's own outputs.

tests/golden/cells.json and queries.json were produced by the unmodified
reference (tests/golden/make_golden.py); the oracle must reproduce every vector
exactly before it may be used to judge the HIP executor.
"""
import ctypes as C
import os

import pytest

import cqtest
from cq_amd import abi

CELLS = cqtest.golden("cells.json")
QUERIES = cqtest.golden("queries.json")


def _cfg_for(key):
    if key.endswith("#noheader"):
        return key.split("#")[0], abi.csv_config(has_header=False)
    if key.endswith("#semicolon"):
        return key.split("#")[0], abi.csv_config(delimiter=";")
    return key, abi.csv_config()


@pytest.mark.parametrize("key", sorted(CELLS))
def test_oracle_cells_match_reference(key):
    fname, cfg = _cfg_for(key)
    with open(os.path.join(cqtest.GOLDEN_DATA, fname), "rb") as fh:
        data = fh.read()
    lib = cqtest.oracle()
    tp = lib.orc_load(data, len(data), cfg)
    got = abi.table_to_py(tp)
    lib.orc_free(tp)
    want = cqtest.table_from_json(CELLS[key])
    cqtest.assert_tables_equal(got, want, ctx=key)


@pytest.mark.skipif(not cqtest.front_available(), reason="reference front end not built")
@pytest.mark.parametrize("idx", range(len(QUERIES)))
def test_oracle_queries_match_reference(idx):
    q = QUERIES[idx]
    got, unsupported = cqtest.oracle_query(cqtest.sql_for(q["sql"]))
    assert not unsupported, q["sql"]
    want = cqtest.table_from_json(q["result"])
    cqtest.assert_tables_equal(got, want, ctx=q["sql"])
