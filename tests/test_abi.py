"""The drop-in boundary on CPU: the C-ABI headers match the reference layout
(tests/golden/abi_layout.json, measured from the reference's own headers), the
ctypes mirror matches the headers, and libcqgpu.so loads and exports every
function include/*.h declares.  No device calls.
"""
import ctypes as C
import json
import os
import re
import subprocess

import pytest

import cq_amd
from cq_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "abi_layout.json")))

# reference name (golden key) -> expression over include/cq_abi.h
FIELDS = {
    "ASTNode.refcount": "offsetof(cq_node, refcount)",
    "ASTNode.type": "offsetof(cq_node, kind)",
    "ASTNode.query.select": "offsetof(cq_node, u.q.select)",
    "ASTNode.query.from": "offsetof(cq_node, u.q.from)",
    "ASTNode.query.joins": "offsetof(cq_node, u.q.joins)",
    "ASTNode.query.join_count": "offsetof(cq_node, u.q.join_count)",
    "ASTNode.query.where": "offsetof(cq_node, u.q.where)",
    "ASTNode.query.group_by": "offsetof(cq_node, u.q.group_by)",
    "ASTNode.query.having": "offsetof(cq_node, u.q.having)",
    "ASTNode.query.order_by": "offsetof(cq_node, u.q.order_by)",
    "ASTNode.query.limit": "offsetof(cq_node, u.q.limit)",
    "ASTNode.query.offset": "offsetof(cq_node, u.q.offset)",
    "ASTNode.select.columns": "offsetof(cq_node, u.sel.texts)",
    "ASTNode.select.column_nodes": "offsetof(cq_node, u.sel.exprs)",
    "ASTNode.select.column_count": "offsetof(cq_node, u.sel.count)",
    "ASTNode.select.distinct": "offsetof(cq_node, u.sel.distinct)",
    "ASTNode.condition.left": "offsetof(cq_node, u.bin.lhs)",
    "ASTNode.condition.right": "offsetof(cq_node, u.bin.rhs)",
    "ASTNode.condition.operator": "offsetof(cq_node, u.bin.op)",
    "ASTNode.binary_op.left": "offsetof(cq_node, u.bin.lhs)",
    "ASTNode.binary_op.right": "offsetof(cq_node, u.bin.rhs)",
    "ASTNode.binary_op.operator": "offsetof(cq_node, u.bin.op)",
    "ASTNode.function.name": "offsetof(cq_node, u.fn.name)",
    "ASTNode.function.args": "offsetof(cq_node, u.fn.args)",
    "ASTNode.function.arg_count": "offsetof(cq_node, u.fn.nargs)",
    "ASTNode.list.nodes": "offsetof(cq_node, u.list.items)",
    "ASTNode.list.node_count": "offsetof(cq_node, u.list.nitems)",
    "ASTNode.order_by.column": "offsetof(cq_node, u.ord.key)",
    "ASTNode.order_by.descending": "offsetof(cq_node, u.ord.desc)",
    "ASTNode.group_by.columns": "offsetof(cq_node, u.grp.keys)",
    "ASTNode.group_by.column_count": "offsetof(cq_node, u.grp.nkeys)",
    "ASTNode.from.table": "offsetof(cq_node, u.from.path)",
    "ASTNode.from.subquery": "offsetof(cq_node, u.from.subquery)",
    "ASTNode.from.alias": "offsetof(cq_node, u.from.alias)",
    "ASTNode.join.join_type": "offsetof(cq_node, u.join.kind)",
    "ASTNode.join.table": "offsetof(cq_node, u.join.path)",
    "ASTNode.join.alias": "offsetof(cq_node, u.join.alias)",
    "ASTNode.join.condition": "offsetof(cq_node, u.join.on)",
    "ASTNode.subquery.query": "offsetof(cq_node, u.sub.query)",
    "ASTNode.identifier": "offsetof(cq_node, u.text)",
    "ASTNode.set_op.op_type": "offsetof(cq_node, u._opaque)",   # set operations: opaque here
    "ASTNode.literal": "offsetof(cq_node, u.text)",
    "Value.type": "offsetof(cq_value, kind)",
    "Value.int_value": "offsetof(cq_value, u.i)",
    "Value.double_value": "offsetof(cq_value, u.f)",
    "Value.string_value": "offsetof(cq_value, u.s)",
    "Value.date_value": "offsetof(cq_value, u.date)",
    "Row.values": "offsetof(cq_row, values)",
    "Row.column_count": "offsetof(cq_row, ncols)",
    "Column.name": "offsetof(cq_column, name)",
    "Column.inferred_type": "offsetof(cq_column, inferred_kind)",
    "CsvTable.filename": "offsetof(cq_table, filename)",
    "CsvTable.data": "offsetof(cq_table, data)",
    "CsvTable.file_size": "offsetof(cq_table, file_size)",
    "CsvTable.fd": "offsetof(cq_table, fd)",
    "CsvTable.columns": "offsetof(cq_table, columns)",
    "CsvTable.column_count": "offsetof(cq_table, ncols)",
    "CsvTable.has_header": "offsetof(cq_table, has_header)",
    "CsvTable.rows": "offsetof(cq_table, rows)",
    "CsvTable.row_count": "offsetof(cq_table, nrows)",
    "CsvTable.row_capacity": "offsetof(cq_table, row_capacity)",
    "CsvTable.delimiter": "offsetof(cq_table, delimiter)",
    "CsvTable.quote": "offsetof(cq_table, quote)",
    "CsvConfig.delimiter": "offsetof(cq_csv_config, delimiter)",
    "CsvConfig.quote": "offsetof(cq_csv_config, quote)",
    "CsvConfig.has_header": "offsetof(cq_csv_config, has_header)",
    "sizeof.ASTNode": "sizeof(cq_node)",
    "sizeof.Value": "sizeof(cq_value)",
    "sizeof.Row": "sizeof(cq_row)",
    "sizeof.Column": "sizeof(cq_column)",
    "sizeof.CsvTable": "sizeof(cq_table)",
    "sizeof.CsvConfig": "sizeof(cq_csv_config)",
    "sizeof.DateValue": "sizeof(cq_date)",
    "enum.NODE_TYPE_QUERY": "CQ_N_QUERY",
    "enum.NODE_TYPE_CONDITION": "CQ_N_CONDITION",
    "enum.NODE_TYPE_BINARY_OP": "CQ_N_BINARY_OP",
    "enum.NODE_TYPE_WINDOW_FUNCTION": "CQ_N_WINDOW_FUNCTION",
    "enum.VALUE_TYPE_DATE": "CQ_V_DATE",
}


@pytest.fixture(scope="module")
def header_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("abi")
    src = d / "layout.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "cq_abi.h"', "int main(void) {"]
    for k, expr in FIELDS.items():
        lines.append(f'    printf("%s %ld\\n", "{k}", (long)({expr}));')
    lines.append("    return 0;\n}")
    src.write_text("\n".join(lines))
    exe = d / "layout"
    subprocess.run(["gcc", "-I", INC, "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {k: int(v) for k, v in (ln.split() for ln in out.splitlines())}


def test_every_golden_field_is_mapped():
    assert set(GOLD) == set(FIELDS)


def test_header_matches_reference(header_layout):
    bad = {k: (header_layout[k], GOLD[k]) for k in GOLD if header_layout[k] != GOLD[k]}
    assert not bad, bad


def test_ctypes_mirror_matches_header(header_layout):
    assert C.sizeof(abi.Node) == header_layout["sizeof.ASTNode"]
    assert C.sizeof(abi.Value) == header_layout["sizeof.Value"]
    assert C.sizeof(abi.Row) == header_layout["sizeof.Row"]
    assert C.sizeof(abi.Column) == header_layout["sizeof.Column"]
    assert C.sizeof(abi.Table) == header_layout["sizeof.CsvTable"]
    assert C.sizeof(abi.CsvConfig) == header_layout["sizeof.CsvConfig"]
    assert abi.Node.u.offset == header_layout["ASTNode.query.select"]


def _declared_functions():
    names = set()
    for h in ("cqgpu.h",):
        text = open(os.path.join(INC, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", text, flags=re.M):
            if m.group(0).startswith("typedef"):          # a function-pointer type, not a symbol
                continue
            if m.group(1) not in ("if", "while", "typedef"):
                names.add(m.group(1))
    return names


def test_library_exports_declared_functions():
    lib = cq_amd.lib()                     # loads without a GPU
    names = _declared_functions()
    assert "evaluate_query" in names and "cqgpu_query_partial" in names
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    cfg = abi.CsvConfig.in_dll(lib, "global_csv_config")    # the reference global
    assert cfg.delimiter == b"," and cfg.quote == b'"'


def test_explain_without_device():
    """the planner runs on the host: compile the bench plan against a header"""
    lib = cq_amd.lib()
    lib.cqgpu_explain.restype = C.c_int
    lib.cqgpu_explain.argtypes = [C.POINTER(abi.Node), C.c_char_p, abi.CsvConfig, C.c_char_p, C.c_size_t]
    P = abi.Plan()
    q = P.query([P.ident("role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("height"))], "x.csv",
                where=P.cond(">", P.ident("age"), P.lit("30")), group_by=["role"])
    buf = C.create_string_buffer(4096)
    assert lib.cqgpu_explain(C.pointer(q), b"name,surname,age,gender,height,role", abi.csv_config(), buf, 4096) == 0
    text = buf.value.decode()
    assert "need: 2 4 5" in text and "group_slot: 2" in text
    q2 = P.query([P.ident("a")], "x.csv", joins=[("y.csv", None, P.cond("=", P.ident("a"), P.ident("b")), 0)])
    assert lib.cqgpu_explain(C.pointer(q2), b"a,b", abi.csv_config(), buf, 4096) != 0


@pytest.mark.parametrize("where,fast", [
    ("age > 30", 1),
    ("age BETWEEN 20 AND 40", 1),                                    # AND(>=, <=)
    ("age > 30 AND gender = 'f'", 1),                                # NUMBER and STRING columns
    ("role IN ('role_001', 'role_002')", 1),
    ("NOT age > 30", 1),
    ("30 < age", 1),                                                 # literal on the left
    ("age > -5", 1),                                                 # unary minus literal
    ("height IN (1.1, 2.25)", 1),
    ("age < 20 OR gender != 'm' AND age > 70", 1),
    ("age = 1 OR age = 2 OR age = 3 OR age = 4 OR age = 5", 0),      # 5 leaves
    ("age > 30 OR age = 'abc'", 0),                                  # one column, both classes
    ("age > 30 AND gender = 'f' AND height > 1.2", 0),               # 3 WHERE columns
    ("age + 1 > 30", 0),                                             # arithmetic
    ("role IN ('a', 'b', 'c', 'd', 'e', 'f', 'g', 'h', 'i')", 0),    # 9 items
    ("gender = 'abcdefghi'", 0),                                     # a 9-byte literal
])
def test_fast_kernel_where_shapes_on_cpu(where, fast):
    """which WHEREs fast_kernel's builds take (fast.hip fast_shape / wx_compile), decided
    on the host from the plan alone: compound trees of <= 4 leaves over <= 2 columns"""
    import cqtest
    lib = cq_amd.lib()
    lib.cqgpu_explain.restype = C.c_int
    lib.cqgpu_explain.argtypes = [C.POINTER(abi.Node), C.c_char_p, abi.CsvConfig, C.c_char_p, C.c_size_t]
    buf = C.create_string_buffer(8192)
    sql = f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM 'x.csv' WHERE {where} GROUP BY role"
    with cqtest.Parsed(sql) as ast:
        if lib.cqgpu_explain(ast, b"name,surname,age,gender,height,role", abi.csv_config(), buf, 8192) != 0:
            assert fast == 0, (where, lib.cqgpu_last_error())    # (outside the GPU subset altogether)
            return
    lines = dict(ln.split(": ", 1) for ln in buf.value.decode().split("\n") if ln.startswith("fast: "))
    assert lines["fast"] == str(fast), (where, buf.value.decode())
