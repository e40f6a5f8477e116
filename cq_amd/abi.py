"""ctypes mirror of include/cq_abi.h -- the reference cq plan/result layout.

The executor's C ABI takes the reference parser's plan (reference
include/parser.h:55-201) and returns the reference's result table
(include/csv_reader.h:47-63).  This module mirrors those layouts for Python
callers: building plans by hand (``Plan`` helpers below, used by bench.py) and
reading result tables back into plain Python values.
"""
from __future__ import annotations

import ctypes as C

# enum cq_node_kind (reference parser.h:11-36)
(N_QUERY, N_SELECT, N_FROM, N_JOIN, N_WHERE, N_GROUP_BY, N_ORDER_BY, N_FUNCTION,
 N_CONDITION, N_LITERAL, N_IDENTIFIER, N_ALIAS, N_LIST, N_SUBQUERY, N_BINARY_OP,
 N_SET_OP) = range(16)
JOIN_INNER, JOIN_LEFT, JOIN_RIGHT, JOIN_FULL = range(4)
V_NULL, V_INT, V_DOUBLE, V_STRING, V_DATE = range(5)


class Node(C.Structure):
    pass


NodeP = C.POINTER(Node)


class _Q(C.Structure):
    _fields_ = [("select", NodeP), ("from_", NodeP), ("joins", C.POINTER(NodeP)),
                ("join_count", C.c_int), ("where", NodeP), ("group_by", NodeP),
                ("having", NodeP), ("order_by", NodeP), ("limit", C.c_int), ("offset", C.c_int)]


class _Sel(C.Structure):
    _fields_ = [("texts", C.POINTER(C.c_char_p)), ("exprs", C.POINTER(NodeP)),
                ("count", C.c_int), ("distinct", C.c_bool)]


class _Bin(C.Structure):
    _fields_ = [("lhs", NodeP), ("rhs", NodeP), ("op", C.c_char_p)]


class _Fn(C.Structure):
    _fields_ = [("name", C.c_char_p), ("args", C.POINTER(NodeP)), ("nargs", C.c_int)]


class _List(C.Structure):
    _fields_ = [("items", C.POINTER(NodeP)), ("nitems", C.c_int)]


class _Ord(C.Structure):
    _fields_ = [("key", C.c_char_p), ("desc", C.c_bool)]


class _Grp(C.Structure):
    _fields_ = [("keys", C.POINTER(C.c_char_p)), ("nkeys", C.c_int)]


class _From(C.Structure):
    _fields_ = [("path", C.c_char_p), ("subquery", NodeP), ("alias", C.c_char_p)]


class _Join(C.Structure):
    _fields_ = [("kind", C.c_int), ("path", C.c_char_p), ("alias", C.c_char_p), ("on", NodeP)]


class _U(C.Union):
    _fields_ = [("q", _Q), ("sel", _Sel), ("bin", _Bin), ("fn", _Fn), ("list", _List),
                ("ord", _Ord), ("grp", _Grp), ("from_", _From), ("join", _Join),
                ("text", C.c_char_p), ("_opaque", C.c_ubyte * 72)]


Node._fields_ = [("refcount", C.c_int), ("kind", C.c_int), ("u", _U)]


class Date(C.Structure):
    _fields_ = [("y", C.c_int), ("m", C.c_int), ("d", C.c_int)]


class _VU(C.Union):
    _fields_ = [("i", C.c_longlong), ("f", C.c_double), ("s", C.c_void_p), ("date", Date)]


class Value(C.Structure):
    _fields_ = [("kind", C.c_int), ("u", _VU)]


class Row(C.Structure):
    _fields_ = [("values", C.POINTER(Value)), ("ncols", C.c_int)]


class Column(C.Structure):
    _fields_ = [("name", C.c_char_p), ("inferred_kind", C.c_int)]


class Table(C.Structure):
    _fields_ = [("filename", C.c_char_p), ("data", C.c_void_p), ("file_size", C.c_size_t),
                ("fd", C.c_int), ("columns", C.POINTER(Column)), ("ncols", C.c_int),
                ("has_header", C.c_bool), ("rows", C.POINTER(Row)), ("nrows", C.c_int),
                ("row_capacity", C.c_int), ("delimiter", C.c_char), ("quote", C.c_char)]


class CsvConfig(C.Structure):
    _fields_ = [("delimiter", C.c_char), ("quote", C.c_char), ("has_header", C.c_bool)]


def csv_config(delimiter: str = ",", quote: str = '"', has_header: bool = True) -> CsvConfig:
    return CsvConfig(delimiter.encode("latin-1"), quote.encode("latin-1"), has_header)


# ---------------------------------------------------------------- result reading
def value_to_py(v: Value):
    """Cell -> tagged Python tuple: ("N",), ("I", int), ("D", float), ("S", bytes), ("T", (y,m,d))."""
    k = v.kind
    if k == V_NULL:
        return ("N",)
    if k == V_INT:
        return ("I", int(v.u.i))
    if k == V_DOUBLE:
        return ("D", float(v.u.f))
    if k == V_STRING:
        return ("S", C.string_at(v.u.s) if v.u.s else b"")
    if k == V_DATE:
        return ("T", (v.u.date.y, v.u.date.m, v.u.date.d))
    return ("?", k)


def table_to_py(tp) -> dict:
    """cq_table* -> {"columns": [bytes], "rows": [[cell]]}."""
    t = tp.contents
    cols = [t.columns[i].name for i in range(t.ncols)]
    rows = []
    for r in range(t.nrows):
        row = t.rows[r]
        rows.append([value_to_py(row.values[c]) for c in range(row.ncols)])
    return {"columns": cols, "rows": rows}


# ---------------------------------------------------------------- plan building
class Plan:
    """Builds reference-layout plan nodes in Python-owned memory.

    The executor only reads plans, so keeping every node and string alive in
    ``self._keep`` for the lifetime of the Plan object is all that is needed.
    Shapes follow what the reference parser emits (parser_clauses.c:16-131,
    parser_expressions.c:445-592, ast_nodes.c:235-320 for column texts).
    """

    def __init__(self):
        self._keep = []

    def _node(self, kind: int) -> Node:
        n = Node()
        n.refcount = 1
        n.kind = kind
        self._keep.append(n)
        return n

    def _s(self, s):
        if s is None:
            return None
        b = s.encode("latin-1") if isinstance(s, str) else s
        buf = C.c_char_p(b)
        self._keep.append(buf)
        self._keep.append(b)
        return b

    def _arr(self, typ, items):
        a = (typ * max(1, len(items)))(*items)
        self._keep.append(a)
        return C.cast(a, C.POINTER(typ))

    def ident(self, name: str) -> Node:
        n = self._node(N_IDENTIFIER)
        n.u.text = self._s(name)
        return n

    def lit(self, text: str) -> Node:
        n = self._node(N_LITERAL)
        n.u.text = self._s(text)
        return n

    def cond(self, op: str, lhs, rhs=None) -> Node:
        n = self._node(N_CONDITION)
        n.u.bin.lhs = C.pointer(lhs) if lhs is not None else None
        n.u.bin.rhs = C.pointer(rhs) if rhs is not None else None
        n.u.bin.op = self._s(op)
        return n

    def binop(self, op: str, lhs, rhs) -> Node:
        n = self._node(N_BINARY_OP)
        n.u.bin.lhs = C.pointer(lhs) if lhs is not None else None
        n.u.bin.rhs = C.pointer(rhs) if rhs is not None else None
        n.u.bin.op = self._s(op)
        return n

    def inlist(self, items) -> Node:
        n = self._node(N_LIST)
        n.u.list.items = self._arr(NodeP, [C.pointer(x) for x in items])
        n.u.list.nitems = len(items)
        return n

    def func(self, name: str, *args) -> Node:
        n = self._node(N_FUNCTION)
        n.u.fn.name = self._s(name)
        n.u.fn.args = self._arr(NodeP, [C.pointer(a) for a in args])
        n.u.fn.nargs = len(args)
        return n

    @staticmethod
    def column_text(n: Node) -> str:
        """generate_column_name (reference ast_nodes.c:235-320), common shapes."""
        if n.kind in (N_IDENTIFIER, N_LITERAL):
            return n.u.text.decode("latin-1")
        if n.kind == N_FUNCTION:
            args = ", ".join(Plan.column_text(n.u.fn.args[i].contents) for i in range(n.u.fn.nargs))
            return f"{n.u.fn.name.decode('latin-1')}({args})"
        if n.kind == N_BINARY_OP:
            op = n.u.bin.op.decode("latin-1")
            if not n.u.bin.lhs:
                r = n.u.bin.rhs.contents
                rs = Plan.column_text(r)
                return f"{op}({rs})" if r.kind == N_BINARY_OP else f"{op}{rs}"
            l, r = n.u.bin.lhs.contents, n.u.bin.rhs.contents
            ls, rs = Plan.column_text(l), Plan.column_text(r)
            if l.kind == N_BINARY_OP:
                ls = f"({ls})"
            if r.kind == N_BINARY_OP:
                rs = f"({rs})"
            return f"{ls} {op} {rs}"
        return "expr"

    def query(self, select, path: str, alias: str | None = None, where=None,
              group_by=(), joins=(), order_by=None, desc=False, having=None,
              limit=-1, offset=-1, distinct=False) -> Node:
        """select: list of Node | "*" | (Node, alias)."""
        sel = self._node(N_SELECT)
        texts, exprs = [], []
        for item in select:
            if isinstance(item, str) and item == "*":
                texts.append(self._s("*"))
                exprs.append(NodeP())
                continue
            node, al = (item if isinstance(item, tuple) else (item, None))
            t = Plan.column_text(node)
            if al:
                t = f"{t} AS {al}"
            texts.append(self._s(t))
            exprs.append(C.pointer(node))
        sel.u.sel.texts = self._arr(C.c_char_p, texts)
        sel.u.sel.exprs = self._arr(NodeP, exprs)
        sel.u.sel.count = len(texts)
        sel.u.sel.distinct = distinct
        frm = self._node(N_FROM)
        frm.u.from_.path = self._s(path)
        frm.u.from_.alias = self._s(alias)
        q = self._node(N_QUERY)
        q.u.q.select = C.pointer(sel)
        q.u.q.from_ = C.pointer(frm)
        jn = []
        for (jpath, jalias, on, kind) in joins:
            j = self._node(N_JOIN)
            j.u.join.kind = kind
            j.u.join.path = self._s(jpath)
            j.u.join.alias = self._s(jalias)
            j.u.join.on = C.pointer(on) if on is not None else None
            jn.append(C.pointer(j))
        q.u.q.joins = self._arr(NodeP, jn) if jn else None
        q.u.q.join_count = len(jn)
        q.u.q.where = C.pointer(where) if where is not None else None
        if group_by:
            g = self._node(N_GROUP_BY)
            g.u.grp.keys = self._arr(C.c_char_p, [self._s(k) for k in group_by])
            g.u.grp.nkeys = len(group_by)
            q.u.q.group_by = C.pointer(g)
        if order_by is not None:
            o = self._node(N_ORDER_BY)
            o.u.ord.key = self._s(order_by)
            o.u.ord.desc = desc
            q.u.q.order_by = C.pointer(o)
        q.u.q.having = C.pointer(having) if having is not None else None
        q.u.q.limit = limit
        q.u.q.offset = offset
        return q
