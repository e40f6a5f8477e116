"""Repartitioned multi-GPU INNER JOIN, simulated in one process.

Every "rank" holds a record-boundary shard of both inputs.  The device routing
(cqgpu_route_plan / cqgpu_route_fill) is run per rank, the all-to-all is done by
hand (slice d of every rank, concatenated in source-rank order -- exactly what
cq_amd.dist.exchange does over RCCL, tested on gloo in test_dist_gloo.py), each
rank joins what it received (cqgpu_table_from_routed + cqgpu_query_partial) and
cqgpu_merge_partials must reproduce the oracle's nested-loop join over the whole
files (reference evaluator_joins.c:63-181): counts, group set and first-appearance
order exact, SUM/AVG within 1e-6 relative.
"""
import re

import numpy as np
import pytest
import torch

import cqtest
import cq_amd
from cq_amd import abi, datagen
from cq_amd.dist import first_join_cross
from test_gpu_parity import compare, tolerant_columns

pytestmark = pytest.mark.gpu


def _shards(data: bytes, nranks: int, seed: int, cfg=None):
    header, body = data.split(b"\n", 1)
    header += b"\n"
    rng = np.random.default_rng(seed)
    fr = sorted(rng.uniform(0.05, 0.95, nranks - 1)) if nranks > 1 else []
    cuts = [0] + [body.index(b"\n", int(len(body) * f)) + 1 if body else 0 for f in fr] + [len(body)]
    tabs = []
    for r in range(nranks):
        pc = body[cuts[r]:cuts[r + 1]]
        if r == 0:
            tabs.append(cq_amd.Table.from_bytes(header + pc, cfg=cfg))
        else:
            tabs.append(cq_amd.Table.from_bytes(pc, cfg=cfg, base_offset=len(header) + cuts[r], header=header))
    return header, tabs


LAST_KINDS = []   # per rank, the scan kernel kind of its partial (4: the STAR fused join)
LAST_MODE = [0]   # the routing mode of the last _run (cqgpu_route_major)
LAST_BLOBS = []   # per rank, its partial blob


def _run(ast, ldata: bytes, rdata: bytes, nranks: int, rest=(), outer=True, cfg=None):
    """rest: a chain's later JOIN tables, whole on every rank.  outer: run the later
    RIGHT / FULL levels' protocol (cqgpu_join_outer_*, as cq_amd.dist.outer_sets):
    per level every rank's matched flags, OR-ed, handed back to every rank with rank
    0 emitting the records no rank matched"""
    lh, ls = _shards(ldata, nranks, 1, cfg)
    rh, rs = _shards(rdata, nranks, 2, cfg)
    routed = [[None, None] for _ in range(nranks)]
    keep = []
    # the routing mode every rank agrees on (cq_amd.dist.join_partitioned's sequence):
    # a JOIN without ON sends side 1 everywhere; mixed key classes replicate the minority
    cross = first_join_cross(ast)
    mode = 0
    if not cross:
        tot = np.zeros(8, dtype=np.int64)
        for r in range(nranks):
            for side in (0, 1):
                tot[4 * side: 4 * side + 4] += cq_amd.route_plan2(ast, [ls[r], rs[r]], side, nranks, r)[3]
        mode = cq_amd.route_major([int(x) for x in tot[:4]], [int(x) for x in tot[4:]])
    LAST_MODE[:] = [mode]
    for side, (hdr, sh) in enumerate(((lh, ls), (rh, rs))):
        plans = [cq_amd.route_plan2(ast, [ls[r], rs[r]], side, nranks, r, mode) for r in range(nranks)]
        total = sum(p[2] for p in plans)
        sends, base = [], 0
        for r in range(nranks):
            nb, nr, nown, _ = plans[r]
            sb = torch.empty(max(sum(nb), 1), dtype=torch.uint8, device="cuda")
            sg = torch.empty(max(sum(nr), 1), dtype=torch.int64, device="cuda")
            cq_amd.route_fill(sh[r], base, sb.data_ptr(), sg.data_ptr())
            base += nown
            bo = np.concatenate([[0], np.cumsum(nb)]).astype(int)
            ro = np.concatenate([[0], np.cumsum(nr)]).astype(int)
            sends.append((sb, sg, bo, ro))
        torch.cuda.synchronize()
        for d in range(nranks):
            rb = torch.cat([sb[bo[d]:bo[d + 1]] for sb, _, bo, _ in sends])
            rg = torch.cat([sg[ro[d]:ro[d + 1]] for _, sg, _, ro in sends])
            keep += [rb, rg]
            torch.cuda.synchronize()          # torch's copies before the library's stream reads them
            routed[d][side] = cq_amd.table_from_routed(rb.data_ptr(), rb.numel(), rg.data_ptr(), rg.numel(), hdr,
                                                       cfg)
            cq_amd.table_set_record_total(routed[d][side], total)
            cq_amd.table_set_key_stride(routed[d][side], nranks)
            cq_amd.table_set_replicated(routed[d][side], (4 if side == 1 else 0) if cross else mode, d == 0)
    whole = [[cq_amd.Table.from_bytes(x, cfg=cfg) for x in rest] for _ in range(nranks)]
    sets = {}

    def apply(d, upto):                    # rank d's view of the sets of the levels below `upto`
        cq_amd.join_outer_clear()
        for jj, g in sets.items():
            if jj < upto:
                cq_amd.join_outer_set(jj, g, d == 0)
    try:
        for j in range(1, len(rest) + 1 if outer else 1):
            fl = []
            for d in range(nranks):
                apply(d, j)
                fl.append(cq_amd.join_outer_matched(ast, routed[d] + whole[d], j))
            if fl[0] is not None:
                sets[j] = np.bitwise_or.reduce([np.frombuffer(f, np.uint8) for f in fl]).tobytes()
        blobs = []
        LAST_KINDS.clear()
        for d in range(nranks):
            apply(d, len(rest) + 1)
            blobs.append(cq_amd.query_partial(ast, routed[d] + whole[d]))
            LAST_KINDS.append(cq_amd.stats().get("scan_kernel"))
        LAST_BLOBS[:] = blobs
        tp = cq_amd.merge_partials(ast, blobs)
    finally:
        cq_amd.join_outer_clear()
        for t in ls + rs + [x for pr in routed for x in pr] + [x for w in whole for x in w]:
            t.close()
    return tp


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("joindist")
    rng = np.random.default_rng(5)
    f = {}
    f["users"] = datagen.users_bytes(4000, seed=7)
    f["orders"] = datagen.orders_bytes(9000, 4500, seed=8)
    # duplicate keys, NULL keys, INTEGER vs DOUBLE spellings of one key, short rows
    lines = ["id,name,age,role"]
    for i in range(2500):
        uid = int(rng.integers(0, 1800))
        age = "" if rng.integers(0, 40) == 0 else str(int(rng.integers(18, 90)))
        key = "" if rng.integers(0, 70) == 0 else str(uid)
        lines.append(f"{key},n{i % 53},{age},role_{int(rng.integers(0, 23)):02d}")
    lines.append("")
    lines.append("77,short")
    f["du"] = ("\n".join(lines) + "\n").encode()
    lines = ["id,price,quantity,customer_id"]
    for i in range(4000):
        cid = int(rng.integers(0, 2000))
        k = int(rng.integers(0, 50))
        cs = "" if k == 0 else (f"{cid}.0" if k == 1 else str(cid))
        lines.append(f"{i},{rng.integers(100, 99999) / 100:.2f},{rng.integers(1, 9)},{cs}")
    f["do"] = ("\n".join(lines) + "\n").encode()
    f["sa"] = ("k,v\n" + "".join(f"{'' if i % 41 == 0 else 'key%03d' % (i % 150)},{i}\n"
                                  for i in range(900))).encode()
    f["sb"] = ("k,w\n" + "".join(f"{'' if i % 53 == 0 else 'key%03d' % (i % 170)},{i * 3}\n"
                                  for i in range(700))).encode()
    f["mixed"] = b"k,z\n1,a\nx,b\n2,c\n,d\n2020-01-02,e\nx,f\n1.0,g\n"
    # larger mixed-class key columns: numbers (INTEGER and DOUBLE spellings), strings,
    # dates and NULLs on both sides
    def mk_key(r):
        k = int(r.integers(0, 10))
        if k < 5:
            return str(int(r.integers(0, 40))) if k else f"{int(r.integers(0, 40))}.0"
        if k < 8:
            return "s%02d" % int(r.integers(0, 25))
        return "" if k == 8 else "2021-03-%02d" % int(r.integers(1, 9))
    f["mk"] = ("k,v,g\n" + "".join(f"{mk_key(rng)},{i},{i % 3}\n" for i in range(300))).encode()
    f["mk2"] = ("k,w\n" + "".join(f"{mk_key(rng)},{i}\n" for i in range(150))).encode()
    # a column mixing numbers, strings and dates (MIN/MAX keep the class of the
    # group's first non-NULL cell in nested-loop order, evaluator_aggregates.c:311-326)
    tags = ["12", "abc", "2020-01-01", "", "7.5", "zz", "1999-12-31", "-3", "b"]
    lines = ["id,tag,role"]
    for i in range(2200):
        lines.append(f"{int(rng.integers(0, 1800))},{tags[int(rng.integers(0, len(tags)))]},r{int(rng.integers(0, 9))}")
    f["mu"] = ("\n".join(lines) + "\n").encode()
    # chain tables: roles of "du" (role_20..22 missing, role_05 twice, a NULL role) and
    # labels of the order quantities
    f["rl"] = ("role,dept,grade\n" + "".join(f"role_{i:02d},dept{i % 4},{i % 3}\n" for i in range(20))
               + "role_05,dept9,7\n,deptx,0\n").encode()
    f["qt"] = b"q,label\n0,lab0\n2,lab2\n1,lab1\n2,lab2b\n9,lab9\n"
    f["ex"] = b"role,dept,grade\n"          # a later level's table with no records
    paths = {}
    for k, v in f.items():
        p = d / f"{k}.csv"
        p.write_bytes(v)
        paths[k] = str(p)
    return f, paths


QUERIES = [
    ("users", "orders", "SELECT COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id"),
    ("users", "orders", "SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM '{L}' AS u JOIN '{R}' AS o "
                        "ON u.id = o.customer_id GROUP BY u.role"),
    ("du", "do", "SELECT COUNT(*), SUM(o.price), AVG(o.quantity) FROM '{L}' AS u JOIN '{R}' AS o "
                 "ON u.id = o.customer_id WHERE u.age > 40"),
    ("du", "do", "SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM '{L}' AS u JOIN '{R}' AS o "
                 "ON u.id = o.customer_id GROUP BY u.role"),
    ("du", "do", "SELECT o.quantity, COUNT(*), MIN(u.age), MAX(u.name) FROM '{L}' AS u JOIN '{R}' AS o "
                 "ON u.id = o.customer_id GROUP BY o.quantity"),
    ("du", "do", "SELECT u.name, COUNT(*), MIN(o.price) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
                 "WHERE o.price > 300 GROUP BY u.name HAVING COUNT(*) > 5 ORDER BY u.name LIMIT 20"),
    ("sa", "sb", "SELECT a.k, COUNT(*), SUM(b.w), MIN(a.v) FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k GROUP BY a.k"),
    ("sa", "sb", "SELECT COUNT(*), MAX(b.w) FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k WHERE a.v > 5000"),
    # outer joins (evaluator_joins.c:128-171): unmatched rows are exact per rank after the
    # repartition; their global positions come from the pair position keys
    ("du", "do", "SELECT COUNT(*), SUM(o.price) FROM '{L}' AS u LEFT JOIN '{R}' AS o ON u.id = o.customer_id"),
    ("du", "do", "SELECT u.role, COUNT(*), MAX(o.id), MIN(u.name) FROM '{L}' AS u LEFT JOIN '{R}' AS o "
                 "ON u.id = o.customer_id GROUP BY u.role"),
    ("du", "do", "SELECT o.quantity, COUNT(*), MIN(u.age) FROM '{L}' AS u RIGHT JOIN '{R}' AS o "
                 "ON u.id = o.customer_id GROUP BY o.quantity"),
    ("du", "do", "SELECT u.age, COUNT(*), SUM(o.price) FROM '{L}' AS u FULL JOIN '{R}' AS o "
                 "ON u.id = o.customer_id GROUP BY u.age"),
    ("sa", "sb", "SELECT b.k, COUNT(*), SUM(a.v) FROM '{L}' AS a FULL JOIN '{R}' AS b ON a.k = b.k GROUP BY b.k"),
    # row-returning joins (build_result over the joined table): every rank's rows with
    # their global (left id, right id) keys, merged in nested-loop order, then the
    # host's ORDER BY / DISTINCT / LIMIT
    ("du", "do", "SELECT u.name, o.price, o.quantity FROM '{L}' AS u JOIN '{R}' AS o "
                 "ON u.id = o.customer_id WHERE o.quantity > 3"),
    ("du", "do", "SELECT u.role, o.id FROM '{L}' AS u LEFT JOIN '{R}' AS o ON u.id = o.customer_id"),
    ("sa", "sb", "SELECT a.k, b.w FROM '{L}' AS a FULL JOIN '{R}' AS b ON a.k = b.k"),
    ("du", "do", "SELECT o.id, u.name, o.price FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
                 "ORDER BY o.id DESC LIMIT 20"),
    ("du", "do", "SELECT o.id, u.age FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id LIMIT 15 OFFSET 5"),
    ("du", "do", "SELECT DISTINCT u.role FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id"),
    ("sa", "sb", "SELECT * FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k WHERE b.w < 100"),
    # MIN/MAX over a column mixing value classes: every rank's per-class first
    # positions and extremes as global pair keys
    ("mu", "do", "SELECT u.role, COUNT(*), MIN(u.tag), MAX(u.tag) FROM '{L}' AS u JOIN '{R}' AS o "
                 "ON u.id = o.customer_id GROUP BY u.role"),
    ("mu", "do", "SELECT MIN(u.tag), MAX(u.tag), COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id"),
    ("mu", "do", "SELECT o.quantity, MAX(u.tag) FROM '{L}' AS u LEFT JOIN '{R}' AS o ON u.id = o.customer_id "
                 "GROUP BY o.quantity"),
    # STDDEV across partials: per-rank (sum, squared deviations, count), merged exactly
    ("du", "do", "SELECT u.role, STDDEV(o.price), COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o "
                 "ON u.id = o.customer_id GROUP BY u.role"),
]


@pytest.mark.parametrize("nranks", [1, 2, 3, 5])
@pytest.mark.parametrize("case", range(len(QUERIES)))
def test_repartitioned_join(files, case, nranks):
    data, paths = files
    lk, rk, tmpl = QUERIES[case]
    sql = tmpl.replace("{L}", paths[lk]).replace("{R}", paths[rk])
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    with cqtest.Parsed(sql) as ast:
        tp = _run(ast, data[lk], data[rk], nranks)
        assert tp, cq_amd.last_error()
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{sql} @ {nranks} ranks")


DIALECT = [   # ';' delimiter, "'" quote: quoted names holding the delimiter, doubled quotes
    "SELECT u.role, COUNT(*), SUM(o.price), MAX(u.name) FROM '{L}' AS u JOIN '{R}' AS o "
    "ON u.id = o.customer_id GROUP BY u.role",
    "SELECT u.name, o.price FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id WHERE o.price > 900",
    "SELECT o.quantity, COUNT(*), MIN(u.name) FROM '{L}' AS u RIGHT JOIN '{R}' AS o "
    "ON u.id = o.customer_id GROUP BY o.quantity",
]


@pytest.mark.parametrize("nranks", [1, 3])
@pytest.mark.parametrize("case", range(len(DIALECT)))
def test_repartitioned_join_dialect(files, tmp_path, case, nranks):
    """the repartition with another CSV dialect (delimiter ';', quote "'"): the route's
    field projection and the routed tables keep the dialect's field split
    (csv_reader.c:278-338) -- quoted names holding ';' and doubled quotes"""
    data, _ = files
    cfg = abi.csv_config(";", "'")

    def conv(b: bytes, quote_col: int) -> bytes:
        out = []
        for i, ln in enumerate(b.decode().split("\n")):
            f = ln.split(",")
            if i > 0 and 0 <= quote_col < len(f) and f[quote_col]:
                v = f[quote_col]
                v = v + ";x" if i % 3 == 0 else (v + "''q" if i % 3 == 1 else v)
                f[quote_col] = "'" + v + "'"
            out.append(";".join(f))
        return "\n".join(out).encode()
    lb, rb = conv(data["du"], 1), conv(data["do"], -1)
    paths = {}
    for k, v in (("L", lb), ("R", rb)):
        paths[k] = str(tmp_path / f"{k}.csv")
        open(paths[k], "wb").write(v)
    sql = DIALECT[case].replace("{L}", paths["L"]).replace("{R}", paths["R"])
    want, unsup = cqtest.oracle_query(sql, cfg)
    assert not unsup, sql
    with cqtest.Parsed(sql) as ast:
        tp = _run(ast, lb, rb, nranks, cfg=cfg)
        assert tp, cq_amd.last_error()
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{sql} @ {nranks} ranks (dialect ; ')")


@pytest.mark.parametrize("nranks", [1, 2, 3, 5, 8])
def test_repartitioned_fused_join(files, nranks):
    """config 5's shape after the key repartition: whole-number keys are routed by key
    mod N (route.hip route_dest), so every rank's build keys are one dense residue
    class and every rank joins its routed sides with the STAR fused join (slots
    (key - kmin) / N, no pair array), reporting its groups' first pairs by global left
    id; the merge must equal the oracle's nested loop.  g_stats is reset per
    cqgpu_query_partial call, so a rank whose STAR declined reports kind 0 here"""
    data, paths = files
    sql = (f"SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM '{paths['users']}' AS u "
           f"JOIN '{paths['orders']}' AS o ON u.id = o.customer_id GROUP BY u.role")
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    with cqtest.Parsed(sql) as ast:
        tp = _run(ast, data["users"], data["orders"], nranks)
        assert tp, cq_amd.last_error()
        kinds = list(LAST_KINDS)
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{sql} @ {nranks} ranks")
    assert len(kinds) == nranks and all(k == 4 for k in kinds), kinds


def _blob_groups(blob: bytes):
    """a "CQJ1" partial's groups, field by field -- everything but the table addresses
    STRING cells carry in their bits (meaningless across table instances)"""
    import struct
    o = [0]

    def take(fmt):
        v = struct.unpack_from("<" + fmt, blob, o[0])
        o[0] += struct.calcsize("<" + fmt)
        return v[0]

    def text():
        n = take("I")
        o[0] += n
        return blob[o[0] - n:o[0]]

    def cell():
        k, bits, s = take("I"), take("Q"), text()
        return (k, s) if k == 3 else (k, bits)
    assert take("I") == 0x314a5143
    names = [text() for _ in range(take("I"))]
    nacc = take("I")
    classes = [take("I") for _ in range(nacc)]
    nrep, nvla = take("I"), take("I")
    masks = (take("I"), take("I"))
    out = [names, classes, nrep, nvla, masks]
    for _ in range(take("Q")):
        g = [take("I"), take("I"), take("Q"), take("Q"), text(), take("Q"), take("Q")]
        g.append([(take("d"), take("Q"), take("Q"), cell()) for _ in range(nacc)])
        g.append([cell() for _ in range(nrep)])
        assert nvla == 0
        g.append(take("I"))                       # class splits (none for these plans)
        out.append(g)
    assert o[0] == len(blob)
    return out


@pytest.mark.parametrize("nranks", [1, 3])
def test_first_ids_device_equals_host(files, nranks, monkeypatch):
    """the STAR partial's first-pair global ids mapped on the device
    (route.hip pack_first_gid_kernel, the default) and by the host lookup
    (CQGPU_HOST_FIRST_IDS=1): the same blobs, byte for byte"""
    data, paths = files
    sql = (f"SELECT u.role, COUNT(*), SUM(o.price) FROM '{paths['users']}' AS u "
           f"JOIN '{paths['orders']}' AS o ON u.id = o.customer_id GROUP BY u.role")
    got = []
    with cqtest.Parsed(sql) as ast:
        for host in (False, True):
            if host:
                monkeypatch.setenv("CQGPU_HOST_FIRST_IDS", "1")
            tp = _run(ast, data["users"], data["orders"], nranks)
            assert tp, cq_amd.last_error()
            assert all(k == 4 for k in LAST_KINDS), LAST_KINDS
            cq_amd.result_free(tp)
            got.append([_blob_groups(b) for b in LAST_BLOBS])
    assert got[0] == got[1]


def test_partial_stats_reset_per_call(files):
    """a general-join partial after a STAR partial reports its own kernel kind (0),
    not the stale 4 of the call before"""
    data, paths = files
    star = (f"SELECT u.role, COUNT(*), SUM(o.price) FROM '{paths['users']}' AS u "
            f"JOIN '{paths['orders']}' AS o ON u.id = o.customer_id GROUP BY u.role")
    gen = (f"SELECT u.role, COUNT(*), MIN(o.price) FROM '{paths['users']}' AS u "
           f"JOIN '{paths['orders']}' AS o ON u.id = o.customer_id GROUP BY u.role")
    with cqtest.Parsed(star) as ast:
        tp = _run(ast, data["users"], data["orders"], 2)
        assert tp and LAST_KINDS == [4, 4], LAST_KINDS
        cq_amd.result_free(tp)
    with cqtest.Parsed(gen) as ast:
        tp = _run(ast, data["users"], data["orders"], 2)
        assert tp, cq_amd.last_error()
        assert LAST_KINDS == [0, 0], LAST_KINDS
        cq_amd.result_free(tp)


@pytest.mark.parametrize("partitioned", [False, True])
def test_repartitioned_fused_join_1m_8_ranks(monkeypatch, partitioned):
    """1e6 users x 1e6 orders over 8 simulated ranks (no small-table slack in the
    STAR range test): every rank must take STAR, and the merged result must equal the
    exact nested-loop answer computed here with numpy (COUNT exact, SUM/AVG 1e-6
    relative; groups in the order of their first matched user)"""
    if partitioned:      # the partitioned probe on every rank (64 Ki-slot partitions)
        monkeypatch.setenv("CQGPU_PART_PROBE_MIN", "0")
        monkeypatch.setenv("CQGPU_PART_PROBE_SHIFT", "16")
    n = 1_000_000
    users = datagen.users_bytes(n, seed=21)
    orders = datagen.orders_bytes(n, n, seed=22)
    rng = np.random.default_rng(21)
    rng.integers(10, 81, n)
    role = rng.integers(0, 1000, n)
    rng2 = np.random.default_rng(22)
    cust = rng2.integers(0, n, n)
    price = rng2.integers(100, 100000, n)
    cnt = np.bincount(role[cust], minlength=1000)
    cents = np.bincount(role[cust], weights=price, minlength=1000)
    matched = np.zeros(n, dtype=bool)
    matched[cust] = True
    first = np.full(1000, n, dtype=np.int64)
    np.minimum.at(first, role[matched], np.nonzero(matched)[0])
    order = [r for r in np.argsort(first, kind="stable") if cnt[r] > 0]
    sql = ("SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM 'users.csv' AS u "
           "JOIN 'orders.csv' AS o ON u.id = o.customer_id GROUP BY u.role")
    with cqtest.Parsed(sql) as ast:
        tp = _run(ast, users, orders, 8)
        assert tp, cq_amd.last_error()
        kinds = list(LAST_KINDS)
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
    assert kinds == [4] * 8, kinds
    rows = got["rows"]
    assert len(rows) == len(order)
    for row, r in zip(rows, order):
        assert row[0][1] in (b"role_%03d" % r, "role_%03d" % r), (row, r)
        assert row[1][1] == cnt[r], (row, cnt[r])
        want_sum = cents[r] / 100.0
        assert abs(row[2][1] - want_sum) <= 1e-6 * abs(want_sum), (row, want_sum)
        assert abs(row[3][1] - want_sum / cnt[r]) <= 1e-6 * abs(want_sum / cnt[r]), row


CHAINS = [
    # (the reference resolves a chained table's columns by their exact joined names:
    # the last level's "r.x" / "q.x"; earlier levels' "o.x" / "u.x" read NULL -- kept
    # in two queries as a parity check of that rule)
    (["rl"], "SELECT r.dept, COUNT(*), SUM(r.grade), AVG(r.grade) FROM '{L}' AS u JOIN '{R}' AS o "
             "ON u.id = o.customer_id JOIN '{X}' AS r ON u.role = r.role GROUP BY r.dept"),
    (["rl"], "SELECT COUNT(*), MIN(r.grade), MAX(r.dept), SUM(o.price) FROM '{L}' AS u JOIN '{R}' AS o "
             "ON u.id = o.customer_id LEFT JOIN '{X}' AS r ON u.role = r.role"),
    (["rl"], "SELECT r.role, r.dept, r.grade FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
             "JOIN '{X}' AS r ON u.role = r.role WHERE r.grade > 1"),
    (["rl"], "SELECT r.role, r.grade, o.id FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
             "LEFT JOIN '{X}' AS r ON u.role = r.role LIMIT 25 OFFSET 10"),
    (["rl"], "SELECT r.dept, COUNT(*), MAX(r.grade), MIN(r.role) FROM '{L}' AS u LEFT JOIN '{R}' AS o "
             "ON u.id = o.customer_id JOIN '{X}' AS r ON u.role = r.role GROUP BY r.dept"),
    (["rl"], "SELECT r.grade, COUNT(*), SUM(r.grade) FROM '{L}' AS u FULL JOIN '{R}' AS o "
             "ON u.id = o.customer_id LEFT JOIN '{X}' AS r ON u.role = r.role GROUP BY r.grade"),
    (["rl"], "SELECT r.role, r.dept FROM '{L}' AS u RIGHT JOIN '{R}' AS o ON u.id = o.customer_id "
             "LEFT JOIN '{X}' AS r ON u.role = r.role WHERE r.grade = 2 ORDER BY r.dept DESC LIMIT 30"),
    (["rl", "qt"], "SELECT q.label, COUNT(*), SUM(q.q), MIN(q.label) FROM '{L}' AS u JOIN '{R}' AS o "
                   "ON u.id = o.customer_id JOIN '{X}' AS r ON u.role = r.role "
                   "JOIN '{Y}' AS q ON r.grade = q.q GROUP BY q.label"),
    (["rl", "qt"], "SELECT q.label, q.q FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
                   "LEFT JOIN '{X}' AS r ON u.role = r.role LEFT JOIN '{Y}' AS q ON r.grade = q.q "
                   "LIMIT 40 OFFSET 500"),
    # a later RIGHT / FULL level (evaluator_joins.c:143-171 through :268-270): its
    # unmatched records are the ones no rank matched ("rl": role_20..22 missing, a NULL
    # role; "qt": q = 9 matches no grade), emitted once, after every left-driven row
    (["rl"], "SELECT COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
             "RIGHT JOIN '{X}' AS r ON u.role = r.role"),
    (["rl"], "SELECT r.dept, COUNT(*), SUM(o.price), MIN(r.role) FROM '{L}' AS u JOIN '{R}' AS o "
             "ON u.id = o.customer_id FULL JOIN '{X}' AS r ON u.role = r.role GROUP BY r.dept"),
    (["rl"], "SELECT r.role, r.dept, o.id FROM '{L}' AS u LEFT JOIN '{R}' AS o ON u.id = o.customer_id "
             "RIGHT JOIN '{X}' AS r ON u.role = r.role WHERE o.price > 990 OR r.grade = 7 OR r.grade = 0"),
    (["rl", "qt"], "SELECT q.label, COUNT(*), MAX(r.dept) FROM '{L}' AS u JOIN '{R}' AS o "
                   "ON u.id = o.customer_id RIGHT JOIN '{X}' AS r ON u.role = r.role "
                   "FULL JOIN '{Y}' AS q ON r.grade = q.q GROUP BY q.label"),
    (["rl", "qt"], "SELECT r.dept, q.label, u.name FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
                   "FULL JOIN '{X}' AS r ON u.role = r.role RIGHT JOIN '{Y}' AS q ON r.grade = q.q "
                   "ORDER BY q.label LIMIT 30 OFFSET 3"),
    # ... whose table has no records: RIGHT keeps nothing, FULL every joined row
    (["ex"], "SELECT COUNT(*), MIN(r.dept) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
             "RIGHT JOIN '{X}' AS r ON u.role = r.role"),
    (["ex"], "SELECT r.dept, COUNT(*), SUM(o.price) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
             "FULL JOIN '{X}' AS r ON u.role = r.role GROUP BY r.dept"),
]


def _chain_sql(paths, rest, tmpl):
    sql = tmpl.replace("{L}", paths["du"]).replace("{R}", paths["do"])
    for ph, k in zip(("{X}", "{Y}"), rest):
        sql = sql.replace(ph, paths[k])
    return sql


@pytest.mark.parametrize("nranks", [1, 3, 8])
@pytest.mark.parametrize("case", range(len(CHAINS)))
def test_join_chain_across_partials(files, case, nranks):
    """process_joins (evaluator_joins.c:237-274) across partials: the first JOIN on
    the key-routed sides, the later ones against the whole next table on every
    rank; rows and groups in the reference's nested-loop order through the
    mixed-radix chain keys (route.hip chain_key_kernel)"""
    data, paths = files
    rest, tmpl = CHAINS[case]
    sql = _chain_sql(paths, rest, tmpl)
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    with cqtest.Parsed(sql) as ast:
        tp = _run(ast, data["du"], data["do"], nranks, [data[k] for k in rest])
        assert tp, (sql, cq_amd.last_error())
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{sql} @ {nranks} ranks")


def test_join_chain_right_later_needs_sets(files):
    """a later level's RIGHT / FULL JOIN needs every rank's matches: without the
    ranks' OR-ed flags (cqgpu_join_outer_set) it is refused, not approximated"""
    data, paths = files
    sql = _chain_sql(paths, ["rl"], "SELECT COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
                                     "RIGHT JOIN '{X}' AS r ON u.role = r.role")
    with cqtest.Parsed(sql) as ast:
        with pytest.raises(RuntimeError):
            _run(ast, data["du"], data["do"], 3, [data["rl"]], outer=False)
        assert "without the ranks' matched records" in cq_amd.last_ineligible()
        # flags of the wrong length are an error, not a wrong answer
        lt, rt, xt = (cq_amd.Table.from_bytes(data[k]) for k in ("du", "do", "rl"))
        try:
            cq_amd.join_outer_set(1, b"\x00" * 3, True)
            with pytest.raises(RuntimeError, match="flags for a level of"):
                cq_amd.query_partial(ast, [lt, rt, xt])
            cq_amd.join_outer_clear()
            # a level that needs no set: INNER / LEFT, and level 0
            assert cq_amd.join_outer_matched(ast, [lt, rt, xt], 0) is None
            fl = cq_amd.join_outer_matched(ast, [lt, rt, xt], 1)
            assert fl is not None and len(fl) == data["rl"].count(b"\n") - 1
        finally:
            cq_amd.join_outer_clear()
            for t in (lt, rt, xt):
                t.close()


MIXED = [   # keys of several value classes: value_compare calls any two non-NULL keys of
    # different classes equal (csv_reader.c:126-129, the join's compare at
    # evaluator_joins.c:53-55) -- the majority class routes by key, the others go to
    # every rank, and a pair of two replicated records is kept by rank 0 only
    ("mixed", "sa", "SELECT COUNT(*) FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k"),
    ("mk", "mk2", "SELECT COUNT(*), SUM(b.w), MIN(a.v) FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k"),
    ("mk", "mk2", "SELECT a.g, COUNT(*), SUM(b.w), MAX(b.k) FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k "
                  "GROUP BY a.g"),
    ("mk", "mk2", "SELECT a.v, b.w, a.k, b.k FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k WHERE b.w < 60"),
    ("mk", "sa", "SELECT a.g, COUNT(*) FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k GROUP BY a.g"),
    ("mixed", "mixed", "SELECT a.z, b.z FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k"),
    ("mk", "mk2", "SELECT b.w, COUNT(*) FROM '{L}' AS a JOIN '{R}' AS b ON a.k = b.k JOIN '{C}' AS c "
                  "ON a.g = c.q GROUP BY b.w ORDER BY b.w LIMIT 12"),
]


@pytest.mark.parametrize("nranks", [1, 2, 3, 5])
@pytest.mark.parametrize("case", range(len(MIXED)))
def test_mixed_key_classes_across_partials(files, case, nranks):
    """mixed key classes across partials (cqgpu_route_plan2's replication) vs the oracle"""
    data, paths = files
    lk, rk, tmpl = MIXED[case]
    sql = tmpl.replace("{L}", paths[lk]).replace("{R}", paths[rk]).replace("{C}", paths["qt"])
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    with cqtest.Parsed(sql) as ast:
        rest = (data["qt"],) if "{C}" in tmpl else ()
        tp = _run(ast, data[lk], data[rk], nranks, rest=rest)
        assert tp, (cq_amd.last_error(), cq_amd.last_ineligible())
        assert LAST_MODE[0] != 0, "the data mixes key classes: a replicated routing"
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{sql} @ {nranks} ranks")


def test_mixed_key_classes_empty_side():
    """ADVICE r1 layout: 5 ranks, a right side of three INTEGER keys, a left side of
    the same INTEGER keys plus many STRING keys: the STRING rows (the majority) route
    by key, to ranks that receive no right rows, the INTEGER rows of the right side
    go to every rank -- every cross-class pair exactly once, vs the oracle"""
    left = b"k,v\n" + b"".join(b"%s,%d\n" % ((b"%d" % (i % 3 + 1)) if i % 4 == 0 else (b"s%02d" % (i % 40)), i)
                                 for i in range(400))
    right = b"k,w\n1,10\n2,20\n3,30\n"
    want = {"count": 0}
    for i in range(400):
        want["count"] += 1 if i % 4 == 0 else 3      # an INTEGER key matches its own; a STRING key all three
    sql = "SELECT COUNT(*), SUM(b.w) FROM 'l' AS a JOIN 'r' AS b ON a.k = b.k"
    with cqtest.Parsed(sql) as ast:
        for n in (1, 2, 5):
            tp = _run(ast, left, right, n)
            assert tp, (cq_amd.last_error(), cq_amd.last_ineligible())
            got = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            s = sum(((i % 3 + 1) * 10) if i % 4 == 0 else 60 for i in range(400))
            assert got["rows"][0][0][1] == want["count"], (n, got)
            assert abs(got["rows"][0][1][1] - s) < 1e-6 * s, (n, got)
            assert LAST_MODE[0] == 2, LAST_MODE      # strings are the majority class


@pytest.mark.parametrize("kind", ["LEFT", "RIGHT", "FULL"])
def test_mixed_key_classes_outer_refused(files, kind):
    """an outer JOIN over mixed key classes across partials: its unmatched rows would
    need every rank's matches -- refused on every rank, never approximated"""
    data, paths = files
    sql = f"SELECT COUNT(*) FROM '{paths['mixed']}' AS a {kind} JOIN '{paths['sa']}' AS b ON a.k = b.k"
    with cqtest.Parsed(sql) as ast:
        with pytest.raises(RuntimeError, match="outer JOIN over keys of different value classes"):
            _run(ast, data["mixed"], data["sa"], 2)


CROSS = [   # JOIN without ON (evaluator_joins.c:41: every pair matches): side 0 stays on its
    # rank, side 1 goes to every rank; order keys (left id, right id) as ever
    ("sa", "qt", "SELECT COUNT(*), SUM(b.q), MIN(a.k) FROM '{L}' AS a JOIN '{R}' AS b"),
    ("du", "qt", "SELECT u.role, COUNT(*), MAX(b.label) FROM '{L}' AS u JOIN '{R}' AS b GROUP BY u.role"),
    ("sa", "qt", "SELECT a.k, b.label FROM '{L}' AS a JOIN '{R}' AS b WHERE a.v < 40"),
    ("sa", "ex", "SELECT a.k, b.dept FROM '{L}' AS a LEFT JOIN '{R}' AS b WHERE a.v < 30"),
    ("sa", "qt", "SELECT COUNT(*), SUM(a.v) FROM '{L}' AS a RIGHT JOIN '{R}' AS b"),
    ("ex", "qt", "SELECT b.q, b.label, a.role FROM '{L}' AS a RIGHT JOIN '{R}' AS b"),
    ("ex", "qt", "SELECT COUNT(*), MAX(b.label) FROM '{L}' AS a FULL JOIN '{R}' AS b"),
    ("sa", "qt", "SELECT b.label, COUNT(*) FROM '{L}' AS a JOIN '{R}' AS b JOIN '{C}' AS c ON b.q = c.q "
                 "GROUP BY b.label"),
]


@pytest.mark.parametrize("nranks", [1, 2, 3])
@pytest.mark.parametrize("case", range(len(CROSS)))
def test_cross_join_across_partials(files, case, nranks):
    """a JOIN without ON across partials (side 1 on every rank) vs the oracle"""
    data, paths = files
    lk, rk, tmpl = CROSS[case]
    sql = tmpl.replace("{L}", paths[lk]).replace("{R}", paths[rk]).replace("{C}", paths["qt"])
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    with cqtest.Parsed(sql) as ast:
        rest = (data["qt"],) if "{C}" in tmpl else ()
        tp = _run(ast, data[lk], data[rk], nranks, rest=rest)
        assert tp, (cq_amd.last_error(), cq_amd.last_ineligible())
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"{sql} @ {nranks} ranks")


def _project(rec: bytes, keep, last_keep, delim=b",", quote=b'"'):
    """the record with only the fields in `keep` and the delimiters up to the last
    kept one (route.hip project_record); field ends as parse_line finds them
    (csv_reader.c:278-338): blanks, then a quoted run to its closing quote (doubled
    quotes inside), then up to the delimiter; raw bytes copied as they are"""
    d, qt = delim[0], quote[0]
    out, i, col = bytearray(), 0, 0
    n = len(rec)
    at = lambda k: rec[k] if k < n else 10
    while True:
        s = i
        while at(i) in (32, 9, 11, 12):     # isspace minus the terminators
            i += 1
        if at(i) not in (10, 13):
            if at(i) == qt:
                i += 1
                while at(i) not in (10, 13):
                    if at(i) == qt:
                        if at(i + 1) == qt:
                            i += 2
                            continue
                        i += 1
                        break
                    i += 1
            while at(i) != d and at(i) not in (10, 13):
                i += 1
        if col in keep:
            out += rec[s:i]
        if at(i) != d or col >= last_keep:
            break
        out.append(d)
        i += 1
        col += 1
    return bytes(out) if out else delim


def _routed_records(ast, table, side, nranks, base):
    nb, nr = cq_amd.route_plan(ast, [table[0], table[1]], side, nranks)
    sb = torch.empty(max(sum(nb), 1), dtype=torch.uint8, device="cuda")
    sg = torch.empty(max(sum(nr), 1), dtype=torch.int64, device="cuda")
    cq_amd.route_fill(table[side], base, sb.data_ptr(), sg.data_ptr())
    torch.cuda.synchronize()
    got = bytes(sb.cpu().numpy()[:sum(nb)]).split(b"\n")[:-1]
    return nb, nr, got, sg.cpu().numpy()[:sum(nr)] - base


def test_route_counts(files, monkeypatch):
    """every record is routed exactly once; bytes = record bytes + one newline each
    (whole records: projection off)"""
    monkeypatch.setenv("CQGPU_NO_ROUTE_PROJECT", "1")
    data, _ = files
    body = data["do"].split(b"\n", 1)[1]
    recs = [ln for ln in body.split(b"\n") if ln]
    sql = "SELECT COUNT(*) FROM 'u' AS u JOIN 'o' AS o ON u.id = o.customer_id"
    with cqtest.Parsed(sql) as ast:
        lt = cq_amd.Table.from_bytes(data["du"])
        rt = cq_amd.Table.from_bytes(data["do"])
        nb, nr, got, gids = _routed_records(ast, (lt, rt), 1, 4, 100)
        assert sum(nr) == len(recs)
        assert sum(nb) == sum(len(r) + 1 for r in recs)
        assert sorted(gids.tolist()) == list(range(len(recs)))
        assert [recs[i] for i in gids] == got
        lt.close()
        rt.close()


@pytest.mark.parametrize("nranks", [1, 3, 8, 64, 70])
def test_route_runs_equal_sort(files, nranks, monkeypatch):
    """the destination-run routing (route.hip route_runs / route_scatter, nranks <= 64)
    writes the same send buffer, ids and per-rank counts as the sorted-order copy
    (CQGPU_ROUTE_SORT=1; above 64 ranks both take it), projected and whole records"""
    data, _ = files
    for sql in ("SELECT u.role, COUNT(*) FROM 'u' AS u JOIN 'o' AS o ON u.id = o.customer_id GROUP BY u.role",
                "SELECT * FROM 'u' AS u JOIN 'o' AS o ON u.id = o.customer_id"):
        with cqtest.Parsed(sql) as ast:
            tabs = (cq_amd.Table.from_bytes(data["du"]), cq_amd.Table.from_bytes(data["do"]))
            try:
                for side in (0, 1):
                    got = []
                    for sort in (False, True):
                        if sort:
                            monkeypatch.setenv("CQGPU_ROUTE_SORT", "1")
                        else:
                            monkeypatch.delenv("CQGPU_ROUTE_SORT", raising=False)
                        nb, nr = cq_amd.route_plan(ast, list(tabs), side, nranks)
                        sb = torch.empty(max(sum(nb), 1), dtype=torch.uint8, device="cuda")
                        sg = torch.empty(max(sum(nr), 1), dtype=torch.int64, device="cuda")
                        cq_amd.route_fill(tabs[side], 7, sb.data_ptr(), sg.data_ptr())
                        torch.cuda.synchronize()
                        got.append((nb, nr, bytes(sb.cpu().numpy()[:sum(nb)]), sg.cpu().numpy()[:sum(nr)].tolist()))
                    assert got[0] == got[1], (sql, side)
                    assert sorted(got[0][3]) == list(range(7, 7 + sum(got[0][1])))
            finally:
                for t in tabs:
                    t.close()


def test_route_long_records(monkeypatch):
    """records whose 64-record wave spans more than the LDS stage (route.hip RP_CAP:
    the projection and the scatter then read global memory lane by lane) and one record
    of 2^25 bytes and more (the runs' byte sums take the 64-bit scan): the same bytes
    through the destination runs and the sorted-order copy, projected and whole, and
    the projection byte for byte as the field split finds it"""
    rng = np.random.default_rng(11)
    lines = [b"id,pad,v"]
    for i in range(700):
        pad = b"x" * (int(rng.integers(40, 220)) if i != 333 else (1 << 25) + 77)
        lines.append(b"%d,%s,%d" % (int(rng.integers(0, 300)), pad, i * 3))
    data = b"\n".join(lines) + b"\n"
    small = b"id,w\n" + b"".join(b"%d,%d\n" % (i, i) for i in range(300))
    recs = lines[1:]
    for sql, keep in (("SELECT a.v, COUNT(*) FROM 'a' AS a JOIN 'b' AS b ON a.id = b.id GROUP BY a.v", {0, 2}),
                      ("SELECT * FROM 'a' AS a JOIN 'b' AS b ON a.id = b.id", None)):
        with cqtest.Parsed(sql) as ast:
            tabs = (cq_amd.Table.from_bytes(data), cq_amd.Table.from_bytes(small))
            try:
                for nranks in (1, 5):
                    got = []
                    for sort in (False, True):
                        if sort:
                            monkeypatch.setenv("CQGPU_ROUTE_SORT", "1")
                        else:
                            monkeypatch.delenv("CQGPU_ROUTE_SORT", raising=False)
                        nb, nr, out, gids = _routed_records(ast, tabs, 0, nranks, 0)
                        got.append((nb, nr, out, gids.tolist()))
                    assert got[0] == got[1], (sql, nranks)
                    nb, nr, out, gids = got[0]
                    want = [recs[i] if keep is None else _project(recs[i], keep, max(keep)) for i in gids]
                    assert out == want, (sql, nranks)
            finally:
                for t in tabs:
                    t.close()


PROJ_LEFT = (b"id,name,age,role,note\n"
             b"1,ann,30,admin,x\n"
             b' 2 , "b,o""b" ,41, "ops, east" ,"q\n'      # an unclosed quote runs to the line end
             b",,,,\n"
             b"3,c\n"
             b"  \n"
             b'4,"d",,  dev  ,"n,1"\n'
             b"5\r\n"
             b',"e""",52,"r""1",z,extra,more\n'
             b"6,f,60,,\n"
             # \v / \f before a quoted field holding the delimiter
             b'7,\x0b"g,h",61,\x0c"ops,w",\x0b\x0c"n,2"\n')
PROJ_RIGHT = b"id,price,quantity,customer_id\n1,2.5,3,1\n2,4.0,1, 2 \n3,,2,\n4,9.5,1,5\n5,1.0,7,6\n"


@pytest.mark.parametrize("sql,keep", [
    ("SELECT u.role, COUNT(*) FROM 'u' AS u JOIN 'o' AS o ON u.id = o.customer_id GROUP BY u.role",
     ({0, 3}, {3})),
    ("SELECT COUNT(*) FROM 'u' AS u LEFT JOIN 'o' AS o ON u.id = o.customer_id", ({0}, {3})),
    ("SELECT u.name, SUM(o.price) FROM 'u' AS u JOIN 'o' AS o ON u.id = o.customer_id "
     "WHERE u.age > 1 GROUP BY u.name", ({0, 1, 2}, {1, 3})),
    ("SELECT o.quantity, MAX(u.note) FROM 'u' AS u RIGHT JOIN 'o' AS o ON u.id = o.customer_id "
     "GROUP BY o.quantity ORDER BY o.quantity", ({0, 4}, {2, 3})),
])
def test_route_projection_bytes(sql, keep):
    """the routed bytes hold each record's needed fields only (route.hip
    project_record), byte for byte as the field splitter finds them: quoted
    delimiters, doubled quotes, blanks, short and long rows, CR endings, all-empty
    records (a lone delimiter: still a record)"""
    with cqtest.Parsed(sql) as ast:
        tabs = (cq_amd.Table.from_bytes(PROJ_LEFT), cq_amd.Table.from_bytes(PROJ_RIGHT))
        try:
            for side, data in enumerate((PROJ_LEFT, PROJ_RIGHT)):
                recs = [ln for ln in re.split(rb"\r?\n", data.split(b"\n", 1)[1]) if ln]
                nb, nr, got, gids = _routed_records(ast, tabs, side, 3, 0)
                assert sorted(gids.tolist()) == list(range(len(recs))), side
                want = [_project(recs[i], keep[side], max(keep[side])) for i in gids]
                assert got == want, (side, got, want)
                assert sum(nb) == sum(len(r) + 1 for r in want)
        finally:
            for t in tabs:
                t.close()


@pytest.mark.parametrize("case", [1, 4, 8, 9, 10, 11, 13, 16, 19, 20])
def test_route_projection_results(files, case, monkeypatch):
    """the same partial-merge result with whole records and with projected ones"""
    data, paths = files
    lk, rk, tmpl = QUERIES[case]
    sql = tmpl.replace("{L}", paths[lk]).replace("{R}", paths[rk])
    with cqtest.Parsed(sql) as ast:
        res = []
        for off in (False, True):
            if off:
                monkeypatch.setenv("CQGPU_NO_ROUTE_PROJECT", "1")
            tp = _run(ast, data[lk], data[rk], 3)
            assert tp, cq_amd.last_error()
            res.append(abi.table_to_py(tp))
            cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(res[1], res[0], tol, f"{sql}: projected vs whole records")   # (float sums: summation order)


def _dist_worker(rank, world, port, lpath, rpath, sql, q, rest=()):
    """one rank of cq_amd.dist.join_partitioned; gloo group, shared GPU 0"""
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cqtest as ct
        import cq_amd as ca
        from cq_amd import abi as ab
        from cq_amd.dist import join_partitioned
        shards = []
        for path in (lpath, rpath):
            data = open(path, "rb").read()
            header, body = data.split(b"\n", 1)
            header += b"\n"
            cuts = [0] + [body.index(b"\n", len(body) * (k + 1) // world) + 1 for k in range(world - 1)] + [len(body)]
            pc = body[cuts[rank]:cuts[rank + 1]]
            t = ca.Table.from_bytes(header + pc) if rank == 0 else ca.Table.from_bytes(pc, header=header)
            shards.append((t, header))
        with ct.Parsed(sql) as ast:
            whole = [ca.Table.from_bytes(open(p, "rb").read()) for p in rest]
            tp = join_partitioned(ast, shards[0][0], shards[1][0], shards[0][1], shards[1][1], "cuda", "cpu", whole)
            for t in whole:
                t.close()
            res = None
            if rank == 0:
                res = ab.table_to_py(tp) if tp else ca.last_error()
                if tp:
                    ca.result_free(tp)
        q.put((rank, res))
        for t, _ in shards:
            t.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_join_partitioned_processes(files, world):
    """the real driver (route, all_to_all, routed tables, partial, gather, merge)
    in two processes over gloo, vs the oracle; one process takes the no-repartition
    path (its shards are the routed tables)"""
    import socket
    import torch.multiprocessing as mp
    data, paths = files
    sql = (f"SELECT u.role, COUNT(*), SUM(o.price), MAX(o.quantity) FROM '{paths['du']}' AS u "
           f"JOIN '{paths['do']}' AS o ON u.id = o.customer_id GROUP BY u.role")
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, paths["du"], paths["do"], sql, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = res[0]
    assert isinstance(got, dict), got
    with cqtest.Parsed(sql) as ast:
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql + f" @ {world} processes")


@pytest.mark.parametrize("case", [0, 10])
@pytest.mark.parametrize("world", [1, 2])
def test_join_chain_processes(files, world, case):
    """a three-table chain through cq_amd.dist.join_partitioned in separate processes
    (gloo): routed first level, whole third table, merged on rank 0 vs the oracle;
    case 10 a later FULL JOIN (dist.outer_sets: the ranks' matched flags OR-ed by an
    all-reduce)"""
    import socket
    import torch.multiprocessing as mp
    data, paths = files
    assert CHAINS[case][0] == ["rl"]
    sql = _chain_sql(paths, ["rl"], CHAINS[case][1])
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, paths["du"], paths["do"], sql, q, [paths["rl"]]))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = res[0]
    assert isinstance(got, dict), got
    with cqtest.Parsed(sql) as ast:
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql + f" @ {world} processes")


# ---------------------------------------------------------------- the typed exchange
TYPED = [
    "SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM '{u}' AS u JOIN '{o}' AS o ON u.id = o.customer_id "
    "GROUP BY u.role",
    "SELECT COUNT(*) FROM '{u}' AS u JOIN '{o}' AS o ON u.id = o.customer_id",
    "SELECT COUNT(*), SUM(o.price) FROM '{u}' AS u JOIN '{o}' AS o ON u.id = o.customer_id",
    "SELECT u.role, COUNT(*) FROM '{u}' AS u JOIN '{o}' AS o ON u.id = o.customer_id GROUP BY u.role "
    "ORDER BY COUNT(*) DESC LIMIT 5",
    "SELECT u.role, 7, AVG(o.price) FROM '{u}' AS u JOIN '{o}' AS o ON u.id = o.customer_id GROUP BY u.role",
]


def _typed(ast, ldata, rdata, nranks, stats=None):
    from cq_amd.dist import typed_join_local
    _, ls = _shards(ldata, nranks, 1)
    _, rs = _shards(rdata, nranks, 2)
    try:
        blobs = typed_join_local(ast, ls, rs, stats)
        if blobs is None:
            return None, cq_amd.last_ineligible()
        return cq_amd.merge_partials(ast, blobs), LAST_KINDS
    finally:
        for t in ls + rs:
            t.close()


@pytest.mark.parametrize("nranks", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("qi", range(len(TYPED)))
def test_typed_exchange_equals_oracle(files, nranks, qi):
    """SURVEY 8e's typed (key, row id, payload) exchange: every simulated rank's
    16-byte build / 8-byte probe entries routed by key mod N, each destination's STAR
    join over its entries, the partials merged -- the oracle's nested loop: COUNT exact,
    SUM / AVG 1e-6 relative, groups in the order of their first matched user"""
    data, paths = files
    sql = TYPED[qi].format(u=paths["users"], o=paths["orders"])
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    st = {}
    with cqtest.Parsed(sql) as ast:
        tp, why = _typed(ast, data["users"], data["orders"], nranks, st)
        assert tp, (cq_amd.last_error(), why)
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"typed exchange {nranks} ranks: {sql}")
    assert sum(st["recv_entries_u"]) == 4000 and st["attempts"] == 1, st


@pytest.mark.parametrize("nranks", [1, 3, 8])
@pytest.mark.parametrize("qi", range(len(TYPED)))
def test_typed_exchange_partitioned_probe(files, nranks, qi, monkeypatch):
    """the receiver's two-pass probe (jx_ent_part_kernel: entries into key partitions of
    16 slots, then jx_part_probe_kernel per XCD) forced at test size -- the oracle's
    answer, as the one-pass probe gives it"""
    monkeypatch.setenv("CQGPU_PART_PROBE_MIN", "0")
    monkeypatch.setenv("CQGPU_PART_PROBE_SHIFT", "4")
    data, paths = files
    sql = TYPED[qi].format(u=paths["users"], o=paths["orders"])
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    with cqtest.Parsed(sql) as ast:
        tp, why = _typed(ast, data["users"], data["orders"], nranks, {})
        assert tp, (cq_amd.last_error(), why)
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, f"typed exchange, partitioned probe, {nranks} ranks: {sql}")


@pytest.mark.parametrize("mode", ["one_pass", "two_pass", "overflow"])
@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_typed_exchange_probe_pass_forms(files, nranks, mode, monkeypatch):
    """the probe side's entries: one pass by default (jx_extract_kernel ROUTE 3: chunks
    from per-destination cursors, holes at the waves' chunk tails, which the receivers
    skip); the count + emit passes under CQGPU_TYPED_TWO_PASS=1 and when a region
    overflows its capacity (CQGPU_TEST_ONE_PASS_CAP) -- the oracle's answer every way,
    the two-pass entries exactly the probe records with a key in range"""
    data, paths = files
    sql = TYPED[0].format(u=paths["users"], o=paths["orders"])
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup
    if mode == "two_pass":
        monkeypatch.setenv("CQGPU_TYPED_TWO_PASS", "1")
    elif mode == "overflow":
        monkeypatch.setenv("CQGPU_TEST_ONE_PASS_CAP", "5")
    with cqtest.Parsed(sql) as ast:
        st = {}
        tp, why = _typed(ast, data["users"], data["orders"], nranks, st)
        assert tp, (cq_amd.last_error(), why)
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
        monkeypatch.setenv("CQGPU_TYPED_TWO_PASS", "1")
        exact = {}
        tp2, _ = _typed(ast, data["users"], data["orders"], nranks, exact)
        cq_amd.result_free(tp2)
    compare(got, want, tol, f"typed exchange ({mode}) {nranks} ranks: {sql}")
    if mode == "one_pass":          # chunk tails: holes beside the same entries
        assert sum(st["sent_entries_o"]) > sum(exact["sent_entries_o"]), (st, exact)
    else:
        assert st["sent_entries_o"] == exact["sent_entries_o"], (st, exact)


@pytest.mark.parametrize("order", ["rising", "shuffled"])
@pytest.mark.parametrize("flags", [False, True])
def test_typed_exchange_first_pair_forms(tmp_path, monkeypatch, order, flags):
    """a group's first pair: with the build keys rising along the entries (global-id
    order) the probe keeps each group's smallest matched slot; shuffled keys -- or
    CQGPU_TYPED_FLAGS=1 -- take the d16 match flags and the first-pair scan.  Both give
    the oracle's groups in first-appearance order, at 1 and 3 ranks"""
    if flags:
        monkeypatch.setenv("CQGPU_TYPED_FLAGS", "1")
    rng = np.random.default_rng(17)
    ids = np.arange(3000) + 500
    if order == "shuffled":
        rng.shuffle(ids)
    users = "id,name,role\n" + "".join("%d,n%d,r%02d\n" % (k, i, rng.integers(0, 40)) for i, k in enumerate(ids))
    orders = "id,price,customer_id\n" + "".join(
        "%d,%d.%d,%d\n" % (i, rng.integers(0, 999), rng.integers(0, 9), 500 + rng.integers(0, 3200))
        for i in range(12000))
    up, op = tmp_path / "u.csv", tmp_path / "o.csv"
    up.write_text(users)
    op.write_text(orders)
    sql = (f"SELECT u.role, COUNT(*), SUM(o.price) FROM '{up}' AS u JOIN '{op}' AS o "
           f"ON u.id = o.customer_id GROUP BY u.role")
    want, _ = cqtest.oracle_query(sql)
    for nranks in (1, 3):
        with cqtest.Parsed(sql) as ast:
            tp, why = _typed(ast, users.encode(), orders.encode(), nranks, {})
            assert tp, (cq_amd.last_error(), why)
            got = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            tol = tolerant_columns(ast)
        compare(got, want, tol, f"typed exchange, {order} keys, flags {flags}, {nranks} ranks")


def test_typed_exchange_partition_overflow(tmp_path, monkeypatch):
    """skewed probe keys (90 % of 120 K orders on one user) overflow a partition
    segment: the receive reruns unpartitioned and still gives the oracle's answer"""
    monkeypatch.setenv("CQGPU_PART_PROBE_MIN", "0")
    monkeypatch.setenv("CQGPU_PART_PROBE_SHIFT", "4")
    rng = np.random.default_rng(9)
    users = "id,name,role\n" + "".join("%d,n%d,r%d\n" % (i, i, i % 7) for i in range(1000))
    orders = "id,price,customer_id\n" + "".join(
        "%d,%d.%d,%d\n" % (i, rng.integers(0, 99), rng.integers(0, 9), 5 if i % 10 else rng.integers(0, 1000))
        for i in range(120_000))
    up, op = tmp_path / "u.csv", tmp_path / "o.csv"
    up.write_text(users)
    op.write_text(orders)
    sql = (f"SELECT u.role, COUNT(*), SUM(o.price) FROM '{up}' AS u JOIN '{op}' AS o "
           f"ON u.id = o.customer_id GROUP BY u.role")
    want, _ = cqtest.oracle_query(sql)
    with cqtest.Parsed(sql) as ast:
        tp, why = _typed(ast, users.encode(), orders.encode(), 1, {})
        assert tp, (cq_amd.last_error(), why)
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    compare(got, want, tol, "typed exchange, partition overflow")


def test_typed_exchange_large_keys_retry(tmp_path):
    """keys near 10^14: key / N does not fit 32 bits, the first attempt flags it and the
    second runs with qbase = the keys' minimum / N; and a probe side with keys outside
    the build window, NULL keys and NULL / negative prices"""
    rng = np.random.default_rng(41)
    n = 3000
    users = "id,name,role\n" + "".join("%d,n%d,r%02d\n" % (10**14 + i, i, rng.integers(0, 30)) for i in range(n))
    rows = []
    for i in range(9000):
        k = int(rng.integers(0, n + 200))                 # (k >= n: a key no user has)
        cid = "" if i % 97 == 0 else str(10**14 + k if k < n else 10**14 + 5 * k)
        pr = "" if i % 89 == 0 else ("-%d.%02d" % (rng.integers(0, 50), rng.integers(0, 100)) if i % 31 == 0
                                     else "%d.%d" % (rng.integers(0, 999), rng.integers(0, 10)))
        rows.append("%d,%s,%s" % (i, pr, cid))
    orders = "id,price,customer_id\n" + "\n".join(rows) + "\n"
    up, op = tmp_path / "u.csv", tmp_path / "o.csv"
    up.write_text(users)
    op.write_text(orders)
    sql = (f"SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM '{up}' AS u JOIN '{op}' AS o "
           f"ON u.id = o.customer_id GROUP BY u.role")
    want, _ = cqtest.oracle_query(sql)
    for nranks in (1, 3, 8):
        st = {}
        with cqtest.Parsed(sql) as ast:
            tp, why = _typed(ast, users.encode(), orders.encode(), nranks, st)
            assert tp, (cq_amd.last_error(), why)
            got = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            tol = tolerant_columns(ast)
        compare(got, want, tol, f"typed, large keys, {nranks} ranks")
        assert st["attempts"] <= 2 and st["qbase"] > 0, st


@pytest.mark.parametrize("case", ["dup", "null", "quote", "sparse", "tags", "canon"])
def test_typed_exchange_declines_or_merges(tmp_path, case):
    """data the entries cannot carry exactly leaves the typed exchange (None: the
    caller takes the CSV exchange) -- a repeated or NULL build key, a quote, a sparse key
    range; tags of one canonical key ("1.0", "1.00", "1") merge into one group"""
    users = ["id,name,role"] + ["%d,n%d,%s" % (100 + i, i, "r%d" % (i % 4)) for i in range(400)]
    orders = ["id,price,customer_id"] + ["%d,%d.5,%d" % (i, i % 50, 100 + (i * 7) % 400) for i in range(1500)]
    if case == "dup":
        users.append("150,dup,r1")
    elif case == "null":
        users.append(",nul,r2")
    elif case == "quote":
        users[5] = '104,"q,x",r0'
    elif case == "sparse":
        users.append("100000000,far,r3")
    elif case == "tags":
        users = ["id,name,role"] + ["%d,n%d,%s" % (100 + i, i, ["1.0", "1.00", "1", "2.5"][i % 4]) for i in range(400)]
    elif case == "canon":
        users = ["id,name,role"] + ["%d,n%d,%s" % (100 + i, i, ["x", "y", "", "z"][i % 4]) for i in range(400)]
    up, op = tmp_path / "u.csv", tmp_path / "o.csv"
    up.write_text("\n".join(users) + "\n")
    op.write_text("\n".join(orders) + "\n")
    sql = (f"SELECT u.role, COUNT(*), SUM(o.price) FROM '{up}' AS u JOIN '{op}' AS o "
           f"ON u.id = o.customer_id GROUP BY u.role")
    with cqtest.Parsed(sql) as ast:
        tp, why = _typed(ast, up.read_bytes(), op.read_bytes(), 3)
        if case in ("dup", "null", "quote", "sparse"):
            assert tp is None, case
            return
        assert tp, (cq_amd.last_error(), why)
        got = abi.table_to_py(tp)
        cq_amd.result_free(tp)
        tol = tolerant_columns(ast)
    want, _ = cqtest.oracle_query(sql)
    compare(got, want, tol, f"typed {case}")
