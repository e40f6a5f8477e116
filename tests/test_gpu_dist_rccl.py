"""The N > 1 step inside the library (cqgpu_dist_query over its own RCCL
communicator) and its gather-merge kernels.

* Gather-merge kernels over simulated ranks (cqgpu_gm_local: every shard's pack,
  then rank 0's merge kernels, in one process): the config-3 / config-4 plan and
  the other plans of its shape at 1..16 ranks against the ORACLE on the whole
  file -- counts, group set and first-appearance order, representative cells
  exact, SUM / AVG 1e-6 relative; CR / CRLF cuts; long keys (inline up to 48
  bytes, declined beyond); too many groups (declined).
* cqgpu_dist_query itself at world size 1 over RCCL (torch.distributed.run, one
  rank: a one-GPU box cannot hold two RCCL ranks): the gather-merge, dense and
  blob paths each against the oracle, the path each query took asserted.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import cqtest
import cq_amd
from cq_amd import abi, datagen
from test_gpu_parity import compare, tolerant_columns
from test_gpu_partials import _mixed_terminators

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GM = [
    "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role",
    "SELECT COUNT(*) FROM '{p}' WHERE age > 30",
    "SELECT COUNT(*), SUM(height), AVG(age) FROM '{p}'",
    "SELECT name, COUNT(*), AVG(height) FROM '{p}' WHERE gender = 'f' GROUP BY name",
    "SELECT age, COUNT(*), SUM(height) FROM '{p}' GROUP BY age ORDER BY COUNT(*) DESC LIMIT 7",
    "SELECT role, 42, COUNT(*) FROM '{p}' WHERE height > 1.99 GROUP BY role",
    "SELECT COUNT(*) FROM '{p}' WHERE age > 200",
    "SELECT role, COUNT(*) FROM '{p}' WHERE age > 200 GROUP BY role",
    "SELECT height, COUNT(*) FROM '{p}' GROUP BY height HAVING COUNT(*) > 100",
]


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("gm"))
    out = {}
    out["plain"] = os.path.join(d, "plain.csv")
    with open(out["plain"], "wb") as fh:
        fh.write(datagen.shape_a_bytes(150_000, seed=21, with_role=True))
    out["mixed"] = os.path.join(d, "mixed.csv")
    with open(out["mixed"], "wb") as fh:
        fh.write(_mixed_terminators(datagen.shape_a_bytes(40_000, seed=22, with_role=True), 5))
    rng = np.random.default_rng(3)
    keys = ["key_of_twenty_bytes_%02d" % i for i in range(40)] + ["k%d" % i for i in range(30)]
    out["longkey"] = os.path.join(d, "longkey.csv")
    with open(out["longkey"], "w") as fh:
        fh.write("k,v,w\n" + "\n".join("%s,%d,%d.%d" % (keys[rng.integers(0, len(keys))], rng.integers(0, 99),
                                                       rng.integers(0, 9), rng.integers(0, 9))
                                       for _ in range(50_000)) + "\n")
    out["verylong"] = os.path.join(d, "verylong.csv")
    with open(out["verylong"], "w") as fh:
        fh.write("k,v\n" + "\n".join("%s,%d" % ("x" * 60 + str(i % 5), i % 7) for i in range(20_000)) + "\n")
    out["users"] = os.path.join(d, "users.csv")
    with open(out["users"], "wb") as fh:
        fh.write(datagen.users_bytes(4000, seed=7))
    out["orders"] = os.path.join(d, "orders.csv")
    with open(out["orders"], "wb") as fh:
        fh.write(datagen.orders_bytes(9000, 4500, seed=8))
    out["roles"] = os.path.join(d, "roles.csv")
    with open(out["roles"], "w") as fh:
        fh.write("role,dept\n" + "".join("role_%03d,dept%d\n" % (i, i % 7) for i in range(0, 1000, 3)))
    # join keys mixing value classes (numbers, strings, dates, NULL) on both sides, and a
    # small table for JOINs without ON
    def mk_key(r):
        k = int(r.integers(0, 10))
        if k < 5:
            return str(int(r.integers(0, 40))) if k else f"{int(r.integers(0, 40))}.0"
        if k < 8:
            return "s%02d" % int(r.integers(0, 25))
        return "" if k == 8 else "2021-03-%02d" % int(r.integers(1, 9))
    out["mk"] = os.path.join(d, "mk.csv")
    with open(out["mk"], "w") as fh:
        fh.write("k,v,g\n" + "".join(f"{mk_key(rng)},{i},{i % 3}\n" for i in range(300)))
    out["mk2"] = os.path.join(d, "mk2.csv")
    with open(out["mk2"], "w") as fh:
        fh.write("k,w\n" + "".join(f"{mk_key(rng)},{i}\n" for i in range(150)))
    out["qt"] = os.path.join(d, "qt.csv")
    with open(out["qt"], "w") as fh:
        fh.write("q,label\n0,lab0\n2,lab2\n1,lab1\n2,lab2b\n9,lab9\n")
    out["many"] = os.path.join(d, "many.csv")
    with open(out["many"], "w") as fh:
        fh.write("k,v\n" + "\n".join("%d,%d" % (i % 9000, i % 7) for i in range(40_000)) + "\n")
    return out


def _gm(path, sql, n):
    q = sql.format(p=path)
    tabs = [cq_amd.Table.open_range(path, r, n) for r in range(n)]
    try:
        with cqtest.Parsed(q) as ast:
            got = cq_amd.gm_local(ast, tabs)
            tol = tolerant_columns(ast)
    finally:
        for t in tabs:
            t.close()
    return q, got, tol


@pytest.mark.parametrize("sql", GM)
@pytest.mark.parametrize("n", [1, 3, 8])
def test_gm_local_equals_oracle(files, sql, n):
    q, got, tol = _gm(files["plain"], sql, n)
    assert got is not None, (q, cq_amd.last_error(), cq_amd.last_ineligible())
    want, unsup = cqtest.oracle_query(q)
    assert not unsup
    compare(got, want, tol, f"gather-merge {n} ranks: {q}")


@pytest.mark.parametrize("n", [2, 5, 16])
def test_gm_local_mixed_terminator_cuts(files, n):
    for sql in GM[:4]:
        q, got, tol = _gm(files["mixed"], sql, n)
        assert got is not None, (q, cq_amd.last_error())
        want, _ = cqtest.oracle_query(q)
        compare(got, want, tol, f"gather-merge {n} ranks: {q}")


@pytest.mark.parametrize("n", [1, 4])
def test_gm_local_long_keys(files, n):
    """keys over 16 bytes (GK_LONG: compared by their bytes, carried inline up to 48)"""
    for sql in ("SELECT k, COUNT(*), SUM(w), AVG(v) FROM '{p}' GROUP BY k",
                "SELECT k, COUNT(*) FROM '{p}' WHERE v > 50 GROUP BY k"):
        q, got, tol = _gm(files["longkey"], sql, n)
        assert got is not None, (q, cq_amd.last_error())
        want, _ = cqtest.oracle_query(q)
        compare(got, want, tol, f"gather-merge {n} ranks: {q}")


def test_gm_local_declines(files):
    """texts over 48 bytes and more than 4096 groups on a rank leave the gather-merge"""
    _, got, _ = _gm(files["verylong"], "SELECT k, COUNT(*) FROM '{p}' GROUP BY k", 2)
    assert got is None and "declined" in cq_amd.last_ineligible()
    _, got, _ = _gm(files["many"], "SELECT k, COUNT(*) FROM '{p}' GROUP BY k", 2)
    assert got is None and "declined" in cq_amd.last_ineligible()
    _, got, _ = _gm(files["plain"], "SELECT role, MIN(age) FROM '{p}' GROUP BY role", 2)
    assert got is None and "outside" in cq_amd.last_ineligible()


# ---------------------------------------------------------------- cqgpu_dist_query over RCCL, one rank
DIST = [   # (sql, the merge path it must take, the file)
    (GM[0], 1, "plain"),
    (GM[2], 1, "plain"),
    ("SELECT role, MIN(height), MAX(name), COUNT(*) FROM '{p}' WHERE age > 30 GROUP BY role", 2, "plain"),
    ("SELECT gender, role, COUNT(*), STDDEV(height) FROM '{p}' GROUP BY gender, role", 2, "plain"),
    ("SELECT role, MEDIAN(age) FROM '{p}' GROUP BY role", 3, "plain"),
    ("SELECT name, age FROM '{p}' WHERE age > 78 AND height < 1.05", 3, "plain"),
    # gather-merge plans the DATA declines: more than GM_MAXG groups on a
    # rank, texts over GM_TEXT bytes -- every rank falls to the dense merge together
    ("SELECT k, COUNT(*), SUM(v) FROM '{p}' GROUP BY k", 2, "many"),
    ("SELECT k, COUNT(*) FROM '{p}' GROUP BY k", 2, "verylong"),
]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cell(c):
    return (c[0], c[1].encode("latin-1")) if c[0] == "S" else tuple(c)


def _dist_run(files, tmp_path, items, env=None):
    out = str(tmp_path / "dist.json")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "dist_rccl_worker.py"),
           out, json.dumps([[s, files[f]] for s, f in items])]
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=e)
    assert p.returncode == 0, p.stderr[:6000] + "\n...\n" + p.stderr[-2000:]
    return json.load(open(out))


def test_dist_query_one_rank_rccl(files, tmp_path):
    res = _dist_run(files, tmp_path, [(s, f) for s, _, f in DIST])
    for (sql, path, f), r in zip(DIST, res):
        q = sql.format(p=files[f])
        assert r["status"] == 0, (q, r["error"])
        assert r["path"] == path, (q, r["path"])
        want, _ = cqtest.oracle_query(q)
        got = {"columns": [c.encode("latin-1") for c in r["result"]["columns"]],
               "rows": [[_cell(c) for c in row] for row in r["result"]["rows"]]}
        with cqtest.Parsed(q) as ast:
            tol = tolerant_columns(ast)
        compare(got, want, tol, f"dist_query path {path}: {q}")


@pytest.mark.parametrize("knob", ["CQGPU_TEST_GM_FAIL_PART", "CQGPU_TEST_GM_FAIL_FINISH"])
def test_dist_query_gather_merge_failure_reported(files, tmp_path, knob):
    """a rank-local failure in the gather-merge -- this rank's part, or rank 0's result
    build after the merge kernels -- is status -1 with the message on every rank after
    the same collectives (rank 0 now builds its result before it broadcasts
    the final status), never a hang"""
    res = _dist_run(files, tmp_path, [(GM[0], "plain")], env={knob: "1"})
    assert res[0]["status"] == -1, res[0]
    assert "injected" in res[0]["error"], res[0]["error"]


JOINS = [   # the repartitioned JOIN step inside the library (cqgpu_dist_join)
    ("SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM '{p}' AS u JOIN '{q}' AS o "
     "ON u.id = o.customer_id GROUP BY u.role", ["users", "orders"]),
    ("SELECT COUNT(*), SUM(o.price) FROM '{p}' AS u LEFT JOIN '{q}' AS o ON u.id = o.customer_id", ["users", "orders"]),
    ("SELECT u.name, o.price FROM '{p}' AS u JOIN '{q}' AS o ON u.id = o.customer_id WHERE o.price > 995",
     ["users", "orders"]),
    ("SELECT r.dept, COUNT(*), SUM(o.price) FROM '{p}' AS u JOIN '{q}' AS o ON u.id = o.customer_id "
     "JOIN '{r}' AS r ON u.role = r.role GROUP BY r.dept", ["users", "orders", "roles"]),
    # a later RIGHT / FULL level: the matched flags all-reduced (MAX over bytes) inside
    # the library, rank 0's partial carrying the records no rank matched
    ("SELECT r.dept, COUNT(*), SUM(o.price) FROM '{p}' AS u JOIN '{q}' AS o ON u.id = o.customer_id "
     "RIGHT JOIN '{r}' AS r ON u.role = r.role GROUP BY r.dept", ["users", "orders", "roles"]),
    ("SELECT COUNT(*), MIN(r.role), MAX(u.name) FROM '{p}' AS u JOIN '{q}' AS o ON u.id = o.customer_id "
     "FULL JOIN '{r}' AS r ON u.role = r.role", ["users", "orders", "roles"]),
]


JOINS_X = [   # mixed key classes (the minority classes replicated) and JOINs without ON
    ("SELECT a.g, COUNT(*), SUM(b.w), MAX(b.k) FROM '{p}' AS a JOIN '{q}' AS b ON a.k = b.k GROUP BY a.g",
     ["mk", "mk2"]),
    ("SELECT a.v, b.w FROM '{p}' AS a JOIN '{q}' AS b ON a.k = b.k WHERE b.w < 40", ["mk", "mk2"]),
    ("SELECT u.role, COUNT(*), MAX(b.label) FROM '{p}' AS u JOIN '{q}' AS b GROUP BY u.role", ["users", "qt"]),
    ("SELECT COUNT(*), SUM(u.age) FROM '{p}' AS u RIGHT JOIN '{q}' AS b", ["users", "qt"]),
    ("SELECT b.label, COUNT(*) FROM '{p}' AS u JOIN '{q}' AS b JOIN '{r}' AS c ON b.q = c.q GROUP BY b.label",
     ["mk2", "qt", "qt"]),
]


@pytest.mark.parametrize("world", [1, 2, 3])
def test_dist_join_mixed_and_cross(files, tmp_path, world):
    """cqgpu_dist_join's agreed routing mode (cqgpu_route_plan2): keys of several value
    classes and JOINs without ON at world size 1 over RCCL and 2 / 3 over the host
    backend, against the oracle"""
    if world == 1:
        res = _dist_run_paths(files, tmp_path, JOINS_X)
        per = None
    else:
        res, per = _host_run(files, tmp_path, JOINS_X, world, paths_of=True)
    for i, ((sql, keys), r) in enumerate(zip(JOINS_X, res)):
        q = sql.format(**dict(zip("pqrs", [files[k] for k in keys])))
        assert r["status"] == 0, (q, r["error"])
        if per:
            assert all(pr[i]["status"] == 0 for pr in per), (q, per)
        want, unsup = cqtest.oracle_query(q)
        assert not unsup
        with cqtest.Parsed(q) as ast:
            tol = tolerant_columns(ast)
        compare(_as_got(r), want, tol, f"dist_join {world} ranks: {q}")


def test_dist_join_one_rank_rccl(files, tmp_path):
    """cqgpu_dist_join at world size 1 over RCCL: the routing, the grouped send /
    recv exchange (to itself), the rebuilt sides (key stride 1), the local join and
    the partial merge, each query against the oracle over the whole files"""
    res = _dist_run_paths(files, tmp_path, JOINS)
    for (sql, keys), r in zip(JOINS, res):
        q = sql.format(**dict(zip("pqrs", [files[k] for k in keys])))
        assert r["status"] == 0, (q, r["error"])
        want, unsup = cqtest.oracle_query(q)
        assert not unsup
        got = {"columns": [c.encode("latin-1") for c in r["result"]["columns"]],
               "rows": [[_cell(c) for c in row] for row in r["result"]["rows"]]}
        with cqtest.Parsed(q) as ast:
            tol = tolerant_columns(ast)
        compare(got, want, tol, f"dist_join: {q}")


def _dist_run_paths(files, tmp_path, items, env=None):
    out = str(tmp_path / "distj.json")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "dist_rccl_worker.py"),
           out, json.dumps([[s, [files[k] for k in keys]] for s, keys in items])]
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=e)
    assert p.returncode == 0, p.stderr[:6000] + "\n...\n" + p.stderr[-2000:]
    return json.load(open(out))


@pytest.mark.parametrize("kind", ["verylong", "many"])
def test_gm_decline_then_dense_same_process(files, kind):
    """cqgpu_dist_query's sequence for data the gather-merge declines, without RCCL:
    the gather-merge pack (gm_local: declined), then the dense merge and the blobs on
    the same table in the same process -- every step the oracle's answer"""
    from test_gpu_partials import _dense_merge_by_hand
    path = files[kind]
    q = f"SELECT k, COUNT(*) FROM '{path}' GROUP BY k"
    want, _ = cqtest.oracle_query(q)
    t = cq_amd.Table.open_range(path, 0, 1)
    try:
        with cqtest.Parsed(q) as ast:
            assert cq_amd.gm_local(ast, [t]) is None and "declined" in cq_amd.last_ineligible()
            tp = _dense_merge_by_hand(ast, [t])
            assert tp, cq_amd.last_error()
            got = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            compare(got, want, set(), f"dense after gm: {q}")
            tp = cq_amd.merge_partials(ast, [cq_amd.query_partial(ast, [t])])
            got = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            compare(got, want, set(), f"blobs after gm: {q}")
    finally:
        t.close()


# ---------------------------------------------------------------- the same protocol at world size 2 and 3
# The library's N > 1 code (dist_gm / dist_dense / dist_blob / dist_join: size
# agreements, per-destination offsets, gid bases, grouped send / recv, outer-set
# all-reduces, status broadcasts) through its host-staged collective backend
# (cqgpu_comm_init_host) over gloo, 2 and 3 processes sharing the box's GPU.  Only the
# transport differs from the RCCL runs: every collective call site is the same code.
def _host_run(files, tmp_path, items, world, env=None, paths_of=None):
    out = str(tmp_path / f"host{world}.json")
    if paths_of is None:
        payload = [[s, files[f]] for s, f in items]
    else:
        payload = [[s, [files[k] for k in keys]] for s, keys in items]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "dist_rccl_worker.py"),
           out, json.dumps(payload)]
    e = dict(os.environ)
    e["CQ_TEST_HOST_COMM"] = "1"
    e.update(env or {})
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=e)
    assert p.returncode == 0, p.stderr[:6000] + "\n...\n" + p.stderr[-2000:]
    per_rank = [json.load(open(f"{out}.{r}")) for r in range(world)]
    return json.load(open(out)), per_rank


def _as_got(r):
    return {"columns": [c.encode("latin-1") for c in r["result"]["columns"]],
            "rows": [[_cell(c) for c in row] for row in r["result"]["rows"]]}


@pytest.mark.parametrize("world", [2, 3])
def test_dist_query_multi_rank_host_backend(files, tmp_path, world):
    """cqgpu_dist_query at world size 2 and 3: gather-merge, dense and blob paths (and
    the gather-merge declines falling to the dense merge together) vs the oracle"""
    res, per = _host_run(files, tmp_path, [(s, f) for s, _, f in DIST], world)
    for (sql, path, f), r in zip(DIST, res):
        q = sql.format(p=files[f])
        assert r["status"] == 0, (q, r["error"])
        assert r["path"] == path, (q, r["path"])
        for pr in per:
            assert pr[DIST.index((sql, path, f))]["status"] == 0
        want, _ = cqtest.oracle_query(q)
        with cqtest.Parsed(q) as ast:
            tol = tolerant_columns(ast)
        compare(_as_got(r), want, tol, f"dist_query {world} ranks, path {path}: {q}")


@pytest.mark.parametrize("world", [2, 3])
def test_dist_join_multi_rank_host_backend(files, tmp_path, world):
    """cqgpu_dist_join at world size 2 and 3: routing, the exchange with per-destination
    offsets and gid bases, rebuilt sides with key stride N, chains with a later RIGHT /
    FULL level (the outer-set all-reduces) -- each against the oracle"""
    res, per = _host_run(files, tmp_path, JOINS, world, paths_of=True)
    for i, ((sql, keys), r) in enumerate(zip(JOINS, res)):
        q = sql.format(**dict(zip("pqrs", [files[k] for k in keys])))
        assert r["status"] == 0, (q, r["error"])
        if i == 0:                                   # config 5's shape: the typed exchange
            assert r["kernel"] == 5, (q, r)
        assert all(pr[i]["status"] == 0 for pr in per), (q, per)
        want, unsup = cqtest.oracle_query(q)
        assert not unsup
        with cqtest.Parsed(q) as ast:
            tol = tolerant_columns(ast)
        compare(_as_got(r), want, tol, f"dist_join {world} ranks: {q}")


@pytest.mark.parametrize("knob,kind", [
    ("CQGPU_TEST_GM_FAIL_PART", "query"),            # one rank's gather-merge part
    ("CQGPU_TEST_GM_FAIL_FINISH", "query"),          # (read by rank 0 only)
    ("CQGPU_TEST_DIST_FAIL_ALLOC", "join"),          # one rank's CSV-exchange buffers
    ("CQGPU_TEST_DIST_CHAIN_MISSING", "chain"),      # one rank lacks a chain level's table
    ("CQGPU_TEST_TYPED_FAIL", "typed"),              # one rank's typed-exchange send
])
def test_dist_one_rank_failure_reaches_every_rank(files, tmp_path, knob, kind):
    """a failure on ONE rank of three is status -1 on EVERY rank after the same
    collectives -- no rank left waiting in a transfer or reduce its peer never posts
    (exchange allocations and the chain loop inside the agreement)"""
    fail_rank = 0 if knob == "CQGPU_TEST_GM_FAIL_FINISH" else 1
    env = {"CQ_TEST_RANK_ENV": f"{fail_rank}:{knob}=1"}
    if kind == "join":
        env["CQGPU_NO_TYPED_JOIN"] = "1"              # (the CSV exchange's allocation)
    if kind == "query":
        res, per = _host_run(files, tmp_path, [(GM[0], "plain")], 3, env=env)
    else:
        item = JOINS[0] if kind in ("join", "typed") else JOINS[4]
        res, per = _host_run(files, tmp_path, [item], 3, env=env, paths_of=True)
    for r, pr in enumerate(per):
        assert pr[0]["status"] == -1, (r, pr)
    assert "injected" in per[fail_rank][0]["error"] or "missing" in per[fail_rank][0]["error"], per[fail_rank]


@pytest.mark.parametrize("world", [2, 3])
def test_dist_join_multi_rank_csv_exchange(files, tmp_path, world):
    """the CSV-record exchange (CQGPU_NO_TYPED_JOIN=1: every plan takes it) at world size
    2 and 3 -- the fallback the typed exchange leaves to -- against the oracle"""
    res, per = _host_run(files, tmp_path, JOINS[:2], world, env={"CQGPU_NO_TYPED_JOIN": "1"}, paths_of=True)
    for (sql, keys), r in zip(JOINS[:2], res):
        q = sql.format(**dict(zip("pqrs", [files[k] for k in keys])))
        assert r["status"] == 0, (q, r["error"])
        assert r["kernel"] != 5, (q, r)
        want, _ = cqtest.oracle_query(q)
        with cqtest.Parsed(q) as ast:
            tol = tolerant_columns(ast)
        compare(_as_got(r), want, tol, f"dist_join (CSV exchange) {world} ranks: {q}")
