#!/usr/bin/env python3
"""Join benchmark: BASELINE.json configs[4] shape (users x orders hash join), weak-scaled.

Per GPU: `--users` users rows and `--orders` orders rows (synthetic, seed 42;
users id = 10^10 + i, orders customer_id = 10^10 + U[0, N x users)), resident in HBM
as CSV bytes; the default 62.5 M + 62.5 M is one rank's share of SURVEY.md section
8d's config 5 (500 M x 500 M over 8 GPUs).  One step = the whole repartitioned join of
    SELECT u.role, COUNT(*), SUM(o.price) FROM 'users.csv' AS u
    JOIN 'orders.csv' AS o ON u.id = o.customer_id GROUP BY u.role
on every rank: device key routing of both shards (route.hip), the record
all-to-all over RCCL (cq_amd.dist.exchange; skipped at N = 1), rebuilding both
sides from the received records, the device join + group aggregate (run_join),
the partial-blob all_gather and the merge on rank 0.

    python bench_join.py [--gpus N] [--steps K] [--warmup W] [--users U] [--orders O]

Prints one JSON line (rank 0): rows/s = (users + orders rows, all ranks) / step
time; `roofline`: the step's algorithmic HBM bytes (both CSV shards read once, the
minimum any implementation moves) / step time against 8 TB/s; `verified`: the
joined pair count (= all orders rows: every customer_id exists) and, at N = 1, the
per-role COUNT / SUM(price) recomputed from the generators' draws (counts exact,
sums 1e-6 relative); the reference CPU evaluator timed in the same run on an
n x n sample (row-pairs/s: its join is a nested loop, so not comparable).
Not the driver's bench line (bench.py is); a measurement of the join path.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _digits(v: np.ndarray, w: int) -> np.ndarray:
    out = np.empty((v.size, w), dtype=np.uint8)
    x = v.astype(np.int64).copy()
    for k in range(w - 1, -1, -1):
        out[:, k] = 48 + x % 10
        x //= 10
    return out


def users_shard(n: int, first_id: int, rng) -> bytes:
    """`id,name,age,role` rows, fixed width: 10^10+i, 6 letters, 10-80, role_000-999"""
    m = np.empty((n, 31), dtype=np.uint8)
    m[:, 0:11] = _digits(np.arange(n, dtype=np.int64) + 10**10 + first_id, 11)
    m[:, 11] = 44
    m[:, 12:18] = rng.integers(65, 81, n).astype(np.uint8)[:, None]
    m[:, 18] = 44
    m[:, 19:21] = _digits(rng.integers(10, 81, n), 2)
    m[:, 21] = 44
    m[:, 22:27] = np.frombuffer(b"role_", dtype=np.uint8)
    m[:, 27:30] = _digits(rng.integers(0, 1000, n), 3)
    m[:, 30] = 10
    return m.tobytes()


def orders_shard(n: int, first_id: int, n_users_total: int, rng) -> bytes:
    """`id,price,quantity,customer_id` rows: 10^10+i, ddd.dd, 1-9, 10^10+U[0, users)"""
    m = np.empty((n, 33), dtype=np.uint8)
    m[:, 0:11] = _digits(np.arange(n, dtype=np.int64) + 10**10 + first_id, 11)
    m[:, 11] = 44
    price = rng.integers(100, 100000, n)
    m[:, 12:15] = _digits(price // 100, 3)
    m[:, 15] = 46
    m[:, 16:18] = _digits(price % 100, 2)
    m[:, 18] = 44
    m[:, 19] = 48 + rng.integers(1, 10, n).astype(np.uint8)
    m[:, 20] = 44
    m[:, 21:32] = _digits(rng.integers(0, n_users_total, n) + 10**10, 11)
    m[:, 32] = 10
    return m.tobytes()


def expected_roles(users: int, orders: int, seed: int):
    """per-role (COUNT, SUM(price) in cents) of the N = 1 join, from the same draws
    users_shard / orders_shard make (rank 0's generator)"""
    rng = np.random.default_rng([seed, 0])
    rng.integers(65, 81, users)                        # names
    rng.integers(10, 81, users)                        # ages
    role = rng.integers(0, 1000, users)
    price = rng.integers(100, 100000, orders)
    rng.integers(1, 10, orders)                        # quantities
    cust = rng.integers(0, users, orders)
    r = role[cust]
    return np.bincount(r, minlength=1000), np.bincount(r, weights=price, minlength=1000)


def _digits_t(v, w: int):
    """int64 tensor -> [n, w] uint8 ASCII digits (zero padded), on v's device"""
    import torch
    out = torch.empty((v.numel(), w), dtype=torch.uint8, device=v.device)
    x = v.clone()
    for k in range(w - 1, -1, -1):
        out[:, k] = (torch.remainder(x, 10) + 48).to(torch.uint8)
        x = torch.div(x, 10, rounding_mode="floor")
    return out


def gen_config5_device(n: int, seed: int, device):
    """BASELINE config 5's whole inputs on the device (torch's Philox generator):
    n users `10^10+i,<6 letters>,<10-80>,role_<000-999>` and n orders
    `10^10+i,<ddd.dd>,<1-9>,10^10+U[0, n)` as '\n'-terminated records (no header),
    plus per role the exact COUNT and SUM(price) in cents of the join and the
    first matched user of each role (the groups' first-appearance order)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    ri = lambda lo, hi: torch.randint(lo, hi, (n,), generator=g, device=device, dtype=torch.int64)  # noqa: E731
    ids = torch.arange(n, dtype=torch.int64, device=device) + 10**10
    u = torch.empty((n, 31), dtype=torch.uint8, device=device)
    u[:, 0:11] = _digits_t(ids, 11)
    u[:, 11] = 44
    u[:, 12:18] = ri(65, 81).to(torch.uint8)[:, None]
    u[:, 18] = 44
    u[:, 19:21] = _digits_t(ri(10, 81), 2)
    u[:, 21] = 44
    u[:, 22:27] = torch.tensor(list(b"role_"), dtype=torch.uint8, device=device)
    role = ri(0, 1000)
    u[:, 27:30] = _digits_t(role, 3)
    u[:, 30] = 10
    o = torch.empty((n, 33), dtype=torch.uint8, device=device)
    o[:, 0:11] = _digits_t(ids, 11)
    o[:, 11] = 44
    price = ri(100, 100000)
    o[:, 12:15] = _digits_t(torch.div(price, 100, rounding_mode="floor"), 3)
    o[:, 15] = 46
    o[:, 16:18] = _digits_t(torch.remainder(price, 100), 2)
    o[:, 18] = 44
    o[:, 19] = (ri(1, 10) + 48).to(torch.uint8)
    o[:, 20] = 44
    cust = ri(0, n)
    o[:, 21:32] = _digits_t(cust + 10**10, 11)
    o[:, 32] = 10
    del ids
    r = role[cust]
    cnt = torch.bincount(r, minlength=1000).cpu().numpy()
    cents = torch.bincount(r, weights=price.to(torch.float64), minlength=1000).cpu().numpy()
    matched = torch.zeros(n, dtype=torch.bool, device=device)
    matched[cust] = True
    idx = torch.nonzero(matched).squeeze(1)
    first = torch.full((1000,), n, dtype=torch.int64, device=device)
    first.scatter_reduce_(0, role[idx], idx, reduce="amin")
    first = first.cpu().numpy()
    del r, matched, idx, cust, price, role
    return u.reshape(-1), o.reshape(-1), cnt, cents, first


def gen_config5_shard_device(n: int, rank: int, world: int, seed: int, device):
    """rank's shard of BASELINE config 5's inputs on the device: users 10^10 + rank n + i
    (i < n) and n orders with customer ids uniform over all world * n users; every
    user's role is drawn from one generator shared by all ranks (so each rank can
    price its orders' groups), the rest from per-rank generators.  Returns the two
    '\n'-terminated record buffers and this rank's per-role (COUNT, SUM(price) cents)
    and matched-user mask over all users (summed / or-ed across ranks by the caller)."""
    import torch
    ga = torch.Generator(device=device)
    ga.manual_seed(seed)
    role_all = torch.randint(0, 1000, (world * n,), generator=ga, device=device, dtype=torch.int64)
    g = torch.Generator(device=device)
    g.manual_seed(seed * 1000 + 17 + rank)
    ri = lambda lo, hi: torch.randint(lo, hi, (n,), generator=g, device=device, dtype=torch.int64)  # noqa: E731
    ids = torch.arange(n, dtype=torch.int64, device=device) + 10**10 + rank * n
    u = torch.empty((n, 31), dtype=torch.uint8, device=device)
    u[:, 0:11] = _digits_t(ids, 11)
    u[:, 11] = 44
    u[:, 12:18] = ri(65, 81).to(torch.uint8)[:, None]
    u[:, 18] = 44
    u[:, 19:21] = _digits_t(ri(10, 81), 2)
    u[:, 21] = 44
    u[:, 22:27] = torch.tensor(list(b"role_"), dtype=torch.uint8, device=device)
    u[:, 27:30] = _digits_t(role_all[rank * n:(rank + 1) * n], 3)
    u[:, 30] = 10
    o = torch.empty((n, 33), dtype=torch.uint8, device=device)
    o[:, 0:11] = _digits_t(ids, 11)
    o[:, 11] = 44
    price = ri(100, 100000)
    o[:, 12:15] = _digits_t(torch.div(price, 100, rounding_mode="floor"), 3)
    o[:, 15] = 46
    o[:, 16:18] = _digits_t(torch.remainder(price, 100), 2)
    o[:, 18] = 44
    o[:, 19] = (ri(1, 10) + 48).to(torch.uint8)
    o[:, 20] = 44
    cust = torch.randint(0, world * n, (n,), generator=g, device=device, dtype=torch.int64)
    o[:, 21:32] = _digits_t(cust + 10**10, 11)
    o[:, 32] = 10
    del ids
    r = role_all[cust]
    cnt = torch.bincount(r, minlength=1000).to(torch.float64)
    cents = torch.bincount(r, weights=price.to(torch.float64), minlength=1000)
    matched = torch.zeros(world * n, dtype=torch.uint8, device=device)
    matched[cust] = 1
    return u.reshape(-1), o.reshape(-1), cnt, cents, matched, role_all


def dist_join_leg(n: int, rank: int, world: int, steps: int, warmup: int, seed: int, device, ast, dist):
    """BASELINE config 5 at N = world: every rank holds n users and n orders (device-
    generated CSV shards), and one step is the whole repartitioned join inside the
    library (cqgpu_dist_join over its RCCL communicator: routing by key mod N, one
    grouped send / recv per side, rebuilt sides, the STAR join with key stride N, the
    partial blobs merged on rank 0).  Timed between barriers, max over ranks; rank 0
    verifies per-role COUNT / SUM(price) and the group order against the generators'
    draws (reduced over ranks)."""
    import torch
    import cq_amd
    from cq_amd import abi
    from cq_amd.dist import join_partitioned_rccl
    uh, oh = b"id,name,age,role\n", b"id,price,quantity,customer_id\n"
    t0 = time.time()
    ub, ob, cnt, cents, matched, role_all = gen_config5_shard_device(n, rank, world, seed, device)
    torch.cuda.synchronize(device)
    gen_s = time.time() - t0
    gids = torch.arange(n, dtype=torch.int64, device=device)
    U = cq_amd.table_from_routed(ub.data_ptr(), ub.numel(), gids.data_ptr(), n, uh)
    O = cq_amd.table_from_routed(ob.data_ptr(), ob.numel(), gids.data_ptr(), n, oh)
    nbytes = ub.numel() + ob.numel()
    del ub, ob, gids
    dist.all_reduce(cnt)
    dist.all_reduce(cents)
    dist.all_reduce(matched, op=dist.ReduceOp.MAX)
    first = None
    if rank == 0:
        idx = torch.nonzero(matched).squeeze(1)
        fr = torch.full((1000,), world * n, dtype=torch.int64, device=device)
        fr.scatter_reduce_(0, role_all[idx], idx, reduce="amin")
        first = fr.cpu().numpy()
        del idx
    cnt, cents = cnt.cpu().numpy().astype(np.int64), cents.cpu().numpy()
    del matched, role_all
    torch.cuda.empty_cache()
    last = None
    for _ in range(warmup):
        tp = join_partitioned_rccl(ast, U, O)
        if tp:
            cq_amd.result_free(tp)
    dist.barrier()
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    for _ in range(steps):
        tp = join_partitioned_rccl(ast, U, O)
        if tp:
            if last:
                cq_amd.result_free(last)
            last = tp
    dist.barrier()
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t1
    t = torch.tensor([el], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    kind = cq_amd.stats().get("scan_kernel")
    kinds = [None] * world
    dist.all_gather_object(kinds, kind)
    ok = None
    if rank == 0:
        res = abi.table_to_py(last)
        cq_amd.result_free(last)
        rows = res["rows"]
        want = [r for r in np.argsort(first, kind="stable") if cnt[r] > 0]
        ok = len(rows) == len(want) and all(k in (4, 5) for k in kinds)     # (5: the typed exchange)
        for row, r in zip(rows, want if ok else []):
            name = row[0][1].decode() if isinstance(row[0][1], bytes) else row[0][1]
            ws = cents[r] / 100.0
            if name != "role_%03d" % r or row[1][1] != cnt[r] or abs(row[2][1] - ws) > 1e-6 * ws:
                ok = False
                break
    U.close()
    O.close()
    return {"step_s": el / steps, "rows_total": 2 * n * world, "bytes_per_rank": nbytes, "verified": ok,
            "kinds": kinds, "gen_s": gen_s, "joined_pairs": int(cnt.sum())}


def routed_share_leg(n_total: int, nranks: int, steps: int, warmup: int, seed: int, device, ast, check_order=True):
    """BASELINE config 5 as a rank of an `nranks`-GPU node runs it, on one GPU: the whole
    n_total x n_total inputs are generated on the device, routed with the product's
    own key routing (cqgpu_route_plan / cqgpu_route_fill: whole keys by key mod N)
    into `nranks` shards, and each shard is rebuilt as that rank would receive it
    (cqgpu_table_from_routed: its records in file order with global ids, key stride N,
    record total).  Rank 0's cqgpu_query_partial is timed (warmup + steps; everything
    but the exchange and the merge); every rank's partial runs once and
    cqgpu_merge_partials must reproduce the exact per-role answer and group order."""
    import ctypes as C
    import torch
    import cq_amd
    from cq_amd import abi
    uh, oh = b"id,name,age,role\n", b"id,price,quantity,customer_id\n"
    t0 = time.time()
    ub, ob, cnt, cents, first = gen_config5_device(n_total, seed, device)
    torch.cuda.synchronize(device)
    gen_s = time.time() - t0
    gids = torch.arange(n_total, dtype=torch.int64, device=device)
    U = cq_amd.table_from_routed(ub.data_ptr(), ub.numel(), gids.data_ptr(), n_total, uh)
    O = cq_amd.table_from_routed(ob.data_ptr(), ob.numel(), gids.data_ptr(), n_total, oh)
    if not U or not O:
        raise RuntimeError(cq_amd.last_error())
    del ub, ob, gids
    torch.cuda.empty_cache()
    sends = []
    t0 = time.perf_counter()
    for side, tab in enumerate((U, O)):
        nb, nr = cq_amd.route_plan(ast, [U, O], side, nranks)
        sb = torch.empty(max(sum(nb), 1), dtype=torch.uint8, device=device)
        sg = torch.empty(max(sum(nr), 1), dtype=torch.int64, device=device)
        cq_amd.route_fill(tab, 0, sb.data_ptr(), sg.data_ptr())
        torch.cuda.synchronize(device)
        sends.append((sb, sg, np.concatenate([[0], np.cumsum(nb)]).astype(np.int64),
                      np.concatenate([[0], np.cumsum(nr)]).astype(np.int64)))
    route_s = time.perf_counter() - t0
    # rank 0's share of the two input files (algorithmic bytes = file
    # bytes): its routed rows as whole CSV records -- the route's plan with the field
    # projection off; the shard it reads holds only the fields the plan needs
    file_share = 0
    old = os.environ.get("CQGPU_NO_ROUTE_PROJECT")
    os.environ["CQGPU_NO_ROUTE_PROJECT"] = "1"
    try:
        for side, tab in enumerate((U, O)):
            nb, _ = cq_amd.route_plan(ast, [U, O], side, nranks)
            file_share += int(nb[0])
    finally:
        if old is None:
            os.environ.pop("CQGPU_NO_ROUTE_PROJECT", None)
        else:
            os.environ["CQGPU_NO_ROUTE_PROJECT"] = old
    U.close()
    O.close()
    rank_rows = [int(sends[0][3][d + 1] - sends[0][3][d]) + int(sends[1][3][d + 1] - sends[1][3][d])
                 for d in range(nranks)]
    blobs, kinds, rank_bytes = [], [], []
    ms = []
    step_s = None
    for d in range(nranks):
        tabs = []
        nbytes = 0
        for (sb, sg, bo, ro), hdr in zip(sends, (uh, oh)):
            rb, rg = sb[int(bo[d]):int(bo[d + 1])], sg[int(ro[d]):int(ro[d + 1])]
            t = cq_amd.table_from_routed(rb.data_ptr(), rb.numel(), rg.data_ptr(), rg.numel(), hdr)
            if not t:
                raise RuntimeError(cq_amd.last_error())
            cq_amd.table_set_record_total(t, n_total)
            cq_amd.table_set_key_stride(t, nranks)
            tabs.append(t)
            nbytes += rb.numel()
        rank_bytes.append(nbytes)
        if d == 0:
            for _ in range(warmup):
                cq_amd.query_partial(ast, tabs)
            torch.cuda.synchronize(device)
            t1 = time.perf_counter()
            for _ in range(steps):
                blob = cq_amd.query_partial(ast, tabs)
                ms.append(cq_amd.stats()["scan_ms"])
            torch.cuda.synchronize(device)
            step_s = (time.perf_counter() - t1) / steps
        else:
            blob = cq_amd.query_partial(ast, tabs)
        kinds.append(cq_amd.stats()["scan_kernel"])
        blobs.append(blob)
        for t in tabs:
            t.close()
    del sends
    torch.cuda.empty_cache()
    tp = cq_amd.merge_partials(ast, blobs)
    if not tp:
        raise RuntimeError(cq_amd.last_error())
    res = abi.table_to_py(tp)
    cq_amd.result_free(tp)
    ok = all(k == 4 for k in kinds)
    rows = res["rows"]
    want = [r for r in np.argsort(first, kind="stable") if cnt[r] > 0]
    ok = ok and len(rows) == len(want)
    for row, r in zip(rows, want if ok else []):
        name = row[0][1].decode() if isinstance(row[0][1], bytes) else row[0][1]
        ws = cents[r] / 100.0
        if (check_order and name != "role_%03d" % r) or row[1][1] != cnt[r] or abs(row[2][1] - ws) > 1e-6 * ws:
            ok = False
            break
    return {"step_s": step_s, "kernel_ms": sum(ms) / len(ms), "rows": rank_rows[0], "bytes": rank_bytes[0],
            "file_bytes": file_share,
            "rank_rows": rank_rows, "kinds": kinds, "verified": ok, "route_s": route_s, "gen_s": gen_s,
            "joined_pairs": int(cnt.sum())}


def typed_rank_step_leg(n_total: int, nranks: int, steps: int, warmup: int, seed: int, device, ast):
    """BASELINE config 5 as rank 0 of an `nranks`-GPU node runs its WHOLE step, on one
    GPU, with the typed exchange (include/cqgpu.h cqgpu_typed_*): the n_total x n_total
    inputs are generated on the device and cut into `nranks` range shards (the files'
    byte ranges every rank holds); ranks 1..N-1's sends and partials are prepared once,
    untimed.  One timed step is everything rank 0 does:
      count    its users shard's records per window (the global ids' bases)
      send     both shards typed into 16-byte users / 8-byte orders entries by key mod N
      receive  region 0 of every rank's entries gathered into its receive buffers (a
               device copy standing in for the xGMI transfer, whose bytes are reported)
      join     the STAR join over the received entries, its partial blob
      merge    cqgpu_merge_partials of the N blobs (rank 0's role)
    The merged answer is verified against the generators' exact per-role COUNT /
    SUM(price) and first-appearance order."""
    import torch
    import cq_amd
    from cq_amd import abi
    uh, oh = b"id,name,age,role\n", b"id,price,quantity,customer_id\n"
    t0 = time.time()
    ub, ob, cnt, cents, first = gen_config5_device(n_total, seed, device)
    torch.cuda.synchronize(device)
    gen_s = time.time() - t0
    if n_total % nranks:
        raise ValueError("rows not divisible by ranks")
    n = n_total // nranks
    U, O = [], []
    for r in range(nranks):
        gids = torch.arange(n, dtype=torch.int64, device=device)
        us, os_ = ub[r * n * 31:(r + 1) * n * 31], ob[r * n * 33:(r + 1) * n * 33]
        U.append(cq_amd.table_from_routed(us.data_ptr(), us.numel(), gids.data_ptr(), n, uh))
        O.append(cq_amd.table_from_routed(os_.data_ptr(), os_.numel(), gids.data_ptr(), n, oh))
    file_bytes = n * 31 + n * 33
    del ub, ob
    torch.cuda.empty_cache()
    pair = lambda r: [U[r], O[r]]  # noqa: E731
    if not cq_amd.typed_plan(ast, pair(0)):
        raise RuntimeError("config 5's plan outside the typed exchange: " + cq_amd.last_ineligible())
    smin = min(cq_amd.typed_sample_kmin(ast, pair(r)) for r in range(nranks))
    qbase = smin // nranks
    cu, co, nrec, kmin, kmax, flags = [], [], [], (1 << 64) - 1, 0, 0
    for r in range(nranks):
        nu, c1, kr, f1 = cq_amd.typed_count(ast, pair(r), 0, nranks, qbase)
        _, c2, _, f2 = cq_amd.typed_count(ast, pair(r), 1, nranks, qbase)
        cu.append(c1)
        co.append(c2)
        nrec.append(nu)
        kmin, kmax, flags = min(kmin, kr[0]), max(kmax, kr[1]), flags | f1 | f2
    gbase = [sum(nrec[:r]) for r in range(nranks)]
    for r in range(nranks):
        flags |= cq_amd.typed_send(ast, pair(r), 0, gbase[r]) | cq_amd.typed_send(ast, pair(r), 1, 0)
    if flags:
        raise RuntimeError(f"typed exchange flags {flags:#x}")
    qoff, rng = kmin // nranks - qbase, kmax // nranks - kmin // nranks + 1
    recv_u = [sum(cu[s][d] for s in range(nranks)) for d in range(nranks)]
    recv_o = [sum(co[s][d] for s in range(nranks)) for d in range(nranks)]
    bu = torch.empty(max(recv_u) * 16 + 16, dtype=torch.uint8, device=device)
    bo = torch.empty(max(recv_o) * 8 + 16, dtype=torch.uint8, device=device)
    blobs = [None] * nranks
    kinds = [None] * nranks
    for d in range(1, nranks):                      # the other ranks' partials (untimed)
        torch.cuda.synchronize(device)
        nu = cq_amd.typed_gather(U, d, bu.data_ptr(), recv_u[d])
        no = cq_amd.typed_gather(O, d, bo.data_ptr(), recv_o[d])
        blobs[d] = cq_amd.typed_partial(ast, pair(d), bu.data_ptr(), nu, bo.data_ptr(), no, qoff, rng)
        kinds[d] = cq_amd.stats().get("scan_kernel")
        if blobs[d] is None:
            raise RuntimeError(cq_amd.last_ineligible() or cq_amd.last_error())
    phases = {}

    def step(timed_phases=False):
        def mark(name):
            if timed_phases:
                torch.cuda.synchronize(device)
                phases[name] = phases.get(name, 0.0) + time.perf_counter() - mark.t
                mark.t = time.perf_counter()
        mark.t = time.perf_counter()
        cq_amd.typed_reset(U[0])
        cq_amd.typed_reset(O[0])
        cq_amd.typed_count(ast, pair(0), 0, nranks, qbase)
        cq_amd.typed_count(ast, pair(0), 1, nranks, qbase)
        mark("count")
        f = cq_amd.typed_send(ast, pair(0), 0, gbase[0]) | cq_amd.typed_send(ast, pair(0), 1, 0)
        if f:
            raise RuntimeError(f"typed send flags {f:#x}")
        mark("send")
        nu = cq_amd.typed_gather(U, 0, bu.data_ptr(), recv_u[0])
        no = cq_amd.typed_gather(O, 0, bo.data_ptr(), recv_o[0])
        mark("receive")
        blob = cq_amd.typed_partial(ast, pair(0), bu.data_ptr(), nu, bo.data_ptr(), no, qoff, rng)
        if blob is None:
            raise RuntimeError(cq_amd.last_ineligible() or cq_amd.last_error())
        kinds[0] = cq_amd.stats().get("scan_kernel")
        mark("join")
        tp = cq_amd.merge_partials(ast, [blob] + blobs[1:])
        mark("merge")
        return tp
    for _ in range(warmup):
        cq_amd.result_free(step())
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    last = None
    for _ in range(steps):
        tp = step()
        if last:
            cq_amd.result_free(last)
        last = tp
    torch.cuda.synchronize(device)
    step_s = (time.perf_counter() - t1) / steps
    cq_amd.result_free(step(timed_phases=True))      # one more step, synchronised per phase
    res = abi.table_to_py(last)
    cq_amd.result_free(last)
    rows = res["rows"]
    want = [r for r in np.argsort(first, kind="stable") if cnt[r] > 0]
    ok = len(rows) == len(want) and all(k == 5 for k in kinds)
    for row, r in zip(rows, want if ok else []):
        name = row[0][1].decode() if isinstance(row[0][1], bytes) else row[0][1]
        ws = cents[r] / 100.0
        if name != "role_%03d" % r or row[1][1] != cnt[r] or abs(row[2][1] - ws) > 1e-6 * ws:
            ok = False
            break
    sent = sum(16 * cu[0][d] + 8 * co[0][d] for d in range(1, nranks))
    received = sum(16 * cu[s][0] + 8 * co[s][0] for s in range(1, nranks))
    entry_bytes_written = 16 * sum(cu[0]) + 8 * sum(co[0])
    entry_bytes_read = 16 * recv_u[0] + 8 * recv_o[0]
    for t in U + O:
        t.close()
    return {"step_s": step_s, "rows": 2 * n, "file_bytes": file_bytes, "entry_bytes_written": entry_bytes_written,
            "entry_bytes_read": entry_bytes_read, "xgmi_sent_bytes": sent, "xgmi_received_bytes": received,
            "phases_ms": {k: round(v * 1e3, 4) for k, v in phases.items()}, "kinds": kinds, "verified": ok,
            "gen_s": gen_s, "joined_pairs": int(cnt.sum()), "recv_entries": [recv_u[0], recv_o[0]]}


def cpu_baseline(n: int, seed: int):
    """The unmodified reference (oracle/_ref/ref_probe, 1 core) on an n x n sample of
    the same generators.  Its nested-loop join is O(L x R) (evaluator_joins.c:63-181),
    so the sample is small and the figure is row-pairs/s: non-comparable with the
    GPU's rows/s, reported beside it as SURVEY.md 8d asks."""
    import subprocess
    import tempfile
    probe = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
    if not os.path.exists(probe):
        return None
    rng = np.random.default_rng([seed, 99])
    with tempfile.TemporaryDirectory() as d:
        up, op = os.path.join(d, "users.csv"), os.path.join(d, "orders.csv")
        with open(up, "wb") as fh:
            fh.write(b"id,name,age,role\n" + users_shard(n, 0, rng))
        with open(op, "wb") as fh:
            fh.write(b"id,price,quantity,customer_id\n" + orders_shard(n, 0, n, rng))
        sql = (f"SELECT u.role, COUNT(*), SUM(o.price) FROM '{up}' AS u JOIN '{op}' AS o "
               f"ON u.id = o.customer_id GROUP BY u.role")
        out = subprocess.run(["taskset", "-c", "0", probe, "time", sql], capture_output=True, timeout=600)
        if out.returncode != 0:
            out = subprocess.run([probe, "time", sql], capture_output=True, timeout=600)
        secs = json.loads(out.stdout.decode())["seconds"]
    return {"value": n * n / secs, "unit": "row-pairs/s", "cores": 1, "kind": "reference",
            "rows_per_s": 2 * n / secs, "seconds": secs, "comparable": False,
            "sample": f"{n} users x {n} orders of the same generators; reference parse + evaluate_query "
                      f"(nested-loop join incl. csv_load) = {secs:.2f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--users", type=int, default=62_500_000, help="users rows per GPU")
    ap.add_argument("--orders", type=int, default=62_500_000, help="orders rows per GPU")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-rows", type=int, default=5000, help="n of the reference's n x n join sample")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.zeros(1, device=dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import ctypes as C
    import cq_amd
    from cq_amd import abi
    from cq_amd.dist import exchange, exclusive_base, gather_blobs
    L = cq_amd.lib()

    t0 = time.time()
    rng = np.random.default_rng([args.seed, rank])
    uh, oh = b"id,name,age,role\n", b"id,price,quantity,customer_id\n"
    ub = users_shard(args.users, rank * args.users, rng)
    ob = orders_shard(args.orders, rank * args.orders, world * args.users, rng)
    ut = cq_amd.Table.from_bytes(uh + ub if rank == 0 else ub, header=None if rank == 0 else uh)
    ot = cq_amd.Table.from_bytes(oh + ob if rank == 0 else ob, header=None if rank == 0 else oh)
    in_bytes = len(ub) + len(ob)
    del ub, ob
    gen_s = time.time() - t0

    P = abi.Plan()
    q = P.query([P.ident("u.role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("o.price"))],
                "users.csv", alias="u", group_by=["u.role"],
                joins=[("orders.csv", "o", P.cond("=", P.ident("u.id"), P.ident("o.customer_id")),
                        abi.JOIN_INNER)])
    ast = C.pointer(q)
    phase = {}
    last_res = [None]

    def step():
        ts = time.perf_counter()
        routed = []
        # one rank routes every record to itself in its own order: the shards are the
        # routed tables (cq_amd.dist.join_partitioned does the same)
        for side, (tab, hdr) in enumerate(((ut, uh), (ot, oh)) if world > 1 else ()):
            nb, nr = cq_amd.route_plan(ast, [ut, ot], side, world)
            base = exclusive_base(sum(nr), dev) if dist is not None else 0
            sb = torch.empty(max(sum(nb), 1), dtype=torch.uint8, device=dev)
            sg = torch.empty(max(sum(nr), 1), dtype=torch.int64, device=dev)
            cq_amd.route_fill(tab, base, sb.data_ptr(), sg.data_ptr())
            if dist is not None:
                rb, _ = exchange(sb[: sum(nb)], nb)
                rg, _ = exchange(sg[: sum(nr)], nr)
                torch.cuda.synchronize(dev)
            else:
                rb, rg = sb[: sum(nb)], sg[: sum(nr)]
            routed.append(cq_amd.table_from_routed(rb.data_ptr(), rb.numel(), rg.data_ptr(), rg.numel(), hdr))
            del sb, sg, rb, rg
        tr = time.perf_counter()
        if world == 1:     # one rank: the whole join is local (the fused aggregate join)
            tp = L.cqgpu_query(ast, (C.c_void_p * 2)(ut.handle.value, ot.handle.value), 2)
            st = cq_amd.stats()
            tj = time.perf_counter()
        else:
            blob = cq_amd.query_partial(ast, routed)
            st = cq_amd.stats()
            tj = time.perf_counter()
            blobs = gather_blobs(blob, dev)
            tp = cq_amd.merge_partials(ast, blobs) if rank == 0 else None
        pairs = 0
        if rank == 0:
            if not tp:
                raise RuntimeError(cq_amd.last_error() or cq_amd.last_ineligible())
            res = abi.table_to_py(tp)
            cq_amd.result_free(tp)
            pairs = int(sum(r[1][1] for r in res["rows"]))   # COUNT(*) cells: ("I", n)
            last_res[0] = res
        for t in routed:
            t.close()
        te = time.perf_counter()
        phase.setdefault("route_exchange_ms", []).append((tr - ts) * 1e3)
        phase.setdefault("join_agg_ms", []).append((tj - tr) * 1e3)
        phase.setdefault("merge_ms", []).append((te - tj) * 1e3)
        phase.setdefault("pair_agg_kernel_ms", []).append(st["scan_ms"])
        return pairs

    pairs = 0
    for _ in range(args.warmup):
        pairs = step()
    for k in phase:
        phase[k].clear()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        pairs = step()
    barrier()
    elapsed = time.perf_counter() - t1
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    rows_total = (args.users + args.orders) * world
    verified = True
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            try:
                cpu = cpu_baseline(args.cpu_rows, args.seed)
            except Exception as e:  # reported, never fatal
                print(f"cpu baseline failed: {e}", file=sys.stderr)
        verified = pairs == args.orders * world
        if not verified:
            print(f"VERIFY FAILED: {pairs} joined pairs, expected {args.orders * world}", file=sys.stderr)
        verified_against = "pair count = orders rows"
        if world == 1 and verified:
            cnt, cents = expected_roles(args.users, args.orders, args.seed)
            got = {r[0][1].decode(): (r[1][1], r[2][1]) for r in last_res[0]["rows"]}
            for k in range(1000):
                if not cnt[k]:
                    continue
                g = got.get("role_%03d" % k)
                want_sum = cents[k] / 100.0
                if g is None or g[0] != cnt[k] or abs(g[1] - want_sum) > 1e-6 * want_sum:
                    verified = False
                    print(f"VERIFY FAILED: role_{k:03d} got {g} want ({cnt[k]}, {want_sum})", file=sys.stderr)
                    break
            verified_against = "per-role COUNT / SUM(price) from the generators' draws (numpy)"
        step_s = elapsed / args.steps
        achieved = in_bytes * world / step_s / 1e9 / world
        line = {
            "metric": "join rows/s (users + orders rows, key-repartitioned device hash join + GROUP BY)",
            "value": rows_total / (elapsed / args.steps),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic users/orders CSV (SURVEY.md 8d config 5 shape, seed {args.seed}), resident in HBM",
            "config": {
                "workload": "config5 per GPU: SELECT u.role, COUNT(*), SUM(o.price) FROM users u "
                            "JOIN orders o ON u.id = o.customer_id GROUP BY u.role",
                "users_per_gpu": args.users,
                "orders_per_gpu": args.orders,
                "bytes_per_gpu": in_bytes,
                "joined_pairs": pairs,
                "parallelism": (f"dp{world} (hash repartition all_to_all over RCCL)" if world > 1
                                else "dp1 (one rank: no repartition)"),
            },
            "verified": verified,
            "verified_against": verified_against,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0, "traffic": None,
                         "algorithmic_bytes": "both CSV shards read once per step (bytes_per_gpu); the "
                                              "pipeline also writes and re-reads routed copies, cells and pairs"},
            "phases_ms": {k: sum(v) / len(v) for k, v in phase.items()},
            "cpu_baseline": cpu,
            "setup_s": gen_s,
        }
        print(json.dumps(line), flush=True)
    ut.close()
    ot.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not verified:
        sys.exit(3)


if __name__ == "__main__":
    main()
