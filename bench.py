#!/usr/bin/env python3
"""Benchmark: rows/s of cq's SELECT hot path (CSV scan + WHERE + GROUP BY) on MI355X.

Workload (BASELINE.json): the logical Shape A+role CSV of cq_amd/datagen.py
(reference utils/generate_big_dataset.py columns + role_%03d, 1,000 groups,
seed 42), resident in HBM, and
    SELECT role, COUNT(*), SUM(height), AVG(height) FROM 'big.csv'
    WHERE age > 30 GROUP BY role
  * N = 1: configs[2] -- rows [0, 1e8) on one GPU (3.89 GB);
  * N > 1: configs[3] -- rows [0, 1e9) range-partitioned over the N ranks (each
    rank generates and uploads only its own rows; ~38.9 GB in all).
One step = one full query over the resident bytes: the fused scan kernel
(tokenize + type + filter + LDS hash aggregate), compaction, first-row gather,
result table; with N > 1 each rank scans its shard (cqgpu_query_partial), the
partial group states are exchanged over RCCL and merged on rank 0.

The last step's result is checked against tests/golden/big.json (the reference
itself at 1e8 rows; the generator's draws at 1e9) or, for other sizes, against
datagen.expected_filter_groupby; a mismatch exits non-zero.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints one JSON line (rank 0) with the roofline of the scan kernel (file bytes /
HIP-event kernel time vs 8 TB/s), an end-to-end evaluate_query timing on the same
file (mmap + H2D + scan), config 2 (filter + COUNT) as an extra key, and a CPU
baseline: the unmodified reference (oracle/_ref/ref_probe built from
/root/reference by oracle/ref.mk) timed on a bounded sample of the same workload.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ProcessPoolExecutor

import torch  # first: libcqgpu binds to the HIP runtime torch loads

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from cq_amd import datagen  # noqa: E402  (numpy only: safe before the GPU is touched)

METRIC = "rows/sec scanned (filter+GROUP BY) at 1/2/4/8 GPUs; % of HBM read peak"
QUERY = ("SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{path}' "
         "WHERE age > 30 GROUP BY role")
QUERY2 = "SELECT COUNT(*) FROM '{path}' WHERE age > 30"
KERNEL_NAMES = {
    (2, True): "cq::fast::fast_kernel<true, true, 1, true, true> (+ slow_kernel, raw_merge_kernel)",
    (2, False): "cq::fast::fast_kernel<false, true, 0, true, true> (+ slow_kernel)",
    (1, True): "cq::lean::lean_kernel<true, LW_NUM, 1, false> (+ slow_kernel, raw_merge_kernel)",
    (1, False): "cq::lean::lean_kernel<false, LW_NUM, 0, false> (+ slow_kernel)",
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GOLDEN = os.path.join(ROOT, "tests", "golden", "big.json")


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=None,
                    help="data rows of the logical file (default 1e8 at N=1, 1e9 at N>1)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-rows", type=int, default=8_000_000,
                    help="rows of the CPU-baseline sample (reference evaluator)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end evaluate_query timing")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 (filter + COUNT) key")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 (users x orders join) key")
    ap.add_argument("--join-rows", type=int, default=62_500_000,
                    help="users and orders rows per rank of the config-5 leg (500 M x 500 M over 8)")
    ap.add_argument("--join-ranks", type=int, default=8, help="ranks the config-5 inputs are routed over")
    ap.add_argument("--gen-workers", type=int, default=4, help="processes generating this rank's rows")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "hbm_traffic.json"))
    ap.add_argument("--config", type=int, default=3, choices=(2, 3),
                    help="3: the bench line (filter + GROUP BY); 2: Shape A filter + COUNT as the line")
    return ap.parse_args()


def build_plan(path, config=3):
    from cq_amd import abi
    P = abi.Plan()
    if config == 2:
        q = P.query([P.func("COUNT", P.lit("*"))], path, where=P.cond(">", P.ident("age"), P.lit("30")))
        return P, q
    q = P.query([P.ident("role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("height")),
                 P.func("AVG", P.ident("height"))], path,
                where=P.cond(">", P.ident("age"), P.lit("30")), group_by=["role"])
    return P, q


def _gen(args):
    seed, lo, hi, role = args
    return datagen.logical_rows(seed, lo, hi, role)


def gen_rows(seed, lo, hi, role, workers):
    """rows [lo, hi) of the logical file, generated chunk-parallel (before any GPU call)"""
    step = datagen.CHUNK_ROWS
    parts = [(seed, a, min(hi, (a // step + 1) * step), role) for a in
             [lo] + list(range((lo // step + 1) * step, hi, step))] if hi > lo else []
    if workers <= 1 or len(parts) <= 1:
        return b"".join(_gen(p) for p in parts)
    with ProcessPoolExecutor(max_workers=workers) as ex:
        return b"".join(ex.map(_gen, parts))


def expected_for(config, rows, seed):
    """(expected answer, source) for the whole logical file rows [0, rows)"""
    try:
        with open(GOLDEN) as fh:
            gj = json.load(fh)
        if gj.get("seed") == seed:
            for key in ("config3", "config4") if config == 3 else ("config2",):
                ent = gj.get(key)
                if ent and ent["rows"] == rows:
                    src = ("reference (tests/golden/big.json %s)" % key if "reference" in ent
                           else "generator draws (tests/golden/big.json %s)" % key)
                    return ent["expected"], src
    except FileNotFoundError:
        pass
    return datagen.expected_filter_groupby(seed, 0, rows, with_role=config == 3), "generator draws (computed)"


def verify(res, exp, config):
    """res: abi.table_to_py of the result; exp: expected_filter_groupby layout"""
    rows = res["rows"]
    if config == 2:
        return len(rows) == 1 and rows[0][0] == ("I", exp["count"][0])
    if len(rows) != len(exp["count"]):
        return False
    for r, name, cnt, cents in zip(rows, exp["groups"], exp["count"], exp["sum_cents"]):
        if r[0] != ("S", name.encode()) or r[1] != ("I", cnt):
            return False
        s, a = r[2][1], r[3][1]
        want = cents / 100.0
        if abs(s - want) > 1e-6 * want or abs(a - want / cnt) > 1e-6 * (want / cnt):
            return False
    return True


def cpu_baseline(rows, seed, config=3):
    """Reference evaluator (single-threaded C, -O2) on a bounded sample, 1 core."""
    probe = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
    if not os.path.exists(probe):
        return None
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "sample.csv")
        datagen.write_logical(path, rows, seed=seed, with_role=config == 3)
        query = (QUERY if config == 3 else QUERY2).format(path=path)
        out = subprocess.run(["taskset", "-c", "0", probe, "time", query], capture_output=True, timeout=600)
        if out.returncode != 0:
            out = subprocess.run([probe, "time", query], capture_output=True, timeout=600)
        res = json.loads(out.stdout.decode())
    secs = res["seconds"]
    cpu = {"value": rows / secs, "unit": "rows/s", "cores": 1, "kind": "reference",
           "sample": f"rows [0, {rows}) of the same logical file (seed {seed}); reference parse + "
                     f"evaluate_query wall time incl. csv_load = {secs:.2f} s, 1 core (taskset)",
           "seconds": secs, "host_cores": os.cpu_count()}
    host_full = os.path.join(ROOT, "profiles", "r5_ref_full_bench_host.json")
    if config == 3 and os.path.exists(host_full):
        # the full 1e8-row file on a GPU box's own host (scripts/archive/r5_ref_full.py): same
        # kind of box as this run, measured separately because it takes ~2.5 minutes
        try:
            with open(host_full) as fh:
                h = json.load(fh)
            cpu["full_size_reference"] = {
                "rows": h["rows"], "seconds": h["reference_seconds"], "rows_per_s": h["rows_per_s"],
                "where": "a GPU box's host: %s, %d logical CPUs, %.1f TB RAM (profiles/r5_ref_full_bench_host.json)"
                         % (h["host"]["cpu_model"], h["host"]["logical_cpus"], h["host"]["mem_total_bytes"] / 1e12),
                "why_not_here": "~2.5 minutes of one core: outside the bench's few-minute budget, so the same-run "
                                "number is the bounded sample above"}
            return cpu
        except Exception:
            pass
    try:
        with open(GOLDEN) as fh:
            g = json.load(fh)["config%d" % config]
        cpu["full_size_reference"] = {
            "rows": g["rows"], "seconds": g["reference_seconds"], "rows_per_s": g["rows"] / g["reference_seconds"],
            "where": "build container (8 vCPU Xeon), tests/golden/make_big_golden.py",
            "why_not_here": "a 1e8-row reference run takes ~6 min and ~35 GB RSS: outside the bench's "
                            "few-minute budget, so the same-run number is the bounded sample above"}
    except Exception:
        pass
    return cpu


def main():
    args = parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    role = args.config == 3
    total = args.rows if args.rows is not None else (100_000_000 if world == 1 else 1_000_000_000)

    # ---- this rank's rows of the logical file, generated before the GPU is touched
    t0 = time.time()
    lo, hi = total * rank // world, total * (rank + 1) // world
    header = datagen.header_of(role)
    body = gen_rows(args.seed, lo, hi, role, args.gen_workers)
    shard = header + body if rank == 0 else body
    del body
    data2 = None   # config 2's file (Shape A, no role), also generated before the GPU is touched
    if world == 1 and args.config == 3 and not args.no_config2:
        data2 = datagen.header_of(False) + gen_rows(args.seed, 0, 100_000_000, False, args.gen_workers)
    gen_s = time.time() - t0

    torch.cuda.set_device(local)
    torch.zeros(1, device="cuda")
    dist = None
    # CQ_BENCH_FORCE_DIST=1 under torchrun: the N > 1 step (range partial + dense RCCL
    # merge) even at world size 1, so one-GPU boxes exercise the collective path
    if world > 1 or (os.environ.get("CQ_BENCH_FORCE_DIST") and "WORLD_SIZE" in os.environ):
        import torch.distributed as dist
        # RCCL prints a version banner on stdout when its communicator comes up: keep
        # stdout for the one JSON line (the banner goes to stderr)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist.barrier()
            torch.cuda.synchronize()
            if not os.environ.get("CQ_BENCH_DIST_PY"):
                # the library's own RCCL communicator (the whole N > 1 step runs inside it)
                from cq_amd.dist import init_library_comm
                init_library_comm()
                torch.cuda.synchronize()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    import cq_amd
    from cq_amd import abi
    from cq_amd.dist import scan_partitioned_dense, scan_partitioned_rccl
    L = cq_amd.lib()

    t0 = time.time()
    sizes = [len(shard)]
    if dist is not None:
        allsz = [None] * world
        dist.all_gather_object(allsz, len(shard))
        sizes = allsz
    base = sum(sizes[:rank])
    table = cq_amd.Table.from_bytes(shard, abi.csv_config(), base_offset=base,
                                    header=None if rank == 0 else header)
    nbytes = len(shard)
    upload_s = time.time() - t0

    P, q = build_plan("big.csv", args.config)
    ast = C.pointer(q)
    kernel_used = [1]
    last_stats = [{}]
    merge_path = [None]

    def step():
        """one query; returns (result pointer on rank 0 or None, scan ms)"""
        if dist is None:
            tp = L.cqgpu_query(ast, (C.c_void_p * 1)(table.handle.value), 1)
            if not tp:
                raise RuntimeError(cq_amd.last_error())
            st = cq_amd.stats()
            if os.environ.get("CQ_BENCH_DEBUG"):
                print("stats", st, file=sys.stderr)
            kernel_used[0] = st.get("scan_kernel", 0)
            last_stats[0] = st
            return tp, st["scan_ms"]
        if os.environ.get("CQ_BENCH_DIST_PY"):
            # A/B: round 3's Python-driven dense merge (torch.distributed collectives)
            tp = scan_partitioned_dense(ast, table)
            merge_path[0] = "dense (python-driven)"
        else:
            # the whole step inside the library over its RCCL communicator: config 4's
            # plan takes the gather-merge (one grouped send/recv to rank 0, device merge)
            tp, path = scan_partitioned_rccl(ast, table)
            merge_path[0] = path + " inside libcqgpu over RCCL"
        st = cq_amd.stats()                   # the merge runs no scan: still this rank's partial
        kernel_used[0] = st.get("scan_kernel", 0)
        last_stats[0] = st
        return tp, st["scan_ms"]

    for _ in range(args.warmup):
        tp, _ = step()
        if tp:
            cq_amd.result_free(tp)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    scan_ms = []
    last = None
    barrier()
    t1 = time.perf_counter()
    for i in range(args.steps):
        tp, ms = step()
        scan_ms.append(ms)
        if tp:
            if last:
                cq_amd.result_free(last)
            last = tp
    barrier()
    elapsed = time.perf_counter() - t1
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    value = total / (elapsed / args.steps)

    cfg5_dist = None
    if world > 1 and not args.no_config5 and dist is not None:
        # configs[4] at N = world: the repartitioned join step inside the library, every rank
        try:
            cfg5_dist = config5_dist_leg(args, rank, world, dist)
        except Exception as e:
            print(f"config 5 (N > 1) leg failed: {e}", file=sys.stderr)
    rc = 0
    if rank == 0:
        # ---- the last step's answer against the expected one (outside the timed region)
        res = abi.table_to_py(last)
        cq_amd.result_free(last)
        exp, exp_src = expected_for(args.config, total, args.seed)
        ok = verify(res, exp, args.config)
        if not ok:
            print("VERIFY FAILED: result differs from " + exp_src, file=sys.stderr)
            print("got rows[:3]", res["rows"][:3], file=sys.stderr)
            rc = 3
        avg_scan_ms = sum(scan_ms) / len(scan_ms)
        achieved = nbytes / (avg_scan_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic) as fh:
                tj = json.load(fh)
            if tj.get("rows") == hi - lo:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            pass

        # ---- end-to-end: evaluate_query on the file (mmap + H2D + scan + result), cold table cache
        e2e = None
        if world == 1 and not args.no_e2e:
            try:
                e2e = end_to_end(shard, args.config, L, cq_amd, exp, total)
            except Exception as e:  # reported, never fatal
                print(f"end-to-end timing failed: {e}", file=sys.stderr)
        cfg2 = None
        if data2 is not None:
            table.close()
            del shard
            try:
                cfg2 = config2_leg(args, cq_amd, abi, L, data2)
                if cfg2 and not cfg2["verified"]:
                    rc = 3
            except Exception as e:
                print(f"config 2 leg failed: {e}", file=sys.stderr)
        cfg5 = None
        if world > 1 and cfg5_dist is not None:
            cfg5 = cfg5_dist
            if not cfg5["verified"]:
                rc = 3
        if world == 1 and not args.no_config5:
            if table.handle:
                table.close()
            try:
                cfg5 = config5_leg(args, cq_amd, L)
                if cfg5 and not cfg5["verified"]:
                    rc = 3
            except Exception as e:
                print(f"config 5 leg failed: {e}", file=sys.stderr)
        cpu = None
        if world == 1 and not args.no_cpu:
            try:
                cpu = cpu_baseline(args.cpu_rows, args.seed, args.config)
            except Exception as e:  # reported, never fatal
                print(f"cpu baseline failed: {e}", file=sys.stderr)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "scaling_note": ("total rows fixed per run: --rows (default 1e8 at N=1, config 3; 1e9 at N>1, "
                             "config 4, range-partitioned); `--gpus 1 --rows 1000000000` runs config 4's "
                             "own file on one GPU, the N=1 point of the same curve"),
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic: logical Shape A+role CSV (generate_big_dataset.py columns + role_%03d, "
                     if role else "synthetic: logical Shape A CSV (generate_big_dataset.py columns, ")
                    + f"seed {args.seed}, cq_amd/datagen.py), resident in HBM before timing",
            "config": {
                "workload": (("config3: " if world == 1 else "config4: ") +
                             "SELECT role, COUNT(*), SUM(height), AVG(height) FROM 'big.csv' "
                             "WHERE age > 30 GROUP BY role" if role else
                             "config2: SELECT COUNT(*) FROM 'big.csv' WHERE age > 30"),
                "rows_total": total,
                "rows_per_gpu": hi - lo,
                "bytes_per_gpu": nbytes,
                "groups": 1000 if role else 1,
                "parallelism": (f"dp{world} (rows [r*T/N, (r+1)*T/N) per rank; merge: " + str(merge_path[0]) +
                                ")" if dist is not None else "dp1"),
            },
            "verified": ok,
            "verified_against": exp_src,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": KERNEL_NAMES.get((kernel_used[0], role), "cq::scan_kernel"),
                "kernel_ms": avg_scan_ms,
                "bytes_per_launch": nbytes,
            },
            "plan_sample": {
                # the plan's choices come from the first 256 KiB (group-key seed, tag width,
                # window stride); records they do not cover show up here
                "slow_records": last_stats[0].get("slow_records"),
                "lds_spills": last_stats[0].get("lds_spills"),
                "retries": last_stats[0].get("retries"),
                "records": last_stats[0].get("records"),
            },
            "end_to_end": e2e,
            "config2": cfg2,
            "config5": cfg5,
            "cpu_baseline": cpu,
            "setup_s": {"generate": round(gen_s, 2), "upload": round(upload_s, 2)},
        }
        print(json.dumps(line), flush=True)
    else:
        if last:
            cq_amd.result_free(last)
    if table.handle:
        table.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    sys.exit(rc)


def end_to_end(data, config, L, cq_amd, exp, rows):
    """evaluate_query (the drop-in entry point) on the same bytes written as a file:
    mmap + pinned H2D upload + scan + result, the device table cache cleared
    before every call; median of 3."""
    from cq_amd import abi
    d = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    fd, path = tempfile.mkstemp(suffix=".csv", dir=d)
    try:
        with os.fdopen(fd, "wb") as fh:
            fh.write(data)
        P, q = build_plan(path, config)
        times = []
        ok = True
        for _ in range(3):
            L.cqgpu_cache_clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tp = L.evaluate_query(C.pointer(q))
            t = time.perf_counter() - t0
            if not tp:
                raise RuntimeError(cq_amd.last_error())
            ok = ok and verify(abi.table_to_py(tp), exp, config)
            cq_amd.result_free(tp)
            times.append(t)
        L.cqgpu_cache_clear()
        times.sort()
        t = times[1]
        return {"seconds": t, "rows_per_s": rows / t, "file_bytes": len(data),
                "GB_per_s": len(data) / t / 1e9, "verified": ok,
                "includes": "evaluate_query on a page-cached file (%s): mmap, 32 MiB pinned chunks filled by up "
                            "to 8 host threads while earlier chunks copy to the device, scan, result; table "
                            "cache cleared before each call; median of 3" % d}
    finally:
        os.unlink(path)


def config5_leg(args, cq_amd, L):
    """configs[4] as rank 0 of the 8-GPU node runs its WHOLE step, on one GPU: users x
    orders of 500 M rows each (`--join-rows` x `--join-ranks`), generated on the
    device and cut into 8 range shards; the step is everything rank 0 does with the
    typed exchange (bench_join.typed_rank_step_leg): count its users shard's records,
    type both shards into 16-byte users / 8-byte orders entries routed by key mod 8,
    receive region 0 of every rank's entries (a device copy standing in for the xGMI
    transfer, whose bytes are reported beside it), the STAR join over them, the
    partial blob and the merge of all 8 partials.  Verified against the exact per-role
    COUNT / SUM(price) and group order of the generators' draws.  Roofline bytes
    (SURVEY.md 8d): the rank's share of both files + the entries it writes and the
    entries it reads.  CPU baseline: the reference's nested-loop join at 5 K x 5 K and
    20 K x 20 K (row-pairs/s, not comparable)."""
    import ctypes as C
    import bench_join as bj
    from cq_amd import abi
    n, N = args.join_rows, args.join_ranks
    P = abi.Plan()
    q = P.query([P.ident("u.role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("o.price"))],
                "users.csv", alias="u", group_by=["u.role"],
                joins=[("orders.csv", "o", P.cond("=", P.ident("u.id"), P.ident("o.customer_id")), abi.JOIN_INNER)])
    ast = C.pointer(q)
    r = bj.typed_rank_step_leg(n * N, N, args.steps, args.warmup, args.seed, torch.device("cuda"), ast)
    step_s = r["step_s"]
    alg = r["file_bytes"] + r["entry_bytes_written"] + r["entry_bytes_read"]
    cpu = None
    if not args.no_cpu:
        cpu = {}
        for m in (5000, 20000):
            try:
                cpu["%dx%d" % (m, m)] = bj.cpu_baseline(m, args.seed)
            except Exception as e:
                cpu["%dx%d" % (m, m)] = {"error": str(e)}
    xgmi = 7 * 153e9                     # 7 xGMI links per GPU at ~153 GB/s each (peak)
    traffic = None                       # HBM bytes per step from the last PMC passes (profiles/)
    try:
        with open(os.path.join(ROOT, "profiles", "config5_traffic.json")) as fh:
            traffic = json.load(fh).get("hbm_bytes_per_step")
    except (OSError, ValueError):
        pass
    return {"workload": "config5 (rank 0 of %d, its whole step): SELECT u.role, COUNT(*), SUM(o.price) "
                        "FROM users u JOIN orders o ON u.id = o.customer_id GROUP BY u.role" % N,
            "users_total": n * N, "orders_total": n * N, "ranks": N,
            "rank_rows": r["rows"], "rank_file_bytes": r["file_bytes"],
            "value": r["rows"] / step_s, "unit": "rows/s (rank 0's share of the users + orders rows)",
            "ms_per_step": step_s * 1e3,
            "step": "count + typed send of both shards (key mod %d) + receive (device copy of the entries the "
                    "rank receives) + STAR join over the entries + partial blob + merge of the %d partials" % (N, N),
            "phases_ms": r["phases_ms"],
            "kernel_kinds_per_rank": r["kinds"],
            "exchange": {"sent_bytes": r["xgmi_sent_bytes"], "received_bytes": r["xgmi_received_bytes"],
                         "entries_received": r["recv_entries"],
                         "entry_bytes": "16 per users record {key/N - qbase, global id, GROUP BY bytes}, 8 per "
                                        "orders record {key/N - qbase, price in 10^-3}; the orders counts include "
                                        "the one-pass send's holes (chunk tails, skipped by the receiver)",
                         "xgmi_bound_ms": max(r["xgmi_sent_bytes"], r["xgmi_received_bytes"]) / xgmi * 1e3,
                         "note": "not in ms_per_step: one GPU has no peer; xgmi_bound_ms = the larger direction "
                                 "over 7 links at their 153 GB/s peak"},
            "roofline": {"bound": "hbm", "achieved": alg / step_s / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": alg / step_s / 1e9 / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": "profiles/config5_traffic.json (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE "
                                           "summed over the step's kernels)",
                         "algorithmic_bytes": alg,
                         "algorithmic": "rank 0's share of both files (%d B) + the entries its send pass writes "
                                        "(%d B) + the entries its join reads (%d B) (SURVEY.md 8d)"
                                        % (r["file_bytes"], r["entry_bytes_written"], r["entry_bytes_read"])},
            "joined_pairs": r["joined_pairs"],
            "verified": r["verified"],
            "verified_against": "every rank's partial merged (cqgpu_merge_partials) vs the exact per-role COUNT / "
                                "SUM(price) and first-appearance order of the generators' draws (torch, on device)",
            "cpu_baseline": cpu, "setup_s": round(r["gen_s"], 2)}


def config5_dist_leg(args, rank, world, dist):
    """configs[4] at N = world (every rank): `--join-rows` users and orders per rank,
    one step = cqgpu_dist_join (route, exchange over RCCL, STAR join with key stride N,
    merge on rank 0); value = all ranks' users + orders rows / step time"""
    import ctypes as C
    import bench_join as bj
    from cq_amd import abi
    P = abi.Plan()
    q = P.query([P.ident("u.role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("o.price"))],
                "users.csv", alias="u", group_by=["u.role"],
                joins=[("orders.csv", "o", P.cond("=", P.ident("u.id"), P.ident("o.customer_id")), abi.JOIN_INNER)])
    r = bj.dist_join_leg(args.join_rows, rank, world, max(3, args.steps // 4), 1, args.seed,
                         torch.device("cuda", torch.cuda.current_device()), C.pointer(q), dist)
    if rank != 0:
        return None
    step_s = r["step_s"]
    return {"workload": "config5 at N = %d: SELECT u.role, COUNT(*), SUM(o.price) FROM users u JOIN orders o "
                        "ON u.id = o.customer_id GROUP BY u.role" % world,
            "users_total": args.join_rows * world, "orders_total": args.join_rows * world, "ranks": world,
            "value": r["rows_total"] / step_s, "unit": "rows/s (all ranks' users + orders rows)",
            "ms_per_step": step_s * 1e3,
            "step": "cqgpu_dist_join: device routing (key mod N), grouped ncclSend/ncclRecv of records + "
                    "global ids per side, rebuilt sides, STAR join (key stride N), partial blobs merged on rank 0",
            "kernel_kinds_per_rank": r["kinds"],
            "roofline": {"bound": "hbm", "achieved": r["bytes_per_rank"] / step_s / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": r["bytes_per_rank"] / step_s / 1e9 / HBM_PEAK_GBS, "traffic": None,
                         "algorithmic_bytes": "each rank's two CSV shards read once (the exchange's xGMI bytes "
                                              "and the routed copies come on top)"},
            "joined_pairs": r["joined_pairs"], "verified": r["verified"],
            "verified_against": "per-role COUNT / SUM(price) and first-appearance order of the generators' draws "
                                "(reduced over ranks)",
            "setup_s": round(r["gen_s"], 2)}


def config2_leg(args, cq_amd, abi, L, data):
    """configs[1]: 1e8 rows of Shape A (no role), SELECT COUNT(*) ... WHERE age > 30"""
    rows = 100_000_000
    t = cq_amd.Table.from_bytes(data, abi.csv_config())
    nb = len(data)
    del data
    P, q = build_plan("big.csv", 2)
    ast = C.pointer(q)
    arr = (C.c_void_p * 1)(t.handle.value)
    for _ in range(args.warmup):
        cq_amd.result_free(L.cqgpu_query(ast, arr, 1))
    torch.cuda.synchronize()
    ms = []
    t0 = time.perf_counter()
    last = None
    st = {}
    for _ in range(args.steps):
        tp = L.cqgpu_query(ast, arr, 1)
        if not tp:
            raise RuntimeError(cq_amd.last_error())
        st = cq_amd.stats()
        ms.append(st["scan_ms"])
        if last:
            cq_amd.result_free(last)
        last = tp
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res = abi.table_to_py(last)
    cq_amd.result_free(last)
    t.close()
    exp, src = expected_for(2, rows, args.seed)
    kms = sum(ms) / len(ms)
    return {"workload": "config2: SELECT COUNT(*) FROM 'big.csv' WHERE age > 30 (Shape A, 1e8 rows)",
            "value": rows / (el / args.steps), "unit": "rows/s", "ms_per_step": el * 1000 / args.steps,
            "kernel_ms": kms, "bytes_per_launch": nb,
            "kernel": KERNEL_NAMES.get((st.get("scan_kernel", 0), False), "cq::scan_kernel"),
            "plan_sample": {"slow_records": st.get("slow_records"), "lds_spills": st.get("lds_spills")},
            "roofline_frac": nb / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "verified": verify(res, exp, 2), "verified_against": src}


if __name__ == "__main__":
    main()
