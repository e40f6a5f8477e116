#!/usr/bin/env python3
"""Benchmark: rows/s of cq's SELECT hot path (CSV scan + WHERE + GROUP BY) on MI355X.

Workload (BASELINE.json configs[2] per GPU; configs[3] shape when N > 1):
  synthetic Shape A+role CSV (reference utils/generate_big_dataset.py columns +
  role_%03d, 1,000 groups), 100M rows per GPU, resident in HBM, and
      SELECT role, COUNT(*), SUM(height), AVG(height) FROM 'big.csv'
      WHERE age > 30 GROUP BY role
One step = one full query over the resident bytes: the fused scan kernel
(tokenize + type + filter + LDS hash aggregate), compaction, first-row gather,
result materialisation; with N > 1 each rank scans its own row-range shard of
one N x 100M-row file, partial group states are exchanged over RCCL
(torch.distributed all_gather) and merged on rank 0 (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints one JSON line (rank 0) with roofline (scan kernel HBM bytes/s vs 8 TB/s)
and a CPU baseline: the unmodified reference (oracle/_ref/ref_probe built from
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

import torch  # first: libcqgpu binds to the HIP runtime torch loads

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rows/sec scanned (filter+GROUP BY) at 1/2/4/8 GPUs; % of HBM read peak"
QUERY = ("SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{path}' "
         "WHERE age > 30 GROUP BY role")
# --config 2 (not the bench line; a measurement of BASELINE configs[1]):
# Shape A without role, filter + COUNT
QUERY2 = "SELECT COUNT(*) FROM '{path}' WHERE age > 30"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000, help="data rows per GPU")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-rows", type=int, default=8_000_000,
                    help="rows of the CPU-baseline sample (reference evaluator)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "hbm_traffic.json"))
    ap.add_argument("--config", type=int, default=3, choices=(2, 3),
                    help="3: the bench line (filter + GROUP BY); 2: Shape A filter + COUNT")
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


def cpu_baseline(rows, seed, config=3):
    """Reference evaluator (single-threaded C, -O2) on a bounded sample, 1 core."""
    from cq_amd import datagen
    probe = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
    kind = "reference"
    if not os.path.exists(probe):
        return None
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "sample.csv")
        datagen.write_shape_a(path, rows, seed=seed, with_role=config == 3)
        query = (QUERY if config == 3 else QUERY2).format(path=path)
        out = subprocess.run(["taskset", "-c", "0", probe, "time", query], capture_output=True, timeout=600)
        if out.returncode != 0:
            out = subprocess.run([probe, "time", query], capture_output=True, timeout=600)
        res = json.loads(out.stdout.decode())
    secs = res["seconds"]
    return {"value": rows / secs, "unit": "rows/s", "cores": 1, "kind": kind,
            "sample": f"{rows} rows of the same workload (same generator, seed {seed}); "
                      f"reference parse+evaluate_query wall time incl. csv_load = {secs:.2f} s",
            "seconds": secs, "host_cores": os.cpu_count()}


def main():
    args = parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    torch.cuda.set_device(local)
    torch.zeros(1, device="cuda")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import cq_amd
    from cq_amd import abi, datagen
    from cq_amd.dist import gather_blobs
    cq_amd.lib()

    # ---- synthetic shard of this rank (one N x rows file, row-range partitioned)
    t0 = time.time()
    role = args.config == 3
    header = b"name,surname,age,gender,height,role\n" if role else b"name,surname,age,gender,height\n"
    import numpy as np
    rng = np.random.default_rng([args.seed, rank])
    chunks = []
    left = args.rows
    while left > 0:
        n = min(1 << 22, left)
        chunks.append(datagen.shape_a_chunk(rng, n, role))
        left -= n
    body = b"".join(chunks)
    del chunks
    shard = header + body if rank == 0 else body
    sizes = [len(shard)]
    if dist is not None:
        allsz = [None] * world
        dist.all_gather_object(allsz, len(shard))
        sizes = allsz
    base = sum(sizes[:rank])
    table = cq_amd.Table.from_bytes(shard, abi.csv_config(), base_offset=base,
                                    header=None if rank == 0 else header)
    nbytes = len(shard)
    del body, shard
    gen_s = time.time() - t0

    P, q = build_plan("big.csv", args.config)
    ast = C.pointer(q)
    L = cq_amd.lib()

    kernel_used = [1]

    def step():
        if dist is None:
            tp = L.cqgpu_query(ast, (C.c_void_p * 1)(table.handle.value), 1)
            if not tp:
                raise RuntimeError(cq_amd.last_error())
            ng = tp.contents.nrows
            cq_amd.result_free(tp)
            st = cq_amd.stats()
            if os.environ.get("CQ_BENCH_DEBUG"):
                print("stats", st, file=sys.stderr)
            kernel_used[0] = st.get("scan_kernel", 0)
            return ng, st["scan_ms"]
        blob = C.c_void_p()
        n = L.cqgpu_query_partial(ast, (C.c_void_p * 1)(table.handle.value), 1, C.byref(blob))
        if n == 0:
            raise RuntimeError(cq_amd.last_error())
        scan_ms = cq_amd.stats()["scan_ms"]
        mine = C.string_at(blob, n)
        C.CDLL(None).free(blob)
        blobs = gather_blobs(mine, device=torch.device("cuda", local))
        ng = 0
        if rank == 0:
            tp = cq_amd.merge_partials(ast, blobs)
            if not tp:
                raise RuntimeError(cq_amd.last_error())
            ng = tp.contents.nrows
            cq_amd.result_free(tp)
        return ng, scan_ms

    ng = None
    for _ in range(args.warmup):
        ng, _ = step()
    want_groups = 1000 if role else 1
    if rank == 0 and ng is not None and ng != want_groups:
        print(f"warning: {ng} groups (expected {want_groups})", file=sys.stderr)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    scan_ms = []
    barrier()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        _, ms = step()
        scan_ms.append(ms)
    barrier()
    elapsed = time.perf_counter() - t1
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    rows_total = args.rows * world
    value = rows_total / (elapsed / args.steps)

    if rank == 0:
        avg_scan_ms = sum(scan_ms) / len(scan_ms)
        achieved = nbytes / (avg_scan_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic) as fh:
                tj = json.load(fh)
            if tj.get("rows") == args.rows:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            pass
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic: Shape A+role CSV (generate_big_dataset.py columns + role_%03d, "
                     if role else "synthetic: Shape A CSV (generate_big_dataset.py columns, ")
                    + f"seed {args.seed}), resident in HBM before timing",
            "config": {
                "workload": ("config3 per GPU: SELECT role, COUNT(*), SUM(height), AVG(height) "
                             "FROM 'big.csv' WHERE age > 30 GROUP BY role" if role else
                             "config2 per GPU: SELECT COUNT(*) FROM 'big.csv' WHERE age > 30"),
                "rows_per_gpu": args.rows,
                "bytes_per_gpu": nbytes,
                "groups": want_groups,
                "parallelism": f"dp{world} (newline-snapped row ranges, RCCL all_gather of partials)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": (("cq::lean::lean_kernel<true, LW_NUM, 1> (+ slow_kernel, raw_merge_kernel)" if role
                            else "cq::lean::lean_kernel<false, LW_NUM, 0> (+ slow_kernel)")
                           if kernel_used[0] else "cq::scan_kernel"),
                "kernel_ms": avg_scan_ms,
                "bytes_per_launch": nbytes,
            },
            "cpu_baseline": cpu,
            "setup_s": gen_s,
        }
        print(json.dumps(line), flush=True)
    table.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
