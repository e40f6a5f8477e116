"""Worker for tests/test_gpu_dist_rccl.py (run under torch.distributed.run): the
library's own RCCL communicator (cq_amd.dist.init_library_comm) -- or, with
CQ_TEST_HOST_COMM=1, its host-staged test backend over gloo (init_host_comm, ranks
sharing one GPU) -- then every query
of argv through cqgpu_dist_query on this rank's range shard; rank 0 writes the
results (and the merge path each took) as JSON to the output file."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    out, items = sys.argv[1], json.loads(sys.argv[2])     # items: [[sql, path], ...]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    host = os.environ.get("CQ_TEST_HOST_COMM") == "1"
    if host:
        # the library's collectives through its host-staged test backend over gloo:
        # every rank on the one GPU of the box (RCCL would refuse a shared device)
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import cqtest
    import cq_amd
    from cq_amd import abi
    from cq_amd.dist import init_host_comm, init_library_comm
    if host:
        init_host_comm()
    else:
        init_library_comm()
    # failure injection on one rank only: CQ_TEST_RANK_ENV="<rank>:<NAME>=<value>"
    spec = os.environ.get("CQ_TEST_RANK_ENV", "")
    if spec:
        r, kv = spec.split(":", 1)
        if int(r) == rank:
            k, v = kv.split("=", 1)
            os.environ[k] = v
    results = []
    for sql, path in items:
        # path: one file (cqgpu_dist_query over its range shard), or a JOIN's files
        # [FROM, JOIN, later chain tables] (cqgpu_dist_join: range shards of the first
        # two, the chain's tables whole); the SQL names them {p}, {q}, {r}, ...
        paths = path if isinstance(path, list) else [path]
        text = sql.format(**dict(zip("pqrs", paths)))
        print(f"dist worker: {text}", file=sys.stderr, flush=True)   # (a failure names its query)
        tabs = [cq_amd.Table.open_range(x, rank, world) if i < 2 else cq_amd.Table.open(x)
                for i, x in enumerate(paths)]
        t = tabs[0]
        with cqtest.Parsed(text) as ast:
            got = None
            for _ in range(2):                      # a warm-up step, then the kept one
                if len(paths) > 1:
                    tp, status = cq_amd.dist_join_raw(ast, tabs)
                    p = 0
                else:
                    tp, status, p = cq_amd.dist_query_raw(ast, t)
                if got is not None or status != 0:
                    break
                if tp:
                    got = abi.table_to_py(tp)
                    cq_amd.result_free(tp)
                else:
                    got = "none"
            results.append({"sql": sql, "status": status, "path": p, "error": cq_amd.last_error(),
                            "kernel": cq_amd.stats().get("scan_kernel"),
                            "result": None if got in (None, "none") else
                            {"columns": got["columns"], "rows": [[list(c) for c in r] for r in got["rows"]]}})
        for x in tabs:
            x.close()
    cq_amd.comm_destroy()
    with open(f"{out}.{rank}", "w") as fh:         # every rank's statuses and errors
        json.dump([{"status": r["status"], "error": r["error"]} for r in results], fh)
    if rank == 0:
        with open(out, "w") as fh:
            json.dump(results, fh, default=lambda b: b.decode("latin-1") if isinstance(b, bytes) else str(b))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
