"""Same-process A/B of the config-5 rank share (bench_join.routed_share_leg's rank 0):
the routed 62.5 M + 62.5 M shard is built once, then each variant (a set of
environment knobs the library reads per call) is timed over the same steps.
    python scripts/r5_join_ab.py '[{}, {"CQGPU_PART_PROBE_SHIFT": "19"}, {"CQGPU_PART_PROBE_MIN": "1000000000"}]'
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_join as bj  # noqa: E402
import cq_amd  # noqa: E402
from cq_amd import abi  # noqa: E402


def main():
    variants = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [{}]
    n_total, N, steps = 500_000_000, 8, int(os.environ.get("AB_STEPS", "10"))
    dev = torch.device("cuda")
    P = abi.Plan()
    q = P.query([P.ident("u.role"), P.func("COUNT", P.lit("*")), P.func("SUM", P.ident("o.price"))],
                "users.csv", alias="u", group_by=["u.role"],
                joins=[("orders.csv", "o", P.cond("=", P.ident("u.id"), P.ident("o.customer_id")), abi.JOIN_INNER)])
    ast = C.pointer(q)
    uh, oh = b"id,name,age,role\n", b"id,price,quantity,customer_id\n"
    ub, ob, cnt, cents, first = bj.gen_config5_device(n_total, 42, dev)
    gids = torch.arange(n_total, dtype=torch.int64, device=dev)
    U = cq_amd.table_from_routed(ub.data_ptr(), ub.numel(), gids.data_ptr(), n_total, uh)
    O = cq_amd.table_from_routed(ob.data_ptr(), ob.numel(), gids.data_ptr(), n_total, oh)
    del ub, ob, gids
    torch.cuda.empty_cache()
    tabs = []
    for side, (tab, hdr) in enumerate(((U, uh), (O, oh))):
        nb, nr = cq_amd.route_plan(ast, [U, O], side, N)
        sb = torch.empty(max(sum(nb), 1), dtype=torch.uint8, device=dev)
        sg = torch.empty(max(sum(nr), 1), dtype=torch.int64, device=dev)
        cq_amd.route_fill(tab, 0, sb.data_ptr(), sg.data_ptr())
        torch.cuda.synchronize(dev)
        t = cq_amd.table_from_routed(sb.data_ptr(), int(nb[0]), sg.data_ptr(), int(nr[0]), hdr)
        cq_amd.table_set_record_total(t, n_total)
        cq_amd.table_set_key_stride(t, N)
        tabs.append(t)
        del sb, sg
    U.close()
    O.close()
    torch.cuda.empty_cache()
    for rnd in range(2):
        for v in variants:
            old = {k: os.environ.get(k) for k in v}
            os.environ.update(v)
            for _ in range(3):
                cq_amd.query_partial(ast, tabs)
            torch.cuda.synchronize(dev)
            ms, t1 = [], time.perf_counter()
            for _ in range(steps):
                cq_amd.query_partial(ast, tabs)
                ms.append(cq_amd.stats()["scan_ms"])
            torch.cuda.synchronize(dev)
            step = (time.perf_counter() - t1) / steps * 1e3
            print(json.dumps({"round": rnd, "variant": v, "step_ms": round(step, 4),
                              "scan_ms": round(float(np.mean(ms)), 4), "kind": cq_amd.stats()["scan_kernel"]}),
                  flush=True)
            for k, o in old.items():
                if o is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = o


if __name__ == "__main__":
    main()
