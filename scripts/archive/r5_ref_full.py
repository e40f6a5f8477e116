"""The reference evaluator (oracle/_ref/ref_probe, built from the reference's own
sources) on the full 1e8-row config-3 file, one core, on the GPU box's host: the
same-box CPU baseline the bench's bounded sample stands in for.
    python scripts/r5_ref_full.py out.json [--rows N]"""
import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cq_amd import datagen  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--rows", type=int, default=100_000_000)
a = ap.parse_args()
mem = {}
for line in open("/proc/meminfo"):
    k, v = line.split(":", 1)
    if k in ("MemTotal", "MemAvailable"):
        mem[k] = int(v.split()[0]) * 1024
model = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), platform.processor())
probe = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
with tempfile.TemporaryDirectory(dir="/tmp") as d:
    path = os.path.join(d, "big.csv")
    t0 = time.time()
    datagen.write_logical(path, a.rows, seed=42, with_role=True)
    gen_s = time.time() - t0
    print(json.dumps({"generated_s": round(gen_s, 1), "bytes": os.path.getsize(path)}), flush=True)
    q = bench.QUERY.format(path=path)
    # progress lines while the single-threaded reference runs (a silent minute looks hung)
    p = subprocess.Popen(["taskset", "-c", "0", probe, "time", q], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    t0 = time.time()
    while p.poll() is None:
        time.sleep(30)
        print(json.dumps({"reference_running_s": round(time.time() - t0)}), flush=True)
    out, err = p.communicate()
    if p.returncode != 0:
        print(err.decode()[-2000:], file=sys.stderr)
        sys.exit(1)
    res = json.loads(out.decode())
doc = {"rows": a.rows, "query": bench.QUERY.format(path="big.csv"), "reference_seconds": res["seconds"],
       "rows_per_s": a.rows / res["seconds"], "cores": 1, "kind": "reference",
       "host": {"cpu_model": model, "logical_cpus": os.cpu_count(), "mem_total_bytes": mem.get("MemTotal"),
                "mem_available_bytes": mem.get("MemAvailable")},
       "how": "oracle/_ref/ref_probe (the reference's parser + evaluate_query built from its own sources) under "
              "taskset -c 0 on the GPU box's host, config 3's 1e8-row file generated there (seed 42)"}
json.dump(doc, open(a.out, "w"), indent=1)
print(json.dumps(doc))
