#!/usr/bin/env python3
"""Golden answers of the UNMODIFIED reference at 1e6 rows (no-WHERE plans).

Run in the build container (needs the reference built by oracle/ref.mk, ~1 GB of
RAM, ~15 s):   python tests/golden/make_mid_golden.py

Writes rows [0, 1e6) of the logical Shape A file (cq_amd/datagen.py, seed 42 --
the same bytes the GPU test regenerates) and runs oracle/_ref/ref_probe on the
queries below.  `SELECT COUNT(*) FROM f` with no WHERE is the plan with no
column role at all (fast_kernel's NR = 0 instantiation).

Writes tests/golden/mid.json.
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from cq_amd import datagen  # noqa: E402

PROBE = os.path.join(REPO, "oracle", "_ref", "ref_probe")
ROWS = 1_000_000
SEED = 42
QUERIES = [
    "SELECT COUNT(*) FROM '{p}'",
    "SELECT COUNT(*), SUM(height), AVG(height) FROM '{p}'",
    "SELECT name, COUNT(*) FROM '{p}' GROUP BY name",
]


def main():
    if not os.path.exists(PROBE):
        sys.exit("build the reference first: make -f oracle/ref.mk")
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "mid.csv")
        size = datagen.write_logical(path, ROWS, SEED, with_role=False)
        out = {"rows": ROWS, "seed": SEED, "with_role": False, "bytes": size, "queries": []}
        for q in QUERIES:
            r = subprocess.run([PROBE, "query", q.format(p=path)], capture_output=True, check=True, timeout=300)
            out["queries"].append({"sql": q, "result": json.loads(r.stdout.decode("latin-1"))})
    with open(os.path.join(HERE, "mid.json"), "w") as fh:
        json.dump(out, fh, indent=0)
    print(f"wrote tests/golden/mid.json ({len(out['queries'])} queries over {ROWS} rows, {size} bytes)")


if __name__ == "__main__":
    main()
