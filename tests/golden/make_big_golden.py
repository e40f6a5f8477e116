#!/usr/bin/env python3
"""Golden answers at the benchmarked sizes.

Run in the build container (needs the reference built by oracle/ref.mk, ~40 GB
of RAM and ~10 minutes):   python tests/golden/make_big_golden.py

1. Writes rows [0, 1e8) of the logical Shape A+role file (cq_amd/datagen.py,
   seed 42) and runs the UNMODIFIED reference (oracle/_ref/ref_probe query) on
   config 3's query; the same for Shape A (no role) and config 2's query.
2. Computes the same answers from the generator's draws
   (datagen.expected_filter_groupby) and checks that the reference agrees:
   group set and first-appearance order and COUNT exact, SUM within 1e-9
   relative of the exact hundredths.
3. Computes config 4's answer (rows [0, 1e9), too large for the reference's
   ~335 GB of RSS) from the draws alone -- pinned to the reference by step 2.

Writes tests/golden/big.json (what bench.py checks its result against).
"""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from cq_amd import datagen  # noqa: E402

PROBE = os.path.join(REPO, "oracle", "_ref", "ref_probe")
SEED = 42
Q3 = "SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role"
Q2 = "SELECT COUNT(*) FROM '{p}' WHERE age > 30"


def run_ref(query):
    t0 = time.time()
    out = subprocess.run([PROBE, "query", query], capture_output=True, check=True)
    return json.loads(out.stdout.decode()), time.time() - t0


def check(ref, exp, grouped):
    rows = ref["rows"]
    assert len(rows) == len(exp["count"]), (len(rows), len(exp["count"]))
    for i, r in enumerate(rows):
        if grouped:
            assert r[0] == {"t": "S", "v": exp["groups"][i]}, (i, r[0], exp["groups"][i])
            assert r[1] == {"t": "I", "v": exp["count"][i]}, (i, r[1], exp["count"][i])
            s = float(r[2]["v"])
            want = exp["sum_cents"][i] / 100.0
            assert abs(s - want) <= 1e-9 * want, (i, s, want)
        else:
            assert r[0] == {"t": "I", "v": exp["count"][0]}, (r, exp)


def main(rows=100_000_000, big_rows=1_000_000_000, tmp="/tmp"):
    out = {"seed": SEED, "generator": "cq_amd/datagen.py logical file (chunks of %d rows, "
           "chunk k drawn from default_rng([seed, k]))" % datagen.CHUNK_ROWS}
    for cfg, role, q in ((3, True, Q3), (2, False, Q2)):
        path = os.path.join(tmp, f"cq_big_config{cfg}.csv")
        size = datagen.write_logical(path, rows, SEED, with_role=role)
        print(f"config {cfg}: {rows} rows, {size} bytes; running the reference ...", flush=True)
        ref, secs = run_ref(q.format(p=path))
        os.unlink(path)
        exp = datagen.expected_filter_groupby(SEED, 0, rows, with_role=role)
        check(ref, exp, role)
        print(f"config {cfg}: reference {secs:.1f} s, agrees with the generator's draws", flush=True)
        out[f"config{cfg}"] = {"rows": rows, "bytes": size, "query": q, "reference": ref,
                               "reference_seconds": round(secs, 2), "expected": exp}
    exp4 = datagen.expected_filter_groupby(SEED, 0, big_rows, with_role=True)
    out["config4"] = {"rows": big_rows, "query": Q3, "expected": exp4,
                      "note": "from the generator's draws; pinned to the reference by config3"}
    with open(os.path.join(HERE, "big.json"), "w") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote tests/golden/big.json")


if __name__ == "__main__":
    main()
