"""one-off: which kernel runs for the fast-shape test query, and parity vs the oracle"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import tempfile
import cqtest, cq_amd
rng = np.random.default_rng(1)
rows = ["n%d,s,%d,%s,%d.%02d,role_%03d" % (i % 7, rng.integers(10, 81), "fm"[i % 2], rng.integers(1, 3),
                                            rng.integers(0, 100), rng.integers(0, 1000)) for i in range(200_000)]
d = tempfile.mkdtemp()
p = os.path.join(d, "bench.csv")
open(p, "w").write("name,surname,age,gender,height,role\n" + "\n".join(rows) + "\n")
for sql in [f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM '{p}' WHERE age > 30 GROUP BY role",
            f"SELECT COUNT(*) FROM '{p}' WHERE age > 30"]:
    for mode in (0, 2):
        cq_amd.set_scan_kernel(mode)
        with cqtest.Parsed(sql) as ast:
            got = cq_amd.evaluate(ast)
        st = cq_amd.stats()
        want, _ = cqtest.oracle_query(sql)
        ok = got["rows"][:3] == want["rows"][:3]
        print(mode, st, "groups", len(got["rows"]), len(want["rows"]), "first rows equal:", ok, got["rows"][:2], want["rows"][:2], flush=True)
