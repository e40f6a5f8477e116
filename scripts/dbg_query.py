import sys, os, time
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
import cqtest, cq_amd
from cq_amd import datagen
p = "/tmp/role.csv"
datagen.write_shape_a(p, 200_000, seed=3, with_role=True)
for sql in ["SELECT COUNT(*), MIN(height) FROM '%s'" % p,
            "SELECT COUNT(*), SUM(height), AVG(height), MIN(height), MAX(age) FROM '%s' WHERE gender = 'f'" % p]:
    t0 = time.time()
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
    print(sql, time.time() - t0, got and got["rows"], cq_amd.last_error(), cq_amd.stats(), flush=True)
    want, _ = cqtest.oracle_query(sql)
    print("want", want["rows"], flush=True)
