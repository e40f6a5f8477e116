"""The fused aggregate join (executor.hip run_fast_join, fast.hip jx_* kernels) against
the oracle's nested-loop join (reference evaluator_joins.c:63-181 feeding
evaluate_aggregate): counts, group sets and first-pair order exact, SUM/AVG within
1e-6 relative.  Each case also checks which path ran: stats()["scan_kernel"] == 3 is
the fused path; shapes it must decline (a quote, a short row, a non-canonical key, a
wide numeral) still give the oracle's answer through the general pipeline.
"""
import numpy as np
import pytest

import cqtest
import cq_amd
from test_gpu_parity import compare, tolerant_columns

pytestmark = pytest.mark.gpu


def _run(sql):
    want, unsup = cqtest.oracle_query(sql)
    assert not unsup, sql
    with cqtest.Parsed(sql) as ast:
        got = cq_amd.evaluate(ast)
        assert not cq_amd.last_ineligible(), (sql, cq_amd.last_ineligible())
        tol = tolerant_columns(ast)
    compare(got, want, tol, sql)
    return cq_amd.stats()["scan_kernel"]


def _write(tmp_path, name, header, rows):
    p = tmp_path / name
    p.write_text(header + "\n" + "\n".join(rows) + "\n")
    return str(p)


@pytest.fixture(scope="module")
def tables(tmp_path_factory):
    d = tmp_path_factory.mktemp("fj")
    rng = np.random.default_rng(3)
    f = {}
    # dense primary keys (the direct table), shuffled order
    ids = rng.permutation(4000) + 1000
    f["u"] = _write(d, "u.csv", "id,name,age,role",
                    [f"{i},n{i % 91},{18 + i % 60},role_{int(rng.integers(0, 40)):02d}" for i in ids])
    f["o"] = _write(d, "o.csv", "id,price,quantity,customer_id",
                    [f"{j},{rng.integers(100, 99999) / 100:.2f},{rng.integers(1, 9)},{int(rng.integers(900, 5100))}"
                     for j in range(6000)])
    # sparse keys with repeats on the build side (the hash table, many-to-many pairs)
    # (11-12 digits: keys of 8-10 digits may type as DATEs and take the general join)
    hot = [int(x) for x in rng.integers(10**10, 10**12, 700)]
    f["us"] = _write(d, "us.csv", "id,role",
                     [f"{hot[i % 700] if i % 3 == 0 else int(rng.integers(10**10, 10**12))},r{int(rng.integers(0, 7))}"
                      for i in range(3000)]
                     + [f"{10**11 + k},dup{k % 3}" for k in range(50) for _ in range(3)])
    f["os"] = _write(d, "os.csv", "k,v",
                     [f"{10**11 + k},{int(rng.integers(0, 100))}" for k in range(60)]
                     + [f"{hot[i % 700] if i % 2 else int(rng.integers(10**10, 10**12))},{i % 17}" for i in range(2000)])
    # NULL keys on both sides (NULL = NULL pairs), empty and decimal values, numeric group keys
    f["un"] = _write(d, "un.csv", "id,g",
                     [f"{'' if i % 13 == 0 else i},{['1', '01', '1.0', '', 'x'][i % 5]}" for i in range(500)])
    f["on"] = _write(d, "on.csv", "cid,amt",
                     [f"{'' if i % 11 == 0 else int(rng.integers(0, 520))},{['', '1.5', '2', '3.125', '-4'][i % 5]}"
                      for i in range(1500)])
    # shapes the fused path declines
    f["uq"] = _write(d, "uq.csv", "id,role", [f"{i},\"r,{i % 3}\"" for i in range(200)])
    f["uz"] = _write(d, "uz.csv", "id,role", [f"{i:04d},r{i % 3}" for i in range(200)])      # leading zeros
    f["ow"] = _write(d, "ow.csv", "cid,amt", [f"{i % 200},{i * 1234.5678:.4f}" for i in range(600)])
    f["ud"] = _write(d, "ud.csv", "id,role", [f"{20240100 + i},r{i % 3}" for i in range(40)] +
                     [f"{i + 1000},q{i % 2}" for i in range(300)])          # 8-digit keys: DATE-shaped
    return f


FUSED = [
    ("u", "o", "SELECT u.role, COUNT(*), SUM(o.price), AVG(o.price) FROM '{L}' AS u JOIN '{R}' AS o "
               "ON u.id = o.customer_id GROUP BY u.role"),
    ("u", "o", "SELECT COUNT(*), SUM(o.quantity) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id"),
    ("u", "o", "SELECT u.name, COUNT(*), AVG(o.price) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id "
               "GROUP BY u.name HAVING COUNT(*) > 60 ORDER BY u.name"),
    ("u", "o", "SELECT u.age, u.role, COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id GROUP BY u.age"),
    ("us", "os", "SELECT u.role, COUNT(*), SUM(o.v) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.k GROUP BY u.role"),
    ("us", "os", "SELECT COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.k"),
    ("un", "on", "SELECT u.g, COUNT(*), SUM(o.amt), AVG(o.amt) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.cid GROUP BY u.g"),
    ("un", "on", "SELECT COUNT(*), SUM(o.amt) FROM '{L}' AS u JOIN '{R}' AS o ON o.cid = u.id"),
]
DECLINED = [
    ("uq", "o", "SELECT u.role, COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id GROUP BY u.role"),
    ("uz", "o", "SELECT u.role, COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id GROUP BY u.role"),
    ("u", "ow", "SELECT u.role, SUM(o.amt) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.cid GROUP BY u.role"),
    ("ud", "o", "SELECT u.role, COUNT(*) FROM '{L}' AS u JOIN '{R}' AS o ON u.id = o.customer_id GROUP BY u.role"),
]


@pytest.mark.parametrize("case", range(len(FUSED)))
def test_fused_join(tables, case):
    lk, rk, tmpl = FUSED[case]
    sql = tmpl.replace("{L}", tables[lk]).replace("{R}", tables[rk])
    kind = _run(sql)
    # "ON o.cid = u.id" resolves each operand against its own side first (the ON quirk)
    assert kind == 3 or "o.cid = u.id" in sql, (sql, kind)


@pytest.mark.parametrize("case", range(len(DECLINED)))
def test_declined_shapes_match_oracle(tables, case):
    lk, rk, tmpl = DECLINED[case]
    sql = tmpl.replace("{L}", tables[lk]).replace("{R}", tables[rk])
    assert _run(sql) != 3, sql
