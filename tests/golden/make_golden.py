#!/usr/bin/env python3
"""Regenerate the golden vectors in tests/golden/ from the UNMODIFIED reference.

Run in the build container (needs /root/reference and the reference build from
oracle/ref.mk):   python tests/golden/make_golden.py

Writes:
  data/*.csv          input fixtures: the reference's own data/*.csv files,
                      our adversarial edge-case CSVs and small seeded synthetic
                      files of the benchmark shapes (cq_amd/datagen.py)
  abi_layout.json     sizeof/offsetof of the reference ABI types
  cells.json          typed cells csv_load produces for every data/*.csv
  queries.json        parse + evaluate_query results for the query corpus
Every expected output here was computed by the reference itself
(oracle/_ref/ref_probe linked with oracle/_ref/libcqref.so).
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from cq_amd import datagen  # noqa: E402

REF = os.environ.get("CQ_REFERENCE", "/root/reference")
PROBE = os.path.join(REPO, "oracle", "_ref", "ref_probe")
DATA = os.path.join(HERE, "data")

# ---------------------------------------------------------------- edge CSVs
EDGE = {
    # typing: infer_type / parse_value (csv_reader.c:133-240)
    "edge_numbers.csv": (
        b"a,b,c,d\n"
        b"+5,-0,.5,1.\n"
        b".,-,1e5,12345678901234567890\n"
        b"-99999999999999999999, 7 ,\"8\",\"  9  \"\n"
        b"1.2.3,+-1,--1,0.0000001\n"
        b"3.14159265358979323846,1e-5,123.,-.5\n"
        b"00042,-007.50,9007199254740993,0.1\n"
        b"179769313486231570000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000.0,4.9e-324,0.000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000049,2.2250738585072011e-308\n"
        b"123456789.123456789,0.30000000000000004,7.0,-0.0\n"
        b"2.5,1.0000005,1.0000015,-1.0000005\n"
    ),
    # dates: parse_date (date_utils.c:26-100) tried for 8..10-char cells
    "edge_dates.csv": (
        b"d1,d2,d3,d4\n"
        b"2024-01-15,1/2/2024,13/12/2024,20240115\n"
        b"2024-1-5x,20240115.5,2024-02-30,2023-02-29\n"
        b"2024-02-29,12345678,99999999,\"2024-03-01\"\n"
        b" 2024-01-05 ,2024- 1- 5,  20240101,0999-01-01\n"
        b"1900-02-29,2000-02-29,12/31/1999,31/12/1999\n"
        b"+2024-1-1,2024-+1-+1,20241301,1000-01-01\n"
        b"9999-12-31,10000-1-1,2024/01/15,2024.01.15\n"
        b"19991231,1999123,199912310,-2024-1-1\n"
    ),
    # quotes: parse_line quoted-field handling (csv_reader.c:294-317)
    "edge_quotes.csv": (
        b"q1,q2,q3,q4\n"
        b"\"a,b\",c\"\"d,\"e\"\"f\",\"g\"h\n"
        b"\"\",\"\"\"\",\"x\"\"\"\"y\",z\n"
        b"\"12\",\" 13 \",\"1.5\",\"2024-01-01\"\n"
        b"\"12\"\"\",p,q,\"unclosed,tail\n"
        b"\"1234\"\"\",\"1.5\"\"\",r,s\n"
        b"  \"lead\" ,\"trail\"  ,  plain  ,\"a\"\"b\"\"c\"\n"
    ),
    # composite GROUP BY text parts holding a tab (evaluator.c:124 joins parts with '\t')
    "edge_tabs.csv": (
        b"t1,t2,t3,n\n"
        b"a\tb,c,x,1\n"
        b"a,b\tc,x,2\n"
        b"a,b,c,3\n"
        b"a\tb,c,y,4\n"
        b"p\tq\tr,s,x,5\n"
        b"p,q\tr\ts,x,6\n"
        b"p\tq,r\ts,x,7\n"
        b"a,b,c,8\n"
        b"1\t2,3,x,9\n"
        b"1,2\t3,x,10\n"
    ),
    # whitespace and field splitting (csv_reader.c:285-338)
    "edge_ws.csv": (
        b"w1,w2,w3,w4\n"
        b" a , b ,c,d\n"
        b"\tx\t,\x0by\x0b,\x0cz\x0c,end\n"
        b"1 2,3 ,  4,5\n"
        b",,x,\n"
        b"p,q,r,   \n"
        b"p2,q2,r2,s2,extra\n"
        b"high\xe9,\xff\xfe,mid\x80dle,ok\n"
    ),
    # records: any \n or \r ends a record; blank lines vanish (csv_reader.c:404-427)
    "edge_lines.csv": (
        b"\r\n\n id , name ,score\r\n"
        b"1,a,10\r\n"
        b"\r\n"
        b"2,b,20\r"
        b"3,c,30\n\n\n"
        b"4,d,40\r\r\n"
        b"5,e,50"
    ),
}


def wide_bytes(rows=600, seed=12):
    """12 columns (more than a fused scan's 8 need slots): ints, decimals, short
    strings, a key column, NULL (empty) cells in c10"""
    import numpy as np
    rng = np.random.default_rng(seed)
    out = ["c0,c1,c2,c3,c4,c5,c6,c7,c8,c9,c10,c11"]
    for i in range(rows):
        c = [str(int(rng.integers(0, 100))) for _ in range(4)]
        c.append("%d.%02d" % (rng.integers(0, 9), rng.integers(0, 100)))
        c.append(["x", "yy", "zz", "w w", "alpha"][int(rng.integers(0, 5))])
        c += [str(int(rng.integers(-50, 1000))) for _ in range(3)]
        c.append("k%d" % rng.integers(0, 7))
        c.append("" if rng.integers(0, 30) == 0 else str(int(rng.integers(0, 5000))))
        c.append("%d.%d" % (rng.integers(0, 300), rng.integers(0, 10)))
        out.append(",".join(c))
    return ("\n".join(out) + "\n").encode()


def write_fixtures():
    os.makedirs(DATA, exist_ok=True)
    for f in sorted(os.listdir(os.path.join(REF, "data"))):
        if f.endswith(".csv"):
            shutil.copyfile(os.path.join(REF, "data", f), os.path.join(DATA, f))
    for name, body in EDGE.items():
        with open(os.path.join(DATA, name), "wb") as fh:
            fh.write(body)
    with open(os.path.join(DATA, "synth_role.csv"), "wb") as fh:
        fh.write(datagen.shape_a_bytes(3000, seed=7, with_role=True))
    with open(os.path.join(DATA, "synth_a.csv"), "wb") as fh:
        fh.write(datagen.shape_a_bytes(3000, seed=8, with_role=False))
    with open(os.path.join(DATA, "synth_users.csv"), "wb") as fh:
        fh.write(datagen.users_bytes(1500, seed=9))
    with open(os.path.join(DATA, "synth_orders.csv"), "wb") as fh:
        fh.write(datagen.orders_bytes(2500, 1800, seed=10))
    with open(os.path.join(DATA, "synth_wide.csv"), "wb") as fh:
        fh.write(wide_bytes())


# ---------------------------------------------------------------- query corpus
T = "'{D}/test_data.csv'"
U = "'{D}/users.csv'"
O = "'{D}/orders.csv'"
R = "'{D}/synth_role.csv'"
A = "'{D}/synth_a.csv'"
SU = "'{D}/synth_users.csv'"
SO = "'{D}/synth_orders.csv'"
P = "'{D}/products.csv'"
W = "'{D}/synth_wide.csv'"
WIDE9 = "c0 > 5 AND c1 < 95 AND c2 != 50 AND c3 >= 3 AND c4 > 0.5 AND c5 != 'yy' AND c6 < 900 AND c7 > -40 AND c8 > 0"
QUERIES = [
    # config 1 (plumbing) and filter + COUNT
    f"SELECT COUNT(*) FROM {T} WHERE age > 30",
    f"SELECT COUNT(*) FROM {T}",
    f"SELECT COUNT(*) FROM {T} WHERE age > 30 AND active = 1",
    f"SELECT COUNT(*) FROM {T} WHERE age < 20 OR age > 40",
    f"SELECT COUNT(*) FROM {T} WHERE role IN ('admin', 'moderator')",
    f"SELECT COUNT(*) FROM {T} WHERE age NOT IN (25, 30, 35)",
    f"SELECT COUNT(*) FROM {T} WHERE NOT (age > 20 AND age < 30)",
    f"SELECT COUNT(*) FROM {T} WHERE NOT NOT age > 30",
    f"SELECT COUNT(*) FROM {T} WHERE age % 2 = 0",
    f"SELECT COUNT(*) FROM {T} WHERE (age & 16) > 0",
    f"SELECT COUNT(*) FROM {T} WHERE (age | 1) > 30",
    f"SELECT COUNT(*) FROM {T} WHERE (age % 10) + (age / 10) > 5",
    f"SELECT COUNT(*) FROM {T} WHERE age * 2 > 30 * 2",
    f"SELECT COUNT(*) FROM {T} WHERE age BETWEEN 25 AND 35",
    f"SELECT COUNT(*) FROM {T} WHERE name BETWEEN 'Alice' AND 'Charlie'",
    f"SELECT COUNT(*) FROM {T} WHERE height > 170.0",
    f"SELECT COUNT(*) FROM {T} WHERE height >= 172",
    f"SELECT COUNT(*) FROM {T} WHERE role = 'user'",
    f"SELECT COUNT(*) FROM {T} WHERE role != 'user'",
    f"SELECT COUNT(*) FROM {T} WHERE role > 'b'",
    f"SELECT COUNT(*) FROM {T} WHERE age > 20 AND age < 40 OR role = 'admin'",
    f"SELECT COUNT(*) FROM {T} WHERE age = '30'",
    f"SELECT COUNT(*) FROM {T} WHERE nosuch = 1",
    f"SELECT COUNT(*) FROM {T} WHERE age > -5",
    f"SELECT COUNT(*) FROM {T} WHERE age + height > 200",
    f"SELECT COUNT(*) FROM {T} WHERE age / 0 = 1",
    f"SELECT COUNT(*) FROM {T} WHERE name LIKE '%a%'",
    f"SELECT COUNT(*) FROM {T} WHERE name ILIKE 'a%'",
    # aggregates without GROUP BY
    f"SELECT COUNT(*), SUM(height), AVG(height) FROM {T} WHERE age > 30",
    f"SELECT MIN(age), MAX(age), MIN(name), MAX(height) FROM {T}",
    f"SELECT COUNT(*), SUM(age), AVG(age) FROM {T} WHERE age > 100",
    f"SELECT MIN(age), MAX(role) FROM {T} WHERE age > 100",
    f"SELECT COUNT(name), COUNT(nosuch), SUM(nosuch) FROM {T}",
    f"SELECT STDDEV(height), MEDIAN(age) FROM {T}",
    f"SELECT SUM(role), AVG(role) FROM {T}",
    # GROUP BY (config 3 shape)
    f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM {T} WHERE age > 30 GROUP BY role",
    f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM {T} GROUP BY role",
    f"SELECT role, AVG(height) AS avg_height FROM {T} GROUP BY role",
    f"SELECT role, COUNT(*) AS count FROM {T} GROUP BY role",
    f"SELECT active, COUNT(*), MIN(age), MAX(age) FROM {T} GROUP BY active",
    f"SELECT height, COUNT(*) FROM {T} GROUP BY height",
    f"SELECT role, COUNT(*) FROM {T} GROUP BY role ORDER BY role",
    f"SELECT role, COUNT(*) FROM {T} GROUP BY role ORDER BY COUNT(*) DESC",
    f"SELECT role, SUM(age) FROM {T} GROUP BY role HAVING SUM(age) > 60",
    f"SELECT role, active, COUNT(*) FROM {T} GROUP BY role, active",
    f"SELECT role, COUNT(*) FROM {T} WHERE age > 100 GROUP BY role",
    f"SELECT role, COUNT(*) FROM {T} GROUP BY role LIMIT 2",
    f"SELECT nosuch, COUNT(*) FROM {T} GROUP BY nosuch",
    f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM {R} WHERE age > 30 GROUP BY role",
    f"SELECT role, COUNT(*), SUM(height), AVG(height) FROM {R} GROUP BY role ORDER BY role",
    f"SELECT gender, COUNT(*), MIN(height), MAX(height) FROM {R} GROUP BY gender",
    f"SELECT age, COUNT(*), AVG(height) FROM {R} WHERE gender = 'f' GROUP BY age",
    f"SELECT name, COUNT(*) FROM {A} WHERE age > 30 GROUP BY name",
    f"SELECT COUNT(*) FROM {A} WHERE age > 30",
    f"SELECT COUNT(*) FROM {R} WHERE age > 30",
    f"SELECT COUNT(*), SUM(height), MIN(age), MAX(age) FROM {R} WHERE age > 30",
    f"SELECT COUNT(*), AVG(height) FROM {R} WHERE age > 30",
    # edge typing through queries
    "SELECT COUNT(*) FROM '{D}/edge_numbers.csv' WHERE a > 0",
    "SELECT a, COUNT(*) FROM '{D}/edge_numbers.csv' GROUP BY a",
    "SELECT b, COUNT(*) FROM '{D}/edge_numbers.csv' GROUP BY b",
    "SELECT d, COUNT(*) FROM '{D}/edge_numbers.csv' GROUP BY d",
    "SELECT SUM(a), SUM(b), SUM(c), SUM(d) FROM '{D}/edge_numbers.csv'",
    "SELECT MIN(a), MAX(a), MIN(b), MAX(b) FROM '{D}/edge_numbers.csv'",
    "SELECT MIN(d), MAX(d) FROM '{D}/edge_numbers.csv'",
    "SELECT d1, COUNT(*) FROM '{D}/edge_dates.csv' GROUP BY d1",
    "SELECT COUNT(*) FROM '{D}/edge_dates.csv' WHERE d1 > '2024-01-01'",
    "SELECT q1, COUNT(*) FROM '{D}/edge_quotes.csv' GROUP BY q1",
    "SELECT q2, q3 FROM '{D}/edge_quotes.csv'",
    "SELECT w1, w2, w3, COUNT(*) FROM '{D}/edge_ws.csv' GROUP BY w1, w2, w3",
    "SELECT COUNT(*), SUM(score) FROM '{D}/edge_lines.csv' WHERE score >= 20",
    "SELECT name, COUNT(*) FROM '{D}/edge_lines.csv' GROUP BY name",
    # joins (config 5 shape)
    f"SELECT COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id",
    f"SELECT u.name, o.price FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id",
    f"SELECT u.role, COUNT(*), SUM(o.price) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id GROUP BY u.role",
    f"SELECT COUNT(*) FROM {U} AS u JOIN {O} AS o ON o.customer_id = u.id",
    f"SELECT COUNT(*) FROM {U} AS u LEFT JOIN {O} AS o ON u.id = o.customer_id",
    f"SELECT COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id WHERE o.price > 60",
    f"SELECT COUNT(*) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id",
    f"SELECT u.role, COUNT(*), SUM(o.price) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id GROUP BY u.role",
    f"SELECT COUNT(*), SUM(o.price), AVG(o.quantity) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id WHERE u.age > 40",
    # JOIN without ON (parser_clauses.c:315-318 makes ON optional; evaluate_join_condition
    # is true for a NULL condition, evaluator_joins.c:42): the cross product
    f"SELECT COUNT(*) FROM {U} AS u JOIN {O} AS o",
    f"SELECT u.name, o.price FROM {U} AS u JOIN {O} AS o WHERE o.price > 100",
    f"SELECT u.role, COUNT(*), SUM(o.price) FROM {U} AS u JOIN {O} AS o GROUP BY u.role",
    f"SELECT COUNT(*), SUM(o.quantity) FROM {U} AS u LEFT JOIN {O} AS o WHERE u.age > 30",
    f"SELECT COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p",
    f"SELECT p.category, COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p GROUP BY p.category",
    # join chains (process_joins, evaluator_joins.c:237-274: level 2 joins "joined")
    f"SELECT COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p ON o.id = p.id",
    f"SELECT p.name, p.category, o.price FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p ON o.id = p.id",
    f"SELECT p.category, COUNT(*), SUM(p.id), MAX(o.price) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p ON o.id = p.id GROUP BY p.category",
    f"SELECT COUNT(*) FROM {U} AS u LEFT JOIN {O} AS o ON u.id = o.customer_id LEFT JOIN {P} AS p ON o.id = p.id",
    f"SELECT COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id RIGHT JOIN {P} AS p ON o.id = p.id",
    f"SELECT COUNT(*), SUM(p.id) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p ON o.id = p.id WHERE p.id > 2",
    f"SELECT COUNT(*) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id JOIN {SU} AS v ON o.customer_id = v.id",
    f"SELECT v.role, COUNT(*), AVG(v.age) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id JOIN {SU} AS v ON o.customer_id = v.id GROUP BY v.role",
    f"SELECT COUNT(*) FROM {U} AS u FULL JOIN {O} AS o ON u.id = o.customer_id JOIN {U} AS w ON o.id = w.id",
    # STDDEV / MEDIAN over joins and with composite / expression keys
    f"SELECT u.role, STDDEV(o.price), MEDIAN(o.price) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id GROUP BY u.role",
    f"SELECT STDDEV(o.price), MEDIAN(o.quantity), COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id",
    f"SELECT u.role, MEDIAN(o.price), STDDEV(u.age) FROM {SU} AS u LEFT JOIN {SO} AS o ON u.id = o.customer_id WHERE u.age > 30 GROUP BY u.role",
    f"SELECT p.category, STDDEV(o.price), MEDIAN(p.id) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p ON o.id = p.id GROUP BY p.category",
    f"SELECT gender, role, STDDEV(height), MEDIAN(age) FROM {R} GROUP BY gender, role",
    f"SELECT age / 10 AS decade, MEDIAN(height), STDDEV(height), COUNT(*) FROM {R} WHERE gender = 'm' GROUP BY decade",
    f"SELECT role, active, MEDIAN(age) FROM {T} GROUP BY role, active",
    # GROUP BY on a joined table by unqualified names: single-column through
    # find_column_index_with_fallback against the joined header (0 groups,
    # evaluator_aggregates.c:114 / evaluator.c:108), composite through
    # csv_get_column_index where a missing name is the part "NULL" (evaluator.c:152)
    f"SELECT role, COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id GROUP BY role",
    f"SELECT COUNT(*), SUM(o.price) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id GROUP BY role",
    f"SELECT u.role, COUNT(*) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id GROUP BY role, u.active",
    f"SELECT u.role, COUNT(*), SUM(o.price) FROM {SU} AS u JOIN {SO} AS o ON u.id = o.customer_id WHERE u.age > 70 GROUP BY u.role, quantity",
    # composite GROUP BY beyond four parts (parser_clauses.c:241-246 grows the list)
    # (at most 4 SELECT items: a 5th overflows the reference's parser)
    f"SELECT name, role, COUNT(*) FROM {T} GROUP BY name, age, role, height, active",
    f"SELECT name, COUNT(*), SUM(age) FROM {T} GROUP BY id, name, age, role, height, active",
    f"SELECT gender, role, COUNT(*), SUM(height) FROM {R} WHERE age > 77 GROUP BY gender, role, age, height, name",
    f"SELECT role, COUNT(*) FROM {R} WHERE age > 78 GROUP BY gender, role, age, height, name, age, gender",
    # composite parts holding a tab: the joined text is the key
    "SELECT t1, t2, COUNT(*), SUM(n) FROM '{D}/edge_tabs.csv' GROUP BY t1, t2",
    "SELECT t1, t2, t3, COUNT(*) FROM '{D}/edge_tabs.csv' GROUP BY t1, t2, t3",
    "SELECT t2, t1, COUNT(*) FROM '{D}/edge_tabs.csv' WHERE n > 1 GROUP BY t2, t1",
    # plans over more than 8 distinct columns (every column copied into the joined
    # row, evaluator_joins.c:30-37; `*` over all of them, evaluator_utils.c:272-417;
    # any condition tree, evaluator_conditions.c:62-164)
    f"SELECT * FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id",
    f"SELECT * FROM {U} AS u LEFT JOIN {O} AS o ON u.id = o.customer_id",
    f"SELECT * FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id WHERE o.price > 60 AND u.age < 40",
    f"SELECT * FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id JOIN {P} AS p ON o.id = p.id",
    f"SELECT u.name, o.price FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id WHERE u.age + u.height + u.active + o.tax + o.quantity + o.id > 100 AND u.city != 'x' AND u.email != 'y' AND u.role != 'z'",
    f"SELECT u.role, COUNT(*), SUM(o.price) FROM {U} AS u JOIN {O} AS o ON u.id = o.customer_id WHERE u.age + u.height + u.active > 0 AND o.tax + o.quantity + o.id > 0 AND u.city != 'x' AND u.email != 'y' GROUP BY u.role",
    f"SELECT COUNT(*), SUM(c11) FROM {W} WHERE {WIDE9}",
    f"SELECT c9, COUNT(*), SUM(c10), AVG(c11) FROM {W} WHERE {WIDE9} GROUP BY c9",
    f"SELECT c9, MIN(c10), MAX(c5), MIN(c4) FROM {W} WHERE c0 + c1 + c2 + c3 + c6 + c7 + c8 > 100 AND c5 != 'x' GROUP BY c9",
    f"SELECT c9, STDDEV(c10), MEDIAN(c11) FROM {W} WHERE c0 + c1 + c2 + c3 + c4 + c6 + c7 + c8 > 60 GROUP BY c9",
    f"SELECT c0, c11 FROM {W} WHERE {WIDE9}",
    f"SELECT * FROM {W} WHERE {WIDE9} AND c10 > 2000",
    f"SELECT c9, c0 + c10, COUNT(*) FROM {W} WHERE {WIDE9} GROUP BY c9",
    # GROUP BY of more than 8 parts (parser_clauses.c:241-246; evaluator.c:113-212)
    f"SELECT c9, COUNT(*) FROM {W} GROUP BY c0, c1, c2, c3, c4, c5, c6, c7, c8, c9",
    f"SELECT c9, COUNT(*), SUM(c11) FROM {W} WHERE c0 > 50 GROUP BY c9, c5, c9, c5, c9, c5, c9, c5, c9, c5, c9, c5",
    f"SELECT c5, COUNT(*) FROM {W} GROUP BY c5, c9, c0 % 3, c1 % 2, c2 % 2, c3 % 2, c6 % 2, c7 % 2, c8 % 2",
    # row-returning (build_result)
    f"SELECT name, age FROM {T} WHERE age > 30",
    f"SELECT * FROM {T} WHERE age > 30",
    f"SELECT name, age * 2, age + height FROM {T}",
    f"SELECT name, age FROM {T} ORDER BY age DESC",
    f"SELECT DISTINCT role FROM {T}",
    f"SELECT name FROM {T} LIMIT 3 OFFSET 2",
]


def probe(*args, cwd=None):
    out = subprocess.run([PROBE, *args], capture_output=True, check=True, cwd=cwd, timeout=120)
    return json.loads(out.stdout.decode("latin-1"))


def main():
    if not os.path.exists(PROBE):
        sys.exit("build the reference first: make -f oracle/ref.mk")
    write_fixtures()
    with open(os.path.join(HERE, "abi_layout.json"), "w") as fh:
        json.dump(probe("layout"), fh, indent=1, sort_keys=True)
    cells = {}
    for f in sorted(os.listdir(DATA)):
        if f.endswith(".csv"):
            cells[f] = probe("cells", os.path.join(DATA, f))
    cells["test_data.csv#noheader"] = probe("cells", os.path.join(DATA, "test_data.csv"), ",", "0")
    cells["synth_a.csv#semicolon"] = probe("cells", os.path.join(DATA, "synth_a.csv"), ";", "1")
    with open(os.path.join(HERE, "cells.json"), "w") as fh:
        json.dump(cells, fh)
    results = []
    for q in QUERIES:
        sql = q.replace("{D}", DATA)
        results.append({"sql": q, "result": probe("query", sql)})
    with open(os.path.join(HERE, "queries.json"), "w") as fh:
        json.dump(results, fh, indent=0)
    print(f"golden: {len(cells)} cell dumps, {len(results)} queries")


if __name__ == "__main__":
    main()
