"""Seeded synthetic CSV generators of the reference's benchmark shapes.

* Shape A  -- reference utils/generate_big_dataset.py:9-18:
  ``name,surname,age,gender,height`` with name = 10 x one letter A-P,
  surname = 8 x one letter A-P, age = randint(10, 80), gender in {f, m},
  height = randint(100, 200) / 100.0 printed by Python ``str`` (``1.0``, ``1.5``,
  ``1.23``: 3 or 4 characters).  ~29.9 B/row.
* Shape A+role -- the GROUP BY configuration: Shape A
  plus ``role`` = ``role_%03d`` uniform over 000-999.  ~38.9 B/row.
* users / orders -- the join configuration:
  ``id,name,age,role`` with id = 10**10 + i (11 digits: never typed DATE) and
  ``id,price,quantity,customer_id`` with customer_id = 10**10 + U[0, n_users).

The reference generator is unseeded; these are numpy-vectorised, seeded and
chunked so a 100M-row file streams to disk in well under a minute.
"""
from __future__ import annotations

import numpy as np

_HEIGHT_TXT = [str(v / 100.0).encode() for v in range(100, 201)]


def _height_table():
    w = 4
    tab = np.full((101, w), ord(" "), dtype=np.uint8)
    lens = np.zeros(101, dtype=np.int64)
    for i, t in enumerate(_HEIGHT_TXT):
        tab[i, : len(t)] = np.frombuffer(t, dtype=np.uint8)
        lens[i] = len(t)
    return tab, lens


def _digits(vals: np.ndarray, width: int) -> np.ndarray:
    out = np.empty((vals.shape[0], width), dtype=np.uint8)
    v = vals.copy()
    for k in range(width - 1, -1, -1):
        out[:, k] = ord("0") + (v % 10)
        v //= 10
    return out


def shape_a_chunk(rng: np.random.Generator, n: int, with_role: bool) -> bytes:
    """n data rows (no header) as bytes."""
    name = rng.integers(65, 81, n, dtype=np.int64).astype(np.uint8)
    sur = rng.integers(65, 81, n, dtype=np.int64).astype(np.uint8)
    age = rng.integers(10, 81, n, dtype=np.int64)
    gender = np.where(rng.integers(0, 2, n) == 0, ord("f"), ord("m")).astype(np.uint8)
    hidx = rng.integers(0, 101, n, dtype=np.int64)
    htab, hlen = _height_table()
    parts = [np.repeat(name[:, None], 10, axis=1), np.full((n, 1), ord(","), np.uint8),
             np.repeat(sur[:, None], 8, axis=1), np.full((n, 1), ord(","), np.uint8),
             _digits(age, 2), np.full((n, 1), ord(","), np.uint8),
             gender[:, None], np.full((n, 1), ord(","), np.uint8),
             htab[hidx]]
    if with_role:
        role = rng.integers(0, 1000, n, dtype=np.int64)
        parts += [np.full((n, 1), ord(","), np.uint8),
                  np.frombuffer(b"role_", dtype=np.uint8)[None, :].repeat(n, axis=0),
                  _digits(role, 3)]
    parts.append(np.full((n, 1), ord("\n"), np.uint8))
    mat = np.concatenate(parts, axis=1)
    # the height cell is padded to 4 chars with a space: drop the pad byte
    hcol = 10 + 1 + 8 + 1 + 2 + 1 + 1 + 1 + 3
    keep = np.ones(mat.shape, dtype=bool)
    keep[:, hcol] = hlen[hidx] == 4
    return mat[keep].tobytes()


def write_shape_a(path: str, rows: int, seed: int = 42, with_role: bool = True,
                  chunk: int = 1 << 20) -> int:
    """Write header + rows; returns file size in bytes."""
    rng = np.random.default_rng(seed)
    header = b"name,surname,age,gender,height" + (b",role" if with_role else b"") + b"\n"
    size = 0
    with open(path, "wb") as f:
        f.write(header)
        size += len(header)
        left = rows
        while left > 0:
            n = min(chunk, left)
            b = shape_a_chunk(rng, n, with_role)
            f.write(b)
            size += len(b)
            left -= n
    return size


def shape_a_bytes(rows: int, seed: int = 42, with_role: bool = True) -> bytes:
    rng = np.random.default_rng(seed)
    header = b"name,surname,age,gender,height" + (b",role" if with_role else b"") + b"\n"
    return header + (shape_a_chunk(rng, rows, with_role) if rows else b"")


# ------------------------------------------------------------------ logical files
#
# The benchmark files are views of one LOGICAL file per
# (seed, shape): a header plus an endless sequence of CHUNK_ROWS-row chunks, chunk
# k drawn from default_rng([seed, k]).  Config 3 is rows [0, 1e8), config 4 rows
# [0, 1e9) range-partitioned over the ranks; every rank generates its own rows
# without touching the others', and the bytes of row i do not depend on N.

CHUNK_ROWS = 1_000_000


def header_of(with_role: bool) -> bytes:
    return b"name,surname,age,gender,height" + (b",role" if with_role else b"") + b"\n"


def _chunk_rng(seed: int, k: int) -> np.random.Generator:
    return np.random.default_rng([seed, k])


def logical_rows(seed: int, row_lo: int, row_hi: int, with_role: bool = True) -> bytes:
    """Data rows [row_lo, row_hi) of the logical file (no header)."""
    out = []
    k = row_lo // CHUNK_ROWS
    while k * CHUNK_ROWS < row_hi:
        c0 = k * CHUNK_ROWS
        b = shape_a_chunk(_chunk_rng(seed, k), CHUNK_ROWS, with_role)
        lo, hi = max(row_lo, c0) - c0, min(row_hi, c0 + CHUNK_ROWS) - c0
        if lo or hi < CHUNK_ROWS:
            a = np.frombuffer(b, dtype=np.uint8)
            ends = np.flatnonzero(a == 10) + 1           # byte after each row's '\n'
            starts = np.concatenate(([0], ends[:-1]))
            b = b[int(starts[lo]):int(ends[hi - 1])]
        out.append(b)
        k += 1
    return b"".join(out)


def write_logical(path: str, rows: int, seed: int = 42, with_role: bool = True) -> int:
    """Header + rows [0, rows) of the logical file; returns the file size."""
    size = 0
    with open(path, "wb") as f:
        h = header_of(with_role)
        f.write(h)
        size += len(h)
        for lo in range(0, rows, CHUNK_ROWS):
            b = logical_rows(seed, lo, min(rows, lo + CHUNK_ROWS), with_role)
            f.write(b)
            size += len(b)
    return size


def _draws(rng: np.random.Generator, n: int, with_role: bool):
    """The same draws, in the same order, as shape_a_chunk (values only)."""
    rng.integers(65, 81, n, dtype=np.int64)             # name
    rng.integers(65, 81, n, dtype=np.int64)             # surname
    age = rng.integers(10, 81, n, dtype=np.int64)
    rng.integers(0, 2, n)                               # gender
    hidx = rng.integers(0, 101, n, dtype=np.int64)      # height = (100 + hidx) / 100
    role = rng.integers(0, 1000, n, dtype=np.int64) if with_role else None
    return age, hidx, role


def expected_filter_groupby(seed: int, row_lo: int, row_hi: int, with_role: bool = True,
                            age_gt: int = 30) -> dict:
    """What `... WHERE age > age_gt [GROUP BY role]` with COUNT(*) and SUM(height)
    must return on rows [row_lo, row_hi) of the logical file, computed from the
    generator's draws (no CSV parsing): per group the row count, the height sum
    in exact hundredths (integer) and the groups in first-appearance order."""
    ngroups = 1000 if with_role else 1
    cnt = np.zeros(ngroups, dtype=np.int64)
    cents = np.zeros(ngroups, dtype=np.int64)
    first = np.full(ngroups, np.iinfo(np.int64).max, dtype=np.int64)
    k = row_lo // CHUNK_ROWS
    while k * CHUNK_ROWS < row_hi:
        c0 = k * CHUNK_ROWS
        age, hidx, role = _draws(_chunk_rng(seed, k), CHUNK_ROWS, with_role)
        lo, hi = max(row_lo, c0) - c0, min(row_hi, c0 + CHUNK_ROWS) - c0
        age, hidx = age[lo:hi], hidx[lo:hi]
        g = role[lo:hi] if with_role else np.zeros(hi - lo, dtype=np.int64)
        m = age > age_gt
        gm = g[m]
        cnt += np.bincount(gm, minlength=ngroups)
        cents += np.rint(np.bincount(gm, weights=hidx[m] + 100, minlength=ngroups)).astype(np.int64)   # < 2^53: exact
        pos = np.flatnonzero(m) + (c0 + lo)
        # first filtered row of each group in this chunk: reversed assignment keeps the smallest
        f = np.full(ngroups, np.iinfo(np.int64).max, dtype=np.int64)
        f[gm[::-1]] = pos[::-1]
        first = np.minimum(first, f)
        k += 1
    order = [int(i) for i in np.argsort(first, kind="stable") if cnt[i] > 0]
    return {"groups": [("role_%03d" % i) if with_role else None for i in order],
            "count": [int(cnt[i]) for i in order],
            "sum_cents": [int(cents[i]) for i in order]}


def users_bytes(n: int, seed: int = 42) -> bytes:
    rng = np.random.default_rng(seed)
    ids = np.arange(n, dtype=np.int64) + 10**10
    age = rng.integers(10, 81, n)
    role = rng.integers(0, 1000, n)
    name = rng.integers(65, 81, n)
    lines = [b"id,name,age,role\n"]
    for i in range(n):
        lines.append(b"%d,%s,%d,role_%03d\n" % (ids[i], bytes([name[i]]) * 6, age[i], role[i]))
    return b"".join(lines)


def orders_bytes(n: int, n_users: int, seed: int = 43) -> bytes:
    rng = np.random.default_rng(seed)
    cust = rng.integers(0, n_users, n) + 10**10
    price = rng.integers(100, 100000, n)
    qty = rng.integers(1, 10, n)
    lines = [b"id,price,quantity,customer_id\n"]
    for i in range(n):
        lines.append(b"%d,%d.%02d,%d,%d\n" % (i + 1, price[i] // 100, price[i] % 100, qty[i], cust[i]))
    return b"".join(lines)
