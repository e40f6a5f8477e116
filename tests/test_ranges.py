"""Range partition of one file over N ranks (cqgpu_range_bounds, host code only).

SURVEY.md section 8e: cut the data region into N byte ranges, snapping each cut
to the byte after the next '\\n' / '\\r' run (records split on any terminator,
quote-blind, reference csv_reader.c:404-408).  Checked here without a device:
the oracle's csv_load restatement (oracle/cq_oracle.c orc_load) over every
rank's range (rank > 0 with the header record prepended) must give exactly the
whole file's rows, in order, for files whose terminator runs (CR, CRLF, LF,
blank-line runs, a missing final terminator) land on and around the cuts.
"""
import random

import pytest

import cqtest
import cq_amd
from cq_amd import abi


def _rows(data: bytes):
    lib = cqtest.oracle()
    tp = lib.orc_load(data, len(data), abi.csv_config())
    assert tp
    try:
        return abi.table_to_py(tp)
    finally:
        lib.orc_free(tp)


def _split_rows(data: bytes, n: int):
    out = []
    prev_hi = 0
    for r in range(n):
        lo, hi, hl, hh = cq_amd.range_bounds(data, r, n)
        assert lo == prev_hi and lo <= hi <= len(data), (r, lo, hi, prev_hi)
        prev_hi = hi
        if r == 0:
            assert lo == 0
        else:
            # a range starts at a record start: the byte before it ends a record
            assert lo == len(data) or data[lo - 1:lo] in (b"\n", b"\r"), (r, lo)
            assert lo >= hh
        piece = data[lo:hi]
        if r > 0:
            piece = data[hl:hh] + b"\n" + piece
        out.append(_rows(piece)["rows"])
    assert prev_hi == len(data)
    return out


def _random_file(rng: random.Random, nrec: int) -> bytes:
    terms = [b"\n", b"\r\n", b"\r", b"\n\n", b"\r\n\r\n", b"\n\r\n\n"]
    parts = [rng.choice([b"", b"\n", b"\r\n"]), b"id,name,v", rng.choice(terms)]
    for i in range(nrec):
        parts.append(b"%d,%s,%d" % (i, rng.choice([b"a", b"bb", b'"q,x"', b" sp"]), rng.randrange(1000)))
        if i + 1 < nrec or rng.random() < 0.7:
            parts.append(rng.choice(terms))
    return b"".join(parts)


@pytest.mark.parametrize("seed", range(12))
def test_ranges_cover_every_record_once(seed):
    rng = random.Random(seed)
    data = _random_file(rng, rng.choice([0, 1, 3, 17, 60]))
    whole = _rows(data)["rows"]
    for n in (1, 2, 3, 4, 5, 7, 8, 13):
        got = _split_rows(data, n)
        assert [r for part in got for r in part] == whole, (seed, n)


def test_cuts_inside_terminator_runs():
    # every nominal cut of a 2-rank split of these files lands in or next to a run
    hdr = b"a,b\n"
    for run in (b"\n", b"\r", b"\r\n", b"\n\n\n", b"\r\n\r\n\r\n"):
        for pad in range(0, 8):
            data = hdr + b"1," + b"x" * pad + run + b"2,y" + run + b"3,z"
            whole = _rows(data)["rows"]
            for n in (2, 3, 4, 6):
                got = _split_rows(data, n)
                assert [r for part in got for r in part] == whole, (run, pad, n)


def test_large_file_balanced():
    from cq_amd import datagen
    data = datagen.shape_a_bytes(20_000, seed=5, with_role=True)
    sizes = [cq_amd.range_bounds(data, r, 8)[1] - cq_amd.range_bounds(data, r, 8)[0] for r in range(8)]
    assert sum(sizes) == len(data)
    assert max(sizes) - min(sizes) < 200          # within a few records of equal
    whole = _rows(data)["rows"]
    assert [r for part in _split_rows(data, 8) for r in part] == whole


def test_headerless_config():
    cfg = abi.csv_config()
    cfg.has_header = False
    data = b"1,a\n2,b\r\n3,c\n"
    lo0, hi0, _, _ = cq_amd.range_bounds(data, 0, 2, cfg)
    lo1, hi1, _, _ = cq_amd.range_bounds(data, 1, 2, cfg)
    assert lo0 == 0 and hi0 == lo1 and hi1 == len(data)
    assert data[lo1 - 1:lo1] == b"\n" or data[lo1 - 1:lo1] == b"\r"


def test_bad_arguments():
    with pytest.raises(ValueError):
        cq_amd.range_bounds(b"a\n1\n", 2, 2)
    with pytest.raises(ValueError):
        cq_amd.range_bounds(b"a\n1\n", 0, 0)
