"""The composite GROUP BY key text of a DOUBLE part (cell.h dbl_text via
joined_text_add): the reference renders it with snprintf(key_part, 256, "%.6f")
(evaluator.c:113-212), i.e. the exact binary value rounded half-even to 6 decimals,
kept to its first 255 bytes.  Checked against Python's correctly rounded "%.6f"
over edge values and random bit patterns (the library's host build of cell.h; no
GPU needed)."""
import ctypes as C
import math
import struct

import numpy as np

import cq_amd


def _text(x: float) -> str:
    L = cq_amd.lib()
    f = L.cq_host_double_key_text
    f.restype = C.c_uint32
    f.argtypes = [C.c_uint64, C.c_char_p]
    buf = C.create_string_buffer(256)
    n = f(struct.unpack("<Q", struct.pack("<d", x))[0], buf)
    return buf.raw[:n].decode()


def _want(x: float) -> str:
    if math.isnan(x):
        s = "-nan" if math.copysign(1.0, x) < 0 else "nan"
    elif math.isinf(x):
        s = "-inf" if x < 0 else "inf"
    else:
        s = "%.6f" % x
    return s[:255]


def test_double_key_text_edges():
    vals = [0.0, -0.0, 1.5, 0.0000005, 0.0000015, 2.0 ** 43, 2.0 ** 43 + 2.0 ** -9, 2.0 ** 43 + 1 / 128,
            2.0 ** 43 + 3 / 128, 2.0 ** 44 + 0.5, 2.0 ** 53 - 1, 2.0 ** 53, 2.0 ** 53 + 2, 2.0 ** 63, 2.0 ** 64,
            2.0 ** 64 + 4096, 1e17, 1e20, 1e22, 1e23, 123456789.123456789, 1e200, 1.7976931348623157e308,
            -1e250, 5e-324, 2.2250738585072014e-308, 8796093022207.9999999, 9007199254740991.5,
            float("inf"), float("-inf")]
    for x in vals:
        assert _text(x) == _want(x), x


def test_double_key_text_random_bits():
    rng = np.random.default_rng(5)
    bits = rng.integers(0, 2 ** 63, size=4000, dtype=np.uint64)
    # exponents spread over the whole range, and many just above 2^43
    ex = rng.integers(1023 + 43, 1023 + 54, size=1000).astype(np.uint64)      # 2^43 .. 2^53
    near = (ex << np.uint64(52)) | (bits[:1000] & np.uint64((1 << 52) - 1))
    for b in list(bits) + list(near):
        x = struct.unpack("<d", struct.pack("<Q", int(b)))[0]
        if math.isnan(x):
            continue
        assert _text(x) == _want(x), (hex(int(b)), x)
        assert _text(-x) == _want(-x), (hex(int(b)), -x)
