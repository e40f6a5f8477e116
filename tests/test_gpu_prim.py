"""The executor's own device primitives (prim.hip): stable LSD radix sorts and
exclusive scans, called through their C entry points on device buffers and
checked against numpy (stable argsort, cumsum) -- sizes across tile boundaries,
duplicate-heavy and all-equal keys, partial last digits, empty inputs."""
import ctypes as C

import numpy as np
import pytest
import torch

import cq_amd

pytestmark = pytest.mark.gpu


def _lib():
    L = cq_amd.lib()
    vp, sz = C.c_void_p, C.c_size_t
    L.cq_sort_codes.argtypes = [vp, C.POINTER(sz), vp, vp, vp, vp, sz, vp]
    L.cq_sort_u32.argtypes = [vp, C.POINTER(sz), vp, vp, vp, vp, sz, C.c_int, vp]
    L.cq_sort_offsets.argtypes = [vp, C.POINTER(sz), vp, vp, sz, C.c_int, vp]
    L.cq_excl_sum_u64.argtypes = [vp, C.POINTER(sz), vp, vp, sz, vp]
    L.cq_excl_sum_u32.argtypes = [vp, C.POINTER(sz), vp, vp, sz, vp]
    for f in (L.cq_sort_codes, L.cq_sort_u32, L.cq_sort_offsets, L.cq_excl_sum_u64, L.cq_excl_sum_u32):
        f.restype = C.c_int
    return L


def _call(fn, *args):
    tb = C.c_size_t(0)
    assert fn(None, C.byref(tb), *args) == 0
    temp = torch.empty(max(tb.value, 1), dtype=torch.uint8, device="cuda")
    assert fn(temp.data_ptr(), C.byref(tb), *args) == 0
    torch.cuda.synchronize()


SIZES = [0, 1, 255, 4096, 4097, 70_001, 1_000_003]


@pytest.mark.parametrize("n", SIZES)
def test_sort_u64_pairs_stable(n):
    L = _lib()
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 2 ** 63, n, dtype=np.int64).astype(np.uint64)
    keys[: n // 3] = keys[0] if n else 0                      # many duplicates
    keys[n // 3: n // 2] = rng.integers(0, 5, n // 2 - n // 3).astype(np.uint64)
    kin = torch.from_numpy(keys.view(np.int64)).cuda()
    vin = torch.arange(n, dtype=torch.int32, device="cuda")
    kout, vout = torch.empty_like(kin), torch.empty_like(vin)
    _call(L.cq_sort_codes, kin.data_ptr(), kout.data_ptr(), vin.data_ptr(), vout.data_ptr(), n, None)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(kout.cpu().numpy().view(np.uint64), keys[order])
    assert np.array_equal(vout.cpu().numpy(), order.astype(np.int32))


@pytest.mark.parametrize("bits", [1, 2, 7, 8, 9, 17, 32])
def test_sort_u32_low_bits(bits):
    L = _lib()
    n = 300_007
    rng = np.random.default_rng(bits)
    keys = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    kin = torch.from_numpy(keys.view(np.int32)).cuda()
    vin = torch.from_numpy(rng.integers(0, 2 ** 31, n).astype(np.int32)).cuda()
    kout, vout = torch.empty_like(kin), torch.empty_like(vin)
    _call(L.cq_sort_u32, kin.data_ptr(), kout.data_ptr(), vin.data_ptr(), vout.data_ptr(), n, bits, None)
    low = keys & np.uint32((1 << bits) - 1 if bits < 32 else 0xFFFFFFFF)
    order = np.argsort(low, kind="stable")
    assert np.array_equal(kout.cpu().numpy().view(np.uint32), keys[order])
    assert np.array_equal(vout.cpu().numpy(), vin.cpu().numpy()[order])


def test_sort_offsets_keys_only():
    L = _lib()
    n = 2_000_000
    rng = np.random.default_rng(3)
    keys = rng.permutation(np.arange(n, dtype=np.uint64) * 37 + 5)
    kin = torch.from_numpy(keys.view(np.int64)).cuda()
    kout = torch.empty_like(kin)
    _call(L.cq_sort_offsets, kin.data_ptr(), kout.data_ptr(), n, 27, None)
    assert np.array_equal(kout.cpu().numpy().view(np.uint64), np.sort(keys))


@pytest.mark.parametrize("n", [1, 2048, 2049, 4_194_305, 9_000_001])
def test_exclusive_scans(n):
    L = _lib()
    rng = np.random.default_rng(n)
    x64 = rng.integers(0, 1 << 20, n, dtype=np.int64)
    x32 = rng.integers(0, 3, n, dtype=np.int32)
    a, b = torch.from_numpy(x64).cuda(), torch.from_numpy(x32).cuda()
    oa, ob = torch.empty_like(a), torch.empty_like(b)
    _call(L.cq_excl_sum_u64, a.data_ptr(), oa.data_ptr(), n, None)
    _call(L.cq_excl_sum_u32, b.data_ptr(), ob.data_ptr(), n, None)
    ea = np.concatenate([[0], np.cumsum(x64)[:-1]])
    eb = np.concatenate([[0], np.cumsum(x32)[:-1]]).astype(np.int32)
    assert np.array_equal(oa.cpu().numpy(), ea)
    assert np.array_equal(ob.cpu().numpy(), eb)
