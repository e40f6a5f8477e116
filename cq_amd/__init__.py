"""cq_amd -- MI355X executor for cq's SELECT path (CSV scan, WHERE, GROUP BY, JOIN).

The product is the native library ``cq_amd/lib/libcqgpu.so`` (HIP for gfx950 +
C++ host), whose C ABI is declared in ``include/cqgpu.h``.  This module is a thin
ctypes binding used by bench.py, __graft_entry__.py and the tests; it never
computes results itself and raises if the native library is missing.
"""
from __future__ import annotations

import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
# CQ_AMD_LIB: profiling builds of the same library (scripts/build_lean_variants.sh, scripts/bench_variants.sh)
LIB_PATH = os.environ.get("CQ_AMD_LIB") or os.path.join(HERE, "lib", "libcqgpu.so")

_lib = None


# cqgpu_coll_fn (include/cqgpu.h): the test backend's collective callback
COLL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                      C.c_uint64)


class Coll(C.Structure):
    """cqgpu_coll: the next collective of the device-side merge (cqgpu.h)"""
    _fields_ = [("op", C.c_int32), ("pad", C.c_int32), ("count", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [("scan_ms", C.c_double), ("total_ms", C.c_double), ("scan_bytes", C.c_uint64),
                ("records", C.c_uint64), ("groups", C.c_uint64), ("lds_spills", C.c_uint64),
                ("grid", C.c_int), ("path", C.c_int), ("retries", C.c_int),
                ("slow_records", C.c_uint64), ("passed", C.c_uint64), ("scan_kernel", C.c_int),
                ("wide", C.c_int)]


def lib():
    """Load libcqgpu.so (fails loudly: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"cq_amd native library missing: {LIB_PATH} (run __graft_entry__.build())")
        # One HIP runtime per process: the torch wheel ships its own libamdhip64 /
        # libhsa-runtime64 / librccl.  Loaded first, they also serve libcqgpu's
        # dependencies (same sonames); loaded after libcqgpu pulled in /opt/rocm's,
        # both runtimes live in the process and their teardown frees twice at exit.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        TP = C.POINTER(abi.Table)
        L.evaluate_query.restype = TP
        L.evaluate_query.argtypes = [C.POINTER(abi.Node)]
        L.cqgpu_table_open.restype = C.c_void_p
        L.cqgpu_table_open.argtypes = [C.c_char_p, abi.CsvConfig]
        L.cqgpu_table_from_bytes.restype = C.c_void_p
        L.cqgpu_table_from_bytes.argtypes = [C.c_void_p, C.c_size_t, abi.CsvConfig, C.c_uint64,
                                             C.c_char_p, C.c_size_t]
        L.cqgpu_table_open_range.restype = C.c_void_p
        L.cqgpu_table_open_range.argtypes = [C.c_char_p, abi.CsvConfig, C.c_int, C.c_int]
        L.cqgpu_range_bounds.restype = C.c_int
        L.cqgpu_range_bounds.argtypes = [C.c_void_p, C.c_size_t, abi.CsvConfig, C.c_int, C.c_int,
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.cqgpu_table_base_offset.restype = C.c_uint64
        L.cqgpu_table_base_offset.argtypes = [C.c_void_p]
        L.cqgpu_table_free.argtypes = [C.c_void_p]
        L.cqgpu_table_bytes.restype = C.c_size_t
        L.cqgpu_table_bytes.argtypes = [C.c_void_p]
        L.cqgpu_query.restype = TP
        L.cqgpu_query.argtypes = [C.POINTER(abi.Node), C.POINTER(C.c_void_p), C.c_int]
        L.cqgpu_result_free.argtypes = [TP]
        L.cqgpu_query_partial.restype = C.c_size_t
        L.cqgpu_query_partial.argtypes = [C.POINTER(abi.Node), C.POINTER(C.c_void_p), C.c_int,
                                          C.POINTER(C.c_void_p)]
        L.cqgpu_merge_partials.restype = TP
        L.cqgpu_merge_partials.argtypes = [C.POINTER(abi.Node), C.POINTER(C.c_void_p),
                                           C.POINTER(C.c_size_t), C.c_int]
        L.cqgpu_route_plan.restype = C.c_int
        L.cqgpu_route_plan.argtypes = [C.POINTER(abi.Node), C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.cqgpu_route_plan2.restype = C.c_int64
        L.cqgpu_route_plan2.argtypes = [C.POINTER(abi.Node), C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64)]
        L.cqgpu_route_major.restype = C.c_uint32
        L.cqgpu_route_major.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.cqgpu_table_set_replicated.restype = C.c_int
        L.cqgpu_table_set_replicated.argtypes = [C.c_void_p, C.c_uint32, C.c_int]
        L.cqgpu_route_fill.restype = C.c_int
        L.cqgpu_route_fill.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
        L.cqgpu_join_outer_matched.restype = C.c_int
        L.cqgpu_join_outer_matched.argtypes = [C.POINTER(abi.Node), C.POINTER(C.c_void_p), C.c_int, C.c_int,
                                               C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_uint64)]
        L.cqgpu_join_outer_set.restype = C.c_int
        L.cqgpu_join_outer_set.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_int]
        L.cqgpu_join_outer_clear.restype = None
        L.cqgpu_join_outer_clear.argtypes = []
        L.cqgpu_table_set_record_total.restype = C.c_int
        L.cqgpu_table_set_record_total.argtypes = [C.c_void_p, C.c_uint64]
        L.cqgpu_table_set_key_stride.restype = C.c_int
        L.cqgpu_table_set_key_stride.argtypes = [C.c_void_p, C.c_uint32]
        L.cqgpu_table_from_routed.restype = C.c_void_p
        L.cqgpu_table_from_routed.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, abi.CsvConfig,
                                              C.c_char_p, C.c_size_t]
        vp = C.c_void_p
        L.cqgpu_partial_new.restype = vp
        L.cqgpu_partial_new.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int]
        L.cqgpu_partial_next.restype = C.c_int
        L.cqgpu_partial_next.argtypes = [vp, vp, C.POINTER(C.c_uint64), C.c_int, C.c_int, C.POINTER(Coll)]
        L.cqgpu_partial_put.restype = C.c_int
        L.cqgpu_partial_put.argtypes = [vp, vp]
        L.cqgpu_partial_result.restype = TP
        L.cqgpu_partial_result.argtypes = [vp, C.POINTER(abi.Node)]
        L.cqgpu_partial_free.argtypes = [vp]
        L.cqgpu_comm_unique_id.restype = C.c_int
        L.cqgpu_comm_unique_id.argtypes = [vp]
        L.cqgpu_comm_init.restype = C.c_int
        L.cqgpu_comm_init.argtypes = [vp, C.c_int, C.c_int]
        L.cqgpu_comm_destroy.argtypes = []
        L.cqgpu_typed_plan.restype = C.c_int
        L.cqgpu_typed_plan.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int]
        L.cqgpu_typed_sample_kmin.restype = C.c_uint64
        L.cqgpu_typed_sample_kmin.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int]
        L.cqgpu_typed_count.restype = C.c_int64
        L.cqgpu_typed_count.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int, C.c_int, C.c_int, C.c_uint64,
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        L.cqgpu_typed_send.restype = C.c_int
        L.cqgpu_typed_send.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int, C.c_int, C.c_uint64,
                                       C.POINTER(C.c_uint32)]
        L.cqgpu_typed_region.restype = vp
        L.cqgpu_typed_region.argtypes = [vp, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.cqgpu_typed_reset.argtypes = [vp]
        L.cqgpu_typed_gather.restype = C.c_int64
        L.cqgpu_typed_gather.argtypes = [C.POINTER(vp), C.c_int, C.c_int, vp, C.c_uint64]
        L.cqgpu_typed_partial.restype = C.c_size_t
        L.cqgpu_typed_partial.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int, vp, C.c_uint64, vp, C.c_uint64,
                                          C.c_uint64, C.c_uint64, C.POINTER(vp)]
        L.cqgpu_comm_init_host.restype = C.c_int
        L.cqgpu_comm_init_host.argtypes = [C.c_int, C.c_int, COLL_FN, vp]
        L.cqgpu_dist_query.restype = TP
        L.cqgpu_dist_query.argtypes = [C.POINTER(abi.Node), vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.cqgpu_dist_join.restype = TP
        L.cqgpu_dist_join.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int, C.POINTER(C.c_int)]
        L.cqgpu_gm_local.restype = TP
        L.cqgpu_gm_local.argtypes = [C.POINTER(abi.Node), C.POINTER(vp), C.c_int]
        L.cqgpu_last_stats.argtypes = [C.POINTER(Stats)]
        L.cqgpu_last_error.restype = C.c_char_p
        L.cqgpu_last_ineligible.restype = C.c_char_p
        L.cqgpu_set_scan_kernel.restype = C.c_int
        L.cqgpu_set_scan_kernel.argtypes = [C.c_int]
        _lib = L
    return _lib


def global_csv_config() -> abi.CsvConfig:
    return abi.CsvConfig.in_dll(lib(), "global_csv_config")


class Table:
    """A CSV table resident in HBM on the current HIP device."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("cq_amd: " + (lib().cqgpu_last_error() or b"").decode())
        self.handle = C.c_void_p(handle)

    @classmethod
    def open(cls, path: str, cfg: abi.CsvConfig | None = None) -> "Table":
        return cls(lib().cqgpu_table_open(path.encode(), cfg or abi.csv_config()))

    @classmethod
    def from_bytes(cls, data: bytes, cfg: abi.CsvConfig | None = None, base_offset: int = 0,
                   header: bytes | None = None) -> "Table":
        # bytes: pass the object's own buffer (no copy); the library copies it to HBM
        ptr = C.cast(C.c_char_p(data), C.c_void_p) if isinstance(data, bytes) else C.cast(data, C.c_void_p)
        h = lib().cqgpu_table_from_bytes(ptr, len(data), cfg or abi.csv_config(),
                                         base_offset, header, len(header) if header else 0)
        return cls(h)

    @classmethod
    def open_range(cls, path: str, rank: int, nranks: int, cfg: abi.CsvConfig | None = None) -> "Table":
        """rank's newline-snapped byte range of the file (cqgpu_table_open_range)"""
        return cls(lib().cqgpu_table_open_range(path.encode(), cfg or abi.csv_config(), rank, nranks))

    @property
    def nbytes(self) -> int:
        return lib().cqgpu_table_bytes(self.handle)

    @property
    def base_offset(self) -> int:
        return lib().cqgpu_table_base_offset(self.handle)

    def close(self):
        if self.handle:
            lib().cqgpu_table_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def range_bounds(data: bytes, rank: int, nranks: int, cfg: abi.CsvConfig | None = None):
    """(lo, hi, header_lo, header_hi) of rank's range (cqgpu_range_bounds; host code only)"""
    lo, hi, hl, hh = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    buf = C.c_char_p(data)
    if lib().cqgpu_range_bounds(C.cast(buf, C.c_void_p), len(data), cfg or abi.csv_config(), rank, nranks,
                                C.byref(lo), C.byref(hi), C.byref(hl), C.byref(hh)) != 0:
        raise ValueError("cqgpu_range_bounds: bad arguments")
    return lo.value, hi.value, hl.value, hh.value


def _tables_arg(tables):
    arr = (C.c_void_p * len(tables))(*[t.handle.value for t in tables])
    return arr, len(tables)


def query(ast, tables) -> dict | None:
    """Run a plan (pointer to a reference-layout node) over resident tables."""
    arr, n = _tables_arg(tables)
    tp = lib().cqgpu_query(ast, arr, n)
    if not tp:
        return None
    res = abi.table_to_py(tp)
    lib().cqgpu_result_free(tp)
    return res


def query_raw(ast, tables):
    """Like query() but returns the result pointer (caller frees with result_free)."""
    arr, n = _tables_arg(tables)
    return lib().cqgpu_query(ast, arr, n)


def result_free(tp):
    lib().cqgpu_result_free(tp)


def evaluate(ast) -> dict | None:
    """The drop-in entry point: evaluate_query(ASTNode*) on files named in the plan."""
    tp = lib().evaluate_query(ast)
    if not tp:
        return None
    res = abi.table_to_py(tp)
    lib().cqgpu_result_free(tp)
    return res


def query_partial(ast, tables) -> bytes:
    """Partial group state of this shard (cqgpu_query_partial), as bytes."""
    arr, n = _tables_arg(tables)
    blob = C.c_void_p()
    size = lib().cqgpu_query_partial(ast, arr, n, C.byref(blob))
    if size == 0:
        raise RuntimeError(last_error() or "cqgpu_query_partial failed")
    try:
        return C.string_at(blob, size)
    finally:
        C.CDLL(None).free(blob)


def join_outer_matched(ast, tables, level: int) -> bytes | None:
    """This rank's matched flags over a chain's later RIGHT / FULL level's records
    (cqgpu_join_outer_matched, one byte per record); None when the level needs no
    global set."""
    arr, n = _tables_arg(tables)
    fl = C.POINTER(C.c_uint8)()
    nrec = C.c_uint64(0)
    r = lib().cqgpu_join_outer_matched(ast, arr, n, level, C.byref(fl), C.byref(nrec))
    if r < 0:
        raise RuntimeError(last_error() or "cqgpu_join_outer_matched failed")
    if r == 0:
        return None
    return C.string_at(fl, nrec.value) if nrec.value else b""


def join_outer_set(level: int, matched: bytes, emit: bool) -> None:
    """The ranks' OR of join_outer_matched for `level` (cqgpu_join_outer_set); emit on
    exactly one rank."""
    buf = C.create_string_buffer(bytes(matched), max(len(matched), 1))
    if lib().cqgpu_join_outer_set(level, buf, len(matched), 1 if emit else 0) != 0:
        raise RuntimeError(last_error() or "cqgpu_join_outer_set failed")


def join_outer_clear() -> None:
    lib().cqgpu_join_outer_clear()


def route_plan(ast, tables, side: int, nranks: int) -> tuple[list[int], list[int]]:
    """Join-key routing of tables[side] (tables = [FROM shard, JOIN shard]):
    per destination rank the send-buffer byte count and record count."""
    arr, n = _tables_arg(tables)
    nb = (C.c_uint64 * nranks)()
    nr = (C.c_uint64 * nranks)()
    if lib().cqgpu_route_plan(ast, arr, n, side, nranks, nb, nr) != 0:
        raise RuntimeError(last_error() or "cqgpu_route_plan failed")
    return list(nb), list(nr)


def route_fill(table: "Table", gid_base: int, dev_bytes_ptr: int, dev_gids_ptr: int) -> None:
    """Write the planned send buffer (device pointers, e.g. torch tensors' data_ptr())."""
    if lib().cqgpu_route_fill(table.handle, gid_base, dev_bytes_ptr, dev_gids_ptr) != 0:
        raise RuntimeError(last_error() or "cqgpu_route_fill failed")


def table_from_routed(dev_bytes_ptr: int, nbytes: int, dev_gids_ptr: int, nrec: int, header: bytes,
                      cfg: abi.CsvConfig | None = None) -> "Table":
    """A join side rebuilt from received records (device memory) and their global ids."""
    return Table(lib().cqgpu_table_from_routed(dev_bytes_ptr, nbytes, dev_gids_ptr, nrec,
                                               cfg or abi.csv_config(), header, len(header)))


def route_plan2(ast, tables, side: int, nranks: int, rank: int, mode: int = 0):
    """cqgpu_route_plan2: the routing of tables[side] for `rank` in routing mode `mode`
    (0 key routing; 1-3 the majority key class of cqgpu_route_major, other non-NULL
    classes to every rank; a JOIN without ON: side 0 stays, side 1 to every rank).
    Returns (bytes per destination, records per destination, this side's record
    count on this rank, its ON keys per value class [NULL, number, string, date])."""
    arr, n = _tables_arg(tables)
    nb = (C.c_uint64 * nranks)()
    nr = (C.c_uint64 * nranks)()
    cc = (C.c_uint64 * 4)()
    own = lib().cqgpu_route_plan2(ast, arr, n, side, nranks, rank, mode, nb, nr, cc)
    if own < 0:
        raise RuntimeError(last_error() or "cqgpu_route_plan2 failed")
    return list(nb), list(nr), int(own), list(cc)


def route_major(lcounts, rcounts) -> int:
    """cqgpu_route_major over the ranks' summed class counts of both sides."""
    return int(lib().cqgpu_route_major((C.c_uint64 * 4)(*lcounts), (C.c_uint64 * 4)(*rcounts)))


def table_set_replicated(table: "Table", mode: int, owner: bool) -> None:
    """cqgpu_table_set_replicated: a routed side's replication mode (0-3, 4 whole on
    every rank) and whether this rank owns what every rank finds."""
    if lib().cqgpu_table_set_replicated(table.handle, mode, 1 if owner else 0) != 0:
        raise RuntimeError(last_error() or "cqgpu_table_set_replicated failed")


def table_set_key_stride(table: "Table", stride: int) -> None:
    """A routed table's join-key stride: the rank count of the key-mod-N routing
    (cqgpu_table_set_key_stride; the STAR join then indexes keys by (key - kmin) / N)."""
    if lib().cqgpu_table_set_key_stride(table.handle, stride) != 0:
        raise RuntimeError(last_error() or "cqgpu_table_set_key_stride failed")


def table_set_record_total(table: "Table", total: int) -> None:
    """The whole input's record count for a routed table (cqgpu_table_set_record_total)."""
    if lib().cqgpu_table_set_record_total(table.handle, total) != 0:
        raise RuntimeError(last_error() or "cqgpu_table_set_record_total failed")


def merge_partials(ast, blobs):
    """cqgpu_merge_partials over byte blobs; returns the result pointer (free with result_free)."""
    bufs = [C.create_string_buffer(b, len(b)) for b in blobs]
    ptrs = (C.c_void_p * len(bufs))(*[C.cast(b, C.c_void_p).value for b in bufs])
    sizes = (C.c_size_t * len(bufs))(*[len(b) for b in blobs])
    return lib().cqgpu_merge_partials(ast, ptrs, sizes, len(bufs))


def stats() -> dict:
    s = Stats()
    lib().cqgpu_last_stats(C.byref(s))
    return {f: getattr(s, f) for f, _ in Stats._fields_}


def set_scan_kernel(mode: int) -> int:
    """0: automatic (fast_kernel, else lean_kernel, else scan_kernel by plan shape),
    1: always the general scan_kernel, 2: never fast_kernel.  Returns the old mode."""
    return lib().cqgpu_set_scan_kernel(mode)


def last_error() -> str:
    return (lib().cqgpu_last_error() or b"").decode("latin-1")


def last_ineligible() -> str:
    return (lib().cqgpu_last_ineligible() or b"").decode("latin-1")


# ---- the N > 1 step inside the library over RCCL (cqgpu.h cqgpu_dist_query)
COMM_ID_BYTES = 128
DIST_PATHS = {1: "gather-merge", 2: "dense", 3: "blobs"}


def comm_unique_id() -> bytes:
    """rank 0: a fresh RCCL unique id (to broadcast to the other ranks)"""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    if lib().cqgpu_comm_unique_id(buf) != 0:
        raise RuntimeError(last_error() or "cqgpu_comm_unique_id failed")
    return buf.raw


def comm_init(uid: bytes, rank: int, world: int) -> None:
    """every rank, once: the library's RCCL communicator on the current HIP device"""
    buf = C.create_string_buffer(bytes(uid), COMM_ID_BYTES)
    if lib().cqgpu_comm_init(buf, rank, world) != 0:
        raise RuntimeError(last_error() or "cqgpu_comm_init failed")


def comm_destroy() -> None:
    lib().cqgpu_comm_destroy()


def dist_query_raw(ast, table: "Table"):
    """(result pointer or None, status, path): rank 0 gets the result; status -1
    on every rank when any rank failed"""
    st, path = C.c_int(0), C.c_int(0)
    tp = lib().cqgpu_dist_query(ast, table.handle, C.byref(st), C.byref(path))
    return (tp if tp else None), st.value, path.value


def dist_join_raw(ast, tables):
    """(result pointer or None, status): the repartitioned JOIN step over the
    library's RCCL communicator (cqgpu_dist_join); status -1 on every rank when any
    rank failed"""
    arr, n = _tables_arg(tables)
    st = C.c_int(0)
    tp = lib().cqgpu_dist_join(ast, arr, n, C.byref(st))
    return (tp if tp else None), st.value


def gm_local(ast, shards):
    """test entry: the gather-merge over shards held by this process (simulated ranks)"""
    arr, n = _tables_arg(shards)
    tp = lib().cqgpu_gm_local(ast, arr, n)
    if not tp:
        return None
    out = abi.table_to_py(tp)
    lib().cqgpu_result_free(tp)
    return out



# ---- the typed exchange of the repartitioned JOIN (include/cqgpu.h cqgpu_typed_*)
def typed_plan(ast, tables) -> bool:
    return lib().cqgpu_typed_plan(ast, *_tables_arg(tables)) == 1


def typed_sample_kmin(ast, tables) -> int:
    return lib().cqgpu_typed_sample_kmin(ast, *_tables_arg(tables))


def typed_count(ast, tables, side: int, nranks: int, qbase: int):
    """the count pass: (records (build) / entries (probe), counts per destination,
    (build keys' min, max), flags)"""
    counts = (C.c_uint64 * nranks)()
    kr = (C.c_uint64 * 2)()
    fl = C.c_uint32(0)
    n = lib().cqgpu_typed_count(ast, *_tables_arg(tables), side, nranks, qbase, counts, kr, C.byref(fl))
    if n < 0:
        raise RuntimeError(last_error() or "cqgpu_typed_count failed")
    return n, list(counts), (kr[0], kr[1]), fl.value


def typed_send(ast, tables, side: int, gid_base: int) -> int:
    """the emit pass after typed_count; returns its flags"""
    fl = C.c_uint32(0)
    if lib().cqgpu_typed_send(ast, *_tables_arg(tables), side, gid_base, C.byref(fl)) != 0:
        raise RuntimeError(last_error() or "cqgpu_typed_send failed")
    return fl.value


def typed_reset(table) -> None:
    lib().cqgpu_typed_reset(table.handle)


def typed_gather(senders, dest: int, dev_out: int, cap_entries: int) -> int:
    arr = (C.c_void_p * len(senders))(*[t.handle.value for t in senders])
    n = lib().cqgpu_typed_gather(arr, len(senders), dest, dev_out, cap_entries)
    if n < 0:
        raise RuntimeError(last_error() or "cqgpu_typed_gather failed")
    return n


def typed_partial(ast, tables, build_ptr: int, nbuild: int, probe_ptr: int, nprobe: int, qoff: int, rng: int):
    """the blob, or None with last_ineligible() saying why the entries left the STAR join"""
    out = C.c_void_p()
    n = lib().cqgpu_typed_partial(ast, *_tables_arg(tables), build_ptr, nbuild, probe_ptr, nprobe, qoff,
                                  rng, C.byref(out))
    if n == 0:
        return None
    try:
        return C.string_at(out, n)
    finally:
        C.CDLL(None).free(out)
