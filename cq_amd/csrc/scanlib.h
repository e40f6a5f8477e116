// scanlib.h -- device helpers shared by the scan kernels (scan.hip, lean.hip):
// byte-class SWAR tests, DPP wave scans, the fast field typers (infer_type +
// parse_value restated for short fields, reference csv_reader.c:133-240), the
// HBM group-table insert and the LDS slot header/key words.
#pragma once
#include <hip/hip_runtime.h>
#include "plan.h"

namespace cq {

constexpr uint64_t NOPOS = ~0ULL;            // no position (no extreme, no first row)

// WHERE shapes the fast kernels are specialised for
enum : int { W_NONE = 0, W_SIMPLE = 1, W_VM = 2 };

typedef uint32_t v4u __attribute__((ext_vector_type(4)));   // one 16-byte load

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ bool is_nl(uint32_t c) { return c == '\n' || c == '\r'; }
__device__ __forceinline__ bool is_blank(uint32_t c) { return c == ' ' || c == '\t' || c == 0x0b || c == 0x0c; }

// LDS-only barrier: waits for this wave's LDS traffic, not for in-flight global
// loads (the next window's prefetch must stay in flight across it)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// exact per-byte tests on a dword.  nonzero_bytes: 0x80 in every nonzero byte.
__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t t) {
    return (((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
// 0x80 in every byte < n, for 0 < n <= 0x80 (rep_n = n * 0x01010101): no borrows
// cross bytes because every byte of (x | 0x80..) is >= 0x80 >= n
__device__ __forceinline__ uint32_t lt_bytes(uint32_t x, uint32_t rep_n) {
    return ~((x | 0x80808080u) - rep_n) & ~x & 0x80808080u;
}

// inclusive prefix sum over a wave with DPP row shifts and row broadcasts
// (no LDS round trips, unlike shuffles)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
__device__ __forceinline__ bool cmp_result(uint32_t op, int c) {
    switch (op) {
        case CMP_EQ: return c == 0;
        case CMP_NE: return c != 0;
        case CMP_LT: return c < 0;
        case CMP_GT: return c > 0;
        case CMP_LE: return c <= 0;
        default: return c >= 0;
    }
}
// ------------------------------------------------------------------ global table
__device__ __forceinline__ uint32_t tag_of(uint64_t h) {
    uint32_t t = (uint32_t)(h >> 32);
    return t < 2 ? t + 2 : t;
}

// Lock-free find-or-insert into the HBM group table.  Every access to a slot's
// tag and key words is a relaxed agent-scope atomic (global_load / global_store
// sc1: past the CU's L1, coherent across XCDs), so no probe pays an acquire's L1
// invalidate or an insert a release's L2 write-back: an inserter claims the tag
// by CAS (0 -> 1), stores the key words, drains them with s_waitcnt vmcnt(0) and
// only then stores the final tag; a reader that sees that tag issues its key loads
// after the tag load returned (the compare depends on it), so it sees the words
// (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores drained before
// the flag, sc1 loads).
static __device__ int g_insert(const GroupTable& gt, const GKey k, uint64_t h, ScanStats* st) {
    const uint32_t tg = tag_of(h);
    const uint32_t mask = gt.cap - 1;
    const uint32_t cl = gk_clslen(k);
    for (uint32_t probe = 0; probe < gt.cap; probe++) {
        uint32_t i = (uint32_t)(h + probe) & mask;
        uint32_t t = __hip_atomic_load(&gt.tag[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0) {
            uint32_t old = atomicCAS(&gt.tag[i], 0u, 1u);
            if (old == 0) {
                __hip_atomic_store(&gt.clslen[i], cl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&gt.w0[i], k.w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&gt.w1[i], k.w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint32_t used = atomicAdd(gt.used, 1u) + 1;
                if (used * 2 > gt.cap) atomicExch(&st->overflow, 1ULL);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // key words performed before the tag
                __hip_atomic_store(&gt.tag[i], tg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return (int)i;
            }
            t = old;
        }
        for (uint32_t spin = 0; t == 1; spin++) {
            if (spin > (1u << 20)) { atomicExch(&st->overflow, 3ULL); return -1; }   // never hang
            __builtin_amdgcn_s_sleep(1);
            t = __hip_atomic_load(&gt.tag[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (t == tg) {
            GKey o;
            uint32_t ocl = __hip_atomic_load(&gt.clslen[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o.cls = ocl >> 16;
            o.len = ocl & 0xffff;
            o.w0 = __hip_atomic_load(&gt.w0[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o.w1 = __hip_atomic_load(&gt.w1[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (gk_equal(o, k)) return (int)i;
        }
    }
    atomicExch(&st->overflow, 1ULL);
    return -1;
}
__device__ __forceinline__ uint32_t lds_hdr(const GKey& k, uint64_t h) {
    return 0x80000000u | (((uint32_t)(h >> 40) & 0xFFFu) << 19) | gk_clslen(k);
}
__device__ __forceinline__ v4u key_words(const GKey& k) {
    v4u r;
    r.x = (uint32_t)k.w0; r.y = (uint32_t)(k.w0 >> 32); r.z = (uint32_t)k.w1; r.w = (uint32_t)(k.w1 >> 32);
    return r;
}
__device__ __forceinline__ bool key_match(const GKey& k, const v4u& mine, const v4u& slot) {
    if (mine.z != slot.z || mine.w != slot.w) return false;
    if (mine.x == slot.x && mine.y == slot.y) return true;
    if (k.cls != GK_LONG) return false;
    GKey o = k;                                     // long keys: same hash and length, compare bytes
    o.w0 = (uint64_t)slot.x | ((uint64_t)slot.y << 32);
    return gk_equal(o, k);
}
// ------------------------------------------------------------------ fast field path
// 16 bytes of the tile at byte offset `o` (any alignment), as four dwords
__device__ __forceinline__ void load16(const uint8_t* tile, uint32_t o, uint32_t& e0, uint32_t& e1,
                                       uint32_t& e2, uint32_t& e3) {
    const uint32_t* t32 = (const uint32_t*)tile;
    const uint32_t a = o >> 2, sh = o & 3;
    const uint32_t d0 = t32[a], d1 = t32[a + 1], d2 = t32[a + 2], d3 = t32[a + 3], d4 = t32[a + 4];
    e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
    e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    e2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    e3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
}

// bytes [0, len) of a dword holding bytes [4j, 4j + 4) of a field
__device__ __forceinline__ uint32_t len_mask(uint32_t len, uint32_t j) {
    const uint32_t n = len > 4 * j ? len - 4 * j : 0;
    return n >= 4 ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1);
}

// 10^e for e <= 15, exact in double (every partial product is exact), branch-free
__device__ __forceinline__ double pow10_exact(uint32_t e) {
    double r = 1.0, b = 10.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        r = ((e >> i) & 1) ? r * b : r;
        b = b * b;
    }
    return r;
}

// four decimal digit values in bytes 0..3 (byte 0 most significant) -> 0..9999
__device__ __forceinline__ uint32_t dig4(uint32_t h) {
    const uint32_t t = (h << 3) + (h << 1) + (h >> 8);   // bytes 0, 2: 10*b0+b1, 10*b2+b3
    return (t & 0xffu) * 100u + ((t >> 16) & 0xffu);
}
__device__ __forceinline__ uint32_t dig8(uint64_t v) {
    return dig4((uint32_t)v) * 10000u + dig4((uint32_t)(v >> 32));
}

// 0x80 in every byte that is a decimal digit
__device__ __forceinline__ uint32_t digit_bytes(uint32_t x) { return lt_bytes(x ^ 0x30303030u, 0x0A0A0A0Au); }
// 0x80 flags -> 0xFF bytes
__device__ __forceinline__ uint32_t spread(uint32_t f) { return f | (f - (f >> 7)); }

enum : int { FF_OK = 0, FF_SLOW = 1 };

// 8 bytes of the tile at byte offset `o` (any alignment), as two dwords
__device__ __forceinline__ void load8(const uint8_t* tile, uint32_t o, uint32_t& e0, uint32_t& e1) {
    const uint32_t* t32 = (const uint32_t*)tile;
    const uint32_t a = o >> 2, sh = o & 3;
    const uint32_t d0 = t32[a], d1 = t32[a + 1], d2 = t32[a + 2];
    e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
    e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
}

// Shape flags of a numeral candidate over one dword of field bytes (f: 0x80 in
// the bytes inside the field): digits, dots, and bytes that are neither.
struct NumFlags {
    uint32_t dig, dot, other;
};
__device__ __forceinline__ NumFlags num_flags(uint32_t d, uint32_t f) {
    NumFlags r;
    r.dig = digit_bytes(d) & f;
    r.dot = ~nonzero_bytes(d ^ 0x2E2E2E2Eu) & f;
    r.other = f & ~r.dig & ~r.dot;
    return r;
}

// Type a field of `len` bytes at tile offset `to` whose bytes hold no record
// terminator or delimiter (infer_type + parse_value, csv_reader.c:136-240).
// FF_OK: `out` (and `key` when want_key) are final; FF_SLOW: the general record
// path decides -- a byte <= ' ' (blank, control, NUL: leading blanks move the
// field start and a blank-only last field is dropped), a date-shaped field, a
// leading '+', a numeral past the exact fast cases, a field over 16 bytes, or a
// delimiter strtod/strtoll could read across (num_ok false).  Branches follow
// the field's shape, which is normally the same for every record of a column,
// so the wave rarely diverges here; fields of <= 8 bytes take the 64-bit path.
__device__ __forceinline__ int fast_field(const uint8_t* tile, uint32_t to, uint32_t len, bool num_ok,
                                          bool want_key, Cell& out, GKey& key) {
    out = cell_null();
    if (len == 0) {
        if (want_key) key = group_key(out);
        return FF_OK;
    }
    if (len > 16) return FF_SLOW;
    const bool wide = len > 8;
    uint32_t d0, d1, d2 = 0, d3 = 0;
    if (!wide) load8(tile, to, d0, d1);
    else load16(tile, to, d0, d1, d2, d3);
    const uint32_t m0 = len_mask(len, 0), m1 = len_mask(len, 1);
    const uint32_t m2 = wide ? len_mask(len, 2) : 0u, m3 = wide ? len_mask(len, 3) : 0u;
    uint32_t low = lt_bytes(d0 | ~m0, 0x21212121u) | lt_bytes(d1 | ~m1, 0x21212121u);
    if (wide) low |= lt_bytes(d2 | ~m2, 0x21212121u) | lt_bytes(d3 | ~m3, 0x21212121u);
    d0 &= m0; d1 &= m1; d2 &= m2; d3 &= m3;
    const uint32_t c0 = d0 & 0xffu;
    if (low || c0 == '+') return FF_SLOW;
    const uint64_t w0 = (uint64_t)d0 | ((uint64_t)d1 << 32), w1 = (uint64_t)d2 | ((uint64_t)d3 << 32);
    const bool lead = is_digit(c0) || c0 == '-' || c0 == '.';
    if (lead) {
        if (c0 != '.' && len >= 8 && len <= 10) return FF_SLOW;   // parse_date may accept it
        const bool neg = c0 == '-';
        // infer_type's numeric shape: [-] digits with at most one '.', at least one digit
        const NumFlags n0 = num_flags(d0, m0 & 0x80808080u), n1 = num_flags(d1, m1 & 0x80808080u);
        NumFlags n2 = {0, 0, 0}, n3 = {0, 0, 0};
        if (wide) { n2 = num_flags(d2, m2 & 0x80808080u); n3 = num_flags(d3, m3 & 0x80808080u); }
        const uint32_t other = (n0.other & ~(neg ? 0x80u : 0u)) | n1.other | n2.other | n3.other;
        const uint32_t ndig = __popc(n0.dig) + __popc(n1.dig) + __popc(n2.dig) + __popc(n3.dig);
        const uint32_t ndot = __popc(n0.dot) + __popc(n1.dot) + __popc(n2.dot) + __popc(n3.dot);
        if (other == 0 && ndig != 0 && ndot <= 1) {
            if (!num_ok) return FF_SLOW;
            // digit values (sign and dot bytes -> 0), dot removed, right-aligned
            const uint64_t dm0 = (uint64_t)n0.dot | ((uint64_t)n1.dot << 32);
            const uint64_t dm1 = (uint64_t)n2.dot | ((uint64_t)n3.dot << 32);
            const uint32_t pa = (uint32_t)__builtin_ctzg(dm0, 64), pz = (uint32_t)__builtin_ctzg(dm1, 64);
            const uint32_t p = (pa < 64 ? pa : 64 + pz) >> 3;       // dot byte index (16: none)
            const uint32_t lc = len - ndot;                         // digit positions (sign counted as 0)
            uint64_t W;
            if (!wide) {
                uint64_t v = (w0 ^ 0x3030303030303030ULL) & ((uint64_t)spread(n0.dig) | ((uint64_t)spread(n1.dig) << 32));
                if (ndot) {
                    const uint64_t k = (1ULL << (8 * p)) - 1;       // p <= 7
                    v = (v & k) | ((v >> 8) & ~k);
                }
                v <<= 8 * (8 - lc);
                W = dig8(v);
            } else {
                uint64_t v0 = (w0 ^ 0x3030303030303030ULL) &
                              ((uint64_t)spread(n0.dig) | ((uint64_t)spread(n1.dig) << 32));
                uint64_t v1 = (w1 ^ 0x3030303030303030ULL) &
                              ((uint64_t)spread(n2.dig) | ((uint64_t)spread(n3.dig) << 32));
                if (ndot) {
                    const uint64_t k0 = p >= 8 ? ~0ULL : ((1ULL << (8 * p)) - 1);
                    const uint64_t k1 = p >= 8 ? ((1ULL << (8 * (p - 8))) - 1) : 0ULL;
                    const uint64_t s0 = (v0 >> 8) | (v1 << 56), s1 = v1 >> 8;
                    v0 = (v0 & k0) | (s0 & ~k0);
                    v1 = (v1 & k1) | (s1 & ~k1);
                }
                const uint32_t sh = 8 * (16 - lc);                  // 0..120
                uint64_t a0, a1;
                if (sh >= 64) {
                    a1 = v0 << (sh - 64);
                    a0 = 0;
                } else {
                    a1 = sh ? (v1 << sh) | (v0 >> (64 - sh)) : v1;
                    a0 = v0 << sh;
                }
                W = (uint64_t)dig8(a0) * 100000000ULL + dig8(a1);
            }
            if (!ndot) {
                out = cell_int(neg ? -(int64_t)W : (int64_t)W);
            } else {
                if (W > (1ULL << 53)) return FF_SLOW;               // Clinger's exact case only
                const double v = (double)W / pow10_exact(len - 1 - p);   // one correctly rounded division
                out = cell_dbl(neg ? -v : v);
            }
            if (want_key) key = group_key(out);
            return FF_OK;
        }
    }
    // STRING with no blank or NUL: exactly what cq_strndup + trim_whitespace give
    out.kind = K_STR;
    out.len = len;
    out.bits = 0;                                              // caller sets the address
    if (want_key) {
        key.cls = GK_STR;
        key.len = len;
        key.w0 = w0;
        key.w1 = w1;
    }
    return FF_OK;
}

// 64-bit SWAR byte tests (0x80 in the matching bytes; no carries or borrows
// cross bytes, so 64-bit adds/subs are exact)
constexpr uint64_t H80 = 0x8080808080808080ULL, L7F = 0x7F7F7F7F7F7F7F7FULL, B01 = 0x0101010101010101ULL;
__device__ __forceinline__ uint64_t nz64(uint64_t t) { return (((t & L7F) + L7F) | t) & H80; }
__device__ __forceinline__ uint64_t lt64(uint64_t x, uint64_t rep) { return ~((x | H80) - rep) & ~x & H80; }
__device__ __forceinline__ uint64_t spread64(uint64_t f) { return f | (f - (f >> 7)); }

// The common short fields in one straight pass: 1-8 bytes, no byte <= ' ', not
// signed, and -- when digit-led -- at most 7 bytes (so never date-shaped).
// Returns false when the field is not of that kind (fast_field decides then).
// On true, `out` is the cell and `w` the field bytes zero-padded (the inline
// group key of a STRING).
__device__ __forceinline__ bool lean_field(const uint8_t* tile, uint32_t to, uint32_t len, bool num_ok, Cell& out,
                                           uint64_t& w) {
    if (len == 0 || len > 8) return false;
    uint32_t d0, d1;
    load8(tile, to, d0, d1);
    const uint64_t k = len == 8 ? ~0ULL : ((1ULL << (8 * len)) - 1);
    w = ((uint64_t)d0 | ((uint64_t)d1 << 32)) & k;
    const uint64_t f = k & H80;
    const uint32_t c0 = d0 & 0xffu;
    const bool numlead = is_digit(c0) || c0 == '.';
    if ((lt64(w | ~k, 0x21 * B01) != 0) | (c0 == '-') | (c0 == '+') | (numlead && (len == 8 || !num_ok))) return false;
    if (numlead) {
        const uint64_t dig = lt64(w ^ (0x30 * B01), 0x0A * B01) & f;
        const uint64_t dot = ~nz64(w ^ (0x2E * B01)) & f;
        const uint32_t ndot = (uint32_t)__popcll(dot);
        if ((f & ~dig & ~dot) == 0 && dig != 0 && ndot <= 1) {
            uint64_t v = (w ^ (0x30 * B01)) & spread64(dig);
            const uint32_t p = (uint32_t)__builtin_ctzg(dot, 64) >> 3;   // dot byte (8: none)
            if (ndot) {
                const uint64_t m = (1ULL << (8 * p)) - 1;                 // p <= 6
                v = (v & m) | ((v >> 8) & ~m);
            }
            v <<= 8 * (8 - (len - ndot));
            const uint64_t W = dig8(v);
            if (!ndot) out = cell_int((int64_t)W);
            else out = cell_dbl((double)W / pow10_exact(len - 1 - p));  // exact operands: correctly rounded
            return true;
        }
    }
    out.kind = K_STR;                 // STRING: no blank or NUL, so already what trim_whitespace gives
    out.len = len;
    out.bits = 0;                     // caller sets the address
    return true;
}
// one counter atomic per wave: this lane's slot among the wave's lanes with `on`
__device__ __forceinline__ unsigned long long wave_slot(bool on, unsigned long long* ctr) {
    const uint64_t m = __ballot(on);
    if (!m) return 0;
    const uint32_t lane = threadIdx.x & 63, lead = (uint32_t)__builtin_ctzll(m);
    unsigned long long base = 0;
    if (lane == lead) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
    base = __shfl(base, (int)lead, 64);
    return base + (unsigned long long)__popcll(m & ((1ull << lane) - 1));
}

__device__ __forceinline__ uint32_t popc_below(uint32_t m, uint32_t b) {
    return (uint32_t)__popc(m & ((1u << b) - 1));
}

// ------------------------------------------------------------------ MIN/MAX order
// reference keeps the first cell that compares strictly better (evaluator_aggregates.c:311-326);
// within one value class that is the lexicographic (value, position) extreme
__device__ __forceinline__ bool ext_better(uint8_t kind, const Cell& a, uint64_t pa, const Cell& b,
                                           uint64_t pb) {
    if (pb == NOPOS) return true;
    int c = compare(a, b);
    if (kind == ACC_MIN) return c < 0 || (c == 0 && pa < pb);
    return c > 0 || (c == 0 && pa < pb);
}
__device__ __forceinline__ uint32_t class_bit(const Cell& c) {
    return c.kind == K_NULL ? 0u : (c.kind == K_STR ? 2u : (c.kind == K_DATE ? 4u : 1u));
}


// the record's field `col` from global memory (the record passed a fast path: no
// quote before it, the field exists), typed by the general parser
static __device__ __noinline__ Cell field_cell(const uint8_t* __restrict__ g, uint64_t rec, uint32_t col,
                                               uint32_t delim) {
    const uint8_t* p = g + rec;
    for (uint32_t c = 0; c < col; p++) {
        const uint32_t ch = *p;
        if (ch == delim) c++;
        else if (ch == '\n' || ch == '\r') return cell_null();
    }
    uint32_t len = 0;
    while (len < 64 && p[len] != delim && p[len] != '\n' && p[len] != '\r') len++;
    return parse_cell(p, len);
}

// MIN/MAX merges take a per-slot lock.  A lock loop written per lane deadlocks
// on SIMT hardware (the compiler may park the lane that won the lock until every
// lane of the wave has won it), so every lock loop here is wave-uniform: the loop
// runs while ANY lane of the wave still needs the lock, and a lane that takes the
// lock releases it in the same trip.  Callers must reach these with the whole
// wave (uniform control flow), passing `need` = false for idle lanes.
__device__ inline void g_ext_update(bool need, const GroupTable& gt, int a, uint8_t kind, uint32_t i,
                             const Cell c, uint64_t pos, ScanStats* st) {
    if (pos == NOPOS) need = false;
    // the lock word is a sequence number (even free, odd held, +2 per update): a
    // candidate that loses against a consistent snapshot drops out without the lock
    // (the extreme only improves), so a hot group serialises only its improvements
    uint32_t* lk = &gt.lock[a][i];
    Cell* ec = &gt.ext[a][i];
    if (need) {
        const uint32_t v1 = __hip_atomic_load(lk, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        Cell cur;
        cur.kind = __hip_atomic_load(&ec->kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cur.len = __hip_atomic_load(&ec->len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cur.bits = __hip_atomic_load(&ec->bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t cp = __hip_atomic_load(&gt.extpos[a][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const uint32_t v2 = __hip_atomic_load(lk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(v1 & 1u) && v1 == v2 && !ext_better(kind, c, pos, cur, cp)) need = false;
    }
    uint32_t trips = 0;
    while (__any(need)) {
        if (need) {
            const uint32_t v = __hip_atomic_load(lk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!(v & 1u) && atomicCAS(lk, v, v + 1u) == v) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                Cell cur;
                cur.kind = __hip_atomic_load(&ec->kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                cur.len = __hip_atomic_load(&ec->len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                cur.bits = __hip_atomic_load(&ec->bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint64_t cp = __hip_atomic_load(&gt.extpos[a][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (ext_better(kind, c, pos, cur, cp)) {
                    __hip_atomic_store(&ec->kind, c.kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&ec->len, c.len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&ec->bits, c.bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&gt.extpos[a][i], (unsigned long long)pos, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                __hip_atomic_store(lk, v + 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                need = false;
            }
        }
        if (++trips > (1u << 20)) {                    // never hang: report and give up
            if (need) atomicExch(&st->overflow, 2ULL);
            break;
        }
    }
}


}  // namespace cq
