// lean.hip -- the wave-autonomous CSV scan for the common SELECT plan shapes.
//
// Same job as scan_kernel (scan.hip) -- csv_load + filter_rows + create_groups +
// evaluate_aggregate in one pass over the HBM-resident bytes (reference
// csv_reader.c:375-465, evaluator_utils.c:986, evaluator_aggregates.c:108-414) --
// for plans whose WHERE is absent or `column op literal` and whose aggregates are
// COUNT / SUM / AVG (at most 4 parsed columns, 2 distinct SUM arguments).
//
// Every wave works on its own windows with no block barrier in the loop, so one
// wave's byte classification overlaps another's record work on the same SIMD.
// The record work is arranged as a few batched LDS round trips (record start ->
// bitmap view -> field bytes -> hash slot) with the arithmetic between them:
//
//   load      a window stages 2 KiB, lane l bytes [32l, 32l + 32) (two 16-byte
//             non-temporal loads, issued one window ahead): the 16 bytes before
//             the window's own range (record-start context), its WS = 1952 owned
//             bytes, and 80 bytes after them for the record views.  Windows start
//             WS bytes apart and own the records that start in their range
//   classify  per lane two 32-bit masks -- separators (delimiter and record
//             terminators '\n' '\r') and terminators -- plus a quote mask when
//             the window holds a quote; stored as the window's LDS bitmaps
//   starts    record starts owned by the window (previous byte a terminator);
//             one DPP wave scan numbers them, 64 per pass go to an LDS list
//   fields    one lane per record: a funnel shift gives the 64 separator and
//             terminator bits from the record start, field c ends at the c-th
//             set separator bit.  A record whose needed fields are not all inside
//             those 64 bytes, or that has a quote in front of its last needed
//             field, goes whole to the slow list and slow_kernel (scan.hip)
//   values    WHERE / SUM fields of 1-7 bytes shaped `digits[.digits]` are typed
//             in registers: M = the digits, k = digits after the dot, exactly
//             parse_value's INTEGER M or DOUBLE strtod = RN(M / 10^k).  A WHERE
//             against a numeric literal L compares INTEGER fields with integer
//             thresholds ceil(L) / floor(L) and DOUBLE fields as RN(M / 10^k)
//             against L (value_compare, csv_reader.c:98-130); a short STRING
//             literal compares big-endian byte words (strcmp).  Any other field
//             shape runs the exact field typers (scanlib.h) or goes slow
//   group     the block's LDS open-addressing table is keyed by the RAW bytes of
//             the GROUP BY field (<= 16 bytes): a raw key partitions the rows at
//             least as finely as the reference's printf-canonical key.  Blocks
//             flush (and a full LDS table spills) into an HBM table of raw keys;
//             raw_merge_kernel then types every distinct raw key once with the
//             general parser (parse_cell + group_key) and merges it into the
//             canonical HBM table -- so "1.5" and "1.50" still meet there
//   aggregate COUNT and SUM are fire-and-forget LDS atomics; the block flushes once
//
// SUM addends of DOUBLE fields are M * RN(10^-k) (within 2 ulp of the reference's
// RN(M / 10^k); SUM / AVG parity is 1e-6 relative, north_star), INTEGER addends
// are exact.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstring>
#include "plan.h"
#include "scanlib.h"

namespace cq {
namespace lean {

constexpr int LT = 1024;                  // threads per block
constexpr int NWV = LT / 64;              // waves per block
constexpr int LB = 32;                    // staged bytes per lane
constexpr int WB = 64 * LB;               // staged window bytes (2 KiB)
constexpr int HEAD = 16;                  // staged bytes before the owned range
constexpr int WS = 1952;                  // largest window stride = owned bytes (LeanPlan.ws: the file's)
constexpr int NMW = WB / 32;              // 32-bit bitmap words per window
constexpr int WBYTES = WB + 32;           // staged bytes + slack for 16-byte field loads
constexpr int RSN = 64;                   // record slots per pass
constexpr int MAXS = 2;                   // distinct SUM arguments
constexpr int KN = 4;                     // need slots
constexpr uint32_t NOFIRST = 0xFFFFFFFFu;
static_assert(HEAD + WS + 64 + 16 <= WB, "a record view (64 bytes) plus a field load stays in the window");
static_assert(WS % 16 == 0, "16-byte aligned window loads");

// profiling build LEAN_CLK: shader cycles per phase, summed over waves into ScanStats.clk
#ifdef LEAN_CLK
#define LCLK(i)                                                   \
    do {                                                          \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();          \
        clk_[i] += t_ - clk_last_;                                \
        clk_last_ = t_;                                           \
    } while (0)
#elif defined(LEAN_MARK)   // asm listing markers (section sizes of the hot path)
#define LCLK(i) asm volatile(";@@LCLK " #i ::: "memory")
#else
#define LCLK(i) do {} while (0)
#endif

// WHERE shapes of this kernel
enum : int { LW_NONE = 0, LW_NUM = 1, LW_STR = 2, LW_GEN = 3 };

// per-wave LDS area
struct WaveLds {
    uint8_t bytes[WBYTES];
    uint2 bm[NMW + 2];          // {separator bits, terminator bits} per 32 window bytes
    uint32_t qt[NMW + 4];       // quote bits (written only when the window holds a quote)
    uint16_t rs[RSN];           // record starts of the current pass (window offsets)
};
static_assert(sizeof(WaveLds) % 16 == 0, "16-byte aligned wave areas");

// everything the kernel reads from constant memory
struct LeanPlan {
    uint64_t lo_ok, hi_ok;       // records starting in [lo_ok, hi_ok) are owned by this launch
    uint64_t first_win, last_win;
    uint32_t wcol;               // WHERE: CSV column compared
    uint32_t wop;                // CMP_*
    uint32_t wtt;                // its truth table (tt_result)
    int32_t wlo, whi;            // LW_NUM: INTEGER M < L <=> M < wlo; M > L <=> M > whi
    double wl;                   // LW_NUM: the literal as a double
    uint64_t wstr;               // LW_STR: literal bytes, big-endian word (zero padded)
    uint32_t pass_null;          // WHERE outcome of a NULL / missing field
    Cell wconst;                 // LW_GEN: the literal cell
    int32_t ns;                  // distinct SUM argument slots
    int32_t sum_slot[MAXS];      // need slot of each
    uint32_t scol[MAXS];         // CSV column of each
    int32_t nacc;
    int32_t acc_sidx[MAX_ACC];   // accumulator -> SUM index
    uint32_t gcol;               // GROUP BY CSV column
    uint32_t delim, quote;
    uint32_t ws;                 // window stride: multiple of 16, <= WS
    uint32_t rcol[KN];           // the roles' CSV columns, ascending
    uint32_t rrole[KN];          // their roles: R_WHERE, R_SUM0, R_SUM1, R_GROUP
};
enum : uint32_t { R_WHERE = 0, R_SUM0 = 1, R_SUM1 = 2, R_GROUP = 3 };

// kernel arguments (kernarg segment).  The two HBM group tables (canonical keys,
// shared with slow_kernel, and raw-byte keys for block flushes and LDS spills) are
// read through a pointer to a device copy instead: only the rare spill path and
// the final flush touch them, and their ~1 KB of pointers held in scalar
// registers across the window loop spilled SGPRs into VGPR lanes.
struct LeanArgs {
    LeanPlan lp;
};
enum : int { TAB_GT = 0, TAB_RT = 1 };
__device__ GroupTable g_lean_tabs[2];

constexpr uint32_t GK_RAW = 6;       // raw field bytes as key (cell.h GK_* never produce 6)
__device__ __forceinline__ GKey raw_key(uint32_t len, uint64_t w0, uint64_t w1) {
    GKey k;
    k.cls = GK_RAW; k.len = len; k.w0 = w0; k.w1 = w1;
    return k;
}

#ifndef LEAN_PF
#define LEAN_PF 1          // windows in flight per wave (1 or 2; 2 measured 2.58 vs 2.52 ms on config 3)
#endif
struct Win {            // one window in flight
    v4u a, b;           // staged bytes [32l, 32l + 32)
};

__device__ __forceinline__ void load_win(const uint8_t* g, uint64_t w, uint32_t ws, Win& x) {
    const v4u* src = (const v4u*)(g + w * ws - HEAD);   // g has 64 padding bytes before byte 0
    const int lane = threadIdx.x & 63;
    x.a = __builtin_nontemporal_load(src + 2 * lane);
    x.b = __builtin_nontemporal_load(src + 2 * lane + 1);
}

// 0x80 flags -> a nibble (bit i = byte i)
__device__ __forceinline__ uint32_t nib(uint32_t f) {
    uint32_t t = f >> 7;
    t |= t >> 7;
    t |= t >> 14;
    return t & 0xFu;
}

// separator / terminator / quote bits of 32 bytes (bit i = byte i).
//
// Byte classes by v_perm_b32 lookups: a selector byte 0-7 picks a table byte,
// 8-11 the sign of table byte 1/3/5/7, 12 gives 0x00 and 13-255 give 0xFF.  With
// z = x ^ 0x08 the terminators land on selectors 2 ('\n') and 5 ('\r'), with
// z = x ^ delim the delimiter on 0; those table bytes are 0x40, all others 0, so
// a byte's lookup is 0x40 exactly when it is in the class, else 0x00 or 0xFF
// (bit 6 and not bit 7 is the flag).  Needs delim >= 0x10, so that '\n' / '\r'
// xor delim and delim xor 0x08 are never selectors 0-12 (lean_shape: delim > ' ').
// The 0x40 flags of two dwords become a byte of bits with one v_dot4_u32_u8
// each (weights 1..128), four such bytes the 32-bit mask.  Quote presence is
// the borrow-based zero-byte test (exact for "any").
__device__ __forceinline__ uint32_t flags40(uint32_t r) {
    return r & ~(r >> 1) & 0x40404040u;
}
__device__ __forceinline__ void classify(const v4u a, const v4u b, uint32_t rep_d, uint32_t rep_q, uint32_t& sep,
                                         uint32_t& nl, uint32_t& qf) {
    uint32_t us[4], un[4], q = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t x = j < 4 ? a[j & 3] : b[j & 3];
        const uint32_t rn = __builtin_amdgcn_perm(0x00004000u, 0x00400000u, x ^ 0x08080808u);
        const uint32_t rd = __builtin_amdgcn_perm(0u, 0x00000040u, x ^ rep_d);
        const uint32_t fs = flags40(rn & rd), fn = flags40(rn);
        const uint32_t w = (j & 1) ? 0x80402010u : 0x08040201u;
        if (j & 1) {
            us[j >> 1] = __builtin_amdgcn_udot4(fs, w, us[j >> 1], false);
            un[j >> 1] = __builtin_amdgcn_udot4(fn, w, un[j >> 1], false);
        } else {
            us[j >> 1] = __builtin_amdgcn_udot4(fs, w, 0u, false);
            un[j >> 1] = __builtin_amdgcn_udot4(fn, w, 0u, false);
        }
        const uint32_t t = x ^ rep_q;
        q |= (t - 0x01010101u) & ~t;
    }
    // us[p] = 0x40 * (bits of bytes 8p .. 8p + 7)
    sep = (us[0] >> 6) | (us[1] << 2) | (us[2] << 10) | (us[3] << 18);
    nl = (un[0] >> 6) | (un[1] << 2) | (un[2] << 10) | (un[3] << 18);
    qf = q & 0x80808080u;
}
__device__ __forceinline__ uint32_t byte_bits(const v4u a, const v4u b, uint32_t rep) {
    uint32_t m = 0;
#pragma unroll
    for (int v = 0; v < 2; v++) {
#pragma unroll
        for (int j = 0; j < 4; j++) m |= nib(~nonzero_bytes((v ? b[j] : a[j]) ^ rep) & 0x80808080u) << ((v * 4 + j) * 4);
    }
    return m;
}

// same-wave LDS hand-off: DS operations of one wave execute in issue order, so only
// the compiler must not move LDS accesses across this point
__device__ __forceinline__ void wave_order() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint32_t ctz64(uint64_t x) { return (uint32_t)__builtin_ctzg(x, 64); }
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }

// 64 bitmap bits starting at window offset p
__device__ __forceinline__ void views(const WaveLds& W, uint32_t p, uint64_t& sv, uint64_t& nv) {
    const uint32_t wi = p >> 5, sh = p & 31;
    const uint2 b0 = W.bm[wi], b1 = W.bm[wi + 1], b2 = W.bm[wi + 2];
    sv = (uint64_t)__builtin_amdgcn_alignbit(b1.x, b0.x, sh) |
         ((uint64_t)__builtin_amdgcn_alignbit(b2.x, b1.x, sh) << 32);
    nv = (uint64_t)__builtin_amdgcn_alignbit(b1.y, b0.y, sh) |
         ((uint64_t)__builtin_amdgcn_alignbit(b2.y, b1.y, sh) << 32);
}
__device__ __forceinline__ uint64_t qview(const WaveLds& W, uint32_t p) {
    const uint32_t wi = p >> 5, sh = p & 31;
    const uint32_t q0 = W.qt[wi], q1 = W.qt[wi + 1], q2 = W.qt[wi + 2];
    return (uint64_t)__builtin_amdgcn_alignbit(q1, q0, sh) | ((uint64_t)__builtin_amdgcn_alignbit(q2, q1, sh) << 32);
}

// 4 bytes of the tile at byte offset o (any alignment)
__device__ __forceinline__ void load4(const uint8_t* tile, uint32_t o, uint32_t& e0) {
    const uint32_t* t32 = (const uint32_t*)tile;
    const uint32_t a = o >> 2, sh = o & 3;
    e0 = __builtin_amdgcn_alignbyte(t32[a + 1], t32[a], sh);
}

// bytes [0, len) of two dwords (len <= 8)
__device__ __forceinline__ void mask8(uint32_t len, uint32_t& d0, uint32_t& d1) {
    const uint32_t n1 = len > 4 ? len - 4 : 0;
    d0 &= len >= 4 ? 0xFFFFFFFFu : ((1u << (8 * len)) - 1);
    d1 &= n1 >= 4 ? 0xFFFFFFFFu : ((1u << (8 * n1)) - 1);
}

// 0x80 in every byte < 0x21 (blank, control, NUL) among the bytes of f-flags
__device__ __forceinline__ uint32_t low_bytes(uint32_t d, uint32_t f) { return lt_bytes(d, 0x21212121u) & f; }

// A field of 1..7 bytes shaped [digits][.][digits] with at least one digit (no sign,
// so never date-shaped: parse_date needs 8-10 bytes): infer_type gives INTEGER
// (no dot) or DOUBLE, parse_value M or strtod = RN(M / 10^k).  d0/d1: the field's
// first 8 bytes, unmasked.  Branch-free; M, k and dot are meaningful when ok.
struct Num {
    uint32_t M, k;
    bool ok, dot;
};
__device__ __forceinline__ Num num7(uint32_t d0, uint32_t d1, uint32_t len) {
    Num r;
    const uint32_t f0 = len_mask(len, 0) & 0x80808080u, f1 = len_mask(len, 1) & 0x80808080u;
    const uint32_t x0 = d0 ^ 0x30303030u, x1 = d1 ^ 0x30303030u;
    const uint32_t g0 = lt_bytes(x0, 0x0A0A0A0Au) & f0, g1 = lt_bytes(x1, 0x0A0A0A0Au) & f1;   // digits
    const uint32_t t0 = ~nonzero_bytes(d0 ^ 0x2E2E2E2Eu) & f0, t1 = ~nonzero_bytes(d1 ^ 0x2E2E2E2Eu) & f1;  // dots
    const uint32_t ndot = (uint32_t)__popc(t0) + (uint32_t)__popc(t1);
    r.ok = (len - 1 <= 6u) & ((g0 | t0) == f0) & ((g1 | t1) == f1) & (ndot <= 1) & ((g0 | g1) != 0);
    uint64_t v = ((uint64_t)(x0 & spread(g0)) | ((uint64_t)(x1 & spread(g1)) << 32));   // digit values, dot -> 0
    const uint64_t tm = (uint64_t)t0 | ((uint64_t)t1 << 32);
    uint32_t pd = ctz64(tm) >> 3;                                       // dot byte (8: none)
    pd = pd > 7 ? 7u : pd;
    r.dot = ndot != 0;
    const uint64_t lo = (1ULL << (8 * pd)) - 1;
    v = r.dot ? ((v & lo) | ((v >> 8) & ~lo)) : v;
    r.k = r.dot ? len - 1 - pd : 0u;
    r.k = r.k > 7 ? 7u : r.k;
    uint32_t nd2 = len - ndot;                                            // digits
    nd2 = nd2 - 1 > 7u ? 1u : nd2;
    v <<= 8 * (8 - nd2);                                                 // right-align the digits
    // digits -> value: three byte dot products (v_dot4_u32_u8) over 3 + 3 + 2 digits
    const uint32_t vl = (uint32_t)v, vh = (uint32_t)(v >> 32);
    const uint32_t e1 = __builtin_amdgcn_udot4(vl, 0x00010A64u, 0u, false);
    const uint32_t e2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(vh, vl, 3), 0x00010A64u, 0u, false);
    const uint32_t e3 = __builtin_amdgcn_udot4(vh, 0x010A0000u, 0u, false);
    r.M = __umul24(__umul24(e1, 1000u) + e2, 100u) + e3;
    return r;
}

// num7 for fields of 1..4 bytes (one dword): the same M, k, dot and ok for every
// field num7 accepts with len <= 4; ok is false for longer fields.  The kernel
// takes it when every lane's field of the role fits (a wave-uniform choice).
__device__ __forceinline__ Num num4(uint32_t d0, uint32_t len) {
    Num r;
    const uint32_t f = len_mask(len, 0) & 0x80808080u;
    const uint32_t x = d0 ^ 0x30303030u;
    const uint32_t g = lt_bytes(x, 0x0A0A0A0Au) & f;                   // digits
    const uint32_t t = ~nonzero_bytes(d0 ^ 0x2E2E2E2Eu) & f;            // dots
    const uint32_t ndot = (uint32_t)__popc(t);
    r.ok = (len - 1 <= 3u) & ((g | t) == f) & (ndot <= 1) & (g != 0);
    uint32_t v = x & spread(g);                                         // digit values, dot -> 0
    uint32_t pd = (uint32_t)__builtin_ctz(t | 0x80000000u) >> 3;        // dot byte (3 when none or last)
    r.dot = ndot != 0;
    const uint32_t lo = (1u << (8 * pd)) - 1;
    v = r.dot ? ((v & lo) | ((v >> 8) & ~lo)) : v;
    r.k = r.dot ? len - 1 - pd : 0u;
    r.k = r.k > 3 ? 3u : r.k;
    uint32_t nd = len - ndot;                                           // digits
    nd = nd - 1 > 3u ? 1u : nd;
    v <<= 8 * (4 - nd);                                                 // right-align the digits
    r.M = __builtin_amdgcn_udot4(v, 0x010A6400u, __umul24(v & 0xFFu, 1000u), false);
    return r;
}

// Field `c` of the record at window offset p from its 64-bit separator view sv
// (delimiters and terminators, bit i = byte p + i) and its end e (the first
// terminator; 64: beyond the view).  Clearing the c lowest separator bits leaves
// the field's end as the lowest bit; the cleared bits' highest is its start - 1.
// A column past the record's end is missing (length 0: NULL); a field the view
// cannot bound fails the fast path.  The roles' columns come in ascending order,
// so s and `done` carry the cleared bits from one role to the next (the clears
// of a record total its largest column, not the sum of the columns).  c is
// uniform: a scalar loop.
__device__ __forceinline__ void field_next(uint64_t sv, uint64_t& s, uint32_t& done, uint32_t e, uint32_t c,
                                           uint32_t p, uint32_t& fp, uint32_t& fl, bool& fail, uint32_t& last) {
    for (; done < c; done++) s &= s - 1;
    const uint64_t cl = sv ^ s;
    const uint32_t start = cl ? 64u - (uint32_t)__builtin_clzll(cl) : 0u;
    const uint32_t end = ctz64(s);
    const bool gone = start > e;
    fail |= gone ? (e == 64) : (end == 64);
    fp = p + start;
    fl = gone ? 0u : end - start;
    const uint32_t l = gone ? e : end;
    last = l > last ? l : last;
}

// value_compare outcome through a truth table: bit 0 for <, bit 1 for ==, bit 2 for >
__device__ __forceinline__ bool tt_result(uint32_t tt, int c) { return (tt >> (c < 0 ? 0 : (c == 0 ? 1 : 2))) & 1; }

// 10^k (exact) and ~10^-k (three rounded products, SUM addends only), k = 0..7
__device__ __forceinline__ double p10(uint32_t k) {
    return ((k & 1) ? 10.0 : 1.0) * ((k & 2) ? 100.0 : 1.0) * ((k & 4) ? 1e4 : 1.0);
}
__device__ __forceinline__ double inv10(uint32_t k) {
    return ((k & 1) ? 0.1 : 1.0) * ((k & 2) ? 0.01 : 1.0) * ((k & 4) ? 1e-4 : 1.0);
}

// exact typing of a field (infer_type + parse_value); false: only the general
// parser can tell (dates, signs, long numerals, blanks ...)
__device__ __forceinline__ bool type_field(const uint8_t* bytes, uint32_t o, uint32_t len, Cell& c) {
    if (len == 0) { c = cell_null(); return true; }
    uint64_t kw;
    if (lean_field(bytes, o, len, true, c, kw)) return true;
    GKey unused;
    return fast_field(bytes, o, len, true, false, c, unused) == FF_OK;
}

__device__ __forceinline__ uint64_t bswap64(uint32_t d0, uint32_t d1) {
    return ((uint64_t)__builtin_bswap32(d0) << 32) | __builtin_bswap32(d1);
}

// LDS group table (structure of arrays carved from dynamic LDS), raw-byte keys.
// Slots are grouped in buckets of BS = 16; a key's home bucket is its hash's top
// bits, and a bucket's 16 u16 fingerprints (0: free, FP_BUSY: being written) are
// read with two 16-byte loads.  A lookup is two batched round trips:
// fingerprints, then the first matching slot's key.  Keys missing from their
// home bucket's first match (new keys, bucket overflow, fingerprint collisions)
// take lt_slow: lock-free linear probing over the slots from the home bucket.
constexpr uint32_t BS = 16;
constexpr uint32_t FP_BUSY = 0xFFFEu;   // fingerprints are odd

// LDS bytes per table slot (fingerprint, key, count, SUM/miss per argument) and
// the slots of a plan shape: a compile-time constant of each kernel instance, so
// every table array sits at an immediate LDS offset
constexpr uint32_t slot_bytes(int ns) { return 2 + 16 + 8 + 4 + (uint32_t)ns * 12; }
constexpr uint32_t fixed_bytes() { return (uint32_t)(sizeof(WaveLds) * NWV); }
constexpr uint32_t slots_for(int ns, bool grouped) {
    if (!grouped) return 0;
    uint32_t h = 2048;
    while (h > 64 && fixed_bytes() + h * slot_bytes(ns) + 512 > 160u * 1024u) h >>= 1;
    return h;
}
struct LTab {
    uint32_t H;           // slots (multiple of BS)
    uint32_t NB;          // buckets
    v4u* F;               // fingerprints: bucket b = F[2b], F[2b + 1]
    v4u* A;               // {0x80000000 | len, first-row code, key bytes 0-3, key bytes 4-7}
    uint2* B;             // key bytes 8-15
    uint32_t* cnt;
    double* sum[MAXS];
    uint32_t* miss[MAXS]; // SUM arguments that were not numeric
};

__device__ __forceinline__ uint32_t key_hash(uint32_t len, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    uint32_t x = k0 ^ rotl(k1, 7) ^ rotl(k2, 13) ^ rotl(k3, 21) ^ (len << 27);
    x *= 0x9E3779B1u;
    x ^= x >> 15;
    x *= 0x85EBCA6Bu;
    return x ^ (x >> 13);
}
__device__ __forceinline__ uint32_t fp_of(uint32_t h) { return (h & 0xFFFFu) | 1u; }
__device__ __forceinline__ uint32_t bucket_of(uint32_t h, uint32_t nb) { return __umulhi(h, nb); }

// index of the first of the 16 u16 fingerprints equal to fp (16: none).  Per
// dword the borrow-based zero-half test (its lowest flag is exact) leaves flags at
// bits 15 and 31; one v_dot4_u32_u8 per dword weighs them 4^j * {1, 2} into a
// chained 8-bit mask (times 0x80) per four dwords.
__device__ __forceinline__ uint32_t fp_first(const v4u q0, const v4u q1, uint32_t fp) {
    const uint32_t rep = fp * 0x00010001u;
    uint32_t m0 = 0, m1 = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t x0 = q0[j] ^ rep, x1 = q1[j] ^ rep;
        const uint32_t f0 = (x0 - 0x00010001u) & ~x0 & 0x80008000u;
        const uint32_t f1 = (x1 - 0x00010001u) & ~x1 & 0x80008000u;
        const uint32_t w = (1u << (2 * j + 8)) | (2u << (2 * j + 24));     // bytes 1 and 3
        m0 = __builtin_amdgcn_udot4(f0, w, m0, false);
        m1 = __builtin_amdgcn_udot4(f1, w, m1, false);
    }
    return (uint32_t)__builtin_ctz((m0 >> 7) | (m1 << 1) | 0x10000u);
}

// Find the key or insert it: linear probing over slots from the home bucket.  A
// free fingerprint is claimed FP_BUSY by CAS on its dword, the key written, then
// the fingerprint published; every inserter of a key probes the same sequence,
// so two of them meet at the same first free slot and the loser finds the
// winner's key.  -1: the table is full or a claim never resolved (the HBM raw
// table takes the record).
__device__ __forceinline__ int lt_slow(const LTab& t, uint32_t len, uint32_t k0, uint32_t k1, uint32_t k2,
                                       uint32_t k3, uint32_t h, uint32_t& first) {
    const uint32_t hd = 0x80000000u | len, fp = fp_of(h);
    uint32_t slot = bucket_of(h, t.NB) * BS;
    uint32_t* f32 = (uint32_t*)t.F;
    uint32_t n = 0;
    for (uint32_t it = 0; it < 4 * t.H + 4096; it++) {
        const uint32_t sh = 16 * (slot & 1);
        const uint32_t d = __hip_atomic_load(f32 + (slot >> 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t x = (d >> sh) & 0xFFFFu;
        if (x == 0) {
            const uint32_t old = atomicCAS(f32 + (slot >> 1), d, d | (FP_BUSY << sh));
            if (old == d) {                                 // claimed: write the key, publish
                t.A[slot] = v4u{hd, NOFIRST, k0, k1};
                t.B[slot] = make_uint2(k2, k3);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                atomicXor(f32 + (slot >> 1), (FP_BUSY ^ fp) << sh);
                first = NOFIRST;
                return (int)slot;
            }
            continue;                                       // the dword changed: look again
        }
        if (x == FP_BUSY) continue;                         // being written: look again
        if (x == fp) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const v4u a = t.A[slot];
            const uint2 b = t.B[slot];
            if (a.x == hd && a.z == k0 && a.w == k1 && b.x == k2 && b.y == k3) {
                first = a.y;
                return (int)slot;
            }
        }
        if (++n == t.H) return -1;
        slot = slot + 1 == t.H ? 0 : slot + 1;
    }
    return -1;
}

// the canonical group key of a raw key: bytes staged in LDS (zero padded, so
// strtod / strtoll stop at the field end), the general parser, group_key
__device__ __noinline__ GKey canonical_key(uint8_t* sb, uint32_t len, uint64_t w0, uint64_t w1) {
    ((uint64_t*)sb)[0] = w0;
    ((uint64_t*)sb)[1] = w1;
    ((uint64_t*)sb)[2] = 0;
    const Cell c = parse_cell(sb, len);
    return group_key(c);
}

__device__ __forceinline__ uint8_t* carve(uint8_t*& q, size_t bytes) {
    uint8_t* r = q;
    q += (bytes + 15) & ~(size_t)15;
    return r;
}

// GROUPED: GROUP BY (else one group); WM: LW_*; NS: distinct SUM arguments (0-2)
template <bool GROUPED, int WM, int NS>
__global__ __launch_bounds__(LT) void lean_kernel(const uint8_t* __restrict__ g, ScanStats* __restrict__ stats,
                                                  unsigned long long* __restrict__ row_out,
                                                  unsigned long long row_cap, uint32_t lds_h_unused,
                                                  unsigned long long* __restrict__ slow_list,
                                                  unsigned long long slow_cap, const LeanArgs args,
                                                  const GroupTable* __restrict__ tabs) {
    const LeanPlan& LP = args.lp;
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t* q = smem;
    WaveLds* waves = (WaveLds*)carve(q, sizeof(WaveLds) * NWV);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: the window loop is scalar
    WaveLds& W = waves[wv];
    constexpr uint32_t lds_h = slots_for(NS, GROUPED);
    LTab lt;
    lt.H = lds_h;
    lt.NB = 0; lt.F = nullptr;
    lt.A = nullptr; lt.B = nullptr; lt.cnt = nullptr;
#pragma unroll
    for (int s = 0; s < MAXS; s++) { lt.sum[s] = nullptr; lt.miss[s] = nullptr; }
    if (GROUPED) {
        lt.NB = lds_h / BS;
        lt.F = (v4u*)carve(q, (size_t)lds_h * 2);
        lt.A = (v4u*)carve(q, (size_t)lds_h * 16);
        lt.B = (uint2*)carve(q, (size_t)lds_h * 8);
        lt.cnt = (uint32_t*)carve(q, (size_t)lds_h * 4);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            lt.sum[s] = (double*)carve(q, (size_t)lds_h * 8);
            lt.miss[s] = (uint32_t*)carve(q, (size_t)lds_h * 4);
        }
        for (uint32_t i = tid; i < lds_h; i += LT) {
            lt.A[i] = v4u{0u, NOFIRST, 0u, 0u};
            lt.B[i] = make_uint2(0u, 0u);
            lt.cnt[i] = 0;
#pragma unroll
            for (int s = 0; s < NS; s++) { lt.sum[s][i] = 0.0; lt.miss[s][i] = 0; }
        }
        for (uint32_t i = tid; i < lt.NB * 2; i += LT) lt.F[i] = v4u{0u, 0u, 0u, 0u};
        __syncthreads();
    }

    // uniform plan facts
    constexpr int NR = (WM != LW_NONE ? 1 : 0) + NS + (GROUPED ? 1 : 0);   // roles
    uint32_t rcol[KN], rrole[KN];
#pragma unroll
    for (int k = 0; k < KN; k++) {
        rcol[k] = __builtin_amdgcn_readfirstlane(LP.rcol[k]);
        rrole[k] = __builtin_amdgcn_readfirstlane(LP.rrole[k]);
    }
    const uint32_t rep_d = LP.delim * 0x01010101u, rep_q = LP.quote * 0x01010101u;
    const uint64_t lo_ok = LP.lo_ok, hi_ok = LP.hi_ok, last_win = LP.last_win;
    const uint32_t wstr_b = __builtin_amdgcn_readfirstlane(LP.ws);   // window stride
    // WHERE facts in scalar registers (no constant reloads inside the loop)
    const bool pass_null = __builtin_amdgcn_readfirstlane(LP.pass_null) != 0;
    const int wlo = __builtin_amdgcn_readfirstlane(LP.wlo), whi = __builtin_amdgcn_readfirstlane(LP.whi);
    const uint32_t wtt = __builtin_amdgcn_readfirstlane(LP.wtt);
    const double wl = WM == LW_NUM ? LP.wl : 0.0;
    const uint64_t wstr = WM == LW_STR ? LP.wstr : 0ull;
    const uint64_t tile_g = (uint64_t)(uintptr_t)W.bytes;
    const uint64_t wstep = (uint64_t)gridDim.x * NWV;

    // per-lane single-group partials and per-wave statistics
    uint32_t my_cnt = 0;
    unsigned long long my_first = ~0ULL;
    double my_sum[MAXS] = {0.0, 0.0};
    uint32_t my_num[MAXS] = {0u, 0u};
    unsigned long long n_rec = 0, n_pass = 0, n_spill = 0;

#ifdef LEAN_CLK
    uint64_t clk_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t clk_last_ = __builtin_amdgcn_s_memtime();
#endif
    // LEAN_PF windows in flight per wave (the one being processed + LEAN_PF - 1
    // prefetched): 4 waves per SIMD with one 2 KiB window each leave too few bytes
    // in flight to cover HBM latency at full bandwidth (Little's law)
    Win nx;
#if LEAN_PF >= 2
    Win nx2;
#endif
    uint64_t w = LP.first_win + (uint64_t)blockIdx.x * NWV + wv;
    if (w < last_win) load_win(g, w, wstr_b, nx);
#if LEAN_PF >= 2
    if (w + wstep < last_win) load_win(g, w + wstep, wstr_b, nx2);
#endif
    for (uint32_t round = 0; w < last_win; round++, w += wstep) {
        const uint64_t ws = w * wstr_b;
#ifdef LEAN_CLK
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        const Win cur = nx;
        LCLK(0);
#ifndef LEAN_NOMEM   // profiling build LEAN_NOMEM: every window re-processes the first one (no HBM reads)
#if LEAN_PF >= 2
        nx = nx2;
        if (w + 2 * wstep < last_win) load_win(g, w + 2 * wstep, wstr_b, nx2);
#else
        if (w + wstep < last_win) load_win(g, w + wstep, wstr_b, nx);
#endif
#endif

        // ---- stage and classify
        ((v4u*)W.bytes)[2 * lane] = cur.a;
        ((v4u*)W.bytes)[2 * lane + 1] = cur.b;
#if defined(LEAN_PROF) && LEAN_PROF == 0   // profiling build: loads + staging only
        if (lane == 0) n_rec += W.bytes[w & 2047];
        continue;
#endif
        uint32_t sep, nl, qf;
        classify(cur.a, cur.b, rep_d, rep_q, sep, nl, qf);
        W.bm[lane] = make_uint2(sep, nl);
        const bool wq = __ballot(qf != 0) != 0;           // window holds a quote (uniform)
        if (wq) W.qt[lane] = byte_bits(cur.a, cur.b, rep_q);

        // ---- record starts owned by this window: file [ws, ws + WS) within [lo_ok, hi_ok)
        const uint32_t prevnl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(nl >> 31), 0x138, 0xf, 0xf, true);
        uint32_t starts = ~nl & ((nl << 1) | prevnl);
        {
            const uint64_t lo64 = (lo_ok > ws ? lo_ok : ws) - ws;
            const uint64_t hi64 = hi_ok < ws + wstr_b ? hi_ok : ws + wstr_b;
            const uint32_t lo_s = HEAD + (uint32_t)(lo64 < (uint64_t)wstr_b ? lo64 : (uint64_t)wstr_b);   // staged offsets
            const uint32_t hi_s = hi64 > ws ? HEAD + (uint32_t)(hi64 - ws) : (uint32_t)HEAD;
            const uint32_t b0 = (uint32_t)lane * LB;
            if (b0 + LB <= lo_s || b0 >= hi_s) {
                starts = 0;
            } else {
                if (lo_s > b0) starts &= ~0u << (lo_s - b0);
                if (hi_s < b0 + LB) starts &= (1u << (hi_s - b0)) - 1;
            }
        }
        const uint32_t nst = (uint32_t)__popc(starts);
        const uint32_t incl = wave_incl_scan(nst);
        const uint32_t rbase = incl - nst;
        const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);

        LCLK(1);
#if defined(LEAN_PROF) && LEAN_PROF == 1   // profiling build: + classify, bitmaps, record numbering
        n_rec += R;
        continue;
#endif
        for (uint32_t pass = 0; pass < R; pass += RSN) {
            // this pass's record starts -> W.rs
            {
                uint32_t m = starts, r = rbase - pass;
                while (m) {
                    const uint32_t b = (uint32_t)__builtin_ctz(m);
                    m &= m - 1;
                    if (r < (uint32_t)RSN) W.rs[r] = (uint16_t)(lane * LB + b);
                    r++;
                }
            }
            wave_order();
            const bool valid = pass + lane < R;
            const uint32_t p = valid ? W.rs[lane] : (uint32_t)HEAD;

            // ---- role fields (WHERE, SUM 0/1, GROUP BY): position and length (0: NULL / missing)
            uint64_t sv, nv;
            views(W, p, sv, nv);
            const uint32_t e = ctz64(nv);                  // record end (64: beyond the view)
            bool fail = !valid;
            uint32_t lastpos = 0;
            uint32_t wfp = p, wfl = 0, gfp = p, klen = 0;
            uint32_t sfp[MAXS], sfl[MAXS];
#pragma unroll
            for (int j = 0; j < MAXS; j++) { sfp[j] = p; sfl[j] = 0; }
            {
                uint64_t s = sv;
                uint32_t done = 0;
#pragma unroll
                for (int k = 0; k < NR; k++) {
                    uint32_t fp_, fl_;
                    field_next(sv, s, done, e, rcol[k], p, fp_, fl_, fail, lastpos);
                    const uint32_t role = rrole[k];
                    if (WM != LW_NONE && role == R_WHERE) { wfp = fp_; wfl = fl_; }
                    if (NS > 0 && role == R_SUM0) { sfp[0] = fp_; sfl[0] = fl_; }
                    if (NS > 1 && role == R_SUM1) { sfp[MAXS - 1] = fp_; sfl[MAXS - 1] = fl_; }
                    if (GROUPED && role == R_GROUP) { gfp = fp_; klen = fl_; }
                }
            }
            // a quote at or before the last byte examined may hide separators
            if (wq) fail |= (qview(W, p) & ((2ULL << (lastpos < 63 ? lastpos : 63)) - 1)) != 0;

            // ---- wave-uniform field-size classes: every lane's numeric WHERE / SUM field
            //      fits a dword (num4), every GROUP BY key fits 8 bytes (two-word keys)
            const bool w4 = WM == LW_NUM && __all(!valid | (wfl <= 4u));
            bool s4 = NS > 0;
#pragma unroll
            for (int j = 0; j < NS; j++) s4 = s4 && __all(!valid | (sfl[j] <= 4u));
            const bool g8 = GROUPED && __all(!valid | (klen <= 8u));

            // ---- field bytes of the roles (one batch of LDS reads)
            uint32_t wd0 = 0, wd1 = 0;
            if (WM != LW_NONE) {
                if (w4) load4(W.bytes, wfp, wd0);
                else load8(W.bytes, wfp, wd0, wd1);
            }
            uint32_t sd0[MAXS], sd1[MAXS];
#pragma unroll
            for (int j = 0; j < MAXS; j++) {
                sd0[j] = sd1[j] = 0;
                if (j < NS) {
                    if (s4) load4(W.bytes, sfp[j], sd0[j]);
                    else load8(W.bytes, sfp[j], sd0[j], sd1[j]);
                }
            }
            uint32_t k0 = 0, k1 = 0, k2 = 0, k3 = 0;
            if (GROUPED) {
                if (g8) load8(W.bytes, gfp, k0, k1);
                else load16(W.bytes, gfp, k0, k1, k2, k3);
            }

            LCLK(2);
#if defined(LEAN_PROF) && LEAN_PROF == 2   // profiling build: + record list, field walk, field loads
            n_rec += __popcll(__ballot(fail || ((wd0 ^ sd0[0] ^ k0 ^ lastpos) & 1)));
            wave_order();
            continue;
#endif
            // ---- WHERE outcome: numerals and short strings in registers, else the exact typers
            bool pass_ = true;
            if (WM != LW_NONE) {
                bool outcome = pass_null;                  // missing column / empty field: NULL
                bool typed = wfl == 0;
                if (WM == LW_NUM) {
                    const Num n = w4 ? num4(wd0, wfl) : num7(wd0, wd1, wfl);
                    int c = (int)n.M < wlo ? -1 : ((int)n.M > whi ? 1 : 0);
                    if (__any(n.ok & n.dot)) {             // DOUBLE fields: strtod = RN(M / 10^k)
                        const double d = (double)n.M / p10(n.k);
                        if (n.dot) c = d < wl ? -1 : (d > wl ? 1 : 0);
                    }
                    if (n.ok) outcome = tt_result(wtt, c);
                    typed |= n.ok;
                } else if (WM == LW_STR) {
                    // a STRING field of <= 8 bytes: no leading digit / sign / dot (never a
                    // numeral or date), no byte <= ' ' (trim_whitespace is a no-op)
                    uint32_t a0 = wd0, a1 = wd1;
                    const uint32_t c0 = a0 & 0xFFu;
                    mask8(wfl, a0, a1);
                    const uint32_t f0 = len_mask(wfl, 0) & 0x80808080u, f1 = len_mask(wfl, 1) & 0x80808080u;
                    const bool ok = (wfl - 1 < 8u) & !(is_digit(c0) | (c0 == '-') | (c0 == '+') | (c0 == '.')) &
                                    ((low_bytes(a0, f0) | low_bytes(a1, f1)) == 0);
                    const uint64_t x = bswap64(a0, a1);
                    if (ok) outcome = tt_result(wtt, x < wstr ? -1 : (x > wstr ? 1 : 0));
                    typed |= ok;
                }
                const bool gen = !typed & !fail;
                if (__any(gen)) {                          // the exact typers (rare shapes)
                    if (gen) {
                        Cell c;
                        if (!type_field(W.bytes, wfp, wfl, c)) {
                            fail = true;
                        } else {
                            if (c.kind == K_STR) c.bits = tile_g + wfp;
                            outcome = tt_result(wtt, compare(c, LP.wconst));
                        }
                    }
                }
                pass_ = outcome;
            }

            // ---- SUM addends (numeric: true and the value)
            double sval[MAXS];
            bool snum[MAXS];
#pragma unroll
            for (int j = 0; j < MAXS; j++) {
                sval[j] = 0.0;
                snum[j] = false;
                if (j >= NS) continue;
                Num n;
                if (s4) {
                    n = num4(sd0[j], sfl[j]);
                    sval[j] = (double)n.M * (((n.k & 1) ? 0.1 : 1.0) * ((n.k & 2) ? 0.01 : 1.0));   // = inv10(k), k <= 3
                } else {
                    n = num7(sd0[j], sd1[j], sfl[j]);
                    sval[j] = (double)n.M * inv10(n.k);
                }
                snum[j] = n.ok;
                const bool gen = !n.ok & (sfl[j] != 0) & !fail;
                if (__any(gen)) {
                    if (gen) {
                        Cell c;
                        if (!type_field(W.bytes, sfp[j], sfl[j], c)) fail = true;
                        else if (is_num(c)) { sval[j] = num_of(c); snum[j] = true; }
                    }
                }
            }

            // ---- GROUP BY key: the raw field bytes (<= 16, no byte <= ' ')
            uint32_t h = 0;
            if (GROUPED) {
                if (g8) {
                    const uint32_t m0 = len_mask(klen, 0), m1 = len_mask(klen, 1);
                    k0 &= m0; k1 &= m1;
                    const uint32_t lowb = low_bytes(k0, m0 & 0x80808080u) | low_bytes(k1, m1 & 0x80808080u);
                    fail |= lowb != 0;
                    h = key_hash(klen, k0, k1, 0u, 0u);
                } else {
                    const uint32_t m0 = len_mask(klen, 0), m1 = len_mask(klen, 1), m2 = len_mask(klen, 2),
                                   m3 = len_mask(klen, 3);
                    k0 &= m0; k1 &= m1; k2 &= m2; k3 &= m3;
                    const uint32_t lowb = low_bytes(k0, m0 & 0x80808080u) | low_bytes(k1, m1 & 0x80808080u) |
                                          low_bytes(k2, m2 & 0x80808080u) | low_bytes(k3, m3 & 0x80808080u);
                    fail |= (lowb != 0) | (klen > 16);
                    h = key_hash(klen, k0, k1, k2, k3);
                }
            }

            LCLK(3);
            // ---- declined records go whole to slow_kernel
            const uint64_t rec = ws - HEAD + p;
            const bool slow = valid && fail;
            const uint64_t sb = __ballot(slow);
            if (sb) {
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(&stats->slow_records, (unsigned long long)__popcll(sb));
                base = __shfl(base, 0, 64);
                if (slow) {
                    const unsigned long long i = base + __popcll(sb & ((1ULL << lane) - 1));
                    if (i < slow_cap) slow_list[i] = rec;
                }
            }
            const bool ok = valid & !fail;
            pass_ = pass_ & ok;
            n_rec += (unsigned long long)__popcll(__ballot(ok));
            n_pass += (unsigned long long)__popcll(__ballot(pass_));
            if (row_out) {
                const unsigned long long slot = wave_slot(pass_, &stats->rows_emitted);
                if (pass_ && slot < row_cap) row_out[slot] = rec;
            }
#if defined(LEAN_PROF) && LEAN_PROF == 3   // profiling build: + values, filter, keys
            n_rec += __popcll(__ballot((h ^ (uint32_t)sval[0]) & 1));
            wave_order();
            continue;
#endif

            LCLK(4);
            // ---- aggregate
            if (!GROUPED) {
                my_cnt += pass_ ? 1u : 0u;
                my_first = pass_ && rec < my_first ? rec : my_first;
#pragma unroll
                for (int j = 0; j < NS; j++) {
                    my_sum[j] += pass_ && snum[j] ? sval[j] : 0.0;
                    my_num[j] += pass_ && snum[j] ? 1u : 0u;
                }
            } else {
                // home bucket for every lane: fingerprints, then the matching slot's key
                const uint32_t bk = bucket_of(h, lt.NB);
                const v4u q0 = lt.F[2 * bk], q1 = lt.F[2 * bk + 1];
                const uint32_t j = fp_first(q0, q1, fp_of(h));
                const uint32_t s0 = bk * BS + (j < BS ? j : BS - 1);
                const v4u a = lt.A[s0];
                bool hit = (j < BS) & (a.x == (0x80000000u | klen)) & (a.z == k0) & (a.w == k1);
                if (!g8) {           // a stored key of the same length <= 8 has zero words 2-3
                    const uint2 b = lt.B[s0];
                    hit = hit & (b.x == k2) & (b.y == k3);
                }
                int slot = hit ? (int)s0 : -1;
                uint32_t first = a.y;
                const bool miss = pass_ & !hit;
                if (__any(miss)) {                         // new keys (rare after the first windows)
                    if (miss) slot = lt_slow(lt, klen, k0, k1, k2, k3, h, first);
                }
                const bool add = pass_ & (slot >= 0);
                if (add) {
                    const uint32_t fc = (round << 15) | ((uint32_t)wv << 11) | p;
                    atomicAdd(&lt.cnt[slot], 1u);
                    if (fc < first) atomicMin((uint32_t*)(lt.A + slot) + 1, fc);
#pragma unroll
                    for (int j = 0; j < NS; j++) atomicAdd(&lt.sum[j][slot], snum[j] ? sval[j] : 0.0);
                }
#pragma unroll
                for (int j = 0; j < NS; j++) {
                    const bool nn = add & !snum[j];
                    if (__any(nn)) {
                        if (nn) atomicAdd(&lt.miss[j][slot], 1u);
                    }
                }
                const bool spill = pass_ && slot < 0;
                if (__any(spill)) {                        // LDS table full: straight to the HBM raw table
                    n_spill += (unsigned long long)__popcll(__ballot(spill));
                    if (spill) {
                        const GroupTable& rt = tabs[TAB_RT];
                        const GKey kk = raw_key(klen, (uint64_t)k0 | ((uint64_t)k1 << 32), (uint64_t)k2 | ((uint64_t)k3 << 32));
                        const int gi = g_insert(rt, kk, gk_hash(kk), stats);
                        if (gi >= 0) {
                            atomicAdd(&rt.cnt[gi], 1ULL);
                            atomicMin(&rt.first[gi], (unsigned long long)rec);
                            for (int a = 0; a < LP.nacc; a++) {
                                const int j = LP.acc_sidx[a];
                                const bool nm = j == 0 ? snum[0] : snum[MAXS - 1];
                                const double v = j == 0 ? sval[0] : sval[MAXS - 1];
                                if (nm) {
                                    atomicAdd(&rt.sum[a][gi], v);
                                    atomicAdd(&rt.num[a][gi], 1ULL);
                                }
                            }
                        }
                    }
                }
            }
            wave_order();                                  // W.rs is rewritten by the next pass
            LCLK(5);
        }
        LCLK(6);
    }
#ifdef LEAN_CLK
    if (lane == 0)
        for (int i = 0; i < 8; i++) atomicAdd(&stats->clk[i], (unsigned long long)clk_[i]);
#endif

    // ---- statistics
    if (lane == 0) {
        if (n_rec) atomicAdd(&stats->records, n_rec);
        if (n_pass) atomicAdd(&stats->passed, n_pass);
        if (n_spill) atomicAdd(&stats->lds_spills, n_spill);
    }

    if (!GROUPED) {
        unsigned long long c = my_cnt, f = my_first;
        double sm[MAXS];
        unsigned long long nm[MAXS];
#pragma unroll
        for (int j = 0; j < MAXS; j++) { sm[j] = my_sum[j]; nm[j] = my_num[j]; }
        for (int o = 32; o > 0; o >>= 1) {
            c += __shfl_down(c, o, 64);
            const unsigned long long ff = __shfl_down(f, o, 64);
            f = ff < f ? ff : f;
#pragma unroll
            for (int j = 0; j < MAXS; j++) {
                sm[j] += __shfl_down(sm[j], o, 64);
                nm[j] += __shfl_down(nm[j], o, 64);
            }
        }
        if (lane == 0) {
            const GroupTable& gt = tabs[TAB_GT];
            GKey k;
            k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
            const int gi = g_insert(gt, k, 0x12345678ULL, stats);
            if (gi >= 0) {
                if (c) atomicAdd(&gt.cnt[gi], c);
                if (f != ~0ULL) atomicMin(&gt.first[gi], f);
                for (int a = 0; a < LP.nacc; a++) {
                    const int j = LP.acc_sidx[a];
                    const double sa = j == 0 ? sm[0] : sm[MAXS - 1];
                    const unsigned long long na = j == 0 ? nm[0] : nm[MAXS - 1];
                    if (na) {
                        atomicAdd(&gt.sum[a][gi], sa);
                        atomicAdd(&gt.num[a][gi], na);
                    }
                }
            }
        }
        return;
    }

    // ---- flush the block's raw keys into the HBM raw table (raw_merge_kernel
    //      types each distinct raw key once and merges it into the canonical table)
    __syncthreads();
    const GroupTable& rt = tabs[TAB_RT];
    for (uint32_t i = tid; i < lds_h; i += LT) {
        const v4u a = lt.A[i];
        if (a.x < 2) continue;
        const uint2 b = lt.B[i];
        const GKey k = raw_key(a.x & 0x1F, (uint64_t)a.z | ((uint64_t)a.w << 32), (uint64_t)b.x | ((uint64_t)b.y << 32));
        const int gi = g_insert(rt, k, gk_hash(k), stats);
        if (gi < 0) continue;
        const uint32_t n = lt.cnt[i];
        if (n) atomicAdd(&rt.cnt[gi], (unsigned long long)n);
        if (a.y != NOFIRST) {
            const uint64_t fw = LP.first_win + ((uint64_t)(a.y >> 15) * gridDim.x + blockIdx.x) * NWV + ((a.y >> 11) & 15);
            atomicMin(&rt.first[gi], (unsigned long long)(fw * LP.ws - HEAD + (a.y & 2047)));
        }
        for (int acc = 0; acc < LP.nacc; acc++) {
            const int j = LP.acc_sidx[acc];
            const double sa = j == 0 ? lt.sum[0][i] : lt.sum[MAXS - 1][i];
            const uint32_t ms = j == 0 ? lt.miss[0][i] : lt.miss[MAXS - 1][i];
            const uint32_t num = n - ms;
            if (num) {
                atomicAdd(&rt.sum[acc][gi], sa);
                atomicAdd(&rt.num[acc][gi], (unsigned long long)num);
            }
        }
    }
}

// Raw keys -> canonical keys: every distinct raw GROUP BY field is typed once by
// the general parser (infer_type + parse_value, then create_groups' key text,
// evaluator_aggregates.c:122-141) and its partial state merged into c_gt.
__global__ __launch_bounds__(256) void raw_merge_kernel(ScanStats* __restrict__ stats, const GroupTable gt,
                                                        const GroupTable rt, int nacc) {
    __shared__ __align__(16) uint8_t buf[256 * 32];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= rt.cap || rt.tag[i] < 2) return;
    const GKey k = canonical_key(buf + threadIdx.x * 32, rt.clslen[i] & 0xFFFF, rt.w0[i], rt.w1[i]);
    const int gi = g_insert(gt, k, gk_hash(k), stats);
    if (gi < 0) return;
    atomicAdd(&gt.cnt[gi], rt.cnt[i]);
    atomicMin(&gt.first[gi], rt.first[i]);
    for (int a = 0; a < nacc; a++) {
        const unsigned long long n = rt.num[a][i];
        if (n) {
            atomicAdd(&gt.sum[a][gi], rt.sum[a][i]);
            atomicAdd(&gt.num[a][gi], n);
        }
    }
}

}  // namespace lean
}  // namespace cq

// ------------------------------------------------------------------ host side
namespace {

using namespace cq;
using lean::LeanPlan;

bool hcmp_result(uint32_t op, int c) {
    switch (op) {
        case CMP_EQ: return c == 0;
        case CMP_NE: return c != 0;
        case CMP_LT: return c < 0;
        case CMP_GT: return c > 0;
        case CMP_LE: return c <= 0;
        default: return c >= 0;
    }
}

// numeric literal thresholds for INTEGER fields M in [0, 10^7]: M < L <=> M < ceil(L),
// M > L <=> M > floor(L) (L finite; clamped to int32)
void int_thresholds(double L, int32_t* lo, int32_t* hi) {
    const double c = std::ceil(L), f = std::floor(L);
    *lo = c >= 2147483647.0 ? 2147483647 : (c <= -2147483648.0 ? (-2147483647 - 1) : (int32_t)c);
    *hi = f >= 2147483647.0 ? 2147483647 : (f <= -2147483648.0 ? (-2147483647 - 1) : (int32_t)f);
}

bool lean_shape(const ScanPlan* P, LeanPlan* lp, int* wm) {
    if (P->nneed > lean::KN || P->nacc > MAX_ACC) return false;
    // numeral parses (strtod / strtoll) must stop at the delimiter
    const uint32_t d = P->delim;
    if ((d - '0') < 10u || d == '.' || ((d | 32) >= 'a' && (d | 32) <= 'z') || d == '+' || d == '-') return false;
    if (d == '\n' || d == '\r' || d <= ' ') return false;
    *lp = LeanPlan{};
    lp->delim = P->delim;
    lp->quote = P->quote;
    if (P->group_slot >= 0) lp->gcol = (uint32_t)P->need_col[P->group_slot];
    lp->nacc = P->nacc;
    for (int a = 0; a < P->nacc; a++) {
        if (P->acc[a].kind != ACC_SUM) return false;
        const int slot = P->acc[a].slot;
        int j = 0;
        while (j < lp->ns && lp->sum_slot[j] != slot) j++;
        if (j == lp->ns) {
            if (lp->ns == lean::MAXS) return false;
            lp->scol[lp->ns] = (uint32_t)P->need_col[slot];
            lp->sum_slot[lp->ns++] = slot;
        }
        lp->acc_sidx[a] = j;
    }
    if (P->nprog == 0) {
        *wm = lean::LW_NONE;
    } else if (P->nprog == 3 && P->prog[0].op == OP_COL && P->prog[1].op == OP_CONST && P->prog[2].op == OP_CMP) {
        lp->wcol = (uint32_t)P->need_col[P->prog[0].a];
        lp->wop = P->prog[2].a;
        lp->wtt = (hcmp_result(lp->wop, -1) ? 1u : 0u) | (hcmp_result(lp->wop, 0) ? 2u : 0u) | (hcmp_result(lp->wop, 1) ? 4u : 0u);
        const Cell& L = P->consts[P->prog[1].b];
        lp->wconst = L;
        lp->pass_null = hcmp_result(lp->wop, L.kind == K_NULL ? 0 : -1) ? 1u : 0u;   // NULL < any non-NULL
        if (L.kind == K_INT || L.kind == K_DBL) {
            *wm = lean::LW_NUM;
            if (L.kind == K_INT) lp->wl = (double)(int64_t)L.bits;
            else memcpy(&lp->wl, &L.bits, 8);
            int_thresholds(lp->wl, &lp->wlo, &lp->whi);
        } else if (L.kind == K_STR && L.len <= 8) {
            *wm = lean::LW_STR;                    // the bytes are filled in by the caller (device address)
        } else {
            *wm = lean::LW_GEN;
        }
    } else {
        return false;
    }
    return true;
}

int ns_of(const LeanPlan& lp) { return lp.ns; }
size_t lean_slot_bytes(int ns) { return lean::slot_bytes(ns); }
size_t lean_fixed_bytes() { return lean::fixed_bytes(); }

uint32_t lean_slots(int ns, int grouped) { return lean::slots_for(ns, grouped != 0); }
size_t lean_lds(int ns, int grouped) {
    return lean_fixed_bytes() + (size_t)lean_slots(ns, grouped) * lean_slot_bytes(ns) + 512;
}

typedef void (*lean_fn_t)(const uint8_t*, ScanStats*, unsigned long long*, unsigned long long, uint32_t,
                          unsigned long long*, unsigned long long, const lean::LeanArgs, const GroupTable*);

template <bool G, int WM>
lean_fn_t pick_ns(int ns) {
    if (ns == 0) return lean::lean_kernel<G, WM, 0>;
    return ns == 1 ? lean::lean_kernel<G, WM, 1> : lean::lean_kernel<G, WM, 2>;
}
template <bool G>
lean_fn_t pick_fn(int wm, int ns) {
    switch (wm) {
        case lean::LW_NONE: return pick_ns<G, lean::LW_NONE>(ns);
        case lean::LW_NUM: return pick_ns<G, lean::LW_NUM>(ns);
        case lean::LW_STR: return pick_ns<G, lean::LW_STR>(ns);
        default: return pick_ns<G, lean::LW_GEN>(ns);
    }
}

}  // namespace

extern "C" {

// 1 when the lean kernel handles this plan
int cq_lean_eligible(const cq::ScanPlan* P) {
    LeanPlan lp;
    int wm = 0;
    return lean_shape(P, &lp, &wm) ? 1 : 0;
}

// windows covering the records that start in [begin, end)
uint64_t cq_lean_windows(uint64_t begin, uint64_t end, uint32_t ws) {
    if (!ws) ws = lean::WS;
    return (end + ws - 1) / ws - begin / ws;
}

// The window stride for a file: a window's records are handled one per lane, so
// a stride holding ~58 records of the file's average length fills a wave in one
// pass instead of spilling a few records into a second, nearly empty pass (and
// never more than the staged bytes allow).  The average comes from up to 256 KiB
// of the data bytes (records split on '\n' / '\r' runs, as csv_load does).
uint32_t cq_lean_pick_ws(const uint8_t* data, uint64_t n) {
    const uint64_t m = n < (256u << 10) ? n : (256u << 10);
    uint64_t recs = 0;
    bool in_rec = false;
    for (uint64_t i = 0; i < m; i++) {
        const bool term = data[i] == '\n' || data[i] == '\r';
        if (!term && !in_rec) recs++;
        in_rec = !term;
    }
    if (recs < 16) return lean::WS;
    const double avg = (double)m / (double)recs;
    uint64_t ws = (uint64_t)(58.0 * avg) & ~(uint64_t)15;
    if (ws > (uint64_t)lean::WS) ws = lean::WS;
    if (ws < 256) ws = 256;
    return (uint32_t)ws;
}
int cq_lean_waves_per_block() { return lean::NWV; }

size_t cq_lean_lds_bytes(const cq::ScanPlan* P, int grouped) {
    LeanPlan lp;
    int wm = 0;
    if (!lean_shape(P, &lp, &wm)) return 0;
    return lean_lds(ns_of(lp), grouped);
}

// the lean scan (the caller runs slow_kernel over slow_list afterwards)
hipError_t cq_launch_lean(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          const cq::GroupTable* rt, cq::ScanStats* stats, unsigned long long* row_out,
                          unsigned long long row_cap, int grouped, int grid, hipStream_t s,
                          unsigned long long* slow_list, unsigned long long slow_cap) {
    LeanPlan lp;
    int wm = 0;
    if (!lean_shape(P, &lp, &wm)) return hipErrorInvalidValue;
    if (wm == lean::LW_STR) {   // the literal's bytes (a STRING cell points at device memory)
        const Cell& L = P->consts[P->prog[1].b];
        uint8_t b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (L.len) {
            hipError_t e = hipMemcpyAsync(b, (const void*)(uintptr_t)L.bits, L.len, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
        }
        uint64_t x = 0;
        for (int i = 0; i < 8; i++) x = (x << 8) | b[i];
        lp.wstr = x;
        bool nul = false;
        for (uint32_t i = 0; i < L.len; i++) nul = nul || b[i] == 0;
        if (nul) wm = lean::LW_GEN;          // strcmp stops at a NUL: the general compare decides
    }
    const uint64_t hi = P->range_end < P->n ? P->range_end : P->n;
    lp.lo_ok = P->data_begin > P->range_begin ? P->data_begin : P->range_begin;
    lp.hi_ok = hi;
    lp.ws = P->lean_ws ? P->lean_ws : (uint32_t)lean::WS;
    if (lp.ws > (uint32_t)lean::WS || lp.ws % 16) return hipErrorInvalidValue;
    lp.first_win = P->range_begin / lp.ws;
    lp.last_win = (hi + lp.ws - 1) / lp.ws;
    const int ns = ns_of(lp);
    {   // the roles in ascending column order (lean_kernel's field walk)
        uint32_t nr = 0;
        auto add = [&](uint32_t col, uint32_t role) {
            uint32_t i = nr++;
            while (i > 0 && lp.rcol[i - 1] > col) {
                lp.rcol[i] = lp.rcol[i - 1];
                lp.rrole[i] = lp.rrole[i - 1];
                i--;
            }
            lp.rcol[i] = col;
            lp.rrole[i] = role;
        };
        if (wm != lean::LW_NONE) add(lp.wcol, lean::R_WHERE);
        for (int j = 0; j < ns; j++) add(lp.scol[j], j == 0 ? lean::R_SUM0 : lean::R_SUM1);
        if (grouped) add(lp.gcol, lean::R_GROUP);
    }
    const uint32_t h = lean_slots(ns, grouped);
    const size_t lds = lean_lds(ns, grouped);
    lean::LeanArgs args;
    memset(&args, 0, sizeof args);
    args.lp = lp;
    static GroupTable* tabs_dev = nullptr;
    if (!tabs_dev) {
        hipError_t e = hipGetSymbolAddress((void**)&tabs_dev, HIP_SYMBOL(lean::g_lean_tabs));
        if (e != hipSuccess) return e;
    }
    static GroupTable tabs[2];
    tabs[0] = *gt;
    if (rt) tabs[1] = *rt;
    else memset(&tabs[1], 0, sizeof tabs[1]);
    {
        hipError_t e = hipMemcpyAsync(tabs_dev, tabs, sizeof tabs, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
    }
    const lean_fn_t fn = grouped ? pick_fn<true>(wm, ns) : pick_fn<false>(wm, ns);
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(lean::LT), lds, s, g, stats, row_out, row_cap, h, slow_list, slow_cap,
                       args, (const GroupTable*)tabs_dev);
    return hipGetLastError();
}

// raw-key table -> canonical table (after cq_launch_lean of a grouped plan)
hipError_t cq_launch_raw_merge(const cq::GroupTable* gt, const cq::GroupTable* rt, int nacc, cq::ScanStats* stats,
                               hipStream_t s) {
    hipLaunchKernelGGL(lean::raw_merge_kernel, dim3((rt->cap + 255) / 256), dim3(256), 0, s, stats, *gt, *rt, nacc);
    return hipGetLastError();
}

}  // extern "C"
