// lean.hip -- the wave-autonomous CSV scan for the common SELECT plan shapes.
//
// Same job as scan_kernel (scan.hip) -- csv_load + filter_rows + create_groups +
// evaluate_aggregate in one pass over the HBM-resident bytes (reference
// csv_reader.c:375-465, evaluator_utils.c:986, evaluator_aggregates.c:108-414) --
// for plans whose WHERE is absent or `column op literal` and whose aggregates are
// COUNT / SUM / AVG (at most 4 parsed columns, 2 distinct SUM arguments).
//
// Every wave works on its own 4 KiB windows with no block barrier in the loop, so
// one wave's byte classification overlaps another's record work on the same SIMD,
// and every lane carries TWO records through the record pass: two independent
// dependency chains per lane for the LDS round trips to overlap, and one set of
// wave-uniform tests, ballots and loop control per two records.
//
//   load      a window is 4 KiB of the file starting at a multiple of its stride
//             (128-byte aligned) by four coalesced 16-byte non-temporal loads per
//             lane (load i: bytes [1024i, 1024i + 1024)) issued one window ahead,
//             plus the dword before the window (record-start context).  The window
//             owns the records that start in its first `ws` bytes (ws <= WS =
//             3968); the last 128 bytes are the record views' tail and are re-read
//             by the next window
//   classify  the window goes to LDS as loaded and comes back lane-contiguous
//             (lane l: bytes [64l, 64l + 64)); per lane two 64-bit masks --
//             separators (delimiter and record terminators '\n' '\r') and
//             terminators -- plus quote presence (quote bitmap in LDS only when the
//             window holds a quote)
//   starts    record starts (previous byte a terminator) owned by the window; each
//             lane takes the records starting in its own 64 bytes, two per pass
//   fields    per record: 64 separator and terminator bits from the record start,
//             funnel-shifted out of the lane's own and the next lane's masks (one
//             DPP wave shift each, no LDS); field c ends at the c-th set separator
//             bit.  A record whose needed fields are not all inside those 64 bytes,
//             or that has a quote in front of its last needed field, goes whole to
//             the slow list and slow_kernel (scan.hip)
//   values    WHERE / SUM fields of 1-4 bytes shaped `digits[.digits]` are typed
//             in registers (right-aligned digit bytes, the dot squeezed out by one
//             v_perm_b32, a v_dot4 for the value): M and k = digits after the dot,
//             exactly parse_value's INTEGER M or DOUBLE strtod = RN(M / 10^k); 5-7
//             byte numerals by an 8-byte variant, anything else by the exact field
//             typers (scanlib.h) or the slow path.  A WHERE against a numeric
//             literal L compares INTEGER fields with the integer thresholds
//             ceil(L) / floor(L) and DOUBLE fields as RN(M / 10^k) against L
//             (value_compare, csv_reader.c:98-130); a short STRING literal
//             compares big-endian byte words (strcmp)
//   group     the block's LDS table is keyed by the RAW bytes of the GROUP BY
//             field (a raw key partitions rows at least as finely as the
//             reference's printf-canonical key): buckets of 4 slots, every key
//             has two candidate buckets (two-choice hashing keeps the fullest
//             bucket near the mean), and a slot's tag IS the zero-padded key, so
//             one round trip of four 16-byte LDS reads finds the key with no
//             fingerprint or second key read.  New keys are claimed by a 64-bit
//             LDS compare-and-swap of the tag.  COUNT / SUM / first-row are
//             fire-and-forget LDS atomics.  Blocks flush (and keys that find no
//             room spill) into an HBM table of raw keys; raw_merge_kernel types
//             every distinct raw key once with the general parser and merges it
//             into the canonical table -- so "1.5" and "1.50" still meet there
//
// SUM addends of DOUBLE fields are M * RN(10^-k) (within 2 ulp of the reference's
// RN(M / 10^k); SUM / AVG parity is 1e-6 relative, north_star), INTEGER addends
// are exact.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstring>
#include "plan.h"
#include "scanlib.h"
#include "upload.h"

namespace cq {
namespace lean {

#ifndef LEAN_REGPF
#define LEAN_DMA 1      // the next window arrives in LDS by LDS-DMA (no registers held for it)
#endif
#ifndef LEAN_WAVES
#ifdef LEAN_DMA
#define LEAN_WAVES 16   // 4 waves per SIMD at 128 VGPRs: no register prefetch to spill
#else
#define LEAN_WAVES 12   // 3 waves per SIMD: 168 VGPRs, so the prefetched window never spills
#endif
#endif
constexpr int LT = 64 * LEAN_WAVES;       // threads per block
constexpr int NWV = LT / 64;              // waves per block
constexpr int LB = 64;                    // staged bytes per lane
constexpr int WB = 64 * LB;               // staged window bytes (4 KiB)
constexpr int WS = 3968;                  // largest window stride = owned bytes (LeanPlan.ws: the file's)
constexpr int NMW = WB / 32;              // 32-bit quote-bitmap words per window
constexpr int WBYTES = WB + 32;           // staged bytes + slack for 16-byte field loads
constexpr int MAXS = 2;                   // distinct SUM arguments
constexpr int KN = 4;                     // need slots
constexpr uint32_t NOFIRST = 0xFFFFFFFFu;
static_assert(WS + 64 + 16 <= WB, "a record view (64 bytes) plus a field load stays in the window");
static_assert(WS % 128 == 0, "128-byte aligned windows");

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
    uint32_t qt[NMW + 4];       // quote bits (written only when the window holds a quote)
};
static_assert(sizeof(WaveLds) % 16 == 0, "16-byte aligned wave areas");

// everything the kernel reads from its arguments
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
    uint32_t ws;                 // window stride: multiple of 128, <= WS
    uint32_t rcol[KN];           // the roles' CSV columns, ascending
    uint32_t rrole[KN];          // their roles: R_WHERE, R_SUM0, R_SUM1, R_GROUP
};
enum : uint32_t { R_WHERE = 0, R_SUM0 = 1, R_SUM1 = 2, R_GROUP = 3 };

// kernel arguments (kernarg segment).  The two HBM group tables (canonical keys,
// shared with slow_kernel, and raw-byte keys for block flushes and LDS spills) are
// read through a pointer to a device copy instead: only the rare spill path and
// the final flush touch them.
struct LeanArgs {
    LeanPlan lp;
};
enum : int { TAB_GT = 0, TAB_RT = 1 };
// (the pair itself: a per-thread device buffer, cq_launch_lean)

constexpr uint32_t GK_RAW = 6;       // raw field bytes as key (cell.h GK_* never produce 6)
__device__ __forceinline__ GKey raw_key(uint32_t len, uint64_t w0, uint64_t w1) {
    GKey k;
    k.cls = GK_RAW; k.len = len; k.w0 = w0; k.w1 = w1;
    return k;
}

struct Win {            // one window in flight
#ifndef LEAN_DMA
    v4u a[4];           // staged bytes [64l, 64l + 64)
#endif
    uint32_t prev;      // the dword before the window
};

// the dword before the window (g has 256 bytes of '\n' before byte 0) by a buffer load: a
// uniform address would otherwise become a scalar load, whose lgkmcnt the LDS waits of the
// whole window would have to drain
__device__ __forceinline__ uint32_t load_prev(const uint8_t* base) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(base - 4), 0, 4, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0);
}

#ifdef LEAN_DMA
#if defined(LEAN_DMA_NT) && LEAN_DMA_NT   // cache policy bits of the window loads
#define LEAN_DMA_CPOL " nt"
#else
#define LEAN_DMA_CPOL ""
#endif
// the window's 4 KiB straight into the wave's LDS bytes (lds: their wave-uniform LDS
// address) by four LDS-DMA loads, 1 KiB each, lane l's 16 bytes at 16l.  The caller waits
// for them with vmcnt(0) before reading the bytes; the lgkmcnt(0) first retires this
// wave's LDS reads of the window the loads overwrite.  M0 (the LDS base of an LDS-DMA
// load) is set and restored inside the one statement (the compiler owns M0).
__device__ __forceinline__ void load_win(const uint8_t* g, uint64_t w, uint32_t ws, uint32_t lds, Win& x) {
    const uint8_t* base = g + w * ws;                    // 128-byte aligned (g is 256-aligned, ws % 128 == 0)
    const int lane = threadIdx.x & 63;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" LEAN_DMA_CPOL
                     "\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(base + 1024 * i + 16 * lane), "s"(lds + 1024u * i)
                     : "memory");
    }
    x.prev = load_prev(base);
}
#else
__device__ __forceinline__ void load_win(const uint8_t* g, uint64_t w, uint32_t ws, uint32_t, Win& x) {
    const uint8_t* base = g + w * ws;                    // 128-byte aligned (g is 256-aligned, ws % 128 == 0)
    const v4u* src = (const v4u*)base;
    const int lane = threadIdx.x & 63;
#ifdef LEAN_TEMPORAL
#define LEAN_LD(p) (*(p))
#else
#define LEAN_LD(p) __builtin_nontemporal_load(p)
#endif
    // coalesced: load i is bytes [1024i, 1024i + 1024), lane l its 16 bytes at 16l (one load
    // per lane of 64 contiguous bytes was 1.5x slower to stream: 64-byte lane strides)
#pragma unroll
    for (int i = 0; i < 4; i++) x.a[i] = LEAN_LD(src + 64 * i + lane);
#undef LEAN_LD
    x.prev = load_prev(base);
}
#endif

// separator / terminator bits of 32 bytes (bit i = byte i) and quote flags.
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
// r & ~(r >> 1) & 0x40404040 as one v_bitop3_b32 (truth table 0x20: a & ~b & c) after
// the shift; the compiler's own form takes a v_not more
__device__ __forceinline__ uint32_t flags40(uint32_t r) {
    return __builtin_amdgcn_bitop3_b32(r, r >> 1, 0x40404040u, 0x20);
}
// The delimiter and terminator flags are packed separately and the separator mask
// is their OR per 32 bytes (one op there instead of an AND per dword).
__device__ __forceinline__ void classify32(const v4u a, const v4u b, uint32_t rep_d, uint32_t rep_q, uint32_t& sep,
                                           uint32_t& nl, uint32_t& q) {
    uint32_t ud[4], un[4];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t x = j < 4 ? a[j & 3] : b[j & 3];
        const uint32_t rn = __builtin_amdgcn_perm(0x00004000u, 0x00400000u, x ^ 0x08080808u);
        const uint32_t rd = __builtin_amdgcn_perm(0u, 0x00000040u, x ^ rep_d);
        const uint32_t fd = flags40(rd), fn = flags40(rn);
        const uint32_t w = (j & 1) ? 0x80402010u : 0x08040201u;
        if (j & 1) {
            ud[j >> 1] = __builtin_amdgcn_udot4(fd, w, ud[j >> 1], false);
            un[j >> 1] = __builtin_amdgcn_udot4(fn, w, un[j >> 1], false);
        } else {
            ud[j >> 1] = __builtin_amdgcn_udot4(fd, w, 0u, false);
            un[j >> 1] = __builtin_amdgcn_udot4(fn, w, 0u, false);
        }
        const uint32_t t = x ^ rep_q;
        q |= (t - 0x01010101u) & ~t;
    }
    // ud[p] = 0x40 * (bits of bytes 8p .. 8p + 7)
    nl = (un[0] >> 6) | (un[1] << 2) | (un[2] << 10) | (un[3] << 18);
    sep = nl | (ud[0] >> 6) | (ud[1] << 2) | (ud[2] << 10) | (ud[3] << 18);
}
// 0x80 flags -> a nibble (bit i = byte i)
__device__ __forceinline__ uint32_t nib(uint32_t f) {
    uint32_t t = f >> 7;
    t |= t >> 7;
    t |= t >> 14;
    return t & 0xFu;
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
// 64 bits from bit b (< 64) of the 128 bits w0 | w1 << 32 | w2 << 64 | w3 << 96
__device__ __forceinline__ uint64_t view128(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t b) {
    const bool hi = b >= 32;
    const uint32_t sh = b & 31, a = hi ? w1 : w0, c = hi ? w2 : w1, d = hi ? w3 : w2;
    return (uint64_t)__builtin_amdgcn_alignbit(c, a, sh) | ((uint64_t)__builtin_amdgcn_alignbit(d, c, sh) << 32);
}
__device__ __forceinline__ uint64_t qview(const WaveLds& W, uint32_t p) {
    const uint32_t wi = p >> 5, sh = p & 31;
    const uint32_t q0 = W.qt[wi], q1 = W.qt[wi + 1], q2 = W.qt[wi + 2];
    return (uint64_t)__builtin_amdgcn_alignbit(q1, q0, sh) | ((uint64_t)__builtin_amdgcn_alignbit(q2, q1, sh) << 32);
}

// 4 bytes of the tile at byte offset o (any alignment)
__device__ __forceinline__ uint32_t load4(const uint8_t* tile, uint32_t o) {
    const uint32_t* t32 = (const uint32_t*)tile;
    const uint32_t a = o >> 2, sh = o & 3;
    return __builtin_amdgcn_alignbyte(t32[a + 1], t32[a], sh);
}

// bytes [0, len) of two dwords (len <= 8)
__device__ __forceinline__ void mask8(uint32_t len, uint32_t& d0, uint32_t& d1) {
    const uint32_t n1 = len > 4 ? len - 4 : 0;
    d0 &= len >= 4 ? 0xFFFFFFFFu : ((1u << (8 * len)) - 1);
    d1 &= n1 >= 4 ? 0xFFFFFFFFu : ((1u << (8 * n1)) - 1);
}

// 0x80 in every byte < 0x21 (blank, control, NUL) among the bytes of f-flags
__device__ __forceinline__ uint32_t low_bytes(uint32_t d, uint32_t f) { return lt_bytes(d, 0x21212121u) & f; }

// A numeral field shaped [digits][.][digits] with at least one digit (no sign, at
// most 7 bytes, so never date-shaped: parse_date needs 8-10 bytes): infer_type
// gives INTEGER (no dot) or DOUBLE, parse_value M or strtod = RN(M / 10^k).
// M, k and dot are meaningful when ok.
struct Num {
    uint32_t M, k;
    bool ok, dot;
};

// Fields of 1..4 bytes, d = the field's first 4 bytes (unmasked).  The field is
// right-aligned in the dword with its digits as byte values (bytes before it 0,
// i.e. leading zeros); with DOT a '.' is squeezed out by one v_perm_b32 whose
// selector keeps the bytes behind the dot and moves the ones before it up a byte.
// Then every byte must be a digit value, and M is one v_dot4 (weights 100/10/1)
// plus the top byte * 1000.  Without DOT a field holding a '.' is simply not ok.
template <bool DOT>
__device__ __forceinline__ Num num4(uint32_t d, uint32_t len) {
    Num r;
    const uint32_t sh = 32u - 8u * len;                                 // len 1..4 (others: ok false)
    uint32_t v = (d ^ 0x30303030u) << (sh & 31);
    r.dot = false;
    r.k = 0;
    if (DOT) {
        const uint32_t fd = ~nonzero_bytes(v ^ 0x1E1E1E1Eu) & 0x80808080u & (0xFFFFFFFFu << (sh & 31));   // '.' ^ '0'
        const uint32_t low = fd & (0u - fd);                            // the first dot, byte index pd
        const uint32_t below = ((low << 1) - (low != 0 ? 1u : 0u)) & 0x01010100u;   // bytes 1..pd (none: 0)
        v = __builtin_amdgcn_perm(0u, v, (low ? 0x0302010Cu : 0x03020100u) - below);   // bytes <= pd up one, byte 0 := 0
        r.dot = low != 0;
        r.k = r.dot ? (uint32_t)__builtin_clz(low) >> 3 : 0u;           // 3 - pd = digits after the dot
    }
    const bool digits = lt_bytes(v, 0x0A0A0A0Au) == 0x80808080u;
    r.ok = (len - 1u <= 3u) & digits & (!DOT | (len > 1u) | !r.dot);
    r.M = __builtin_amdgcn_udot4(v, 0x010A6400u, __umul24(v & 0xFFu, 1000u), false);
    return r;
}

// Fields of 1..7 bytes (d0/d1: the field's first 8 bytes, unmasked).
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
#ifdef LEAN_NOGEN
    return false;
#endif
    if (len == 0) { c = cell_null(); return true; }
    uint64_t kw;
    if (lean_field(bytes, o, len, true, c, kw)) return true;
    GKey unused;
    return fast_field(bytes, o, len, true, false, c, unused) == FF_OK;
}

__device__ __forceinline__ uint64_t bswap64(uint32_t d0, uint32_t d1) {
    return ((uint64_t)__builtin_bswap32(d0) << 32) | __builtin_bswap32(d1);
}

// ------------------------------------------------------------------ LDS group table
//
// Structure of arrays carved from dynamic LDS at compile-time offsets.  Slots come
// in buckets of BSLOTS = 4; a key may live in either of two buckets (hash bits
// [0, 16) and [16, 32)).  The tag of a slot is the key itself:
//   K8  (keys of <= 8 bytes): one u64, the zero-padded key bytes.  Key bytes are
//       > ' ' (keys with lower bytes take the slow path), so a key's first byte
//       is nonzero and the zero padding encodes its length; the empty key (NULL
//       field) is tag 1 << 32 and a free slot is tag 0.
//   K16 (keys of <= 16 bytes): four u32, words 0-1 as for K8, words 2-3 the key
//       bytes 8-15.  A free slot is claimed by a CAS of words 0-1 to CLAIM,
//       words 2-3 written, then words 0-1 published.
// A key is inserted into the first free slot of the less occupied bucket by CAS;
// two inserters of one key that race into different buckets leave a duplicate,
// which is harmless: lookups take either slot and the flush merges by key.
constexpr uint32_t BSLOTS = 4;
constexpr uint32_t CLAIM = 0xFFFFFFFFu;       // K16 tag word 1 of a slot being written

template <bool K16>
constexpr uint32_t slot_bytes(int ns) { return (K16 ? 16u : 8u) + 4u + 4u + (uint32_t)ns * 12u; }
constexpr uint32_t fixed_bytes() { return (uint32_t)(sizeof(WaveLds) * NWV); }
constexpr uint32_t LDS_MAX = 160u * 1024u - 256u;
template <bool K16>
constexpr uint32_t slots_for(int ns, bool grouped) {
    if (!grouped) return 0;
    uint32_t h = 4096;
    while (h > 64 && fixed_bytes() + h * slot_bytes<K16>(ns) > LDS_MAX) h >>= 1;
    return h;
}

struct LTab {
    uint8_t* T;           // tags: H * (8 | 16) bytes
    uint32_t* cnt;
    uint32_t* first;      // smallest first-row code of the slot's passing records
    double* sum[MAXS];
    uint32_t* miss[MAXS]; // SUM arguments that were not numeric
};

__device__ __forceinline__ uint32_t key_hash(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    uint32_t x = k0 ^ rotl(k1, 11) ^ rotl(k2, 19) ^ rotl(k3, 5);
    x ^= x >> 16;
    x = __umul24(x, 0x2F0B3Du) ^ (x >> 7);
    x ^= x >> 13;
    return __umul24(x, 0x3C6EF3u) ^ (x >> 11) ^ (x << 16);
}

// look the key up in its two buckets: the slot, or -1
template <bool K16>
__device__ __forceinline__ int lt_find(const LTab& t, uint32_t nb, uint32_t h, uint32_t k0, uint32_t k1, uint32_t k2,
                                       uint32_t k3) {
    const uint32_t b1 = h & (nb - 1), b2 = (h >> 16) & (nb - 1);
    int s = -1;
    if (!K16) {
        const v4u* T4 = (const v4u*)t.T;                 // two tags per v4u
        const v4u a0 = T4[2 * b1], a1 = T4[2 * b1 + 1], c0 = T4[2 * b2], c1 = T4[2 * b2 + 1];
        const uint64_t k = (uint64_t)k0 | ((uint64_t)k1 << 32);
#define LT_TRY8(V, HALF, SLOT) \
        s = (((uint64_t)(HALF ? V.z : V.x) | ((uint64_t)(HALF ? V.w : V.y) << 32)) == k) ? (int)(SLOT) : s;
        LT_TRY8(c1, 1, 4 * b2 + 3) LT_TRY8(c1, 0, 4 * b2 + 2) LT_TRY8(c0, 1, 4 * b2 + 1) LT_TRY8(c0, 0, 4 * b2)
        LT_TRY8(a1, 1, 4 * b1 + 3) LT_TRY8(a1, 0, 4 * b1 + 2) LT_TRY8(a0, 1, 4 * b1 + 1) LT_TRY8(a0, 0, 4 * b1)
#undef LT_TRY8
    } else {
        const v4u* T4 = (const v4u*)t.T;                 // one tag per v4u
        v4u x[8];
#pragma unroll
        for (int i = 0; i < 4; i++) { x[i] = T4[4 * b1 + i]; x[4 + i] = T4[4 * b2 + i]; }
#pragma unroll
        for (int i = 7; i >= 0; i--) {
            const bool m = (x[i].x == k0) & (x[i].y == k1) & (x[i].z == k2) & (x[i].w == k3);
            s = m ? (int)((i < 4 ? 4 * b1 : 4 * b2 - 4) + i) : s;
        }
    }
    return s;
}

// find or insert (lanes that missed in lt_find); -1: both buckets full (the
// record spills to the HBM raw table)
template <bool K16>
__device__ int lt_insert(const LTab& t, uint32_t nb, uint32_t h, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    const uint32_t b1 = h & (nb - 1), b2 = (h >> 16) & (nb - 1);
    for (int attempt = 0; attempt < 64; attempt++) {
        const int s = lt_find<K16>(t, nb, h, k0, k1, k2, k3);
        if (s >= 0) return s;
        // occupancy of the two buckets (slots fill in order)
        uint32_t n1 = 0, n2 = 0;
        const uint32_t stride = K16 ? 16u : 8u;
        for (uint32_t i = 0; i < BSLOTS; i++) {
            const uint32_t* a = (const uint32_t*)(t.T + (4 * b1 + i) * stride);
            const uint32_t* c = (const uint32_t*)(t.T + (4 * b2 + i) * stride);
            n1 += (__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) |
                   __hip_atomic_load(a + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
            n2 += (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) |
                   __hip_atomic_load(c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
        }
        if (n1 >= BSLOTS && n2 >= BSLOTS) return -1;
        const uint32_t slot = (n1 <= n2 || n2 >= BSLOTS) && n1 < BSLOTS ? 4 * b1 + n1 : 4 * b2 + n2;
        unsigned long long* w01 = (unsigned long long*)(t.T + slot * stride);
        const unsigned long long key01 = (unsigned long long)k0 | ((unsigned long long)k1 << 32);
        if (!K16) {
            if (atomicCAS(w01, 0ull, key01) == 0ull) return (int)slot;
        } else {
            if (atomicCAS(w01, 0ull, (unsigned long long)CLAIM << 32) == 0ull) {
                uint32_t* w = (uint32_t*)w01;
                w[2] = k2;
                w[3] = k3;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                atomicExch(w01, key01);
                return (int)slot;
            }
        }
        // lost the slot to another inserter: look again
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

// a raw key's length from its zero-padded words (key bytes are nonzero)
__device__ __forceinline__ uint32_t key_len(uint64_t w0, uint64_t w1) {
    if (w1) return 16u - ((uint32_t)__builtin_clzll(w1) >> 3);
    if (w0 == (1ull << 32)) return 0u;                  // the empty key's tag
    return w0 ? 8u - ((uint32_t)__builtin_clzll(w0) >> 3) : 0u;
}

// a record whose key found no LDS slot (a key longer than the tag, both buckets
// full): aggregated straight into the HBM raw table; keys over 16 bytes or with
// low bytes past byte 8 go to the slow list
__device__ __forceinline__ void spill_record(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t kl,
                                          uint64_t off, const GroupTable* tabs, ScanStats* stats,
                                          unsigned long long* slow_list, unsigned long long slow_cap, int nacc,
                                          const int32_t* acc_sidx, bool n0, double v0, bool n1, double v1) {
    const GroupTable& rt = tabs[TAB_RT];
    const uint32_t m0 = len_mask(kl, 0), m1 = len_mask(kl, 1), m2 = len_mask(kl, 2), m3 = len_mask(kl, 3);
    a0 &= m0; a1 &= m1; a2 &= m2; a3 &= m3;
    const bool fits = kl <= 16 && (low_bytes(a2, m2 & 0x80808080u) | low_bytes(a3, m3 & 0x80808080u)) == 0;
    if (!fits) {
        const unsigned long long i = atomicAdd(&stats->slow_records, 1ull);
        if (i < slow_cap) slow_list[i] = off;
        return;
    }
    const GKey kk = raw_key(kl, (uint64_t)a0 | ((uint64_t)a1 << 32), (uint64_t)a2 | ((uint64_t)a3 << 32));
    const int gi = g_insert(rt, kk, gk_hash(kk), stats);
    if (gi < 0) return;
    atomicAdd(&rt.cnt[gi], 1ULL);
    atomicMin(&rt.first[gi], (unsigned long long)off);
    for (int a = 0; a < nacc; a++) {
        const bool nm = acc_sidx[a] == 0 ? n0 : n1;
        if (nm) {
            atomicAdd(&rt.sum[a][gi], acc_sidx[a] == 0 ? v0 : v1);
            atomicAdd(&rt.num[a][gi], 1ULL);
        }
    }
}

// one record's role fields
struct Rec {
    uint32_t p;                 // window offset of the record start
    bool valid, fail;
    uint32_t wfp, wfl, gfp, klen, lastpos;
    uint32_t sfp[MAXS], sfl[MAXS];
};

// Field walk of a record from its 64-bit separator view sv and record end e (first
// terminator bit; 64: beyond the view): the roles' columns come in ascending
// order, and clearing separator bits one by one visits the field ends in order:
// before field c's end is cleared, the lowest remaining bit is that end, and the
// previous one (field c - 1's end) is its start - 1.  A column past the record's
// end is missing (length 0: NULL); a field the view cannot bound fails the fast
// path.
// The same walk for both records of a lane at once, with the roles addressed by
// their rank in column order: skip[k] = separators between role k - 1's field end
// and role k's field start (uniform), so both records' bit-clearing chains run in
// one scalar loop, and each field lands in its role's registers by selects on
// the uniform role ranks (kw: WHERE, ks: SUM 0/1, kg: GROUP BY) -- no branch
// depends on which role a column plays.
// DISTINCT (the roles' columns strictly ascending): skip[k] >= 1 for k >= 1, so the
// first bit role k clears is role k - 1's field end, already known -- a role in the
// column right after the previous one costs no bit search for its start.
template <int NR, int WM, int NS, bool GROUPED, bool DISTINCT>
__device__ __forceinline__ void walk2(Rec (&rec)[2], const uint64_t (&sv)[2], const uint64_t (&nv)[2],
                                      const uint32_t (&skip)[KN], uint32_t kw, const uint32_t (&ks)[MAXS],
                                      uint32_t kg) {
    uint64_t s0 = sv[0], s1 = sv[1];
    const uint32_t e0 = ctz64(nv[0]), e1 = ctz64(nv[1]);
    uint32_t pe0 = 0xFFFFFFFFu, pe1 = 0xFFFFFFFFu;      // start - 1 of the current field
    uint32_t en0 = 0, en1 = 0;                          // the previous role's field end
#pragma unroll
    for (int k = 0; k < NR; k++) {
        const uint32_t n = skip[k];
        if (DISTINCT && k > 0) {
            s0 &= s0 - 1;                               // role k - 1's end
            s1 &= s1 - 1;
            if (n == 1) {
                pe0 = en0;
                pe1 = en1;
            } else {
                for (uint32_t i = 2; i < n; i++) {
                    s0 &= s0 - 1;
                    s1 &= s1 - 1;
                }
                pe0 = ctz64(s0);
                pe1 = ctz64(s1);
                s0 &= s0 - 1;
                s1 &= s1 - 1;
            }
        } else if (n > 0) {
            for (uint32_t i = 1; i < n; i++) {          // fields passed over: only their bits go
                s0 &= s0 - 1;
                s1 &= s1 - 1;
            }
            pe0 = ctz64(s0);
            pe1 = ctz64(s1);
            s0 &= s0 - 1;
            s1 &= s1 - 1;
        }
        en0 = ctz64(s0);
        en1 = ctz64(s1);
#pragma unroll
        for (int u = 0; u < 2; u++) {
            Rec& R = rec[u];
            const uint32_t start = (u ? pe1 : pe0) + 1, end = u ? en1 : en0, e = u ? e1 : e0;
            const bool gone = start > e;
            R.fail |= gone ? (e == 64) : (end == 64);
            const uint32_t fp = R.p + start, fl = gone ? 0u : end - start;
            const uint32_t l = gone ? e : end;
            R.lastpos = l > R.lastpos ? l : R.lastpos;
            if (WM != LW_NONE) {
                R.wfp = kw == (uint32_t)k ? fp : R.wfp;
                R.wfl = kw == (uint32_t)k ? fl : R.wfl;
            }
            if (NS > 0) {
                R.sfp[0] = ks[0] == (uint32_t)k ? fp : R.sfp[0];
                R.sfl[0] = ks[0] == (uint32_t)k ? fl : R.sfl[0];
            }
            if (NS > 1) {
                R.sfp[1] = ks[1] == (uint32_t)k ? fp : R.sfp[1];
                R.sfl[1] = ks[1] == (uint32_t)k ? fl : R.sfl[1];
            }
            if (GROUPED) {
                R.gfp = kg == (uint32_t)k ? fp : R.gfp;
                R.klen = kg == (uint32_t)k ? fl : R.klen;
            }
        }
    }
}

// GROUPED: GROUP BY (else one group); WM: LW_*; NS: distinct SUM arguments (0-2);
// K16: LDS tags of 16 key bytes (else 8)
// CANON: the roles' column order is their canonical order (WHERE, SUM 0, SUM 1, GROUP
// BY, as present) over distinct columns, so the walk's role ranks are compile-time
// constants (no selects) and every later role skips at least one separator
template <bool GROUPED, int WM, int NS, bool K16, bool CANON>
__global__ __launch_bounds__(LT) void lean_kernel(const uint8_t* __restrict__ g, ScanStats* __restrict__ stats,
                                                  unsigned long long* __restrict__ row_out,
                                                  unsigned long long row_cap,
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
    constexpr uint32_t H = slots_for<K16>(NS, GROUPED);
    constexpr uint32_t NB = H / BSLOTS;
    constexpr uint32_t TSTRIDE = K16 ? 16u : 8u;
    LTab lt;
    lt.T = nullptr; lt.cnt = nullptr; lt.first = nullptr;
#pragma unroll
    for (int s = 0; s < MAXS; s++) { lt.sum[s] = nullptr; lt.miss[s] = nullptr; }
    if (GROUPED) {
        lt.T = carve(q, (size_t)H * TSTRIDE);
        lt.cnt = (uint32_t*)carve(q, (size_t)H * 4);
        lt.first = (uint32_t*)carve(q, (size_t)H * 4);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            lt.sum[s] = (double*)carve(q, (size_t)H * 8);
            lt.miss[s] = (uint32_t*)carve(q, (size_t)H * 4);
        }
        for (uint32_t i = tid; i < H * TSTRIDE / 16; i += LT) ((v4u*)lt.T)[i] = v4u{0u, 0u, 0u, 0u};
        for (uint32_t i = tid; i < H; i += LT) {
            lt.cnt[i] = 0;
            lt.first[i] = NOFIRST;
#pragma unroll
            for (int s = 0; s < NS; s++) { lt.sum[s][i] = 0.0; lt.miss[s][i] = 0; }
        }
        __syncthreads();
    }

    // uniform plan facts
    constexpr int NR = (WM != LW_NONE ? 1 : 0) + NS + (GROUPED ? 1 : 0);   // roles
    uint32_t skip[KN];                     // separators before role rank k's field (walk2)
    uint32_t kw = 0, ks[MAXS] = {0, 0}, kg = 0;   // role ranks of WHERE, SUM 0/1, GROUP BY
    constexpr uint32_t CKW = 0, CKS0 = WM != LW_NONE ? 1u : 0u, CKS1 = CKS0 + 1, CKG = (uint32_t)NR - 1;
#pragma unroll
    for (int k = 0; k < KN; k++) {
        const uint32_t c = __builtin_amdgcn_readfirstlane(LP.rcol[k]);
        const uint32_t pc = k ? __builtin_amdgcn_readfirstlane(LP.rcol[k - 1]) : 0u;
        skip[k] = k ? c - pc : c;
        const uint32_t role = __builtin_amdgcn_readfirstlane(LP.rrole[k]);
        if (k < NR) {
            kw = role == R_WHERE ? (uint32_t)k : kw;
            ks[0] = role == R_SUM0 ? (uint32_t)k : ks[0];
            ks[1] = role == R_SUM1 ? (uint32_t)k : ks[1];
            kg = role == R_GROUP ? (uint32_t)k : kg;
        }
    }
    if (CANON) { kw = CKW; ks[0] = CKS0; ks[1] = CKS1; kg = CKG; }
    const uint32_t rep_d = LP.delim * 0x01010101u, rep_q = LP.quote * 0x01010101u;
    const uint64_t lo_ok = LP.lo_ok, hi_ok = LP.hi_ok, last_win = LP.last_win;
    const uint32_t wstr_b = __builtin_amdgcn_readfirstlane(LP.ws);   // window stride
    // WHERE facts in scalar registers (no constant reloads inside the loop)
    const bool pass_null = __builtin_amdgcn_readfirstlane(LP.pass_null) != 0;
    const int wlo = __builtin_amdgcn_readfirstlane(LP.wlo), whi = __builtin_amdgcn_readfirstlane(LP.whi);
    const uint32_t wtt = __builtin_amdgcn_readfirstlane(LP.wtt);
    const double wl = WM == LW_NUM ? LP.wl : 0.0;
    const uint64_t wstr = WM == LW_STR ? LP.wstr : 0ull;
    const uint64_t wstep = (uint64_t)gridDim.x * NWV;

    // per-lane single-group partials and per-wave statistics
    uint32_t my_cnt = 0;
    unsigned long long my_first = ~0ULL;
    double my_sum[MAXS] = {0.0, 0.0};
    uint32_t my_num[MAXS] = {0u, 0u};
    // record / passing counts per lane (vector registers: the scalar file is full)
    uint32_t v_rec = 0, v_pass = 0;
    unsigned long long n_rec = 0;
    uint32_t v_spill = 0;                  // LDS-table misses of this lane (a vector register too)

#ifdef LEAN_CLK
    uint64_t clk_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t clk_last_ = __builtin_amdgcn_s_memtime();
#endif
    Win nx;
    // the wave's LDS window bytes as an LDS address (the LDS-DMA base)
    const uint32_t wlds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)W.bytes);
    uint64_t w = LP.first_win + (uint64_t)blockIdx.x * NWV + wv;
    if (w < last_win) load_win(g, w, wstr_b, wlds, nx);
#ifndef LEAN_L2PF
#define LEAN_L2PF 0
#endif
    // L2 prefetch of the window LEAN_L2PF windows ahead: one dword per lane every
    // 64 bytes touches every 128-byte line of it, so its HBM read starts that many
    // windows before the register load of the same bytes (then an L2 hit).  The
    // dwords are folded into pf_sink two windows later, so the wait for them comes
    // after the next register window's anyway, and never change a result.
    uint32_t pf_sink = 0, pf0 = 0, pf1 = 0;
    for (uint32_t round = 0; w < last_win; round++, w += wstep) {
        const uint64_t ws = w * wstr_b;
#if defined(LEAN_CLK) || defined(LEAN_DMA)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (LEAN_DMA: the window's bytes are in LDS)
#endif
        const Win cur = nx;
        LCLK(0);
#ifdef LEAN_DMA
        // the next window's DMA goes out once this window's bytes are read for the last
        // time: after the key loads of the last pass (LEAN_ISSUE), or after the passes
#ifdef LEAN_NOMEM
        bool issued = true;
#else
        bool issued = false;
#endif
#define LEAN_ISSUE()                                                                \
    do {                                                                            \
        if (!issued && w + wstep < last_win) load_win(g, w + wstep, wstr_b, wlds, nx); \
        issued = true;                                                              \
    } while (0)
#else
#define LEAN_ISSUE() do {} while (0)
#endif
#if !defined(LEAN_NOMEM) && !defined(LEAN_DMA)   // LEAN_NOMEM: every window re-processes the first one (no HBM reads)
        if (w + wstep < last_win) load_win(g, w + wstep, wstr_b, wlds, nx);
        if (LEAN_L2PF > 0) {
            const uint64_t wp = w + (uint64_t)LEAN_L2PF * wstep;
            pf_sink ^= pf1;
            pf1 = pf0;
            if (wp < last_win) pf0 = ((const uint32_t*)(g + wp * wstr_b))[16 * lane];
        }
#endif

        // ---- stage and classify
#ifndef LEAN_DMA
#pragma unroll
        for (int i = 0; i < 4; i++) ((v4u*)W.bytes)[64 * i + lane] = cur.a[i];
        wave_order();
#endif
        v4u la[4];                                                    // lane l: window bytes [64l, 64l + 64)
#pragma unroll
        for (int i = 0; i < 4; i++) la[i] = ((const v4u*)W.bytes)[4 * lane + i];
        uint32_t sep0, nl0, sep1, nl1, qf = 0;
        classify32(la[0], la[1], rep_d, rep_q, sep0, nl0, qf);
        classify32(la[2], la[3], rep_d, rep_q, sep1, nl1, qf);
        const bool wq = __ballot((qf & 0x80808080u) != 0) != 0;   // window holds a quote (uniform)
        if (wq) {
            W.qt[2 * lane] = byte_bits(la[0], la[1], rep_q);
            W.qt[2 * lane + 1] = byte_bits(la[2], la[3], rep_q);
        }

        // ---- record starts owned by this window: file [ws, ws + stride) within [lo_ok, hi_ok)
        const uint64_t nl = (uint64_t)nl0 | ((uint64_t)nl1 << 32);
        const uint32_t prev_top = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(nl1 >> 31), 0x138, 0xf, 0xf, true);
        const uint32_t pb = cur.prev >> 24;                           // the byte before the window
        const uint32_t prevnl = lane == 0 ? (uint32_t)(pb == '\n' || pb == '\r') : prev_top;
        uint64_t starts = ~nl & ((nl << 1) | prevnl);
        {
            const uint64_t lo64 = (lo_ok > ws ? lo_ok : ws) - ws;
            const uint64_t hi64 = hi_ok < ws + wstr_b ? hi_ok : ws + wstr_b;
            const uint32_t lo_s = (uint32_t)(lo64 < (uint64_t)wstr_b ? lo64 : (uint64_t)wstr_b);   // window offsets
            const uint32_t hi_s = hi64 > ws ? (uint32_t)(hi64 - ws) : 0u;
            const uint32_t b0 = (uint32_t)lane * LB;
            if (b0 + LB <= lo_s || b0 >= hi_s) {
                starts = 0;
            } else {
                if (lo_s > b0) starts &= ~0ull << (lo_s - b0);
                if (hi_s < b0 + LB) starts &= (1ull << (hi_s - b0)) - 1;
            }
        }
        // every lane walks the records that start in its own 64 bytes, two per pass
        // the next lane's bitmap words (wave_shl:1): a record starting in this lane's
        // bytes has its 64-byte view inside these 128 bits (lane 63 owns no start:
        // ws <= 3968)
        const uint32_t xs0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sep0, 0x130, 0xf, 0xf, true);
        const uint32_t xs1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sep1, 0x130, 0xf, 0xf, true);
        const uint32_t xn0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nl0, 0x130, 0xf, 0xf, true);
        const uint32_t xn1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nl1, 0x130, 0xf, 0xf, true);
        uint64_t todo = starts;

        LCLK(1);
#if defined(LEAN_PROF) && LEAN_PROF == 1   // profiling build: + classify, bitmaps
        n_rec += (unsigned long long)__popcll(__ballot(((xs0 ^ xs1 ^ xn0 ^ xn1) & 1) != (todo & 1)));
        LEAN_ISSUE();
        continue;
#endif
        while (__any(todo != 0)) {
            Rec rec[2];
            uint64_t sv[2], nv[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                Rec& Rr = rec[u];
                Rr.valid = todo != 0;
                const uint32_t b = Rr.valid ? ctz64(todo) : 0u;
                todo &= todo - 1;
                Rr.p = (uint32_t)lane * LB + b;
                sv[u] = view128(sep0, sep1, xs0, xs1, b);
                nv[u] = view128(nl0, nl1, xn0, xn1, b);
                Rr.fail = !Rr.valid;
                Rr.lastpos = 0;
            }
            const bool last_pass = !__any(todo != 0);
            // ---- role fields (WHERE, SUM 0/1, GROUP BY): position and length (0: NULL / missing)
            {
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    Rec& Rr = rec[u];
                    Rr.wfp = Rr.p; Rr.wfl = 0; Rr.gfp = Rr.p; Rr.klen = 0;
#pragma unroll
                    for (int j = 0; j < MAXS; j++) { Rr.sfp[j] = Rr.p; Rr.sfl[j] = 0; }
                }
                walk2<NR, WM, NS, GROUPED, CANON>(rec, sv, nv, skip, kw, ks, kg);
            }
            // a quote at or before the last byte examined may hide separators
            if (wq) {
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    Rec& Rr = rec[u];
                    Rr.fail |= (qview(W, Rr.p) & ((2ULL << (Rr.lastpos < 63 ? Rr.lastpos : 63)) - 1)) != 0;
                }
            }

            // ---- wave-uniform field-size classes: every lane's numeric WHERE / SUM field
            //      fits a dword (num4), the GROUP BY keys fit the tag (K8: 8 bytes)
            bool w4 = WM == LW_NUM, s4 = NS > 0;
            bool g8 = GROUPED;
            {
                bool wb = true, sb = true, gb = true;
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const Rec& Rr = rec[u];
                    wb = wb & (!Rr.valid | (Rr.wfl <= 4u));
#pragma unroll
                    for (int j = 0; j < NS; j++) sb = sb & (!Rr.valid | (Rr.sfl[j] <= 4u));
                    gb = gb & (!Rr.valid | (Rr.klen <= 8u));
                }
                if (WM == LW_NUM) w4 = __all(wb);
                if (NS > 0) s4 = __all(sb);
                if (GROUPED) g8 = __all(gb);
            }

            // ---- field bytes of the roles (one batch of LDS reads)
            uint32_t wd0[2] = {0, 0}, wd1[2] = {0, 0};
            uint32_t sd0[2][MAXS], sd1[2][MAXS];
            uint32_t k0[2] = {0, 0}, k1[2] = {0, 0}, k2[2] = {0, 0}, k3[2] = {0, 0};
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const Rec& Rr = rec[u];
                if (WM != LW_NONE) {
                    if (w4) wd0[u] = load4(W.bytes, Rr.wfp);
                    else load8(W.bytes, Rr.wfp, wd0[u], wd1[u]);
                }
#pragma unroll
                for (int j = 0; j < MAXS; j++) {
                    sd0[u][j] = sd1[u][j] = 0;
                    if (j < NS) {
                        if (s4) sd0[u][j] = load4(W.bytes, Rr.sfp[j]);
                        else load8(W.bytes, Rr.sfp[j], sd0[u][j], sd1[u][j]);
                    }
                }
                if (GROUPED) {
                    if (g8 || !K16) load8(W.bytes, Rr.gfp, k0[u], k1[u]);
                    else load16(W.bytes, Rr.gfp, k0[u], k1[u], k2[u], k3[u]);
                }
            }

            LCLK(2);
#if defined(LEAN_PROF) && LEAN_PROF == 2   // profiling build: + record list, views, field walk, field loads
            n_rec += __popcll(__ballot(rec[0].fail ^ rec[1].fail ^ ((wd0[0] ^ wd0[1] ^ sd0[0][0] ^ sd0[1][0] ^ k0[0] ^ k1[1]) & 1)));
            wave_order();
            continue;
#endif
            // ---- WHERE outcome: numerals and short strings in registers, else the exact typers
            bool pass_[2] = {true, true};
            if (WM != LW_NONE) {
                bool outcome[2], gen[2];
                Num n[2];
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const Rec& Rr = rec[u];
                    outcome[u] = pass_null;                // missing column / empty field: NULL
                    bool typed = Rr.wfl == 0;
                    if (WM == LW_NUM) {
                        n[u] = w4 ? num4<false>(wd0[u], Rr.wfl) : num7(wd0[u], wd1[u], Rr.wfl);
                        const int c = (int)n[u].M < wlo ? -1 : ((int)n[u].M > whi ? 1 : 0);
                        if (n[u].ok) outcome[u] = tt_result(wtt, c);
                        typed |= n[u].ok;
                    } else if (WM == LW_STR) {
                        // a STRING field of <= 8 bytes: no leading digit / sign / dot (never a
                        // numeral or date), no byte <= ' ' (trim_whitespace is a no-op)
                        uint32_t a0 = wd0[u], a1 = wd1[u];
                        const uint32_t c0 = a0 & 0xFFu;
                        mask8(Rr.wfl, a0, a1);
                        const uint32_t f0 = len_mask(Rr.wfl, 0) & 0x80808080u, f1 = len_mask(Rr.wfl, 1) & 0x80808080u;
                        const bool ok = (int)(Rr.wfl - 1 < 8u) &
                                        (int)!(is_digit(c0) | (c0 == '-') | (c0 == '+') | (c0 == '.')) &
                                        (int)((low_bytes(a0, f0) | low_bytes(a1, f1)) == 0);
                        const uint64_t x = bswap64(a0, a1);
                        if (ok) outcome[u] = tt_result(wtt, x < wstr ? -1 : (x > wstr ? 1 : 0));
                        typed |= ok;
                    }
                    gen[u] = !typed & !Rr.fail;
                }
                if (WM == LW_NUM && w4) {
                    // DOUBLE fields of <= 4 bytes (num4<false> declined them): strtod = RN(M / 10^k)
                    if (__any(gen[0] | gen[1])) {
#pragma unroll
                        for (int u = 0; u < 2; u++) {
                            if (gen[u]) {
                                const Num d = num4<true>(wd0[u], rec[u].wfl);
                                if (d.ok) {
                                    const double v = (double)d.M / p10(d.k);
                                    outcome[u] = tt_result(wtt, v < wl ? -1 : (v > wl ? 1 : 0));
                                    gen[u] = false;
                                }
                            }
                        }
                    }
                } else if (WM == LW_NUM) {
                    if (__any(n[0].ok & n[0].dot) || __any(n[1].ok & n[1].dot)) {
#pragma unroll
                        for (int u = 0; u < 2; u++) {
                            if (n[u].ok & n[u].dot) {
                                const double v = (double)n[u].M / p10(n[u].k);
                                outcome[u] = tt_result(wtt, v < wl ? -1 : (v > wl ? 1 : 0));
                            }
                        }
                    }
                }
                if (__any(gen[0] | gen[1])) {              // the exact typers (rare shapes)
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        if (gen[u]) {
                            Cell c;
                            if (!type_field(W.bytes, rec[u].wfp, rec[u].wfl, c)) {
                                rec[u].fail = true;
                            } else {
                                if (c.kind == K_STR) c.bits = (uint64_t)(uintptr_t)(W.bytes + rec[u].wfp);
                                outcome[u] = tt_result(wtt, compare(c, LP.wconst));
                            }
                        }
                    }
                }
                pass_[0] = outcome[0];
                pass_[1] = outcome[1];
            }

            // ---- SUM addends (numeric: true and the value)
            double sval[2][MAXS];
            bool snum[2][MAXS];
#pragma unroll
            for (int j = 0; j < MAXS; j++) {
                bool gen[2] = {false, false};
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    sval[u][j] = 0.0;
                    snum[u][j] = false;
                    if (j >= NS) continue;
                    const uint32_t len = rec[u].sfl[j];
                    Num n;
                    if (s4) {
                        n = num4<true>(sd0[u][j], len);
                        sval[u][j] = (double)n.M * (((n.k & 1) ? 0.1 : 1.0) * ((n.k & 2) ? 0.01 : 1.0));   // = inv10(k), k <= 3
                    } else {
                        n = num7(sd0[u][j], sd1[u][j], len);
                        sval[u][j] = (double)n.M * inv10(n.k);
                    }
                    snum[u][j] = n.ok;
                    gen[u] = !n.ok & (len != 0) & !rec[u].fail;
                }
                if (j < NS && __any(gen[0] | gen[1])) {
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        if (gen[u]) {
                            Cell c;
                            if (!type_field(W.bytes, rec[u].sfp[j], rec[u].sfl[j], c)) rec[u].fail = true;
                            else if (is_num(c)) { sval[u][j] = num_of(c); snum[u][j] = true; }
                        }
                    }
                }
            }

            // ---- GROUP BY key: the raw field bytes (no byte <= ' '), zero padded
            uint32_t h[2] = {0, 0};
            bool longk[2] = {false, false};
            if (GROUPED) {
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const uint32_t klen = rec[u].klen;
                    if (g8 || !K16) {
                        const uint32_t m0 = len_mask(klen, 0), m1 = len_mask(klen, 1);
                        k0[u] &= m0; k1[u] &= m1;
                        if (!K16 && __any(klen - 9u < 8u) && klen - 9u < 8u)   // a 9-16 byte key: its spill
                            load16(W.bytes, rec[u].gfp, k0[u], k1[u], k2[u], k3[u]);   // needs bytes 8-15
                        const uint32_t lowb = low_bytes(k0[u], m0 & 0x80808080u) | low_bytes(k1[u], m1 & 0x80808080u);
                        rec[u].fail |= lowb != 0;
                        longk[u] = klen > 8;
                    } else {
                        const uint32_t m0 = len_mask(klen, 0), m1 = len_mask(klen, 1), m2 = len_mask(klen, 2),
                                       m3 = len_mask(klen, 3);
                        k0[u] &= m0; k1[u] &= m1; k2[u] &= m2; k3[u] &= m3;
                        const uint32_t lowb = low_bytes(k0[u], m0 & 0x80808080u) | low_bytes(k1[u], m1 & 0x80808080u) |
                                              low_bytes(k2[u], m2 & 0x80808080u) | low_bytes(k3[u], m3 & 0x80808080u);
                        rec[u].fail |= lowb != 0;
                        longk[u] = klen > 16;
                    }
                    if (klen == 0) k1[u] = 1u;               // the empty key's tag
                    // 8-byte tags: only keys of <= 8 bytes are looked up (longer ones spill
                    // with their own hash), so words 2-3 never enter the tag hash
                    h[u] = K16 ? key_hash(k0[u], k1[u], k2[u], k3[u]) : key_hash(k0[u], k1[u], 0u, 0u);
                }
            }

            if (last_pass) LEAN_ISSUE();                  // (spills take the key from registers)
            LCLK(3);
#if defined(LEAN_PROF) && LEAN_PROF == 3   // profiling build: + typing, keys and hashes
            n_rec += __popcll(__ballot(pass_[0] ^ pass_[1] ^ ((h[0] ^ h[1] ^ (uint32_t)sval[0][0] ^ (uint32_t)sval[1][0]) & 1)));
            wave_order();
            continue;
#endif
            // ---- declined records go whole to slow_kernel
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const Rec& Rr = rec[u];
                const uint64_t off = ws + Rr.p;
                const bool slow = Rr.valid && Rr.fail;
                const uint64_t sb = __ballot(slow);
                if (sb) {
                    unsigned long long base = 0;
                    if (lane == 0) base = atomicAdd(&stats->slow_records, (unsigned long long)__popcll(sb));
                    base = __shfl(base, 0, 64);
                    if (slow) {
                        const unsigned long long i = base + __popcll(sb & ((1ULL << lane) - 1));
                        if (i < slow_cap) slow_list[i] = off;
                    }
                }
                const bool ok = Rr.valid & !Rr.fail;
                pass_[u] = pass_[u] & ok;
                v_rec += ok ? 1u : 0u;
                v_pass += pass_[u] ? 1u : 0u;
                if (!GROUPED && row_out) {                 // (grouped launches never emit rows)
                    const unsigned long long slot = wave_slot(pass_[u], &stats->rows_emitted);
                    if (pass_[u] && slot < row_cap) row_out[slot] = off;
                }
            }

            LCLK(4);
            // ---- aggregate
            if (!GROUPED) {
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const uint64_t off = ws + rec[u].p;
                    my_cnt += pass_[u] ? 1u : 0u;
                    my_first = pass_[u] && off < my_first ? off : my_first;
#pragma unroll
                    for (int j = 0; j < NS; j++) {
                        my_sum[j] += pass_[u] && snum[u][j] ? sval[u][j] : 0.0;
                        my_num[j] += pass_[u] && snum[u][j] ? 1u : 0u;
                    }
                }
            } else {
                int slot[2];
                bool miss[2];
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    slot[u] = longk[u] ? -1 : lt_find<K16>(lt, NB, h[u], k0[u], k1[u], k2[u], k3[u]);
                    miss[u] = pass_[u] & (slot[u] < 0) & !longk[u];
                }
#if defined(LEAN_PROF) && LEAN_PROF == 4   // profiling build: + table lookups (no atomics)
                n_rec += __popcll(__ballot((slot[0] ^ slot[1]) & 1));
                wave_order();
                continue;
#endif
                if (__any(miss[0] | miss[1])) {           // new keys (rare after the first windows)
#pragma unroll
                    for (int u = 0; u < 2; u++)
                        if (miss[u]) slot[u] = lt_insert<K16>(lt, NB, h[u], k0[u], k1[u], k2[u], k3[u]);
                }
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const bool add = pass_[u] & (slot[u] >= 0);
                    if (add) {
                        const uint32_t fc = (round << 16) | ((uint32_t)wv << 12) | rec[u].p;
#ifndef LEAN_ATOM
#define LEAN_ATOM 7
#endif
                        if (LEAN_ATOM & 1) atomicAdd(&lt.cnt[slot[u]], 1u);
                        if (LEAN_ATOM & 32) lt.cnt[slot[u]] = fc;                       // experiment: plain store
                        if (LEAN_ATOM & 64) atomicAdd(&lt.cnt[(wv * 64 + lane + 128 * u) & (H - 1)], 1u);   // experiment: private
                        if (LEAN_ATOM & 128) atomicAdd(&lt.cnt[h[u] & (H - 1)], 1u);   // experiment: no lookup dependency
                        if (LEAN_ATOM & 2) atomicMin(&lt.first[slot[u]], fc);
#pragma unroll
                        for (int j = 0; j < NS; j++) {
                            if (LEAN_ATOM & 4) atomicAdd(&lt.sum[j][slot[u]], snum[u][j] ? sval[u][j] : 0.0);
                            if (LEAN_ATOM & 8) atomicAdd((unsigned long long*)&lt.sum[j][slot[u]], (unsigned long long)(sval[u][j] * 1000.0));
                            if (LEAN_ATOM & 16) atomicAdd((uint32_t*)&lt.sum[j][slot[u]], (uint32_t)(sval[u][j] * 1000.0));
                        }
                    }
#pragma unroll
                    for (int j = 0; j < NS; j++) {
                        const bool nn = add & !snum[u][j];
                        if (__any(nn)) {
                            if (nn) atomicAdd(&lt.miss[j][slot[u]], 1u);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const bool spill = pass_[u] && slot[u] < 0;
                    if (__any(spill)) {                    // long key or both buckets full: the HBM raw table
                        v_spill += spill ? 1u : 0u;
                        if (spill) {
                            spill_record(k0[u], k1[u], k2[u], k3[u], rec[u].klen, ws + rec[u].p, tabs, stats,
                                         slow_list, slow_cap, LP.nacc, LP.acc_sidx, snum[u][0], sval[u][0],
                                         snum[u][MAXS - 1], sval[u][MAXS - 1]);
                        }
                    }
                }
            }
            wave_order();
            LCLK(5);
        }
        LEAN_ISSUE();                                     // (a window without owned records)
        LCLK(6);
    }
#undef LEAN_ISSUE
    if (LEAN_L2PF > 0 && (pf_sink ^ pf0 ^ pf1) == 0x9E3779B9u && lane == 63 && n_rec == 0x9E3779B9ull)
        stats->clk[7] = 1;       // keeps the prefetch loads (never true in practice)
#ifdef LEAN_CLK
    if (lane == 0)
        for (int i = 0; i < 8; i++) atomicAdd(&stats->clk[i], (unsigned long long)clk_[i]);
#endif

    // ---- statistics
    unsigned long long n_pass = v_pass, n_spill = v_spill;
    n_rec = (lane == 0 ? n_rec : 0ull) + v_rec;     // (profiling builds count uniformly in n_rec)
    for (int o = 32; o > 0; o >>= 1) {
        n_rec += __shfl_down(n_rec, o, 64);
        n_pass += __shfl_down(n_pass, o, 64);
        n_spill += __shfl_down(n_spill, o, 64);
    }
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
    // every block walks its slots from a different start: the blocks' tables hold
    // the same keys in nearly the same slots, and flushing them in the same order
    // would send all blocks' atomics for one key to one HBM slot at once
    const uint32_t rot = (uint32_t)blockIdx.x * (H / 64 + 1);
    for (uint32_t ii = tid; ii < H; ii += LT) {
        const uint32_t i = (ii + rot) & (H - 1);
        const uint32_t* tw = (const uint32_t*)(lt.T + i * TSTRIDE);
        const uint64_t w0 = (uint64_t)tw[0] | ((uint64_t)tw[1] << 32);
        const uint64_t w1 = K16 ? ((uint64_t)tw[2] | ((uint64_t)tw[3] << 32)) : 0ull;
        if (w0 == 0 || (K16 && tw[1] == CLAIM && tw[0] == 0)) continue;   // free (or a never-published claim)
        const uint32_t n = lt.cnt[i];
        if (!n) continue;
        const uint32_t kl = key_len(w0, w1);
        const GKey k = raw_key(kl, kl ? w0 : 0ull, w1);
        const int gi = g_insert(rt, k, gk_hash(k), stats);
        if (gi < 0) continue;
        atomicAdd(&rt.cnt[gi], (unsigned long long)n);
        const uint32_t fc = lt.first[i];
        if (fc != NOFIRST) {
            const uint64_t fw = LP.first_win + ((uint64_t)(fc >> 16) * gridDim.x + blockIdx.x) * NWV + ((fc >> 12) & 15);
            atomicMin(&rt.first[gi], (unsigned long long)(fw * LP.ws + (fc & 4095)));
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
// A raw key's MIN / MAX cell (fast_kernel's EXT builds) merges like every other
// extreme: the wave-uniform seqlock update (scanlib.h g_ext_update), so the thread
// loop has no early exit.  max_mask bit a: accumulator a is a MAX.
// pk_acc >= 0: that accumulator's rt.extpos words hold fast_kernel's packed extreme
// keys (fast.hip ext_packed: value bits above a 40-bit record offset), typed here from
// the record's field pk_col -- once per raw key instead of once per block
__global__ __launch_bounds__(256) void raw_merge_kernel(ScanStats* __restrict__ stats, const GroupTable gt,
                                                        const GroupTable rt, int nacc, uint32_t max_mask,
                                                        const uint8_t* __restrict__ g, int pk_acc, uint32_t pk_col,
                                                        uint32_t delim) {
    __shared__ __align__(16) uint8_t buf[256 * 32];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const bool live = i < rt.cap && rt.tag[i] >= 2;
    int gi = -1;
    if (live) {
        const GKey k = canonical_key(buf + threadIdx.x * 32, rt.clslen[i] & 0xFFFF, rt.w0[i], rt.w1[i]);
        gi = g_insert(gt, k, gk_hash(k), stats);
    }
    if (gi >= 0) {
        atomicAdd(&gt.cnt[gi], rt.cnt[i]);
        atomicMin(&gt.first[gi], rt.first[i]);
        rt.cnt[i] = 0;                    // consumed: a chunked rescan merges each chunk's
        for (int a = 0; a < nacc; a++) {  // raw state once (first offsets merge by MIN)
            if (!rt.num[a]) continue;
            const unsigned long long n = rt.num[a][i];
            if (n) {
                atomicAdd(&gt.sum[a][gi], rt.sum[a][i]);
                atomicAdd(&gt.num[a][gi], n);
                rt.sum[a][i] = 0;
                rt.num[a][i] = 0;
            }
        }
    }
    for (int a = 0; a < nacc; a++) {
        if (!rt.ext[a] || !gt.ext[a]) continue;       // (uniform)
        const unsigned long long w = gi >= 0 ? rt.extpos[a][i] : NOPOS;
        bool need = gi >= 0 && w != NOPOS;
        unsigned long long pos = w;
        Cell c = cell_null();
        if (a == pk_acc) {
            pos = need ? (w & ((1ull << 40) - 1)) : NOPOS;
            if (need) c = field_cell(g, pos, pk_col, delim);
            need = need && c.kind != K_NULL;
        } else if (need) {
            c = rt.ext[a][i];
        }
        g_ext_update(need, gt, a, ((max_mask >> a) & 1) ? ACC_MAX : ACC_MIN, gi >= 0 ? (uint32_t)gi : 0u, c, pos,
                     stats);
        if (need) rt.extpos[a][i] = NOPOS;
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

template <bool K16>
size_t lean_lds_t(int ns, int grouped) {
    return lean::fixed_bytes() + (size_t)lean::slots_for<K16>(ns, grouped != 0) * lean::slot_bytes<K16>(ns) + 256;
}

typedef void (*lean_fn_t)(const uint8_t*, ScanStats*, unsigned long long*, unsigned long long, unsigned long long*,
                          unsigned long long, const lean::LeanArgs, const GroupTable*);

template <bool G, int WM, bool K16, bool CANON>
lean_fn_t pick_ns(int ns) {
    if (ns == 0) return lean::lean_kernel<G, WM, 0, K16, CANON>;
    return ns == 1 ? lean::lean_kernel<G, WM, 1, K16, CANON> : lean::lean_kernel<G, WM, 2, K16, CANON>;
}
template <bool G, bool K16, bool CANON>
lean_fn_t pick_wm(int wm, int ns) {
    switch (wm) {
        case lean::LW_NONE: return pick_ns<G, lean::LW_NONE, K16, CANON>(ns);
        case lean::LW_NUM: return pick_ns<G, lean::LW_NUM, K16, CANON>(ns);
        case lean::LW_STR: return pick_ns<G, lean::LW_STR, K16, CANON>(ns);
        default: return pick_ns<G, lean::LW_GEN, K16, CANON>(ns);
    }
}
template <bool G, bool K16>
lean_fn_t pick_fn(int wm, int ns, bool canon) {
    return canon ? pick_wm<G, K16, true>(wm, ns) : pick_wm<G, K16, false>(wm, ns);
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

// The window stride for a file: a window's records are handled two per lane, so a
// stride holding ~120 records of the file's average length fills a wave's 128
// record slots in one pass (and never more than the staged bytes allow).  The
// average comes from up to 256 KiB of the data bytes (records split on '\n' /
// '\r' runs, as csv_load does).
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
    uint64_t ws = (uint64_t)(120.0 * avg) & ~(uint64_t)127;
    if (ws > (uint64_t)lean::WS) ws = lean::WS;
    if (ws < 512) ws = 512;
    return (uint32_t)ws;
}
int cq_lean_waves_per_block() { return lean::NWV; }

// Columns whose sampled fields (up to 256 KiB of records, quote-blind split) are
// longer than 8 bytes: bit c for column c < 63, bit 63 for every later column.
// A GROUP BY on such a column runs the K16 tag width.
uint64_t cq_cols_longer_than(const uint8_t* data, uint64_t n, uint32_t delim, uint32_t limit);
uint64_t cq_lean_long_cols(const uint8_t* data, uint64_t n, uint32_t delim) {
    return cq_cols_longer_than(data, n, delim, 8);
}
// bit c: a sampled field of column c (the first 256 KiB) is longer than `limit`
// bytes (bit 63 for every column from 63 on, and always set)
uint64_t cq_cols_longer_than(const uint8_t* data, uint64_t n, uint32_t delim, uint32_t limit) {
    const uint64_t m = n < (256u << 10) ? n : (256u << 10);
    uint64_t mask = 1ull << 63, i = 0;
    while (i < m) {
        while (i < m && (data[i] == '\n' || data[i] == '\r')) i++;
        uint32_t c = 0;
        uint64_t fs = i;
        while (i <= m) {
            const bool end = i == m || data[i] == '\n' || data[i] == '\r';
            if (end || data[i] == delim) {
                if (i - fs > limit) mask |= 1ull << (c < 63 ? c : 63);
                c++;
                fs = i + 1;
                if (end) break;
            }
            i++;
        }
    }
    return mask;
}

size_t cq_lean_lds_bytes(const cq::ScanPlan* P, int grouped) {
    LeanPlan lp;
    int wm = 0;
    if (!lean_shape(P, &lp, &wm)) return 0;
    return P->lean_k16 ? lean_lds_t<true>(ns_of(lp), grouped) : lean_lds_t<false>(ns_of(lp), grouped);
}

// the lean scan (the caller runs slow_kernel over slow_list afterwards)
hipError_t cq_launch_lean(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          const cq::GroupTable* rt, cq::ScanStats* stats, unsigned long long* row_out,
                          unsigned long long row_cap, int grouped, int grid, hipStream_t s,
                          unsigned long long* slow_list, unsigned long long slow_cap) {
    LeanPlan lp;
    int wm = 0;
    if (!lean_shape(P, &lp, &wm)) return hipErrorInvalidValue;
    if (((uintptr_t)g & 255) != 0) return hipErrorInvalidValue;   // 128-byte aligned windows
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
    if (lp.ws > (uint32_t)lean::WS || lp.ws % 128) return hipErrorInvalidValue;
    lp.first_win = P->range_begin / lp.ws;
    lp.last_win = (hi + lp.ws - 1) / lp.ws;
    const int ns = ns_of(lp);
    bool canon = true;
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
        // canonical: the walk meets the roles in the order they were added
        uint32_t want[lean::KN], nw = 0;
        if (wm != lean::LW_NONE) want[nw++] = lean::R_WHERE;
        for (int j = 0; j < ns; j++) want[nw++] = j == 0 ? lean::R_SUM0 : lean::R_SUM1;
        if (grouped) want[nw++] = lean::R_GROUP;
        // and the columns are distinct (walk2's DISTINCT: every later role skips >= 1 separator)
        for (uint32_t i = 0; i < nr; i++) canon = canon && lp.rrole[i] == want[i] && (i == 0 || lp.rcol[i] > lp.rcol[i - 1]);
    }
    const bool k16 = grouped && P->lean_k16;
    const size_t lds = k16 ? lean_lds_t<true>(ns, grouped) : lean_lds_t<false>(ns, grouped);
    lean::LeanArgs args;
    memset(&args, 0, sizeof args);
    args.lp = lp;
    // the launch's table pair in device memory of this thread and device (as fast.hip)
    thread_local GroupTable* tabs_devs[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    GroupTable*& tabs_dev = tabs_devs[dev & 63];
    if (!tabs_dev) {
        hipError_t e = hipMalloc((void**)&tabs_dev, 2 * sizeof(GroupTable));
        if (e != hipSuccess) return e;
    }
    GroupTable tabs[2];
    tabs[0] = *gt;
    if (rt) tabs[1] = *rt;
    else memset(&tabs[1], 0, sizeof tabs[1]);
    {
        hipError_t e = cq::upload_buffer(tabs_dev, tabs, sizeof tabs, s);
        if (e != hipSuccess) return e;
    }
    if (grouped && row_out) return hipErrorInvalidValue;   // the grouped kernels emit no rows
    const lean_fn_t fn = !grouped ? pick_fn<false, false>(wm, ns, canon)
                                  : (k16 ? pick_fn<true, true>(wm, ns, canon) : pick_fn<true, false>(wm, ns, canon));
    cq::set_max_lds((const void*)fn, (int)lds);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(lean::LT), lds, s, g, stats, row_out, row_cap, slow_list, slow_cap,
                       args, (const GroupTable*)tabs_dev);
    return hipGetLastError();
}

// raw-key table -> canonical table (after cq_launch_lean of a grouped plan)
hipError_t cq_launch_raw_merge(const cq::GroupTable* gt, const cq::GroupTable* rt, int nacc, cq::ScanStats* stats,
                               hipStream_t s, uint32_t max_mask, const uint8_t* g, int pk_acc, uint32_t pk_col,
                               uint32_t delim) {
    if (pk_acc >= 0 && !g) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lean::raw_merge_kernel, dim3((rt->cap + 255) / 256), dim3(256), 0, s, stats, *gt, *rt, nacc,
                       max_mask, g, pk_acc, pk_col, delim);
    return hipGetLastError();
}

}  // extern "C"
