// fast.hip -- the scan kernel for the plan shape of the benchmark queries.
//
// Same job and semantics as lean_kernel (lean.hip) -- csv_load + filter_rows +
// create_groups + evaluate_aggregate in one pass over the HBM-resident bytes
// (reference csv_reader.c:375-465, evaluator_utils.c:986-1006,
// evaluator_aggregates.c:108-414) -- for the narrower shape the benchmark and most
// aggregate queries have:
//   WHERE absent or `column op numeric-literal`; COUNT / SUM / AVG over at most two
//   distinct columns; GROUP BY absent or one column whose keys fit 8 bytes; the
//   roles' columns strictly ascending in the order WHERE, SUM 0, SUM 1, GROUP BY.
// Everything a record needs is decided on one straight path; any record the path
// cannot type exactly (a quote in front of its fields, a field of another shape, a
// short row, a key with a blank) goes whole to the slow list and slow_kernel
// (scan.hip), which runs the general parser.  That keeps the kernel's vector
// instruction stream short: on gfx950 a wave64 integer VALU instruction holds its
// SIMD for four cycles, and lean_kernel was bound by that stream
// (profiles/r3_valu_rate.txt).
//
// Structure (one 1024-thread block per CU, each wave streaming its own windows):
//   load      4 KiB windows by LDS-DMA straight into the wave's LDS bytes
//   classify  lane l: bytes [64l, 64l+64) -> 64-bit separator and terminator masks
//             (two v_perm_b32 lookups per dword); with the default ',' and '"' the
//             delimiter lookup also flags quotes (its table maps '"' to 0x00, whose
//             zero-byte test costs two instructions per dword)
//   records   each lane walks the records starting in its own 64 bytes, two at a time
//   fields    the roles' field ends by clearing separator bits; compile-time role ranks
//   values    numerals of 1-4 bytes in registers (v_perm + v_dot4); wider ones by a
//             uniform side path
//   SUM       addends of <= 3 decimals as exact fixed-point integers (scale 10^3)
//             accumulated with 64-bit LDS integer atomics; other numerals in doubles
//   GROUP BY  LDS table of 2048 slots in 1024 two-slot buckets; a key lives in one of
//             its two buckets.  The host seeds the table from a sample of the file
//             with a cuckoo placement (no bucket overflows for the sampled keys), so a
//             lookup is two 16-byte LDS reads and four compares; unseen keys take a
//             free slot of their buckets by CAS, or spill to the HBM raw table
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include <unordered_set>
#include "plan.h"
#include "scanlib.h"
#include "upload.h"

namespace cq {
namespace fast {

constexpr int NWV = 16;                   // waves per block
constexpr int LT = 64 * NWV;              // threads per block
constexpr int LB = 64;                    // window bytes per lane
constexpr int WB = 64 * LB;               // window bytes (4 KiB)
constexpr int WS = 3968;                  // largest window stride (records owned per window)
constexpr int NMW = WB / 32;
constexpr int WBYTES = WB + 32;
constexpr int MAXS = 2;
constexpr uint32_t NOFIRST = 0xFFFFFFFFu;
constexpr uint32_t TSLOTS = 2048;         // LDS table slots
constexpr uint32_t TBUCKETS = TSLOTS / 2; // two-slot buckets
static_assert(WS + 64 + 16 <= WB, "a record view plus a field load stays in the window");

struct WaveLds {
    uint8_t bytes[WBYTES];
    uint32_t qt[NMW + 4];       // quote bits (written only when the window holds a quote)
};
static_assert(sizeof(WaveLds) % 16 == 0, "16-byte aligned wave areas");

struct FastPlan {
    uint64_t first_win;         // the first window holding an owned record start
    uint32_t nwin;              // windows [first_win, first_win + nwin) hold the owned starts
    uint32_t lo_s, hi_s;        // owned starts: from lo_s in the first window, below hi_s in the last
    uint32_t ws;                // window stride (multiple of 128, <= WS)
    uint32_t delim, quote;
    uint32_t skip[5];           // field k's column minus field k-1's (field 0: its column); fields = the
                                // roles' columns ascending (equal columns: skip 0)
    uint32_t rank[5];           // field index of WHERE, SUM 0, SUM 1, GROUP BY, WHERE column 1 (WX == 2)
    uint32_t wtt;               // WHERE truth table (bit 0 <, 1 ==, 2 >)
    int32_t wlo, whi;           // INTEGER field M: M < L <=> M < wlo; M > L <=> M > whi
    uint32_t wa, ww, wneg;      // a 1-4 digit INTEGER M passes <=> ((M - wa) <=u ww) != wneg
    double wl;                  // the literal
    uint32_t pass_null;         // WHERE outcome of a NULL (empty) field
    int32_t nacc;
    uint32_t acc1;              // bit a: accumulator a sums SUM argument 1 (else 0)
    const unsigned long long* seed;   // TSLOTS host-placed tags, or null
    // the one MIN / MAX accumulator of an EXT build (its argument: SUM argument 0);
    // sum_mask bit a: accumulator a is a SUM / AVG (the flushes skip the extreme)
    int32_t ext_acc;
    uint32_t ext_col;           // the argument's column (the flushes re-type the extreme's field)
    uint32_t sum_mask;
    // WSTR builds: WHERE `column op 'literal'` with a 1-8 byte STRING literal: its bytes
    // as a big-endian word, zero padded (strcmp order of zero-padded words), cut at a NUL
    uint32_t wstr_lit;          // 1: the WHERE literal is such a STRING
    uint64_t wstr;
    // WX builds: a compound WHERE (evaluate_condition's NOT / AND / OR tree over up to 4
    // leaves `column op literal` or `column [NOT] IN (literals)`, evaluator_conditions.c:
    // 62-164) over up to 2 columns.  Every leaf is evaluated (as the reference evaluates
    // both sides of AND / OR), the tree is the 16-entry truth table wx_tt over the leaf
    // outcomes.  A NUMBER column's fields are typed as exact 10^-3 fixed point V (the SUM
    // path's num4: <= 4 bytes); a comparison is an interval of V whose bounds the host
    // found with the reference's own double compare (RN(V / 1000) against the literal's
    // double); a STRING column's 1-8 byte fields compare as zero-padded big-endian words.
    uint32_t wx_nleaf;
    uint32_t wx_tt;
    uint32_t wx_str;            // bit c: WHERE column c is a STRING column (else a NUMBER one)
    uint32_t lx_col[4];         // the leaf's WHERE column (0 / 1)
    uint32_t lx_kind[4];        // LX_*
    uint32_t lx_a[4], lx_w[4], lx_neg[4];   // LX_NUM: ((V - a) <=u w) != neg; LX_*IN: neg = NOT IN
    uint32_t lx_null[4];        // the leaf's outcome for a NULL (empty) field
    uint32_t lx_tt[4];          // LX_STR: truth table over (<, ==, >)
    uint32_t lx_nin[4];         // LX_*IN: items
    uint64_t lx_lit[4];         // LX_STR: the literal's word
    uint64_t lx_in[4][8];       // LX_*IN: V values (numbers) or words (strings)
};
enum : uint32_t { LX_NUM = 0, LX_STR = 1, LX_NIN = 2, LX_SIN = 3 };
// a leaf's parameters in LDS (WX builds): meta (kind | col << 2 | neg << 3 | null << 4 |
// tt << 5 | nin << 8), a, w, 0, lit (2 words), in[8] (16 words)
constexpr uint32_t LX_WORDS = 22;

// HBM tables: canonical keys (TAB_GT), raw keys (TAB_RT)
enum : int { TAB_GT = 0, TAB_RT = 1 };
// (the pair itself: a per-thread device buffer, cq_launch_fast)
constexpr uint32_t GK_RAW = 6;       // raw field bytes as key (lean.hip's class)

// ------------------------------------------------------------------ helpers
// trailing zeros of x, or >= 64 (0xFFFFFFFF) when x == 0: v_ffbl of each half (all
// ones for a zero half), the high half's index | 32, the smaller (v_ffbl as written:
// the compiler's cttz lowering adds zero tests)
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t ctz64(uint64_t x) {
    const uint32_t lo = ffbl((uint32_t)x), hi = ffbl((uint32_t)(x >> 32)) | 32u;
    return lo < hi ? lo : hi;
}

// The window's 4 KiB straight into the wave's LDS bytes by four LDS-DMA loads, 1 KiB
// each (lane l's 16 bytes at 16l): one scalar base, the lane's constant offset `voff`
// (16 * lane) and the instruction offsets 0 / 1024 / 2048 / 3072, which step the LDS
// destination (M0 + offset + 16 * lane) with the source, so the window costs no vector
// address arithmetic and keeps one scalar pair live.  The caller waits with vmcnt(0);
// the lgkmcnt(0) first retires this wave's LDS reads of the window the loads
// overwrite.  M0 is set and restored inside the statement (the compiler owns M0).
// `prev`: the 4 bytes before the window.
__device__ __forceinline__ void load_win(const uint8_t* g, uint64_t w, uint32_t ws, uint32_t lds, uint32_t voff,
                                         uint32_t& prev) {
    const uint8_t* base = g + w * ws;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:2048\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:3072\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(base), "s"(lds)
        : "memory");
    prev = *(const uint32_t*)(base - 4);
}

// A VGPR-resident copy of a (uniform or constant) value: on gfx950 a VALU instruction
// reading an SGPR operand issues at half rate, and VOP3 instructions cannot take a
// literal, so the constants of the hot VOP3 operations live in VGPRs
__device__ __forceinline__ uint32_t vreg(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
// the same for a 64-bit value or a pointer (cold-path operands: the loop's scalar
// registers stay for its own state instead of spilling into VGPR lanes)
__device__ __forceinline__ uint64_t vreg64(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
template <class T>
__device__ __forceinline__ T* vptr(T* p) { return (T*)(uintptr_t)vreg64((uint64_t)(uintptr_t)p); }
// the classifier's constants (VGPRs)
struct CK {
    uint32_t tn1, tn0, td1, td0;   // v_perm tables: terminators, delimiter
    uint32_t m40;                  // 0x40404040
    uint32_t m80;                  // 0x80808080
    uint32_t w0, w1;               // v_dot4 bit weights
    uint32_t rd, rq;               // delimiter / quote bytes x 4 (non-COMMA)
};
__device__ __forceinline__ uint32_t flags40(uint32_t r, uint32_t m40) { return __builtin_amdgcn_bitop3_b32(r, r >> 1, m40, 0x20); }

// 32 bytes -> separator and terminator bits; quote presence accumulated in q
// (COMMA: the delimiter lookup's zero bytes, else the quote byte's zero test)
#ifndef FAST_OLD_CLS
// COMMA tables with the match in bit 0 (v_perm output & 0x01010101 is 0 exactly
// for the matched bytes, so no flag extraction before v_dot4):
//   terminators: x ^ 0x06 -> '\n' selector 12 (always 0x00), '\r' selector 11 (sign
//     of table byte 7 = 0x01 -> 0x00); byte 0x01 selects table byte 7 itself (0x01);
//     every other table byte 0xFF, selectors >= 13 0xFF: exact, no false match
//   delimiter: x ^ 0x2E -> ',' selector 2 (0x80), '"' selector 12 (0x00: a separator
//     here, and the one zero byte, so the zero-byte test flags exactly the quotes);
//     every other table byte 0xFF (the sign selectors 8-11 give 0xFF)
constexpr uint32_t CLS2_TN1 = 0x01FFFFFFu, CLS2_TN0 = 0xFFFFFFFFu, CLS2_TD1 = 0xFFFFFFFFu, CLS2_TD0 = 0xFF80FFFFu;
#endif
template <bool COMMA>
__device__ __forceinline__ void classify32(const v4u a, const v4u b, const CK& k, uint32_t& sep, uint32_t& nl,
                                           uint32_t& q) {
#ifndef FAST_OLD_CLS
    if (COMMA) {
        uint32_t us[4], un[4];
        uint32_t rdp = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t x = j < 4 ? a[j & 3] : b[j & 3];
            const uint32_t rn = __builtin_amdgcn_perm(k.tn1, k.tn0, x ^ 0x06060606u);
            const uint32_t rd = __builtin_amdgcn_perm(k.td1, k.td0, x ^ 0x2E2E2E2Eu);
#ifndef FAST_NO_Q3
            // q: the AND of the dwords' rd (a quote is the only byte with bit 7 clear),
            // two dwords per v_bitop3 (caller: q starts all ones, a quote clears a bit 7)
            if (j & 1) q = __builtin_amdgcn_bitop3_b32(q, rdp, rd, 0x80);
            else rdp = rd;
#elif defined(FAST_OLD_Q)
            q = __builtin_amdgcn_bitop3_b32(rd - 0x01010101u, rd, q, 0xBA);   // (t & ~rd) | q: quotes
#else
            q = __builtin_amdgcn_bitop3_b32(rd, q, k.m80, 0xCE);                // q | (~rd & 0x80): quotes (rd 0x00)
#endif
            const uint32_t fn = rn & k.m40;                                    // 1: not a terminator
            const uint32_t fs = __builtin_amdgcn_bitop3_b32(rn, rd, k.m40, 0x80);   // 1: not a separator
            const uint32_t w = (j & 1) ? k.w1 : k.w0;
            if (j & 1) {
                us[j >> 1] = __builtin_amdgcn_udot4(fs, w, us[j >> 1], false);
                un[j >> 1] = __builtin_amdgcn_udot4(fn, w, un[j >> 1], false);
            } else {
                us[j >> 1] = __builtin_amdgcn_udot4(fs, w, 0u, false);
                un[j >> 1] = __builtin_amdgcn_udot4(fn, w, 0u, false);
            }
        }
        nl = ~(un[0] | (un[1] << 8) | (un[2] << 16) | (un[3] << 24));
        sep = ~(us[0] | (us[1] << 8) | (us[2] << 16) | (us[3] << 24));
        return;
    }
#endif
    uint32_t ud[4], un[4];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t x = j < 4 ? a[j & 3] : b[j & 3];
        const uint32_t rn = __builtin_amdgcn_perm(k.tn1, k.tn0, x ^ 0x08080808u);
        uint32_t rd;
        if (COMMA) {
            // x ^ '*': ',' -> 6 (0x40); '"' -> 8 = sign of table byte 1 (0x20) -> 0x00; '&' -> 12 -> 0x00;
            // '+' -> 1 (0x20); the other selectors 0-7 -> 0x80, 9-11 -> signs of 0x80 bytes, >= 13 -> 0xFF
            rd = __builtin_amdgcn_perm(k.td1, k.td0, x ^ 0x2A2A2A2Au);
            q = __builtin_amdgcn_bitop3_b32(rd - 0x01010101u, rd, q, 0xBA);   // (t & ~rd) | q
        } else {
            rd = __builtin_amdgcn_perm(k.td1, k.td0, x ^ k.rd);
            const uint32_t t = x ^ k.rq;
            q = __builtin_amdgcn_bitop3_b32(t - 0x01010101u, t, q, 0xBA);
        }
        const uint32_t fd = flags40(rd, k.m40), fn = flags40(rn, k.m40);
        const uint32_t w = (j & 1) ? k.w1 : k.w0;
        if (j & 1) {
            ud[j >> 1] = __builtin_amdgcn_udot4(fd, w, ud[j >> 1], false);
            un[j >> 1] = __builtin_amdgcn_udot4(fn, w, un[j >> 1], false);
        } else {
            ud[j >> 1] = __builtin_amdgcn_udot4(fd, w, 0u, false);
            un[j >> 1] = __builtin_amdgcn_udot4(fn, w, 0u, false);
        }
    }
    nl = (un[0] >> 6) | (un[1] << 2) | (un[2] << 10) | (un[3] << 18);
    sep = nl | (ud[0] >> 6) | (ud[1] << 2) | (ud[2] << 10) | (ud[3] << 18);
}

// exact quote bits of 32 bytes (only for windows that hold a quote)
__device__ __forceinline__ uint32_t nib(uint32_t f) {
    uint32_t t = f >> 7;
    t |= t >> 7;
    t |= t >> 14;
    return t & 0xFu;
}
__device__ __forceinline__ uint32_t quote_bits(const v4u a, const v4u b, uint32_t rep) {
    uint32_t m = 0;
#pragma unroll
    for (int v = 0; v < 2; v++) {
#pragma unroll
        for (int j = 0; j < 4; j++) m |= nib(~nonzero_bytes((v ? b[j] : a[j]) ^ rep) & 0x80808080u) << ((v * 4 + j) * 4);
    }
    return m;
}

// 64 bits from bit b (< 64) of the 128 bits lo | hi << 64, given hi2 = hi << 1 and
// nb = 63 - b: two 64-bit shifts and an or (the view of both bit planes of a record
// shares nb)
__device__ __forceinline__ uint64_t view128(uint64_t lo, uint64_t hi2, uint32_t b, uint32_t nb) {
    return (lo >> b) | (hi2 << nb);
}
__device__ __forceinline__ uint64_t qview(const WaveLds& W, uint32_t p) {
    const uint32_t wi = p >> 5, sh = p & 31;
    const uint32_t q0 = W.qt[wi], q1 = W.qt[wi + 1], q2 = W.qt[wi + 2];
    return (uint64_t)__builtin_amdgcn_alignbit(q1, q0, sh) | ((uint64_t)__builtin_amdgcn_alignbit(q2, q1, sh) << 32);
}

// 4 / 8 bytes at LDS byte address a (any alignment; one ds_read2_b32 [+ ds_read_b32]):
// the record positions are absolute LDS addresses, so a field load adds no base
typedef const __attribute__((address_space(3))) uint32_t* lds_u32p;
__device__ __forceinline__ uint32_t ld4a(uint32_t a) {
    const lds_u32p t = (lds_u32p)(size_t)(a & ~3u);
    return __builtin_amdgcn_alignbyte(t[1], t[0], a);   // (v_alignbyte uses the low 2 bits)
}
__device__ __forceinline__ void ld8a(uint32_t a, uint32_t& d0, uint32_t& d1) {
    const lds_u32p t = (lds_u32p)(size_t)(a & ~3u);
    const uint32_t x0 = t[0], x1 = t[1], x2 = t[2];
    d0 = __builtin_amdgcn_alignbyte(x1, x0, a);
    d1 = __builtin_amdgcn_alignbyte(x2, x1, a);
}
// 4 / 8 bytes of the window at byte offset o (one ds_read2_b32 [+ ds_read_b32])
__device__ __forceinline__ uint32_t ld4(const uint8_t* w, uint32_t o) {
    const uint32_t* t = (const uint32_t*)w;
    const uint32_t a = o >> 2;
    return __builtin_amdgcn_alignbyte(t[a + 1], t[a], o & 3);
}
__device__ __forceinline__ void ld8(const uint8_t* w, uint32_t o, uint32_t& d0, uint32_t& d1) {
    const uint32_t* t = (const uint32_t*)w;
    const uint32_t a = o >> 2;
    const uint32_t x0 = t[a], x1 = t[a + 1], x2 = t[a + 2];
    d0 = __builtin_amdgcn_alignbyte(x1, x0, o & 3);
    d1 = __builtin_amdgcn_alignbyte(x2, x1, o & 3);
}

// A numeral of 1-4 bytes shaped [digits][.][digits] with at least one digit: M and
// k (digits after the dot), exactly parse_value's INTEGER M (no dot) or strtod's
// RN(M / 10^k) (csv_reader.c:133-240; never date-shaped: parse_date needs 8-10
// bytes).  d: the field's first 4 bytes, unmasked.  DOT: a dot is allowed.
struct Num {
    uint32_t M, k;
    bool ok, dot;
};
// SWAR constants of the record pass.  A VOP3 instruction cannot take a literal, so
// LLVM keeps them in SGPRs, and on gfx950 a VALU instruction reading an SGPR issues at
// half rate; fast_kernel holds them in VGPRs instead (vreg; FAST_NO_VK: literals)
struct NK {
    uint32_t k80, k7f, k1e, w4;
};
__device__ __forceinline__ NK nk_literals() { return NK{0x80808080u, 0x7F7F7F7Fu, 0x1E1E1E1Eu, 0x010A6400u}; }
__device__ __forceinline__ uint32_t nzb(uint32_t t, const NK& K) { return (((t & K.k7f) + K.k7f) | t) & K.k80; }
__device__ __forceinline__ uint32_t ltb(uint32_t x, uint32_t rep_n, const NK& K) { return ~((x | K.k80) - rep_n) & ~x & K.k80; }
template <bool DOT>
__device__ __forceinline__ Num num4(uint32_t d, uint32_t len, const NK& K = nk_literals()) {
    Num r;
    // (32 - 8 len) mod 32: LLVM folds it into 24 * len, a full-width v_mul_lo_u32
    uint32_t l8 = len << 3;
#ifndef FAST_OLD_SH
    asm volatile("" : "+v"(l8));
#endif
    const uint32_t sh = 32u - l8;
    uint32_t v = (d ^ 0x30303030u) << (sh & 31);
    r.dot = false;
    r.k = 0;
    if (DOT) {
        const uint32_t fd = ~nzb(v ^ K.k1e, K) & K.k80 & (0xFFFFFFFFu << (sh & 31));   // '.' ^ '0'
        const uint32_t low = fd & (0u - fd);
#ifdef FAST_OLD_NUMK
        const uint32_t below = ((low << 1) - (low != 0 ? 1u : 0u)) & 0x01010100u;
        v = __builtin_amdgcn_perm(0u, v, (low ? 0x0302010Cu : 0x03020100u) - below);
        r.dot = low != 0;
        r.k = r.dot ? (uint32_t)__builtin_clz(low) >> 3 : 0u;
#else
        // branch-free: t1 = the bytes up to the dot (all ones without a dot); the
        // digits after the dot are the sign bits above it; the bytes below the dot
        // move up one place (the dot's byte drops out, byte 0 becomes zero)
        const uint32_t t1 = (low << 1) - 1u;
        const uint32_t nzm = low ? 0xFFFFFFFFu : 0u;
        const uint32_t below = t1 & 0x01010100u & nzm;
        v = __builtin_amdgcn_perm(0u, v, 0x03020100u - below + (nzm & 12u));
        r.dot = low != 0;
        r.k = (uint32_t)__popc(~t1 & 0x80808080u);
#endif
    }
    const bool digits = ltb(v, 0x0A0A0A0Au, K) == K.k80;
    r.ok = (len - 1u <= 3u) & digits & (!DOT | (len > 1u) | !r.dot);
    r.M = __builtin_amdgcn_udot4(v, K.w4, __umul24(v & 0xFFu, 1000u), false);
    return r;
}
// 1-7 bytes (d0/d1: the field's first 8 bytes, unmasked)
__device__ __forceinline__ Num num7(uint32_t d0, uint32_t d1, uint32_t len) {
    Num r;
    const uint32_t f0 = len_mask(len, 0) & 0x80808080u, f1 = len_mask(len, 1) & 0x80808080u;
    const uint32_t x0 = d0 ^ 0x30303030u, x1 = d1 ^ 0x30303030u;
    const uint32_t g0 = lt_bytes(x0, 0x0A0A0A0Au) & f0, g1 = lt_bytes(x1, 0x0A0A0A0Au) & f1;
    const uint32_t t0 = ~nonzero_bytes(d0 ^ 0x2E2E2E2Eu) & f0, t1 = ~nonzero_bytes(d1 ^ 0x2E2E2E2Eu) & f1;
    const uint32_t ndot = (uint32_t)__popc(t0) + (uint32_t)__popc(t1);
    r.ok = (len - 1 <= 6u) & ((g0 | t0) == f0) & ((g1 | t1) == f1) & (ndot <= 1) & ((g0 | g1) != 0);
    uint64_t v = ((uint64_t)(x0 & spread(g0)) | ((uint64_t)(x1 & spread(g1)) << 32));
    const uint64_t tm = (uint64_t)t0 | ((uint64_t)t1 << 32);
    uint32_t pd = ctz64(tm) >> 3;
    pd = pd > 7 ? 7u : pd;
    r.dot = ndot != 0;
    const uint64_t lo = (1ULL << (8 * pd)) - 1;
    v = r.dot ? ((v & lo) | ((v >> 8) & ~lo)) : v;
    r.k = r.dot ? len - 1 - pd : 0u;
    r.k = r.k > 7 ? 7u : r.k;
    uint32_t nd2 = len - ndot;
    nd2 = nd2 - 1 > 7u ? 1u : nd2;
    v <<= 8 * (8 - nd2);
    const uint32_t vl = (uint32_t)v, vh = (uint32_t)(v >> 32);
    const uint32_t e1 = __builtin_amdgcn_udot4(vl, 0x00010A64u, 0u, false);
    const uint32_t e2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(vh, vl, 3), 0x00010A64u, 0u, false);
    const uint32_t e3 = __builtin_amdgcn_udot4(vh, 0x010A0000u, 0u, false);
    r.M = __umul24(__umul24(e1, 1000u) + e2, 100u) + e3;
    return r;
}

__device__ __forceinline__ bool tt_result(uint32_t tt, int c) { return (tt >> (c < 0 ? 0 : (c == 0 ? 1 : 2))) & 1; }
__device__ __forceinline__ double p10(uint32_t k) {
    return ((k & 1) ? 10.0 : 1.0) * ((k & 2) ? 100.0 : 1.0) * ((k & 4) ? 1e4 : 1.0);
}

// 0x80 in every byte < 0x21 (blank, control, NUL) among the f-flagged bytes
__device__ __forceinline__ uint32_t low_bytes(uint32_t d, uint32_t f) { return lt_bytes(d, 0x21212121u) & f; }
__device__ __forceinline__ uint32_t low_bytes(uint32_t d, uint32_t f, const NK& K) { return ltb(d, 0x21212121u, K) & f; }

}  // namespace fast

// the bucket hash of an 8-byte key tag (shared with the host's seed placement)
__host__ __device__ __forceinline__ uint32_t fast_key_hash(uint32_t k0, uint32_t k1) {
    uint32_t x = k0 ^ ((k1 << 11) | (k1 >> 21));
    x ^= x >> 16;
    x = ((x & 0xFFFFFFu) * 0x2F0B3Du) ^ (x >> 7);
    x ^= x >> 13;
    return ((x & 0xFFFFFFu) * 0x3C6EF3u) ^ (x >> 11);
}

namespace fast {

__device__ __forceinline__ GKey raw_key(uint32_t len, uint64_t w0) {
    GKey k;
    k.cls = GK_RAW; k.len = len; k.w0 = w0; k.w1 = 0;
    return k;
}
__device__ __forceinline__ uint32_t key_len8(uint64_t w0) {
    if (w0 == (1ull << 32)) return 0u;                 // the empty key's tag
    return w0 ? 8u - ((uint32_t)__builtin_clzll(w0) >> 3) : 0u;
}

// a record whose key found no LDS slot: straight into the HBM raw table
// (acc1: bit a set when accumulator a sums SUM argument 1, else argument 0)
#ifdef FAST_SPILL_INL
#define FAST_SPILL_ATTR __forceinline__
#else
#define FAST_SPILL_ATTR __noinline__
#endif
__device__ FAST_SPILL_ATTR void spill8(uint64_t tag, uint64_t off, const GroupTable* tabs, ScanStats* stats, int nacc,
                                    uint32_t acc1, bool n0, double v0, bool n1, double v1) {
    const GroupTable& rt = tabs[TAB_RT];
    const uint32_t kl = key_len8(tag);
    const GKey kk = raw_key(kl, kl ? tag : 0ull);
    const int gi = g_insert(rt, kk, gk_hash(kk), stats);
    if (gi < 0) return;
    atomicAdd(&rt.cnt[gi], 1ULL);
    atomicMin(&rt.first[gi], (unsigned long long)off);
    for (int a = 0; a < nacc; a++) {
        const bool s1 = (acc1 >> a) & 1;
        const bool nm = s1 ? n1 : n0;
        if (nm) {
            atomicAdd(&rt.sum[a][gi], s1 ? v1 : v0);
            atomicAdd(&rt.num[a][gi], 1ULL);
        }
    }
}

__device__ __forceinline__ uint8_t* carve(uint8_t*& q, size_t bytes) {
    uint8_t* r = q;
    q += (bytes + 15) & ~(size_t)15;
    return r;
}

// A slot's accumulators, one 32-byte record (one address for all of a record's LDS
// atomics): COUNT, first-row code, per SUM argument the fixed-point sum (10^-3) and the
// non-numeric count; with one SUM argument a double sum for the addends outside the
// fixed-point path (two SUM arguments: such addends take the HBM table)
constexpr uint32_t SLOT_BYTES = 32;
enum SlotOff : uint32_t { SO_CNT = 0, SO_FIRST = 4, SO_FIX0 = 8, SO_FIX1 = 16, SO_DBL = 16, SO_MISS0 = 24, SO_MISS1 = 28,
                         SO_EXT = 16 };   // (EXT builds: one SUM argument, no double addends -- the word is free)

// MIN / MAX of narrow numerals in one 64-bit LDS atomic: the value as exact 10^-3
// fixed point (< 10^7 for the <= 4-byte numerals of the fast path) above the
// record's 32-bit first-row code, so one atomicMin takes the smallest value and,
// among equal values, the first record (evaluate_aggregate keeps the first cell
// that compares strictly better, evaluator_aggregates.c:311-326); MAX stores the
// code complemented under atomicMax.  Initial word: no candidate.
template <int EXT>
__device__ __forceinline__ unsigned long long ext_key(uint64_t fix, uint32_t code) {
    return (fix << 32) | (EXT == 1 ? code : ~code);
}
template <int EXT>
__device__ __forceinline__ unsigned long long ext_none() { return EXT == 1 ? ~0ull : 0ull; }
// The block flushes carry each extreme as one 64-bit key, merged by a global
// atomicMin (no lock): the fixed-point value (< 2^24: <= 4-byte numerals, scale 10^3;
// MAX as 2^24 - 1 - value) above the record's byte offset (< 2^40), so the smallest
// key is the extreme and, among equal values, its first record.  raw_merge_kernel
// (grouped) / fast_ext_final_kernel (one group) types the winning field once.
constexpr uint32_t EXT_POS_BITS = 40;
constexpr uint64_t EXT_FIX_MAX = (1ull << 24) - 1;
template <int EXT>
__device__ __forceinline__ unsigned long long ext_packed(uint64_t fix, uint64_t pos) {
    return ((EXT == 1 ? fix : EXT_FIX_MAX - fix) << EXT_POS_BITS) | pos;
}
template <int NS>
constexpr uint32_t table_bytes(bool grouped) {
    // the tags, and a 32-byte slot record (see SlotOff) per slot
    return grouped ? TSLOTS * (8u + SLOT_BYTES) : 0u;
}
constexpr uint32_t fixed_bytes() { return (uint32_t)(sizeof(WaveLds) * NWV); }

// GROUPED: GROUP BY one column (else one group); WHERE: `col op numeric literal`
// (else none); NS: distinct SUM arguments; COMMA: delimiter ',' and quote '"';
// CANON: the roles' columns ascend in the order WHERE, SUM 0, SUM 1, GROUP BY (the
// walk's ranks are compile-time), else rank[] says which field each role reads
// WN: numerals of 5-7 bytes / over 3 decimals are typed here (a side path); without
// it (the plan's sampled WHERE / SUM fields are all <= 4 bytes) such a record goes
// whole to slow_kernel, and the kernel keeps only the fixed-point SUM
// WX: a compound WHERE over WX (1 or 2) columns (FastPlan wx_*, lx_*)
template <bool GROUPED, bool WHERE, int NS, bool COMMA, bool CANON, int RP, bool WN, int EXT = 0, bool WSTR = false,
          int WX = 0>
__global__ __launch_bounds__(LT) void fast_kernel(const uint8_t* __restrict__ g, ScanStats* __restrict__ stats,
                                                  unsigned long long* __restrict__ slow_list,
                                                  unsigned long long slow_cap, const FastPlan fp,
                                                  const GroupTable* __restrict__ tabs) {
    static_assert(EXT == 0 || (NS == 1 && !WN), "MIN / MAX: one fixed-point argument, no double addends");
    static_assert(!WSTR || (WHERE && !WN && EXT == 0), "STRING-literal WHERE: the narrow-numeral builds");
    static_assert(WX == 0 || (WHERE && !WN && EXT == 0 && !WSTR && COMMA && RP == 2), "compound WHERE builds");
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t* q = smem;
    // LDS table: slot records first (LDS address 0: field offsets fold into the
    // atomics), then the tags (bucket b = slots 2b, 2b + 1), then the wave windows
    uint8_t* S = nullptr;
    unsigned long long* T = nullptr;
    if (GROUPED) {
        S = carve(q, TSLOTS * SLOT_BYTES);
        T = (unsigned long long*)carve(q, TSLOTS * 8);
    }
    WaveLds* waves = (WaveLds*)carve(q, sizeof(WaveLds) * NWV);
    // WX builds: the leaves' parameters in LDS, read once per record pass -- as kernel
    // arguments the compiler keeps them in scalar registers across the loop and spills
    // (v_writelane / v_readlane) the loop's own state
    uint32_t* lxl = nullptr;
    if constexpr (WX != 0) {
        lxl = (uint32_t*)carve(q, 4 * LX_WORDS * 4);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int l = 0; l < 4; l++) {
                uint32_t* L = lxl + l * LX_WORDS;
                L[0] = fp.lx_kind[l] | (fp.lx_col[l] << 2) | (fp.lx_neg[l] << 3) | (fp.lx_null[l] << 4) |
                       (fp.lx_tt[l] << 5) | (fp.lx_nin[l] << 8);
                L[1] = fp.lx_a[l];
                L[2] = fp.lx_w[l];
                L[3] = 0;
                L[4] = (uint32_t)fp.lx_lit[l];
                L[5] = (uint32_t)(fp.lx_lit[l] >> 32);
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    L[6 + 2 * t] = (uint32_t)fp.lx_in[l][t];
                    L[7 + 2 * t] = (uint32_t)(fp.lx_in[l][t] >> 32);
                }
            }
        }
        __syncthreads();
    }
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    WaveLds& W = waves[wv];
    if (GROUPED) {
        const unsigned long long* seed = fp.seed;
        for (uint32_t i = tid; i < TSLOTS; i += LT) {
            T[i] = seed ? seed[i] : 0ull;
            uint32_t* r = (uint32_t*)(S + i * SLOT_BYTES);
#pragma unroll
            for (int w = 0; w < 8; w++) r[w] = 0u;
            r[SO_FIRST / 4] = NOFIRST;
            if (EXT) *(unsigned long long*)(r + SO_EXT / 4) = ext_none<EXT>();
        }
        __syncthreads();
    }

    // roles, in column order (CANON: WHERE, WHERE column 1, SUM 0, SUM 1, GROUP BY)
    constexpr int NR = (WHERE ? 1 : 0) + (WX == 2 ? 1 : 0) + NS + (GROUPED ? 1 : 0);
    constexpr int KW = 0, KW1 = 1, KS0 = (WHERE ? 1 : 0) + (WX == 2 ? 1 : 0), KG = NR - 1;
    uint32_t skip[5], rk[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        skip[k] = __builtin_amdgcn_readfirstlane(fp.skip[k]);
        rk[k] = __builtin_amdgcn_readfirstlane(fp.rank[k]);
    }
    const uint32_t rep_q = fp.quote * 0x01010101u;
    CK ck;
#ifndef FAST_OLD_CLS
    ck.tn1 = vreg(COMMA ? CLS2_TN1 : 0x00004000u);
    ck.tn0 = vreg(COMMA ? CLS2_TN0 : 0x00400000u);
    ck.td1 = vreg(COMMA ? CLS2_TD1 : 0u);
    ck.td0 = vreg(COMMA ? CLS2_TD0 : 0x40u);
    ck.m40 = vreg(COMMA ? 0x01010101u : 0x40404040u);   // (COMMA: the bit-0 mask)
    ck.m80 = vreg(0x80808080u);
#else
    ck.tn1 = vreg(0x00004000u);
    ck.tn0 = vreg(0x00400000u);
    ck.td1 = vreg(COMMA ? 0x80408080u : 0u);
    ck.td0 = vreg(COMMA ? 0x80802080u : 0x40u);
    ck.m40 = vreg(0x40404040u);
#endif
    ck.w0 = vreg(0x08040201u);
    ck.w1 = vreg(0x80402010u);
#ifndef FAST_NO_VK
    const NK nk{vreg(0x80808080u), vreg(0x7F7F7F7Fu), vreg(0x1E1E1E1Eu), vreg(0x010A6400u)};
#else
    const NK nk = nk_literals();
#endif
    ck.rd = vreg(fp.delim * 0x01010101u);
    ck.rq = vreg(rep_q);
    const uint64_t first_win = fp.first_win;    // (scalar: the window loads' base)
#ifndef FAST_SR
#ifdef FAST_VPTR   // experiment (round 4): 17 -> 10 SGPR spills, +8 VGPRs, ~1 % slower in a same-box A/B
    if constexpr (!WN) {     // (the wide-numeral builds need those VGPRs themselves)
        stats = vptr(stats);
        slow_list = vptr(slow_list);
        slow_cap = vreg64(slow_cap);
        tabs = vptr(tabs);
    }
#endif
#endif
    const uint32_t nwin = __builtin_amdgcn_readfirstlane(fp.nwin);
    const uint32_t wsb = __builtin_amdgcn_readfirstlane(fp.ws);
#ifndef FAST_SR
    // uniform plan values of the cold paths (and the WHERE's NULL / negation bits)
    // held in VGPRs: the loop's scalar registers stay for its own state
    const bool pass_null = vreg(fp.pass_null) != 0;
    const int wlo = (int)vreg((uint32_t)fp.wlo), whi = (int)vreg((uint32_t)fp.whi);
    const uint32_t wtt = vreg(fp.wtt);
    const uint32_t wa = vreg(fp.wa), ww = vreg(fp.ww);
    const bool wneg = vreg(fp.wneg) != 0;
    const double wl = fp.wl;
    const int nacc = (int)vreg((uint32_t)fp.nacc);
    const uint32_t acc1 = vreg(fp.acc1);
#else
    const bool pass_null = __builtin_amdgcn_readfirstlane(fp.pass_null) != 0;
    const int wlo = __builtin_amdgcn_readfirstlane(fp.wlo), whi = __builtin_amdgcn_readfirstlane(fp.whi);
    const uint32_t wtt = __builtin_amdgcn_readfirstlane(fp.wtt);
    const uint32_t wa = vreg(fp.wa), ww = vreg(fp.ww);
    const bool wneg = __builtin_amdgcn_readfirstlane(fp.wneg) != 0;
    const double wl = fp.wl;
    const int nacc = __builtin_amdgcn_readfirstlane(fp.nacc);
    const uint32_t acc1 = __builtin_amdgcn_readfirstlane(fp.acc1);
#endif
    const uint32_t wstep = gridDim.x * NWV;
    // interior windows own the records starting in their first ws bytes: the lanes below ws / 64
    const uint32_t lane_full = (uint32_t)lane * LB < wsb ? ~0u : 0u;

    uint32_t my_cnt = 0;                       // ungrouped partials (per lane)
    uint32_t my_first = NOFIRST;               // first-row code (round, wave, window offset)
    unsigned long long my_fix[MAXS] = {0ull, 0ull};
    double my_dbl[MAXS] = {0.0, 0.0};
    uint32_t my_num[MAXS] = {0u, 0u};
    uint32_t n_rec = 0, n_pass = 0, n_spill = 0;   // wave totals (uniform)
    unsigned long long my_ext = ext_none<EXT>();   // ungrouped EXT builds: the lane's extreme key
    bool saw_num = false;                          // EXT: a numeric candidate (the class bit)

    uint32_t prev_next = 0;
    const uint32_t voff = vreg(16u * (uint32_t)lane);
    const uint32_t wlds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)W.bytes);
    // window i (0 .. nwin - 1) of the range: file window first_win + i
    const uint32_t lane_lds = vreg(wlds + (uint32_t)lane * LB);   // the LDS address of the lane's bytes
    uint32_t i = blockIdx.x * NWV + wv;
#ifdef FAST_PF_PLAIN
#define FAST_PFLOAD(p) (*(p))
#else
#define FAST_PFLOAD(p) __builtin_nontemporal_load(p)
#endif
#ifdef FAST_REGPF
    // register prefetch: lane l's 64 bytes of the NEXT window are loaded into VGPRs
    // while this window is processed (a whole window of work hides the load), then
    // stored to the wave's LDS bytes for the record pass
    v4u nx[4];
    const v4u* gl = (const v4u*)(g + (size_t)lane * LB);
    if (i < nwin) {
        const v4u* a = (const v4u*)((const uint8_t*)gl + (first_win + i) * wsb);
#pragma unroll
        for (int k = 0; k < 4; k++) nx[k] = FAST_PFLOAD(a + k);
        prev_next = *(const uint32_t*)(g + (first_win + i) * wsb - 4);
    }
#else
    if (i < nwin) load_win(g, first_win + i, wsb, wlds, voff, prev_next);
#endif
    for (uint32_t round = 0; i < nwin; round++, i += wstep) {
        const uint32_t fcw = (round << 16) | ((uint32_t)wv << 12);   // first-row code of this window
#ifdef FAST_REGPF
        v4u la[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            la[k] = nx[k];
            ((v4u*)W.bytes)[4 * lane + k] = la[k];
        }
        const uint32_t prevw = prev_next;
        if (i + wstep < nwin) {
            const v4u* a = (const v4u*)((const uint8_t*)gl + (first_win + i + wstep) * wsb);
#pragma unroll
            for (int k = 0; k < 4; k++) nx[k] = FAST_PFLOAD(a + k);
            prev_next = *(const uint32_t*)(g + (first_win + i + wstep) * wsb - 4);
        }
#define FAST_ISSUE() do {} while (0)
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the window's bytes are in LDS
        const uint32_t prevw = prev_next;
        bool issued = false;
#define FAST_ISSUE()                                                               \
    do {                                                                           \
        if (!issued && i + wstep < nwin) {                                          \
            uint32_t ni = i + wstep;                                               \
            asm volatile("" : "+s"(ni)); /* the address is formed here, not hoisted */ \
            load_win(g, first_win + ni, wsb, wlds, voff, prev_next);               \
        }                                                                          \
        issued = true;                                                             \
    } while (0)

        // ---- classify lane l's 64 bytes
        v4u la[4];
#pragma unroll
        for (int i = 0; i < 4; i++) la[i] = ((const v4u*)W.bytes)[4 * lane + i];
#endif
#ifndef FAST_NO_Q3
        uint32_t sep0, nl0, sep1, nl1, qf = COMMA ? 0xFFFFFFFFu : 0u;
#else
        uint32_t sep0, nl0, sep1, nl1, qf = 0;
#endif
        classify32<COMMA>(la[0], la[1], ck, sep0, nl0, qf);
        classify32<COMMA>(la[2], la[3], ck, sep1, nl1, qf);
#ifndef FAST_NO_Q3
        const bool wq = __ballot(((COMMA ? ~qf : qf) & 0x80808080u) != 0) != 0;   // window may hold a quote (uniform)
#else
        const bool wq = __ballot((qf & 0x80808080u) != 0) != 0;   // window may hold a quote (uniform)
#endif
        if (wq) {
            W.qt[2 * lane] = quote_bits(la[0], la[1], rep_q);
            W.qt[2 * lane + 1] = quote_bits(la[2], la[3], rep_q);
        }

        // ---- record starts owned by this window
        const uint64_t nl = (uint64_t)nl0 | ((uint64_t)nl1 << 32);
        const uint32_t prev_top = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(nl1 >> 31), 0x138, 0xf, 0xf, true);
        const uint32_t pb = prevw >> 24;
        const uint32_t prevnl = lane == 0 ? (uint32_t)(pb == '\n' || pb == '\r') : prev_top;
        uint64_t todo = ~nl & ((nl << 1) | prevnl);
        if (i == 0 || i == nwin - 1) {                      // the range's first / last window: clip
            const uint32_t lo_s = i == 0 ? fp.lo_s : 0u, hi_s = i == nwin - 1 ? fp.hi_s : wsb;
            const uint32_t b0 = (uint32_t)lane * LB;
            const uint32_t a = lo_s > b0 ? lo_s - b0 : 0u, e = hi_s > b0 ? hi_s - b0 : 0u;
            const uint64_t keep_lo = a >= 64 ? 0ull : (~0ull << a);
            const uint64_t keep_hi = e >= 64 ? ~0ull : ((1ull << e) - 1);
            todo &= keep_lo & keep_hi;
        } else {
            todo &= ((uint64_t)lane_full << 32) | lane_full;
        }
        const uint32_t xs0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sep0, 0x130, 0xf, 0xf, true);
        const uint32_t xs1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sep1, 0x130, 0xf, 0xf, true);
        const uint32_t xn0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nl0, 0x130, 0xf, 0xf, true);
        const uint32_t xn1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nl1, 0x130, 0xf, 0xf, true);
        const uint64_t sep64 = (uint64_t)sep0 | ((uint64_t)sep1 << 32);
        const uint64_t xsep2 = ((uint64_t)xs0 | ((uint64_t)xs1 << 32)) << 1;   // the next lane's bits, << 1
        const uint64_t xnl2 = ((uint64_t)xn0 | ((uint64_t)xn1 << 32)) << 1;

#if defined(FAST_PROF) && FAST_PROF == 1      // profiling build: load + classify + record starts only
        n_rec += (uint32_t)__popcll(__ballot(((uint32_t)__popcll(todo) + ((xs0 ^ xs1 ^ xn0 ^ xn1) & 1)) & 1));
        FAST_ISSUE();
        continue;
#endif
        while (__any(todo != 0)) {
            // ---- two records of this lane
            uint32_t p[RP], pa[RP], fst[RP][5], fen[RP][5], e[RP];   // p: window offset, pa: LDS address
            uint64_t sv[RP];
            bool valid[RP], fail[RP];
#pragma unroll
            for (int u = 0; u < RP; u++) {
                valid[u] = todo != 0;
                const uint32_t b = ctz64(todo) & 63u;               // (no start left: any byte of the lane)
                todo &= todo - 1;
                pa[u] = lane_lds + b;
                p[u] = pa[u] - wlds;
                const uint32_t nb = b ^ 63u;
                sv[u] = view128(sep64, xsep2, b, nb);
                e[u] = ctz64(view128(nl, xnl2, b, nb));            // record end (>= 64: past the view)
            }
            // the roles' fields in column order, both records at once: clearing separator
            // bits visits field ends in order (skip 0 after the first role: the same
            // column again).  ctz64 of an exhausted view is >= 64, and so is every later end.
#pragma unroll
            for (int k = 0; k < NR; k++) {
                uint32_t n = skip[k];
                asm volatile("" : "+s"(n));                         // tested here, not hoisted as lane masks
                if (k > 0 && n == 0) {
#pragma unroll
                    for (int u = 0; u < RP; u++) { fst[u][k] = fst[u][k - 1]; fen[u][k] = fen[u][k - 1]; }
                    continue;
                }
                if (k > 0) {
#pragma unroll
                    for (int u = 0; u < RP; u++) sv[u] &= sv[u] - 1;  // the previous field's end
                }
                if (k == 0 && n == 0) {
#pragma unroll
                    for (int u = 0; u < RP; u++) fst[u][k] = 0;
                } else if (k > 0 && n == 1) {
#pragma unroll
                    for (int u = 0; u < RP; u++) fst[u][k] = fen[u][k - 1] + 1;
                } else {
                    for (uint32_t i = k == 0 ? 1u : 2u; i < n; i++) {
#pragma unroll
                        for (int u = 0; u < RP; u++) sv[u] &= sv[u] - 1;
                    }
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        fst[u][k] = ctz64(sv[u]) + 1;
                        sv[u] &= sv[u] - 1;
                    }
                }
#pragma unroll
                for (int u = 0; u < RP; u++) fen[u][k] = ctz64(sv[u]);
            }
#pragma unroll
            for (int u = 0; u < RP; u++) {
                // the last role's field must end inside the view and at or before the
                // record's terminator (else the row is short or longer than the view);
                // with no role at all (COUNT(*), no WHERE) every record counts as it is
                // (record splitting is quote-blind, csv_reader.c:404-408)
                if constexpr (NR == 0) {
                    fail[u] = !valid[u];
                } else {
                    const uint32_t en = fen[u][NR - 1];
                    fail[u] = !valid[u] | (en >= 64u) | (en > e[u]);
                }
            }
            const bool last_pass = !__any(todo != 0);
            if (NR > 0 && wq) {                                      // a quote in front of a needed field
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    const uint32_t lr = fen[u][NR > 0 ? NR - 1 : 0];
                    const uint32_t lp = lr < 63 ? lr : 63u;
                    fail[u] |= (qview(W, p[u]) & ((2ULL << lp) - 1)) != 0;
                }
            }

            // ---- each role's field: compile-time ranks (CANON) or the plan's (uniform selects)
            uint32_t wst[RP] = {}, wen[RP] = {}, gst[RP] = {}, gen[RP] = {}, xst[RP] = {}, xen[RP] = {};
            uint32_t sst[RP][MAXS] = {}, sen[RP][MAXS] = {};
#pragma unroll
            for (int u = 0; u < RP; u++) {
                auto pick = [&](uint32_t r, uint32_t& a, uint32_t& b) {
                    a = fst[u][0];
                    b = fen[u][0];
#pragma unroll
                    for (int k = 1; k < NR; k++) {
                        a = r == (uint32_t)k ? fst[u][k] : a;
                        b = r == (uint32_t)k ? fen[u][k] : b;
                    }
                };
                if (CANON) {
                    if (WHERE) { wst[u] = fst[u][KW]; wen[u] = fen[u][KW]; }
                    if (WX == 2) { xst[u] = fst[u][KW1]; xen[u] = fen[u][KW1]; }
#pragma unroll
                    for (int j = 0; j < NS; j++) { sst[u][j] = fst[u][KS0 + j]; sen[u][j] = fen[u][KS0 + j]; }
                    if (GROUPED) { gst[u] = fst[u][KG]; gen[u] = fen[u][KG]; }
                } else {
                    if (WHERE) pick(rk[0], wst[u], wen[u]);
                    if (WX == 2) pick(rk[4], xst[u], xen[u]);
#pragma unroll
                    for (int j = 0; j < NS; j++) pick(rk[1 + j], sst[u][j], sen[u][j]);
                    if (GROUPED) pick(rk[3], gst[u], gen[u]);
                }
            }

#if defined(FAST_PROF) && FAST_PROF == 2      // + record views and the field walk
            n_rec += (uint32_t)__popcll(__ballot((wst[0] ^ sst[1][0] ^ gen[0] ^ gst[1] ^ (uint32_t)fail[0] ^ (uint32_t)fail[1]) & 1));
            if (last_pass) FAST_ISSUE();
            continue;
#endif
            // ---- field bytes (one batch of LDS reads)
            uint32_t wd[RP], wd1[RP], sd[RP][MAXS], k0[RP], k1[RP], xd[RP], xd1[RP];
#pragma unroll
            for (int u = 0; u < RP; u++) {
                if (WX == 2) ld8a(pa[u] + xst[u], xd[u], xd1[u]);
                if (WSTR || WX) ld8a(pa[u] + wst[u], wd[u], wd1[u]);
                else if (WHERE) wd[u] = ld4a(pa[u] + wst[u]);
#pragma unroll
                for (int j = 0; j < NS; j++) sd[u][j] = ld4a(pa[u] + sst[u][j]);
                if (GROUPED) ld8a(pa[u] + gst[u], k0[u], k1[u]);
            }

            // ---- WHERE outcome (wu: a field the 4-byte numeral path could not type)
            bool pass[RP];
            bool wu[RP];
#pragma unroll
            for (int u = 0; u < RP; u++) { pass[u] = true; wu[u] = false; }
            if constexpr (WX != 0) {
                // per WHERE column its typed value (uniform class), then every leaf, then
                // the tree's truth table (a field this path cannot type: wu, slow_kernel)
                const uint32_t tt16 = fp.wx_tt, nleaf = fp.wx_nleaf;
                if constexpr (WX == 1) {
                    // one WHERE column (BETWEEN, IN, OR / AND over one column): leaf-major
                    bool cnull[RP][2];
                    uint32_t cv[RP][2];
                    uint64_t cx[RP][2];
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        bool cok[2];
#pragma unroll
                        for (int c = 0; c < WX; c++) {
                            const uint32_t len = c ? xen[u] - xst[u] : wen[u] - wst[u];
                            const uint32_t a0r = c ? xd[u] : wd[u], a1r = c ? xd1[u] : wd1[u];
                            cnull[u][c] = len == 0;
                            cv[u][c] = 0;
                            cx[u][c] = 0;
                            if ((fp.wx_str >> c) & 1) {
                                const uint32_t m0 = len_mask(len, 0), m1 = len_mask(len, 1);
                                const uint32_t a0 = a0r & m0, a1 = a1r & m1;
                                const uint32_t c0 = a0 & 0xFFu;
                                cok[c] = (int)(len - 1u < 8u) & (int)!(is_digit(c0) | (c0 == '-') | (c0 == '+') | (c0 == '.')) &
                                         (int)((low_bytes(a0, m0 & nk.k80, nk) | low_bytes(a1, m1 & nk.k80, nk)) == 0);
                                cx[u][c] = ((uint64_t)__builtin_bswap32(a0) << 32) | __builtin_bswap32(a1);
                            } else {
                                const Num n = num4<true>(a0r, len, nk);
                                const uint32_t mul = (uint32_t)(0x0001000A006403E8ull >> (n.k << 4)) & 0xFFFFu;
                                cv[u][c] = __umul24(n.M, mul);
                                cok[c] = n.ok;
                            }
                            wu[u] |= !cok[c] & !cnull[u][c] & !fail[u];
                        }
                }
                    // leaf by leaf, both records at once: a leaf's parameters (and an IN
                    // list's items) are read from LDS once per pass, not once per record
                    uint32_t idx[RP];
#pragma unroll
                    for (int u = 0; u < RP; u++) idx[u] = 0;
#pragma unroll
                    for (int l = 0; l < 4; l++) {
                        if ((uint32_t)l < nleaf) {
                            const uint32_t* L = lxl + l * LX_WORDS;
                            const uint32_t meta = __builtin_amdgcn_readfirstlane(L[0]);
                            const uint32_t c = WX == 2 ? (meta >> 2) & 1u : 0u;
                            const uint32_t kind = meta & 3u;
                            const bool neg = (meta >> 3) & 1u, nulv = (meta >> 4) & 1u;
                            bool b[RP];
                            if (kind == LX_NUM) {
                                const uint32_t la = L[1], lw = L[2];
#pragma unroll
                                for (int u = 0; u < RP; u++) b[u] = ((c ? cv[u][WX - 1] : cv[u][0]) - la <= lw) != neg;
                            } else if (kind == LX_STR) {
                                const uint64_t lit = (uint64_t)L[4] | ((uint64_t)L[5] << 32);
                                const uint32_t tt = (meta >> 5) & 7u;
#pragma unroll
                                for (int u = 0; u < RP; u++) {
                                    const uint64_t X = c ? cx[u][WX - 1] : cx[u][0];
                                    b[u] = tt_result(tt, X < lit ? -1 : (X > lit ? 1 : 0));
                                }
                            } else {
                                bool hit[RP];
#pragma unroll
                                for (int u = 0; u < RP; u++) hit[u] = false;
                                const uint32_t nin = (meta >> 8) & 15u;
                                for (uint32_t t = 0; t < nin; t++) {
                                    const uint64_t v = (uint64_t)L[6 + 2 * t] | ((uint64_t)L[7 + 2 * t] << 32);
#pragma unroll
                                    for (int u = 0; u < RP; u++)
                                        hit[u] |= kind == LX_NIN ? (c ? cv[u][WX - 1] : cv[u][0]) == (uint32_t)v
                                                                 : (c ? cx[u][WX - 1] : cx[u][0]) == v;
                                }
#pragma unroll
                                for (int u = 0; u < RP; u++) b[u] = hit[u] != neg;
                            }
#pragma unroll
                            for (int u = 0; u < RP; u++) {
                                const bool nul = c ? cnull[u][WX - 1] : cnull[u][0];
                                idx[u] |= ((nul ? nulv : b[u]) ? 1u : 0u) << l;
                            }
                        }
                }
#pragma unroll
                    for (int u = 0; u < RP; u++) pass[u] = (tt16 >> idx[u]) & 1u;
                } else {
                    // two WHERE columns: record-major (the leaf-major form's live [RP][2] typed
                    // values pushed this build into scratch: 64 bytes / lane, 3 % slower)
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        bool cnull[2], cok[2];
                        uint32_t cv[2];
                        uint64_t cx[2];
#pragma unroll
                        for (int c = 0; c < WX; c++) {
                            const uint32_t len = c ? xen[u] - xst[u] : wen[u] - wst[u];
                            const uint32_t a0r = c ? xd[u] : wd[u], a1r = c ? xd1[u] : wd1[u];
                            cnull[c] = len == 0;
                            cv[c] = 0;
                            cx[c] = 0;
                            if ((fp.wx_str >> c) & 1) {
                                const uint32_t m0 = len_mask(len, 0), m1 = len_mask(len, 1);
                                const uint32_t a0 = a0r & m0, a1 = a1r & m1;
                                const uint32_t c0 = a0 & 0xFFu;
                                cok[c] = (int)(len - 1u < 8u) & (int)!(is_digit(c0) | (c0 == '-') | (c0 == '+') | (c0 == '.')) &
                                         (int)((low_bytes(a0, m0 & nk.k80, nk) | low_bytes(a1, m1 & nk.k80, nk)) == 0);
                                cx[c] = ((uint64_t)__builtin_bswap32(a0) << 32) | __builtin_bswap32(a1);
                            } else {
                                const Num n = num4<true>(a0r, len, nk);
                                const uint32_t mul = (uint32_t)(0x0001000A006403E8ull >> (n.k << 4)) & 0xFFFFu;
                                cv[c] = __umul24(n.M, mul);
                                cok[c] = n.ok;
                            }
                            wu[u] |= !cok[c] & !cnull[c] & !fail[u];
                        }
                        uint32_t idx = 0;
#pragma unroll
                        for (int l = 0; l < 4; l++) {
                            if ((uint32_t)l < nleaf) {
                                const uint32_t* L = lxl + l * LX_WORDS;
                                const uint32_t meta = __builtin_amdgcn_readfirstlane(L[0]);
                                const uint32_t c = WX == 2 ? (meta >> 2) & 1u : 0u;
                                const uint32_t V = c ? cv[WX - 1] : cv[0];
                                const uint64_t X = c ? cx[WX - 1] : cx[0];
                                const bool nul = c ? cnull[WX - 1] : cnull[0];
                                const uint32_t kind = meta & 3u;
                                const bool neg = (meta >> 3) & 1u;
                                bool b;
                                if (kind == LX_NUM) {
                                    b = (V - L[1] <= L[2]) != neg;
                                } else if (kind == LX_STR) {
                                    const uint64_t lit = (uint64_t)L[4] | ((uint64_t)L[5] << 32);
                                    b = tt_result((meta >> 5) & 7u, X < lit ? -1 : (X > lit ? 1 : 0));
                                } else {
                                    bool hit = false;
                                    const uint32_t nin = (meta >> 8) & 15u;
                                    for (uint32_t t = 0; t < nin; t++) {
                                        const uint64_t v = (uint64_t)L[6 + 2 * t] | ((uint64_t)L[7 + 2 * t] << 32);
                                        hit |= kind == LX_NIN ? V == (uint32_t)v : X == v;
                                    }
                                    b = hit != neg;
                                }
                                b = nul ? ((meta >> 4) & 1u) != 0 : b;
                                idx |= (b ? 1u : 0u) << l;
                            }
                        }
                        pass[u] = (tt16 >> idx) & 1u;
                }
                }
            } else if (WSTR) {
                // a STRING field of 1-8 bytes: no leading digit / sign / dot (never a
                // numeral or a date, infer_type csv_reader.c:133-240), no byte <= ' '
                // (trim_whitespace is a no-op); then strcmp against the literal is the
                // order of the zero-padded big-endian words.  Any other non-empty field
                // goes whole to slow_kernel (wu).
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    const uint32_t len = wen[u] - wst[u];
                    const uint32_t m0 = len_mask(len, 0), m1 = len_mask(len, 1);
                    const uint32_t a0 = wd[u] & m0, a1 = wd1[u] & m1;
                    const uint32_t c0 = a0 & 0xFFu;
                    const bool ok = (int)(len - 1u < 8u) &
                                    (int)!(is_digit(c0) | (c0 == '-') | (c0 == '+') | (c0 == '.')) &
                                    (int)((low_bytes(a0, m0 & nk.k80, nk) | low_bytes(a1, m1 & nk.k80, nk)) == 0);
                    const uint64_t x = ((uint64_t)__builtin_bswap32(a0) << 32) | __builtin_bswap32(a1);
                    const uint64_t ws = fp.wstr;
                    pass[u] = len == 0 ? pass_null : tt_result(wtt, x < ws ? -1 : (x > ws ? 1 : 0));
                    wu[u] = !ok & (len != 0) & !fail[u];
                }
            } else if (WHERE) {
                bool wide = false;
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    const uint32_t len = wen[u] - wst[u];
                    const Num n = num4<false>(wd[u], len, nk);
                    pass[u] = len == 0 ? pass_null : ((n.M - wa <= ww) != wneg);
                    wu[u] = !n.ok & (len != 0) & !fail[u];
                    wide |= wu[u];
                }
                if (WN && __any(wide)) {                             // DOUBLE or 5-7 byte numerals
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        if (wu[u]) {
                            const uint32_t len = wen[u] - wst[u];
                            uint32_t d0, d1;
                            ld8a(pa[u] + wst[u], d0, d1);
                            const Num n = num7(d0, d1, len);
                            if (n.ok) {
                                int c;
                                if (n.dot) {
                                    const double v = (double)n.M / p10(n.k);   // strtod: exact operands, one rounding
                                    c = v < wl ? -1 : (v > wl ? 1 : 0);
                                } else {
                                    c = (int)n.M < wlo ? -1 : ((int)n.M > whi ? 1 : 0);
                                }
                                pass[u] = tt_result(wtt, c);
                                wu[u] = false;
                            }
                        }
                    }
                }
            }

#if defined(FAST_EXP_NOB)      // experiment: the record pass up to the WHERE outcome only
            {
                uint32_t x = 0;
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    x ^= (uint32_t)pass[u] ^ (uint32_t)wu[u] ^ (uint32_t)fail[u];
#pragma unroll
                    for (int j = 0; j < NS; j++) x ^= sd[u][j];
                    if (GROUPED) x ^= k0[u] ^ k1[u];
                }
                n_rec += (uint32_t)__popcll(__ballot(x & 1));
            }
            if (last_pass) FAST_ISSUE();
            continue;
#endif
            // ---- SUM addends: fixed point (10^-3) for numerals of <= 4 bytes (<= 3 decimals);
            //      5-7 byte numerals as strtod's double; su: not typed here
            uint64_t sfix[RP][MAXS];
            double sdbl[RP][MAXS];
            bool hspill[RP] = {};   // an addend only the HBM table can take (NS == 2, > 3 decimals)
            bool snum[RP][MAXS], sfx[RP][MAXS], su[RP] = {};
#pragma unroll
            for (int j = 0; j < NS; j++) {
                bool wide = false, sw[RP];
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    const uint32_t len = sen[u][j] - sst[u][j];
                    const Num n = num4<true>(sd[u][j], len, nk);
#ifdef FAST_OLD_NUMK
                    const uint32_t mul = (n.k & 2) ? ((n.k & 1) ? 1u : 10u) : ((n.k & 1) ? 100u : 1000u);
#else
                    // 10^(3 - k), k <= 3: a 16-bit entry of one 64-bit constant
                    const uint32_t mul = (uint32_t)(0x0001000A006403E8ull >> (n.k << 4)) & 0xFFFFu;
#endif
                    sfix[u][j] = __umul24(n.M, mul);   // < 10^7
                    sdbl[u][j] = 0.0;
                    snum[u][j] = n.ok;
                    sfx[u][j] = true;
                    sw[u] = !n.ok & (len != 0) & !fail[u];
                    wide |= sw[u];
                }
                if (WN && __any(wide)) {
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        if (sw[u]) {
                            const uint32_t len = sen[u][j] - sst[u][j];
                            uint32_t d0, d1;
                            ld8a(pa[u] + sst[u][j], d0, d1);
                            const Num n = num7(d0, d1, len);
                            if (n.ok) {
                                snum[u][j] = true;
                                sw[u] = false;
                                if (n.k <= 3) {                          // exact: M * 10^(3 - k) < 10^10
                                    const uint32_t mul = (n.k & 2) ? ((n.k & 1) ? 1u : 10u) : ((n.k & 1) ? 100u : 1000u);
                                    sfix[u][j] = (uint64_t)n.M * mul;
                                } else {
                                    sdbl[u][j] = (double)n.M / p10(n.k);   // strtod: RN(M / 10^k), exact operands
                                    sfx[u][j] = false;
                                    hspill[u] |= NS == 2;
                                }
                            }
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < RP; u++) su[u] |= sw[u];
            }
#pragma unroll
            for (int u = 0; u < RP; u++) fail[u] |= wu[u] | su[u];

            // ---- GROUP BY key: the raw field bytes (<= 8, none <= ' '), zero padded
            uint64_t tag[RP] = {};
            uint32_t hb[RP] = {};
            if (GROUPED) {
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    const uint32_t klen = gen[u] - gst[u];
                    const uint32_t m0 = len_mask(klen, 0), m1 = len_mask(klen, 1);
                    const uint32_t a0 = k0[u] & m0, a1 = k1[u] & m1;
                    fail[u] |= (klen > 8u) | ((low_bytes(a0, m0 & nk.k80, nk) | low_bytes(a1, m1 & nk.k80, nk)) != 0);
                    tag[u] = klen ? ((uint64_t)a0 | ((uint64_t)a1 << 32)) : (1ull << 32);
                    hb[u] = fast_key_hash((uint32_t)tag[u], (uint32_t)(tag[u] >> 32));
                }
            }
            if (last_pass) FAST_ISSUE();                             // the window's bytes are read
#if defined(FAST_PROF) && FAST_PROF == 3      // + field loads, typing, keys and hashes
            n_rec += (uint32_t)__popcll(__ballot((hb[0] ^ hb[1] ^ (uint32_t)pass[0] ^ (uint32_t)fail[1] ^ (uint32_t)sfix[0][0]) & 1));
            continue;
#endif

            // ---- declined records go whole to slow_kernel
#pragma unroll
            for (int u = 0; u < RP; u++) {
                const bool slow = valid[u] & fail[u];
                const uint64_t sb = __ballot(slow);
                if (sb) {
                    unsigned long long base = 0;
                    if (lane == 0) base = atomicAdd(&stats->slow_records, (unsigned long long)__popcll(sb));
                    base = __shfl(base, 0, 64);
                    if (slow) {
                        const unsigned long long si = base + __popcll(sb & ((1ULL << lane) - 1));
                        if (si < slow_cap) slow_list[si] = (first_win + i) * wsb + p[u];
                    }
                }
                const bool ok = valid[u] & !fail[u];
                pass[u] = pass[u] & ok;
                n_rec += (uint32_t)__popcll(__ballot(ok));
                n_pass += (uint32_t)__popcll(__ballot(pass[u]));
            }

            // ---- aggregate
            if (!GROUPED) {
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    my_cnt += pass[u] ? 1u : 0u;
                    my_first = pass[u] ? min(my_first, fcw | p[u]) : my_first;
#pragma unroll
                    for (int j = 0; j < NS; j++) {
                        const bool on = pass[u] & snum[u][j];
                        my_fix[j] += (on & sfx[u][j]) ? sfix[u][j] : 0u;
                        my_dbl[j] += (on & !sfx[u][j]) ? sdbl[u][j] : 0.0;
                        my_num[j] += on ? 1u : 0u;
                    }
                    if constexpr (EXT != 0) {
                        const bool cand = pass[u] & snum[u][0];
                        const unsigned long long xk = ext_key<EXT>(sfix[u][0], fcw | p[u]);
                        if (cand) my_ext = EXT == 1 ? (xk < my_ext ? xk : my_ext) : (xk > my_ext ? xk : my_ext);
                        saw_num |= cand;
                    }
                }
            } else {
                // lookup: the key's two buckets (one 16-byte LDS read each)
                int slot[RP];
                bool miss[RP];
#ifndef FAST_OLD_LK
                // both records' bucket reads issued before any compare (one LDS wait per pass)
                v4u xs[RP], ys[RP];
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    const uint32_t b1 = hb[u] & (TBUCKETS - 1), b2 = (hb[u] >> 16) & (TBUCKETS - 1);
                    xs[u] = ((const v4u*)T)[b1];
                    ys[u] = ((const v4u*)T)[b2];
                }
#endif
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    const uint32_t b1 = hb[u] & (TBUCKETS - 1), b2 = (hb[u] >> 16) & (TBUCKETS - 1);
#ifndef FAST_OLD_LK
                    const v4u x = xs[u], y = ys[u];
#else
                    const v4u x = ((const v4u*)T)[b1], y = ((const v4u*)T)[b2];
#endif
                    const uint64_t t0 = (uint64_t)x.x | ((uint64_t)x.y << 32), t1 = (uint64_t)x.z | ((uint64_t)x.w << 32);
                    const uint64_t t2 = (uint64_t)y.x | ((uint64_t)y.y << 32), t3 = (uint64_t)y.z | ((uint64_t)y.w << 32);
                    int s = -1;
                    s = t3 == tag[u] ? (int)(2 * b2 + 1) : s;
                    s = t2 == tag[u] ? (int)(2 * b2) : s;
                    s = t1 == tag[u] ? (int)(2 * b1 + 1) : s;
                    s = t0 == tag[u] ? (int)(2 * b1) : s;
#ifdef FAST_NOLOOKUP                                          // experiment: no table reads
                    s = (int)(hb[u] & (TSLOTS - 1));
#endif
                    slot[u] = s;
                    miss[u] = pass[u] & (s < 0) & !hspill[u];
                }
                bool anym = false;
#pragma unroll
                for (int u = 0; u < RP; u++) anym |= miss[u];
                if (__any(anym)) {                                   // keys the seed did not place
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        if (miss[u]) {
                            const uint32_t b1 = hb[u] & (TBUCKETS - 1), b2 = (hb[u] >> 16) & (TBUCKETS - 1);
                            const uint32_t cand[4] = {2 * b1, 2 * b1 + 1, 2 * b2, 2 * b2 + 1};
                            for (int c = 0; c < 4 && slot[u] < 0; c++) {
                                const unsigned long long old = atomicCAS(&T[cand[c]], 0ull, (unsigned long long)tag[u]);
                                if (old == 0ull || old == tag[u]) slot[u] = (int)cand[c];
                            }
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    slot[u] = hspill[u] ? -1 : slot[u];
                    const bool add = pass[u] & (slot[u] >= 0);
                    uint8_t* r = S + (uint32_t)slot[u] * SLOT_BYTES;
                    if (add) {
                        const uint32_t fc = fcw | p[u];
#ifndef FAST_ATOM
#define FAST_ATOM 7                                                  // experiment: which LDS atomics run
#endif
                        if (FAST_ATOM & 1) atomicAdd((uint32_t*)(r + SO_CNT), 1u);
                        if (FAST_ATOM & 2) atomicMin((uint32_t*)(r + SO_FIRST), fc);
#pragma unroll
                        for (int j = 0; j < NS; j++) {
                            if (snum[u][j] && (FAST_ATOM & 4)) {
                                if (sfx[u][j]) atomicAdd((unsigned long long*)(r + (j ? SO_FIX1 : SO_FIX0)), (unsigned long long)sfix[u][j]);
                                else if (NS == 1 && EXT == 0) atomicAdd((double*)(r + SO_DBL), sdbl[u][j]);
                            }
                        }
                        if constexpr (EXT != 0) {
                            if (snum[u][0]) {
                                const unsigned long long xk = ext_key<EXT>(sfix[u][0], fc);
                                if (EXT == 1) atomicMin((unsigned long long*)(r + SO_EXT), xk);
                                else atomicMax((unsigned long long*)(r + SO_EXT), xk);
                            }
                        }
                    }
                    if constexpr (EXT != 0) saw_num |= add & snum[u][0];
#pragma unroll
                    for (int j = 0; j < NS; j++) {
                        const bool nn = add & !snum[u][j];
                        if (__any(nn)) {
                            if (nn) atomicAdd((uint32_t*)(r + (j ? SO_MISS1 : SO_MISS0)), 1u);
                        }
                    }
                    const bool spill = pass[u] & (slot[u] < 0);
                    const uint64_t spb = __ballot(spill);
                    if (EXT != 0 && spb) {
                        // both buckets full: the record goes whole to slow_kernel (which keeps
                        // the extreme in the canonical table); not counted here
                        unsigned long long base = 0;
                        if (lane == 0) base = atomicAdd(&stats->slow_records, (unsigned long long)__popcll(spb));
                        base = __shfl(base, 0, 64);
                        if (spill) {
                            const unsigned long long si = base + __popcll(spb & ((1ULL << lane) - 1));
                            if (si < slow_cap) slow_list[si] = (first_win + i) * wsb + p[u];
                        }
                        n_rec -= (uint32_t)__popcll(spb);
                        n_pass -= (uint32_t)__popcll(spb);
                    } else if (spb) {                                // both buckets full
                        n_spill += (uint32_t)__popcll(spb);
                        if (spill) {
                            double v0 = 0.0, v1 = 0.0;
                            bool n0 = false, n1 = false;
                            if (NS > 0) { n0 = snum[u][0]; v0 = sfx[u][0] ? sfix[u][0] / 1000.0 : sdbl[u][0]; }
                            if (NS > 1) { n1 = snum[u][1]; v1 = sfx[u][1] ? sfix[u][1] / 1000.0 : sdbl[u][1]; }
                            spill8(tag[u], (first_win + i) * wsb + p[u], tabs, stats, nacc, acc1, n0, v0, n1, v1);
                        }
                    }
                }
            }
            asm volatile("" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
        FAST_ISSUE();                                                // (a window without owned records)
#undef FAST_ISSUE
    }

    // ---- statistics
    if (EXT != 0 && __any(saw_num) && lane == 0) atomicOr(&stats->acc_classes[fp.ext_acc], 1u);   // numbers
    if (lane == 0) {
        if (n_rec) atomicAdd(&stats->records, (unsigned long long)n_rec);
        if (n_pass) atomicAdd(&stats->passed, (unsigned long long)n_pass);
        if (n_spill) atomicAdd(&stats->lds_spills, (unsigned long long)n_spill);
    }

    if (!GROUPED) {
        unsigned long long c = my_cnt;
        uint32_t f = my_first;
        double sm[MAXS];
        unsigned long long nm[MAXS];
#pragma unroll
        for (int j = 0; j < MAXS; j++) { sm[j] = (double)my_fix[j] / 1000.0 + my_dbl[j]; nm[j] = my_num[j]; }
        for (int o = 32; o > 0; o >>= 1) {
            c += __shfl_down(c, o, 64);
            const uint32_t ff = __shfl_down(f, o, 64);
            f = ff < f ? ff : f;
#pragma unroll
            for (int j = 0; j < MAXS; j++) {
                sm[j] += __shfl_down(sm[j], o, 64);
                nm[j] += __shfl_down(nm[j], o, 64);
            }
        }
        const GroupTable& gt = tabs[TAB_GT];
        if (lane == 0) {
            GKey k;
            k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
            const int gi = g_insert(gt, k, 0x12345678ULL, stats);
            if (gi >= 0) {
                if (c) atomicAdd(&gt.cnt[gi], c);
                if (f != NOFIRST) {
                    const uint64_t fw = first_win + ((uint64_t)(f >> 16) * gridDim.x + blockIdx.x) * NWV + ((f >> 12) & 15);
                    atomicMin(&gt.first[gi], (unsigned long long)(fw * wsb + (f & 4095)));
                }
                for (int a = 0; a < nacc; a++) {
                    if (EXT != 0 && !((fp.sum_mask >> a) & 1)) continue;
                    const bool j1 = (acc1 >> a) & 1;
                    const double sa = j1 ? sm[MAXS - 1] : sm[0];
                    const unsigned long long na = j1 ? nm[MAXS - 1] : nm[0];
                    if (na) {
                        atomicAdd(&gt.sum[a][gi], sa);
                        atomicAdd(&gt.num[a][gi], na);
                    }
                }
            }
        }
        if constexpr (EXT != 0) {
            // the wave's extreme (one key order for MIN and MAX) as a packed key into the
            // raw table's word 0 (fast_ext_final_kernel merges it into the group)
            unsigned long long x = my_ext;
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long y = __shfl_down(x, o, 64);
                x = EXT == 1 ? (y < x ? y : x) : (y > x ? y : x);
            }
            if (lane == 0 && x != ext_none<EXT>()) {
                const uint32_t code = EXT == 1 ? (uint32_t)x : ~(uint32_t)x;
                const uint64_t fw = first_win + ((uint64_t)(code >> 16) * gridDim.x + blockIdx.x) * NWV + ((code >> 12) & 15);
                atomicMin(&tabs[TAB_RT].extpos[fp.ext_acc][0], ext_packed<EXT>(x >> 32, fw * wsb + (code & 4095)));
            }
        }
        return;
    }

    // ---- flush the block's raw keys into the HBM raw table (raw_merge_kernel types
    //      every distinct raw key once and merges it into the canonical table)
    __syncthreads();
    const GroupTable& rt = tabs[TAB_RT];
    const uint32_t rot = (uint32_t)blockIdx.x * (TSLOTS / 64 + 1);
    static_assert(TSLOTS % LT == 0, "every lane runs every flush trip (the MIN / MAX merge is wave-uniform)");
    for (uint32_t ii = tid; ii < TSLOTS; ii += LT) {
        const uint32_t i = (ii + rot) & (TSLOTS - 1);
        const uint8_t* r = S + i * SLOT_BYTES;
        const uint32_t n = *(const uint32_t*)(r + SO_CNT);
        int gi = -1;
        if (n) {
            const uint64_t w0 = T[i];
            const uint32_t kl = key_len8(w0);
            const GKey k = raw_key(kl, kl ? w0 : 0ull);
            gi = g_insert(rt, k, gk_hash(k), stats);
        }
        if constexpr (EXT != 0) {      // the slot's extreme as a packed key (raw_merge_kernel types it)
            const unsigned long long x = *(const unsigned long long*)(r + SO_EXT);
            if (gi >= 0 && x != ext_none<EXT>()) {
                const uint32_t code = EXT == 1 ? (uint32_t)x : ~(uint32_t)x;
                const uint64_t fw = first_win + ((uint64_t)(code >> 16) * gridDim.x + blockIdx.x) * NWV + ((code >> 12) & 15);
                atomicMin(&rt.extpos[fp.ext_acc][gi], ext_packed<EXT>(x >> 32, fw * wsb + (code & 4095)));
            }
        }
        if (gi < 0) continue;
        atomicAdd(&rt.cnt[gi], (unsigned long long)n);
        const uint32_t fc = *(const uint32_t*)(r + SO_FIRST);
        if (fc != NOFIRST) {
            const uint64_t fw = first_win + ((uint64_t)(fc >> 16) * gridDim.x + blockIdx.x) * NWV + ((fc >> 12) & 15);
            atomicMin(&rt.first[gi], (unsigned long long)(fw * wsb + (fc & 4095)));
        }
        for (int acc = 0; acc < nacc; acc++) {
            if (EXT != 0 && !((fp.sum_mask >> acc) & 1)) continue;
            const bool j1 = (acc1 >> acc) & 1;
            const double sa = j1 ? (double)*(const unsigned long long*)(r + SO_FIX1) / 1000.0
                                 : (double)*(const unsigned long long*)(r + SO_FIX0) / 1000.0 +
                                       (NS == 1 && EXT == 0 ? *(const double*)(r + SO_DBL) : 0.0);
            const uint32_t ms = *(const uint32_t*)(r + (j1 ? SO_MISS1 : SO_MISS0));
            const uint32_t num = n - ms;
            if (num) {
                atomicAdd(&rt.sum[acc][gi], sa);
                atomicAdd(&rt.num[acc][gi], (unsigned long long)num);
            }
        }
    }
}


// ------------------------------------------------------------------ fused join: extraction
// One side of an aggregate-only equi-join (perform_join, evaluator_joins.c:63-181,
// feeding evaluate_aggregate) streamed like fast_kernel: per record the ON key as a
// canonical non-negative INTEGER below 10^15 (then value_compare's double equality is
// integer equality) or NULL, and one payload: BUILD the GROUP BY field's raw bytes
// (<= 8, none <= ' ', as fast_kernel's tags), else the SUM argument in units of 10^-3
// (fast_kernel's fixed-point path; NULL: JX_NOVAL).  Every record lands, in no particular
// order, at a slot reserved per wave: key[], pay[], off[] (its byte offset, the join's
// order key).  A record outside this shape (a quote in the window, a short row, another
// key spelling, a wider numeral) sets *flag: the caller runs the general join instead.
constexpr unsigned long long JX_NULLKEY = ~0ull;
constexpr unsigned long long JX_NOVAL = 0x8000000000000000ull;
struct JxPlan {
    uint64_t first_win;
    uint32_t nwin, lo_s, hi_s, ws;
    uint32_t delim, quote;
    uint32_t skip[2];          // field k's column minus field k-1's (the roles in column order)
    uint32_t rank_key;         // field index of the key (the payload's: 1 - rank_key)
};
struct JxOut {
    unsigned long long* key;
    unsigned long long* pay;
    uint32_t* off;
    unsigned int* wcount;      // COUNT pass: records owned by window i
    const unsigned int* wbase; // emit pass: the first record index of window i (exclusive scan)
    unsigned int cap;
    unsigned int* flag;
    unsigned long long* krange;   // [0] min, [1] max of the non-NULL keys
    // STAR passes (jx_star_*): no record arrays; the build side goes straight into
    // key-indexed arrays over [kmin, kmin + range), the probe side aggregates in place
    unsigned long long kmin, range;
    // key stride S = 2^sshift * m (m odd, sinv = m^-1 mod 2^32): slot i holds key
    // kmin + i S.  A table routed by key mod N (route.hip) holds on rank d only keys
    // = d (mod N): dense with stride N.  S = 1: sshift 0, smask 0, sinv 1.
    uint32_t sshift, smask, sinv;
    uint32_t stride;           // S itself (the build's slot-domain key range back to keys)
    uint16_t* d16;             // build: group id + 1 of key kmin + i S (0: no build record);
                               // probe: | 0x8000 once a probe record met it
    uint32_t* l32;             // build: that record's byte offset
    unsigned long long* ttab;  // build: GROUP BY raw tags, slot = group id (0: free)
    unsigned long long* gsum;  // probe: per group id COUNT, fixed-point SUM, SUM count
    unsigned long long* nbuilt;   // build: records placed
    uint32_t* notmono;         // build / order check: nonzero unless the build keys rise in file order
                               // (probe: zero -> per group the smallest matched key index, no flags)
    unsigned long long* wfl;   // build: per window its first and last key (order check)
    uint32_t* gminix;          // probe: per group id the smallest matched key index
    // partitioned STAR probe, pass 1 (PART): no lookup; every matchable probe record
    // appends (slot, 32-bit payload) to its key partition (slot >> psh) in this block's
    // region of pent: [block][np][pcap] entries, counts in pcnt[block][np]
    unsigned long long* pent;
    uint32_t* pcnt;
    uint32_t np, pcap, psh;
    // ROUTE (the typed exchange of the multi-GPU join): every
    // record with a non-NULL key goes to rank key mod rn as one fixed-size entry:
    //   BUILD  uint4 {q32, gid, tag lo, tag hi}: q32 = key / rn - qbase, gid = gbase +
    //          the record's index in this table (file order), tag = the GROUP BY bytes
    //   PROBE  uint2 {q32, pay}: pay = the SUM argument in 10^-3 units (JX_PNULL: NULL)
    // Two passes, no atomics: ROUTE 1 counts per window i and destination d the entries
    // (rcnt[d * nwin + i]; BUILD: the window's records into wcount as well); the host
    // scans rcnt destination-major (roffs), so destination d's entries fill
    // [roffs[d * nwin], roffs[(d + 1) * nwin]) of rent with no hole; ROUTE 2 writes
    // each entry at roffs[d * nwin + i] + its rank among the window's entries for d.
    // Flags: 8 a NULL build key, 16 a build q32 outside [0, 2^32 - 1) (the host retries
    // with the keys' own minimum), 512 a payload outside 31 bits.  A probe key outside
    // the window matches no build key and is not sent.
    // ROUTE 3 (probe side, rn <= 8): one pass, no count.  Destination d's entries fill
    // region [d * cap, (d + 1) * cap) of rent in chunks of JX_RCHUNK entries, which a
    // wave's lane d reserves from the cursor rcnt[64 d] when its current chunk cannot hold
    // the pass's entries for d (the pass's first ones close the old chunk, the rest open
    // the new one); at the end each wave's unused chunk tails become holes {~0, JX_PNULL}
    // (q32 ~0 is never below qoff + range: the receivers skip them).  The probe's order
    // inside a region is free: its entries only add to sums and counts, and the first
    // pair of a group is its build record's.  A cursor past cap sets 1024 (the host
    // reruns the two passes).
    void* rent;
    unsigned int* rcnt;           // ROUTE 1; ROUTE 3: the destinations' cursors (stride 64)
    const unsigned int* roffs;    // ROUTE 2
    uint64_t rmagic;              // ceil(2^64 / rn) (rn > 1): key / rn = mulhi(key, rmagic) for keys < 2^58
    uint64_t qbase, gbase;
    uint32_t rn;
};
// a key's STAR slot (k - kmin) / S when k = kmin (mod S) and the slot is below 2^32,
// else ~0 (never < range: the host keeps range * S < 2^32).  Exact division by the
// odd part through its inverse: for x divisible by m, (x * m^-1) mod 2^32 = x / m;
// for any other x it is above (2^32 - 1) / m >= range (Granlund-Montgomery)
__device__ __forceinline__ unsigned long long jx_slot(unsigned long long k, const JxOut& jo) {
    const unsigned long long x = k - jo.kmin;
    const uint32_t lo = (uint32_t)x;
    const uint32_t q = (lo >> jo.sshift) * jo.sinv;
    return ((x >> 32) == 0ull && (lo & jo.smask) == 0u) ? (unsigned long long)q : ~0ull;
}

// STAR flags (JxOut.flag): 8 a NULL build key, 16 a key outside [kmin, kmin + range),
// 32 more GROUP BY tags than JX_G, 64 a repeated build key (placed != occupied),
// 128 a partitioned probe's partition region full or a payload outside 31 bits
// (the host reruns the probe unpartitioned)
constexpr uint32_t JX_G = 2048;           // group ids of a STAR join (LDS sums per block)
constexpr uint32_t JX_PMAX = 4096;        // key partitions of a partitioned STAR probe (LDS counters)
constexpr uint32_t JX_PNULL = 0x80000000u;   // a partitioned entry's NULL payload
constexpr uint32_t JX_RCHUNK = 192;          // ROUTE 3 chunk (>= one pass's entries for one destination)

// a GROUP BY raw tag's group id: its slot in the tag table (linear probing; a stale
// 0 read only leads to the CAS, a set slot never changes)
__device__ __forceinline__ uint32_t jx_tag_gid(unsigned long long* __restrict__ tt, unsigned long long tag,
                                               bool& full) {
    uint32_t s = fast_key_hash((uint32_t)tag, (uint32_t)(tag >> 32)) & (JX_G - 1);
    for (uint32_t q = 0; q < JX_G; q++) {
        const unsigned long long t = tt[s];
        if (t == tag) return s;
        if (t == 0ull) {
            const unsigned long long old = atomicCAS(&tt[s], 0ull, tag);
            if (old == 0ull || old == tag) return s;
        }
        s = (s + 1) & (JX_G - 1);
    }
    full = true;
    return 0;
}
// the same through a block's LDS mirror of the tag table (slots as the global table's;
// a slot the mirror has not seen yet ends the walk there and asks the global table)
__device__ __forceinline__ uint32_t jx_tag_gid_lds(unsigned long long* __restrict__ lt,
                                                   unsigned long long* __restrict__ tt, unsigned long long tag,
                                                   bool& full) {
    uint32_t s = fast_key_hash((uint32_t)tag, (uint32_t)(tag >> 32)) & (JX_G - 1);
    for (uint32_t q = 0; q < 8u; q++) {
        const unsigned long long t = lt[s];
        if (t == tag) return s;
        if (t == 0ull) break;
        s = (s + 1) & (JX_G - 1);
    }
    const uint32_t g = jx_tag_gid(tt, tag, full);
    if (!full) lt[g] = tag;
    return g;
}

// the same with fast_kernel's two-choice buckets (slots 2b, 2b + 1 of buckets
// b1, b2 of fast_key_hash), the table seeded by the host's cuckoo placement of the
// build side's sampled tags (cq_fast_seed): a hit is two 16-byte LDS reads and
// four compares, no walk; a tag the sample missed claims a free candidate slot in
// the global table (every block agrees on its slot) and enters the block's mirror.
// No free candidate: `full` (the record-array join takes the query).
static_assert(TSLOTS == JX_G, "the STAR tag table is fast_kernel's seeded layout");
__device__ __forceinline__ uint32_t jx_tag_slot(unsigned long long* __restrict__ lt,
                                                unsigned long long* __restrict__ tt, unsigned long long tag,
                                                bool& full) {
    const uint32_t h = fast_key_hash((uint32_t)tag, (uint32_t)(tag >> 32));
    const uint32_t b1 = h & (TBUCKETS - 1), b2 = (h >> 16) & (TBUCKETS - 1);
    const v4u x = ((const v4u*)lt)[b1], y = ((const v4u*)lt)[b2];
    const unsigned long long t0 = (unsigned long long)x.x | ((unsigned long long)x.y << 32);
    const unsigned long long t1 = (unsigned long long)x.z | ((unsigned long long)x.w << 32);
    const unsigned long long t2 = (unsigned long long)y.x | ((unsigned long long)y.y << 32);
    const unsigned long long t3 = (unsigned long long)y.z | ((unsigned long long)y.w << 32);
    int sl = -1;
    sl = t3 == tag ? (int)(2 * b2 + 1) : sl;
    sl = t2 == tag ? (int)(2 * b2) : sl;
    sl = t1 == tag ? (int)(2 * b1 + 1) : sl;
    sl = t0 == tag ? (int)(2 * b1) : sl;
    if (sl >= 0) return (uint32_t)sl;
    const uint32_t cand[4] = {2 * b1, 2 * b1 + 1, 2 * b2, 2 * b2 + 1};
    for (int c = 0; c < 4 && sl < 0; c++) {
        const unsigned long long old = atomicCAS(&tt[cand[c]], 0ull, tag);
        if (old == 0ull || old == tag) sl = (int)cand[c];
    }
    if (sl < 0) { full = true; return 0; }
    lt[sl] = tag;                                  // (every writer: the same tag)
    return (uint32_t)sl;
}

// the canonical INTEGER key of a field (16 bytes d0..d3 from its start, len bytes):
// digits only, no leading zero, at most 15 digits and not 8-10; NULL (empty) -> JX_NULLKEY
__device__ __forceinline__ bool jx_key(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t len,
                                       unsigned long long& key) {
    if (len == 0) { key = JX_NULLKEY; return true; }
    // (8-10 digits may type as a DATE, infer_type csv_reader.c:139: such keys take the
    // general join, whose class rules pair DATE with every number)
    bool ok = len <= 15u && (len < 8u || len > 10u) && ((d0 & 0xFFu) != '0' || len == 1u);
#ifdef JX_OLD_KEY
    const uint32_t dd[4] = {d0, d1, d2, d3};
    unsigned long long v = 0;
#pragma unroll
    for (int j = 0; j < 15; j++) {
        const uint32_t c = (dd[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        const uint32_t dg = c - '0';
        if ((uint32_t)j < len) {
            ok = ok && dg < 10u;
            v = v * 10ull + dg;
        }
    }
    key = v;
    return ok;
#else
    // the 16 bytes right-aligned (the digits end at byte 15, '0' fill below): a
    // 128-bit shift left by 16 - len bytes drops the bytes past the field
    const uint32_t sb = (16u - (len & 15u)) * 8u;          // 8 .. 120 (len 1 .. 15)
    const unsigned long long lo = (unsigned long long)d0 | ((unsigned long long)d1 << 32);
    const unsigned long long hi = (unsigned long long)d2 | ((unsigned long long)d3 << 32);
    unsigned long long ylo, yhi, fill_lo, fill_hi;
    if (sb < 64u) {
        ylo = lo << sb;
        yhi = (hi << sb) | (lo >> (64u - sb));
        fill_lo = 0x3030303030303030ull & ((1ull << sb) - 1ull);
        fill_hi = 0ull;
    } else {
        ylo = 0ull;
        yhi = lo << (sb - 64u);
        fill_lo = 0x3030303030303030ull;
        fill_hi = 0x3030303030303030ull & ((1ull << (sb - 64u)) - 1ull);
    }
    const unsigned long long dl = (ylo | fill_lo) - 0x3030303030303030ull;   // byte 0: the 10^15 digit
    const unsigned long long dh = (yhi | fill_hi) - 0x3030303030303030ull;
    // every byte < 10 (a byte >= 10 sets bit 7 of itself or of itself + 0x76)
    ok = ok && (((dl + 0x7676767676767676ull) | dl | (dh + 0x7676767676767676ull) | dh) & 0x8080808080808080ull) == 0;
    // four digits per 32-bit word (most significant first): (b0 10 + b1) 100 + b2 10 + b3
    const auto g4 = [](uint32_t w) {
        const uint32_t p = __builtin_amdgcn_udot4(w, 0x0000010Au, 0u, false);
        const uint32_t q = __builtin_amdgcn_udot4(w, 0x010A0000u, 0u, false);
        return __umul24(p, 100u) + q;
    };
    const uint32_t h0 = __umul24(g4((uint32_t)dl), 10000u) + g4((uint32_t)(dl >> 32));
    const uint32_t h1 = __umul24(g4((uint32_t)dh), 10000u) + g4((uint32_t)(dh >> 32));
    key = (unsigned long long)h0 * 100000000ull + h1;
    return ok;
#endif
}

template <bool BUILD, bool COMMA, int NR, bool COUNT, bool STAR = false, int RP = 2, bool PART = false,
          int ROUTE = 0>
__global__ __launch_bounds__(LT) void jx_extract_kernel(const uint8_t* __restrict__ g, const JxPlan jp, const JxOut jo) {
    static_assert(ROUTE == 0 || (!STAR && !COUNT), "ROUTE: the record form's passes");
    static_assert(ROUTE != 3 || !BUILD, "ROUTE 3: the probe side");
    extern __shared__ __align__(16) uint8_t smem[];
    WaveLds* waves = (WaveLds*)smem;
    // STAR probe: per group id COUNT / fixed-point SUM / SUM count of this block;
    // STAR build: the block's mirror of the GROUP BY tag table;
    // partitioned STAR probe (PART): the block's per-partition entry counters
    static_assert(!PART || (STAR && !BUILD), "PART: the STAR probe's first pass");
    constexpr bool SPROBE = STAR && !BUILD && !PART;
    uint32_t* pcl = (uint32_t*)(smem + sizeof(WaveLds) * NWV);
    if constexpr (PART) {
        for (uint32_t k = threadIdx.x; k < jo.np; k += LT) pcl[k] = 0u;
        __syncthreads();
    }
    constexpr bool SBUILD = STAR && BUILD && NR == 2;
    constexpr uint32_t NG = SPROBE ? JX_G : 1;
    unsigned long long* sfix = (unsigned long long*)(smem + sizeof(WaveLds) * NWV);
    uint32_t* scnt = (uint32_t*)(sfix + NG);
    uint32_t* snum = scnt + NG;
    uint32_t* smix = snum + NG;
    unsigned long long* stt = (unsigned long long*)(smem + sizeof(WaveLds) * NWV);
    // (probe: with rising offsets the first pair's build record is the smallest matched
    // key's: no match flags written into d16)
    uint32_t mono = 0;
    if constexpr (SPROBE) {
        for (uint32_t k = threadIdx.x; k < NG; k += LT) { sfix[k] = 0; scnt[k] = 0; snum[k] = 0; smix[k] = ~0u; }
        mono = __builtin_amdgcn_readfirstlane(*jo.notmono) == 0u ? 1u : 0u;
        __syncthreads();
    }
    if constexpr (SBUILD) {                       // the mirror starts as the seeded global table
        for (uint32_t k = threadIdx.x; k < JX_G; k += LT) stt[k] = jo.ttab[k];
        __syncthreads();
    }
    uint32_t sflag = 0;
    unsigned long long nstar = 0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    WaveLds& W = waves[wv];
    const uint32_t rep_q = jp.quote * 0x01010101u;
    CK ck;
#ifndef FAST_OLD_CLS
    ck.tn1 = vreg(COMMA ? CLS2_TN1 : 0x00004000u);
    ck.tn0 = vreg(COMMA ? CLS2_TN0 : 0x00400000u);
    ck.td1 = vreg(COMMA ? CLS2_TD1 : 0u);
    ck.td0 = vreg(COMMA ? CLS2_TD0 : 0x40u);
    ck.m40 = vreg(COMMA ? 0x01010101u : 0x40404040u);   // (COMMA: the bit-0 mask)
    ck.m80 = vreg(0x80808080u);
#else
    ck.tn1 = vreg(0x00004000u);
    ck.tn0 = vreg(0x00400000u);
    ck.td1 = vreg(COMMA ? 0x80408080u : 0u);
    ck.td0 = vreg(COMMA ? 0x80802080u : 0x40u);
    ck.m40 = vreg(0x40404040u);
#endif
    ck.w0 = vreg(0x08040201u);
    ck.w1 = vreg(0x80402010u);
    ck.rd = vreg(jp.delim * 0x01010101u);
    ck.rq = vreg(rep_q);
    const uint64_t first_win = jp.first_win;
    const uint32_t nwin = __builtin_amdgcn_readfirstlane(jp.nwin);
    const uint32_t wsb = __builtin_amdgcn_readfirstlane(jp.ws);
    const uint32_t rkey = __builtin_amdgcn_readfirstlane(jp.rank_key);
    const uint32_t wstep = gridDim.x * NWV;
    const uint32_t lane_full = (uint32_t)lane * LB < wsb ? ~0u : 0u;
    uint32_t prev_next = 0;
    const uint32_t voff = vreg(16u * (uint32_t)lane);
    const uint32_t wlds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)W.bytes);
    const uint32_t lane_lds = vreg(wlds + (uint32_t)lane * LB);
    bool bad = false;
    unsigned long long kmin = ~0ull, kmax = 0ull;
    uint32_t smin = ~0u, smax = 0u;          // STAR build: the in-range keys' extreme slots
    uint32_t ccur = 0, cend = 0;             // ROUTE 3: lane d's chunk for destination d (next, end)
    uint32_t i = blockIdx.x * NWV + wv;
    if (i < nwin) load_win(g, first_win + i, wsb, wlds, voff, prev_next);
    for (; i < nwin; i += wstep) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t prevw = prev_next;
        v4u la[4];
#pragma unroll
        for (int k = 0; k < 4; k++) la[k] = ((const v4u*)W.bytes)[4 * lane + k];
#ifndef FAST_NO_Q3
        uint32_t sep0, nl0, sep1, nl1, qf = COMMA ? 0xFFFFFFFFu : 0u;
#else
        uint32_t sep0, nl0, sep1, nl1, qf = 0;
#endif
        classify32<COMMA>(la[0], la[1], ck, sep0, nl0, qf);
        classify32<COMMA>(la[2], la[3], ck, sep1, nl1, qf);
#ifndef FAST_NO_Q3
        bad = bad || __ballot(((COMMA ? ~qf : qf) & 0x80808080u) != 0) != 0;      // a quote: the general join
#else
        bad = bad || __ballot((qf & 0x80808080u) != 0) != 0;      // a quote: the general join
#endif
        const uint64_t nl = (uint64_t)nl0 | ((uint64_t)nl1 << 32);
        const uint32_t prev_top = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(nl1 >> 31), 0x138, 0xf, 0xf, true);
        const uint32_t pb = prevw >> 24;
        const uint32_t prevnl = lane == 0 ? (uint32_t)(pb == '\n' || pb == '\r') : prev_top;
        uint64_t todo = ~nl & ((nl << 1) | prevnl);
        if (i == 0 || i == nwin - 1) {
            const uint32_t lo_s = i == 0 ? jp.lo_s : 0u, hi_s = i == nwin - 1 ? jp.hi_s : wsb;
            const uint32_t b0 = (uint32_t)lane * LB;
            const uint32_t a = lo_s > b0 ? lo_s - b0 : 0u, e = hi_s > b0 ? hi_s - b0 : 0u;
            const uint64_t keep_lo = a >= 64 ? 0ull : (~0ull << a);
            const uint64_t keep_hi = e >= 64 ? ~0ull : ((1ull << e) - 1);
            todo &= keep_lo & keep_hi;
        } else {
            todo &= ((uint64_t)lane_full << 32) | lane_full;
        }
        const uint32_t xs0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sep0, 0x130, 0xf, 0xf, true);
        const uint32_t xs1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sep1, 0x130, 0xf, 0xf, true);
        const uint32_t xn0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nl0, 0x130, 0xf, 0xf, true);
        const uint32_t xn1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nl1, 0x130, 0xf, 0xf, true);
        const uint64_t sep64 = (uint64_t)sep0 | ((uint64_t)sep1 << 32);
        const uint64_t xsep2 = ((uint64_t)xs0 | ((uint64_t)xs1 << 32)) << 1;
        const uint64_t xnl2 = ((uint64_t)xn0 | ((uint64_t)xn1 << 32)) << 1;
        const uint64_t wbase = (first_win + i) * wsb;
        if (COUNT) {                       // records owned by this window (the emit pass's layout)
            const uint32_t tot = __builtin_amdgcn_readlane(wave_incl_scan((uint32_t)__popcll(todo)), 63);
            if (lane == 0) jo.wcount[i] = tot;
            if (i + wstep < nwin) {
                uint32_t ni = i + wstep;
                asm volatile("" : "+s"(ni));
                load_win(g, first_win + ni, wsb, wlds, voff, prev_next);
            }
            continue;
        }
        // record j of this lane in this window lands at wbase[i] + (the lanes below's
        // records) + j: file order
        const uint32_t nmine = (uint32_t)__popcll(todo);
        uint32_t at_next = (STAR || ROUTE == 1 || ROUTE == 3 || (ROUTE == 2 && !BUILD)) ? 0u
                                                                         : jo.wbase[i] + wave_incl_scan(nmine) - nmine;
        // ROUTE: lane d (< rn) holds destination d's entries of this window so far, and
        // (emit) its first position
        uint32_t rrun = 0, rbase = 0;
        if constexpr (ROUTE == 2) rbase = (uint32_t)lane < jo.rn ? jo.roffs[(uint64_t)lane * nwin + i] : 0u;
        if constexpr (ROUTE == 1 && BUILD) {
            const uint32_t tot = __builtin_amdgcn_readlane(wave_incl_scan(nmine), 63);
            if (lane == 0) jo.wcount[i] = tot;
        }
        bool issued = false;
        // STAR build: this lane's first and last key (its records come in file order),
        // as slots: keys map to slots monotonically, and a key outside the range flags
        // the query for a retry, which discards this round's order anyway
        uint32_t lfirst = ~0u, llast = 0u;
        bool lany = false, lbad = false;
        while (__any(todo != 0)) {
            uint32_t p[RP], pa[RP], fst[RP][2], fen[RP][2], e[RP];
            uint64_t sv[RP];
            bool valid[RP], fail[RP];
#pragma unroll
            for (int u = 0; u < RP; u++) {
                valid[u] = todo != 0;
                const uint32_t b = ctz64(todo) & 63u;
                todo &= todo - 1;
                pa[u] = lane_lds + b;
                p[u] = pa[u] - wlds;
                const uint32_t nb = b ^ 63u;
                sv[u] = view128(sep64, xsep2, b, nb);
                e[u] = ctz64(view128(nl, xnl2, b, nb));
            }
#pragma unroll
            for (int k = 0; k < NR; k++) {
                uint32_t n = jp.skip[k];
                n = __builtin_amdgcn_readfirstlane(n);
                asm volatile("" : "+s"(n));
                if (k > 0 && n == 0) {
#pragma unroll
                    for (int u = 0; u < RP; u++) { fst[u][k] = fst[u][k - 1]; fen[u][k] = fen[u][k - 1]; }
                    continue;
                }
                if (k > 0) {
#pragma unroll
                    for (int u = 0; u < RP; u++) sv[u] &= sv[u] - 1;
                }
                if (k == 0 && n == 0) {
#pragma unroll
                    for (int u = 0; u < RP; u++) fst[u][k] = 0;
                } else if (k > 0 && n == 1) {
#pragma unroll
                    for (int u = 0; u < RP; u++) fst[u][k] = fen[u][k - 1] + 1;
                } else {
                    for (uint32_t j = k == 0 ? 1u : 2u; j < n; j++) {
#pragma unroll
                        for (int u = 0; u < RP; u++) sv[u] &= sv[u] - 1;
                    }
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        fst[u][k] = ctz64(sv[u]) + 1;
                        sv[u] &= sv[u] - 1;
                    }
                }
#pragma unroll
                for (int u = 0; u < RP; u++) fen[u][k] = ctz64(sv[u]);
            }
            const bool last_pass = !__any(todo != 0);
            unsigned long long key[RP], pay[RP];
            uint32_t gpre[RP] = {};   // STAR probe: d16 of the key, loaded before the payload is typed
#pragma unroll
            for (int u = 0; u < RP; u++) {
                const uint32_t en = fen[u][NR - 1];
                fail[u] = (en >= 64u) | (en > e[u]);
                const uint32_t ks = NR == 1 || rkey == 0 ? fst[u][0] : fst[u][1];
                const uint32_t ke = NR == 1 || rkey == 0 ? fen[u][0] : fen[u][1];
                uint32_t d0, d1, d2, d3;
                ld8a(pa[u] + ks, d0, d1);
                ld8a(pa[u] + ks + 8, d2, d3);
                fail[u] |= !jx_key(d0, d1, d2, d3, ke - ks, key[u]);
#ifndef JX_LATE_LOOK
                if constexpr (SPROBE) {    // (out of range or NULL: slot 0, not used)
                    const unsigned long long ix = jx_slot(key[u], jo);
                    gpre[u] = jo.d16[ix < jo.range ? ix : 0ull];
                }
#endif
                pay[u] = 0;
                if (NR == 2) {
                    const uint32_t ps = rkey == 0 ? fst[u][1] : fst[u][0];
                    const uint32_t pe = rkey == 0 ? fen[u][1] : fen[u][0];
                    const uint32_t plen = pe - ps;
                    uint32_t q0, q1;
                    ld8a(pa[u] + ps, q0, q1);
                    if (BUILD) {                                      // the group field's raw bytes
                        const uint32_t m0 = len_mask(plen, 0), m1 = len_mask(plen, 1);
                        const uint32_t a0 = q0 & m0, a1 = q1 & m1;
                        fail[u] |= (plen > 8u) | ((low_bytes(a0, m0 & 0x80808080u) | low_bytes(a1, m1 & 0x80808080u)) != 0);
                        pay[u] = plen ? ((uint64_t)a0 | ((uint64_t)a1 << 32)) : (1ull << 32);
                    } else if (plen == 0) {
                        pay[u] = JX_NOVAL;                            // NULL: counted, not summed
                    } else {                                          // the SUM argument, 10^-3 units
#ifdef JX_AB_NOPAY
                        pay[u] = q0 & 0xFFFu;
                        continue;
#endif
                        // (a leading '-': the rest parsed, then negated; two's complement sums)
                        const bool neg = (q0 & 0xFFu) == '-' && plen > 1u;
                        uint32_t v0 = q0, v1 = q1, vl = plen;
                        if (neg) {
                            ld8a(pa[u] + ps + 1, v0, v1);
                            vl = plen - 1;
                        }
                        // (1-7 bytes in one typing: num7 is exact for the 4-byte shapes too,
                        // and a mix of widths in one wave would run both)
                        const Num n7 = num7(v0, v1, vl);
                        fail[u] |= !n7.ok | (n7.k > 3u);
                        const uint32_t mul = (uint32_t)(0x0001000A006403E8ull >> ((n7.k & 3u) << 4)) & 0xFFFFu;
                        const unsigned long long fx = (unsigned long long)n7.M * mul;
                        pay[u] = neg ? 0ull - fx : fx;
                    }
                }
                bad = bad || (valid[u] && fail[u]);
            }
            if (last_pass && !issued) {                               // the window's bytes are read
                if (i + wstep < nwin) {
                    uint32_t ni = i + wstep;
                    asm volatile("" : "+s"(ni));
                    load_win(g, first_win + ni, wsb, wlds, voff, prev_next);
                }
                issued = true;
            }
            if constexpr (STAR) {
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    if (!valid[u] || fail[u]) continue;
                    const unsigned long long k = key[u];
                    const unsigned long long ix = jx_slot(k, jo);
                    if (BUILD) {
                        if (k == JX_NULLKEY) { sflag |= 8u; continue; }
                        if (ix >= jo.range) {                   // (rare: the retry's range)
                            kmin = k < kmin ? k : kmin;
                            kmax = k > kmax ? k : kmax;
                            sflag |= 16u;
                            continue;
                        }
                        // the in-range keys' extremes and order in 32-bit slots
                        const uint32_t x32 = (uint32_t)ix;
                        smin = x32 < smin ? x32 : smin;
                        smax = x32 > smax ? x32 : smax;
                        lbad = lbad || (lany && x32 <= llast);
                        lfirst = lany ? lfirst : x32;
                        llast = x32;
                        lany = true;
                        bool full = false;
                        uint32_t gid = 0;
#ifndef JX_AB_NOTAG
                        if constexpr (SBUILD) gid = jx_tag_slot(stt, jo.ttab, pay[u], full);
#else
                        gid = (uint32_t)(pay[u] >> 40) & 1023u;
#endif
                        if (full) sflag |= 32u;
#ifndef JX_AB_NOSTORE
                        jo.d16[ix] = (uint16_t)(gid + 1u);
                        jo.l32[ix] = (uint32_t)(wbase + p[u]);
                        nstar++;
#else
                        sflag |= gid == 12345u ? 1u : 0u;
#endif
                    } else if (PART) {
                        // (a NULL key's slot is ~0, >= range: no entry, as it matches nothing)
                        if (ix < jo.range) {
                            const uint32_t pr = (uint32_t)ix >> jo.psh;
                            const unsigned long long pv = pay[u];
                            const bool pok = pv == JX_NOVAL || pv < (1ull << 31);
                            const uint32_t at = atomicAdd(&pcl[pr], 1u);
                            if (at < jo.pcap) {
                                // (a payload outside 31 bits: an entry pass 2 skips, and the flag)
                                const uint32_t p32 = pv == JX_NOVAL ? JX_PNULL : (uint32_t)pv;
                                jo.pent[((size_t)blockIdx.x * jo.np + pr) * jo.pcap + at] =
                                    pok ? ((unsigned long long)(uint32_t)ix | ((unsigned long long)p32 << 32)) : ~0ull;
                            }
                            if (at >= jo.pcap || !pok) sflag |= 128u;
                        }
                    } else if (k != JX_NULLKEY && ix < jo.range) {
#if defined(JX_AB_NOLOOK)
#elif defined(JX_LATE_LOOK)
                        const uint32_t gv = jo.d16[ix];
#else
                        const uint32_t gv = gpre[u];
#endif
#ifdef JX_AB_NOLOOK
                        const uint32_t gv = 1u + (uint32_t)(ix & 1023u);
#endif
                        if (gv) {
                            const uint32_t gi = (gv & 0x7FFFu) - 1u;
#if !defined(JX_AB_NOFLAG)
                            if (mono) {
                                if ((uint32_t)ix < smix[gi]) atomicMin(&smix[gi], (uint32_t)ix);
                            } else if (!(gv & 0x8000u)) {
                                jo.d16[ix] = (uint16_t)(gv | 0x8000u);   // (every writer: the same value)
                            }
#endif
#ifndef JX_AB_NOAGG
                            atomicAdd(&scnt[gi], 1u);
                            if (NR == 2 && pay[u] != JX_NOVAL) {
                                atomicAdd(&sfix[gi], pay[u]);
                                atomicAdd(&snum[gi], 1u);
                            }
#else
                            sflag |= gi == 12345u ? 1u : 0u;
#endif
                            nstar++;
                        }
                    }
                }
            } else if constexpr (ROUTE != 0) {
                // destination and q32 of each record, then per destination its entries'
                // ranks in the window (ballots; the count pass and the emit pass decide
                // `take` alike -- a record either pass fails flags the whole exchange)
                uint32_t dd[RP], q32[RP], gid[RP];
                bool take[RP];
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    gid[u] = valid[u] ? (uint32_t)(jo.gbase + at_next) : 0u;
                    at_next += valid[u] ? 1u : 0u;
                    const unsigned long long k = key[u];
                    take[u] = valid[u] && !fail[u] && k != JX_NULLKEY;
                    if (ROUTE == 1 && BUILD && valid[u] && !fail[u] && k == JX_NULLKEY) sflag |= 8u;
                    const unsigned long long q = jo.rn > 1u ? __umul64hi(k, jo.rmagic) : k;
                    dd[u] = (uint32_t)(k - q * jo.rn);
                    const unsigned long long qq = q - jo.qbase;
                    q32[u] = (uint32_t)qq;
                    if (ROUTE == 1 && BUILD && take[u]) {          // (every build key: a retry's window)
                        kmin = k < kmin ? k : kmin;
                        kmax = k > kmax ? k : kmax;
                    }
                    if (take[u] && (q < jo.qbase || qq >= 0xFFFFFFFFull)) {
                        take[u] = false;                          // (probe: matches no build key)
                        if (ROUTE == 1 && BUILD) sflag |= 16u;
                    }
                    if (ROUTE >= 2 && !BUILD && take[u] && pay[u] != JX_NOVAL &&
                        ((long long)pay[u] < -2147483647ll || (long long)pay[u] > 2147483647ll))
                        sflag |= 512u;                            // (still written: the flag drops the exchange)
                }
                const uint32_t nd = __builtin_amdgcn_readfirstlane(jo.rn);
                const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
                uint32_t pos[RP];
#pragma unroll
                for (int u = 0; u < RP; u++) pos[u] = 0;
                if (nd <= 8u) {
                    // one packed histogram per lane (8-bit fields, destinations 0-3 / 4-7 in
                    // two words; at most 64 * RP <= 192 per field) and two wave scans of it,
                    // instead of a ballot and popcount per destination and record: the
                    // scans' totals are each destination's entries this pass (lane d's
                    // running count); emit: the exclusive scans are the entries of the lanes
                    // below per destination -- a record's file-order rank in its run is that
                    // plus this lane's earlier records of the same destination
                    uint32_t h0 = 0, h1 = 0;
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        const uint32_t one = take[u] ? 1u << (8u * (dd[u] & 3u)) : 0u;
                        h0 += dd[u] < 4u ? one : 0u;
                        h1 += dd[u] < 4u ? 0u : one;
                    }
                    const uint32_t s0 = wave_incl_scan(h0), s1 = wave_incl_scan(h1);
                    const uint32_t t0 = __builtin_amdgcn_readlane(s0, 63), t1 = __builtin_amdgcn_readlane(s1, 63);
                    if constexpr (ROUTE == 2) {
                        const uint32_t e0 = s0 - h0, e1 = s1 - h1;        // exclusive: the lanes below
                        const int base = (int)(rbase + rrun);               // lane d: destination d's next
#pragma unroll
                        for (int u = 0; u < RP; u++) {
                            const uint32_t d = dd[u] & 7u;
                            uint32_t mine = 0;
#pragma unroll
                            for (int v = 0; v < u; v++) mine += (take[v] && dd[v] == dd[u]) ? 1u : 0u;
                            const uint32_t below = ((d < 4u ? e0 : e1) >> (8u * (d & 3u))) & 0xFFu;
                            const uint32_t b = (uint32_t)__shfl(base, (int)d, 64);
                            pos[u] = b + below + mine;
                        }
                    }
                    const uint32_t tw = lane < 4 ? t0 : t1;
                    const uint32_t td = (uint32_t)lane < nd ? (tw >> (8u * ((uint32_t)lane & 3u))) & 0xFFu : 0u;
                    rrun += td;
                    if constexpr (ROUTE == 3) {
                        // lane d: a new chunk when the current one cannot take this pass's
                        // entries for d; an entry of rank r among them lands at cur + r in the
                        // old chunk while r < room, else at the new chunk's r - room
                        const uint32_t room = cend - ccur;
                        uint32_t nb = 0;
                        if (td > room) nb = atomicAdd(&jo.rcnt[(uint32_t)lane * 64u], JX_RCHUNK);
                        const uint32_t e0 = s0 - h0, e1 = s1 - h1;
#pragma unroll
                        for (int u = 0; u < RP; u++) {
                            const uint32_t d = dd[u] & 7u;
                            uint32_t mine = 0;
#pragma unroll
                            for (int v = 0; v < u; v++) mine += (take[v] && dd[v] == dd[u]) ? 1u : 0u;
                            const uint32_t r = (((d < 4u ? e0 : e1) >> (8u * (d & 3u))) & 0xFFu) + mine;
                            const uint32_t cd = (uint32_t)__shfl((int)ccur, (int)d, 64);
                            const uint32_t rd = (uint32_t)__shfl((int)room, (int)d, 64);
                            const uint32_t bd = (uint32_t)__shfl((int)nb, (int)d, 64);
                            pos[u] = r < rd ? cd + r : bd + (r - rd);
                        }
                        if (td > room) {
                            ccur = nb + (td - room);
                            cend = nb + JX_RCHUNK;
                        } else {
                            ccur += td;
                        }
                    }
                } else
                for (uint32_t d = 0; d < nd; d++) {
                    uint64_t m[RP];
                    uint32_t tot = 0;
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        m[u] = __ballot(take[u] && dd[u] == d);
                        tot += (uint32_t)__popcll(m[u]);
                    }
                    if (tot == 0) continue;
                    if constexpr (ROUTE == 2) {
                        // file order within the window's run for d: the lanes below's records,
                        // then this lane's earlier ones (entries in global-id order: the
                        // receiver's STAR sees its build keys rise when the ids do)
                        const uint32_t pre = __builtin_amdgcn_readlane(rbase, d) + __builtin_amdgcn_readlane(rrun, d);
                        uint32_t below = 0;
#pragma unroll
                        for (int u = 0; u < RP; u++) below += (uint32_t)__popcll(m[u] & lt);
                        uint32_t mine = 0;
#pragma unroll
                        for (int u = 0; u < RP; u++) {
                            if ((m[u] >> lane) & 1ull) pos[u] = pre + below + mine++;
                        }
                    }
                    rrun += (uint32_t)lane == d ? tot : 0u;
                }
                if constexpr (ROUTE == 3) {
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        if (!take[u]) continue;
                        if (pos[u] >= jo.cap) { sflag |= 1024u; continue; }     // (the region is full)
                        const uint32_t p32 = pay[u] == JX_NOVAL ? JX_PNULL : (uint32_t)pay[u];
                        ((uint2*)jo.rent)[(uint64_t)(dd[u] & 7u) * jo.cap + pos[u]] = make_uint2(q32[u], p32);
                    }
                }
                if constexpr (ROUTE == 2) {
#pragma unroll
                    for (int u = 0; u < RP; u++) {
                        if (!take[u]) continue;
                        if (BUILD) {
                            ((uint4*)jo.rent)[pos[u]] = make_uint4(q32[u], gid[u], (uint32_t)pay[u], (uint32_t)(pay[u] >> 32));
                        } else {
                            const uint32_t p32 = pay[u] == JX_NOVAL ? JX_PNULL : (uint32_t)pay[u];
                            ((uint2*)jo.rent)[pos[u]] = make_uint2(q32[u], p32);
                        }
                    }
                }
            } else {
#pragma unroll
                for (int u = 0; u < RP; u++) {
                    if (valid[u]) {
                        const uint32_t at = at_next++;
                        if (at < jo.cap) {
                            jo.key[at] = key[u];
                            jo.pay[at] = pay[u];
                            jo.off[at] = (uint32_t)(wbase + p[u]);
                        }
                        if (key[u] != JX_NULLKEY) {
                            kmin = key[u] < kmin ? key[u] : kmin;
                            kmax = key[u] > kmax ? key[u] : kmax;
                        }
                    }
                }
            }
        }
        if (!issued && i + wstep < nwin) {
            uint32_t ni = i + wstep;
            asm volatile("" : "+s"(ni));
            load_win(g, first_win + ni, wsb, wlds, voff, prev_next);
        }
        if constexpr (ROUTE == 1) {
            if ((uint32_t)lane < jo.rn) jo.rcnt[(uint64_t)lane * nwin + i] = rrun;
        }
        if constexpr (STAR && BUILD) {
            // keys rising across the lanes too; the window's first and last for the
            // order check between windows (an empty window: not checked, not rising)
            const uint64_t am = __ballot(lany);
            const uint64_t above = lane < 63 ? am >> (lane + 1) : 0ull;
            const uint32_t nfirst = (uint32_t)__shfl((int)lfirst, above ? (int)(lane + 1 + __builtin_ctzll(above)) : lane, 64);
            lbad = lbad || (lany && above && llast >= nfirst);
            const unsigned long long wf = (uint32_t)__shfl((int)lfirst, am ? __builtin_ctzll(am) : 0, 64);
            const unsigned long long wl = (uint32_t)__shfl((int)llast, am ? 63 - __builtin_clzll(am) : 0, 64);
            if (lane == 0) {
                jo.wfl[2 * (uint64_t)i] = am ? wf : ~0ull;
                jo.wfl[2 * (uint64_t)i + 1] = am ? wl : 0ull;
            }
            if ((__any(lbad) || !am) && lane == 0) atomicOr(jo.notmono, 1u);
        }
    }
    if (COUNT) return;
    if constexpr (ROUTE == 3) {                   // this wave's chunk tails: holes
        const uint32_t nd = __builtin_amdgcn_readfirstlane(jo.rn);
        for (uint32_t d = 0; d < nd; d++) {
            const uint32_t a = __builtin_amdgcn_readlane(ccur, d), b = __builtin_amdgcn_readlane(cend, d);
            for (uint32_t q = a + (uint32_t)lane; q < b && q < jo.cap; q += 64u)
                ((uint2*)jo.rent)[(uint64_t)d * jo.cap + q] = make_uint2(~0u, JX_PNULL);
        }
    }
    if (__any(bad) && lane == 0) atomicOr(jo.flag, 1u);
    if constexpr (STAR || ROUTE) {
        for (int o = 32; o > 0; o >>= 1) {
            sflag |= (uint32_t)__shfl_down((int)sflag, o, 64);
            nstar += __shfl_down(nstar, o, 64);
        }
        if (lane == 0 && sflag) atomicOr(jo.flag, sflag);
        if (lane == 0 && nstar) atomicAdd(jo.nbuilt, nstar);   // build: placed; probe: pairs
    }
    if constexpr (PART) {
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < jo.np; k += LT)
            jo.pcnt[(size_t)blockIdx.x * jo.np + k] = min(pcl[k], jo.pcap);
        return;
    }
    if constexpr (SPROBE) {
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < NG; k += LT) {
            if (!scnt[k]) continue;
            if (mono) atomicMin(&jo.gminix[k], smix[k]);
            atomicAdd(&jo.gsum[3 * k], (unsigned long long)scnt[k]);
            if (snum[k]) {
                atomicAdd(&jo.gsum[3 * k + 1], sfix[k]);
                atomicAdd(&jo.gsum[3 * k + 2], (unsigned long long)snum[k]);
            }
        }
        return;
    }
    if constexpr (STAR && BUILD) {            // slots back to keys: kmin + slot * S
        if (smin != ~0u) {
            const unsigned long long a = jo.kmin + (unsigned long long)smin * jo.stride;
            const unsigned long long b = jo.kmin + (unsigned long long)smax * jo.stride;
            kmin = a < kmin ? a : kmin;
            kmax = b > kmax ? b : kmax;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long a = __shfl_down(kmin, o, 64), b = __shfl_down(kmax, o, 64);
        kmin = a < kmin ? a : kmin;
        kmax = b > kmax ? b : kmax;
    }
    if (lane == 0 && kmin != ~0ull) {
        atomicMin(&jo.krange[0], kmin);
        atomicMax(&jo.krange[1], kmax);
    }
}

// Partitioned STAR probe, pass 2: the entries of key partition p (d16 slots
// [p << psh, (p + 1) << psh): a 2 MiB slice) are looked up by the blocks of one XCD
// only -- blocks b and b + 8 share an XCD (MI355X_MICROARCH.md, workgroup dispatch),
// so block b takes partitions b % 8, b % 8 + 8, ... -- and every block of that XCD
// works on the same partition at once, so its slice stays in the XCD's 4 MiB L2
// instead of each lookup fetching a random line from HBM.  The matches aggregate as
// the unpartitioned probe's do: per group id COUNT / fixed-point SUM / SUM count in
// LDS, the smallest matched key index (rising build keys) or the d16 match flag.
__global__ __launch_bounds__(1024) void jx_part_probe_kernel(const unsigned long long* __restrict__ pent,
                                                             const uint32_t* __restrict__ pcnt, uint32_t nsrc,
                                                             uint32_t np, uint32_t pcap, uint64_t range,
                                                             uint16_t* __restrict__ d16,
                                                             const uint32_t* __restrict__ notmono,
                                                             unsigned long long* __restrict__ gsum,
                                                             uint32_t* __restrict__ gminix,
                                                             unsigned long long* __restrict__ npairs) {
    // per group: fixed-point sum, count, NULL-payload count (the SUM count is count -
    // NULLs: one LDS atomic fewer per match), smallest matched key index
    __shared__ unsigned long long sfix[JX_G];
    __shared__ uint32_t scnt[JX_G], snul[JX_G], smix[JX_G];
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x) { sfix[k] = 0; scnt[k] = 0; snul[k] = 0; smix[k] = ~0u; }
    const bool mono = __builtin_amdgcn_readfirstlane(*notmono) == 0u;
    __syncthreads();
    const uint32_t x = blockIdx.x & 7u, sub = blockIdx.x >> 3, nsub = gridDim.x >> 3;
    unsigned long long pairs = 0;
    // Work items of partition p: chunks of CH entries of the block's segments (sources
    // sub, sub + nsub, ...), SEG segments at a time; wave w takes items w, w + NW, ...
    // A chunk is one segment's entries [c * CH, c * CH + CH): every lane loads U of
    // them (lane-strided: coalesced), then their U d16 lookups, then the LDS updates,
    // so a lane keeps U independent loads in flight and the item -> (segment, chunk)
    // map is scalar work once per chunk, not vector work per entry.
    constexpr uint32_t U = 8, CH = 64 * U, SEG = 16, NW = 1024 / 64;
    __shared__ uint32_t sitem[SEG + 1], scount[SEG];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t p = x; p < np; p += 8) {
        for (uint32_t sb0 = sub; sb0 < nsrc; sb0 += SEG * nsub) {
            __syncthreads();                                   // (the last group's reads)
            if (threadIdx.x < 64) {
                const uint32_t sb = sb0 + threadIdx.x * nsub;
                const uint32_t n = threadIdx.x < SEG && sb < nsrc ? pcnt[(size_t)sb * np + p] : 0u;
                uint32_t c = (n + CH - 1) / CH;                  // chunks of this segment
                for (int o = 1; o < (int)SEG; o <<= 1) {
                    const uint32_t t = (uint32_t)__shfl_up((int)c, o, 64);
                    c += threadIdx.x >= (uint32_t)o ? t : 0u;
                }
                if (threadIdx.x < SEG) { sitem[threadIdx.x + 1] = c; scount[threadIdx.x] = n; }
                if (threadIdx.x == 0) sitem[0] = 0;
            }
            __syncthreads();
            const uint32_t items = __builtin_amdgcn_readfirstlane(sitem[SEG]);
            uint32_t sg = 0;
            for (uint32_t t = wv; t < items; t += NW) {
                while (sg + 1 < SEG && __builtin_amdgcn_readfirstlane(sitem[sg + 1]) <= t) sg++;   // (t rises)
                const uint32_t c0 = (t - __builtin_amdgcn_readfirstlane(sitem[sg])) * CH;
                const uint32_t n = __builtin_amdgcn_readfirstlane(scount[sg]);
                const unsigned long long* e = pent + ((size_t)(sb0 + sg * nsub) * np + p) * pcap;
                unsigned long long v[U];
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    const uint32_t i = c0 + u * 64 + lane;
                    v[u] = i < n ? __builtin_nontemporal_load(e + i) : ~0ull;
                }
                uint32_t gv[U];
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    const uint32_t ix = (uint32_t)v[u];
#ifdef PP_NOLOOK                                           // experiment: no d16 lookups (wrong results)
                    gv[u] = ix < range ? (ix & 1023u) + 1u : 0u;
#else
                    gv[u] = ix < range ? (uint32_t)d16[ix] : 0u;   // (a skipped entry: ~0)
#endif
                }
#ifdef PP_NOATOM                                           // experiment: no LDS updates (wrong results)
#pragma unroll
                for (uint32_t u = 0; u < U; u++) pairs += gv[u] ? 1u : 0u;
                continue;
#endif
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    if (!gv[u]) continue;
                    const uint32_t ix = (uint32_t)v[u], p32 = (uint32_t)(v[u] >> 32);
                    const uint32_t gi = (gv[u] & 0x7FFFu) - 1u;
                    if (mono) {
                        if (ix < smix[gi]) atomicMin(&smix[gi], ix);
                    } else if (!(gv[u] & 0x8000u)) {
                        d16[ix] = (uint16_t)(gv[u] | 0x8000u);     // (every writer: the same value)
                    }
                    atomicAdd(&scnt[gi], 1u);
                    // (signed: a typed entry's payload may be negative; the CSV pass 1's are < 2^31)
                    if (p32 != JX_PNULL) atomicAdd(&sfix[gi], (unsigned long long)(long long)(int32_t)p32);
                    else atomicAdd(&snul[gi], 1u);
                    pairs++;
                }
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) pairs += __shfl_down(pairs, o, 64);
    if ((threadIdx.x & 63) == 0 && pairs) atomicAdd(npairs, pairs);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x) {
        if (!scnt[k]) continue;
        if (mono) atomicMin(&gminix[k], smix[k]);
        atomicAdd(&gsum[3 * k], (unsigned long long)scnt[k]);
        const uint32_t num = scnt[k] - snul[k];
        if (num) {
            atomicAdd(&gsum[3 * k + 1], sfix[k]);
            atomicAdd(&gsum[3 * k + 2], (unsigned long long)num);
        }
    }
}

// STAR, after the build: the windows' keys in file order (first of window i + 1 above
// the last of window i); a fall sets *notmono (then the probe flags the matched keys)
__global__ void jx_star_order_kernel(const unsigned long long* __restrict__ wfl, uint64_t nwin,
                                     uint32_t* __restrict__ notmono) {
    bool bad = false;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w + 1 < nwin;
         w += (uint64_t)gridDim.x * blockDim.x)
        bad = bad || wfl[2 * w + 1] >= wfl[2 * (w + 1)];
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(notmono, 1u);
}

// STAR, before the build: every per-query array in one launch (instead of a fill
// per array and a copy of the tag seed): d16 zero over the key range, the small
// block zero except its 0xFF run [ff0, ff1) (16-byte granular) and the 8-byte word
// at ffw, the tag table from the seed when there is one
__global__ void jx_star_init_kernel(uint4* __restrict__ d16, uint64_t n16, uint4* __restrict__ small, uint32_t nsmall16,
                                    uint32_t ff0, uint32_t ff1, uint32_t ffw, const uint4* __restrict__ seed,
                                    uint32_t nseed16) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u), f = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (uint64_t i = t; i < nsmall16; i += nt) {
        const uint32_t b = (uint32_t)i * 16u;
        uint4 v = (b >= ff0 && b < ff1) ? f : (seed && i < nseed16 ? seed[i] : z);
        if (ffw == b) { v.x = ~0u; v.y = ~0u; }
        if (ffw == b + 8u) { v.z = ~0u; v.w = ~0u; }
        small[i] = v;
    }
    for (uint64_t i = t; i < n16; i += nt) d16[i] = z;
}

// STAR without rising build keys: each group's first pair in (l, r) order has the
// group's smallest matched build record l (the probe flagged the matched keys in d16).
// Also counts the occupied keys: fewer than the records placed means a repeated key.
__global__ __launch_bounds__(1024) void jx_star_first_kernel(const uint16_t* __restrict__ d16,
                                                             const uint32_t* __restrict__ l32, uint64_t range,
                                                             const uint32_t* __restrict__ notmono,
                                                             uint32_t* __restrict__ gfirst,
                                                             unsigned long long* __restrict__ nocc) {
    if (!*notmono) return;
    __shared__ uint32_t sf[JX_G];
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x) sf[k] = ~0u;
    __syncthreads();
    unsigned long long occ = 0;
    const auto take = [&](uint32_t gv, uint32_t l) {
        occ += gv != 0u;
        if (gv & 0x8000u) {
            const uint32_t gi = (gv & 0x7FFFu) - 1u;
            if (l < sf[gi]) atomicMin(&sf[gi], l);        // (an atomic only when it lowers)
        }
    };
    const uint64_t n8 = range / 8;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n8; w += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 dv = ((const uint4*)d16)[w];             // 8 group ids
        const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w};
        if (((dv.x | dv.y | dv.z | dv.w) & 0x80008000u) == 0u) {   // nothing matched here
#pragma unroll
            for (int j = 0; j < 4; j++) occ += ((dw[j] & 0xFFFFu) != 0u) + ((dw[j] >> 16) != 0u);
            continue;
        }
        const uint4 la = ((const uint4*)l32)[2 * w], lb = ((const uint4*)l32)[2 * w + 1];
        const uint32_t lv[8] = {la.x, la.y, la.z, la.w, lb.x, lb.y, lb.z, lb.w};
#pragma unroll
        for (int j = 0; j < 8; j++) take((dw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu, lv[j]);
    }
    for (uint64_t ix = n8 * 8 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; ix < range;
         ix += (uint64_t)gridDim.x * blockDim.x)
        take(d16[ix], l32[ix]);
    for (int o = 32; o > 0; o >>= 1) occ += __shfl_down(occ, o, 64);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd(nocc, occ);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x)
        if (sf[k] != ~0u) atomicMin(&gfirst[k], sf[k]);
}

// STAR: the per-group sums into the join's group table (raw tags -> raw_merge_kernel,
// as jx_probe_kernel's flush; ungrouped: the one GK_ALL group); a repeated build key
// (occupied keys != records placed) sets flag 64 and nothing is written
template <bool GROUPED, bool VALUE>
__global__ __launch_bounds__(1024) void jx_star_flush_kernel(const unsigned long long* __restrict__ ttab,
                                                             const unsigned long long* __restrict__ gsum,
                                                             const uint32_t* __restrict__ gfirst,
                                                             const uint32_t* __restrict__ gminix,
                                                             const uint32_t* __restrict__ l32,
                                                             const uint32_t* __restrict__ notmono,
                                                             const unsigned long long* __restrict__ cnts,
                                                             GroupTable rt, int nacc, ScanStats* __restrict__ stats,
                                                             unsigned int* __restrict__ flag) {
    // cnts: [0] build records placed, [1] pairs, [2] occupied keys (counted when the
    // build keys do not rise in file order; rising keys are distinct)
    const bool mono = *notmono == 0u;
    if (!mono && cnts[0] != cnts[2]) {
        if (threadIdx.x == 0) atomicOr(flag, 64u);
        return;
    }
    if (threadIdx.x == 0 && cnts[1]) atomicAdd(&stats->passed, cnts[1]);
    for (uint32_t s = threadIdx.x; s < (GROUPED ? JX_G : 1u); s += blockDim.x) {
        const unsigned long long cnt = gsum[3 * s];
        if (!cnt) continue;
        GKey kk;
        if (GROUPED) {
            const unsigned long long w0 = ttab[s];
            const uint32_t kl = key_len8(w0);
            kk = raw_key(kl, kl ? w0 : 0ull);
        } else {
            kk.cls = GK_ALL; kk.len = 0; kk.w0 = 0; kk.w1 = 0;
        }
        const int gi = g_insert(rt, kk, GROUPED ? gk_hash(kk) : 0x12345678ULL, stats);
        if (gi < 0) continue;
        atomicAdd(&rt.cnt[gi], cnt);
        const uint32_t first = mono ? l32[gminix[s]] : gfirst[s];
        atomicMin(&rt.first[gi], (unsigned long long)first << 32);
        if (VALUE && gsum[3 * s + 2]) {
            for (int a = 0; a < nacc; a++) {
                atomicAdd(&rt.sum[a][gi], (double)(long long)gsum[3 * s + 1] / 1000.0);
                atomicAdd(&rt.num[a][gi], gsum[3 * s + 2]);
            }
        }
    }
}


// ------------------------------------------------------------------ STAR over typed entries
// The receiving rank of the typed exchange (jx_extract_kernel ROUTE): the same STAR
// arrays as the CSV form -- d16 (group id + 1, bit 15 once a probe entry matched),
// l32 (here the build record's GLOBAL id, so a group's first pair needs no offset
// lookup), the GROUP BY tag table ttab, per group COUNT / fixed-point SUM / SUM count
// in gsum -- filled from the fixed-size entries instead of re-parsing CSV.  Slot =
// q32 - qoff (one residue class of a dense key range: key mod N routing).
// Flags: 16 a q32 outside [qoff, qoff + range), 32 more tags than JX_G.
__global__ __launch_bounds__(1024) void jx_ent_build_kernel(const uint4* __restrict__ ent, uint64_t n, uint32_t qoff,
                                                            uint64_t range, uint16_t* __restrict__ d16,
                                                            uint32_t* __restrict__ l32,
                                                            unsigned long long* __restrict__ ttab,
                                                            unsigned long long* __restrict__ nplaced,
                                                            unsigned int* __restrict__ flag, uint32_t ungrouped,
                                                            uint32_t* __restrict__ notmono) {
    __shared__ unsigned long long lt[JX_G];       // the block's mirror of the tag table
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x) lt[k] = ttab[k];
    __syncthreads();
    uint32_t fl = 0;
    unsigned long long placed = 0;
    bool fall = false;
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    // (latency-bound at two entries in flight per thread: SQ_WAIT_ANY / SQ_WAVE_CYCLES 0.72,
    // profiles/r6_pmc.json; JXB_U entries in flight, streamed past the caches)
#ifndef JXB_U
#define JXB_U 4
#endif
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += JXB_U * nt) {
        uint4 e[JXB_U];
        uint32_t nq[JXB_U];
        bool ok[JXB_U];
#pragma unroll
        for (int u = 0; u < JXB_U; u++) {
            ok[u] = i + u * nt < n;
            const v4u x = ok[u] ? __builtin_nontemporal_load((const v4u*)(ent + i + u * nt)) : v4u{0u, 0u, 0u, 0u};
            e[u] = make_uint4(x.x, x.y, x.z, x.w);
            // the next entry's q32 (lanes 0-62: the line the next lane loads; measured
            // against a ds_bpermute of the next lane's entry, which competed with the tag
            // lookups' LDS: 0.69 -> 0.75 ms)
            nq[u] = i + u * nt + 1 < n ? ((const uint32_t*)(ent + i + u * nt + 1))[0] : ~0u;
        }
#pragma unroll
        for (int u = 0; u < JXB_U; u++) {
            if (!ok[u]) continue;
            const uint64_t slot = (uint64_t)(uint32_t)(e[u].x - qoff);
            if (e[u].x < qoff || slot >= range) { fl |= 16u; continue; }
            bool full = false;
            const unsigned long long tag = (unsigned long long)e[u].z | ((unsigned long long)e[u].w << 32);
            const uint32_t gid = ungrouped ? 0u : jx_tag_gid_lds(lt, ttab, tag, full);
            if (full) { fl |= 32u; continue; }
            d16[slot] = (uint16_t)(gid + 1u);
            l32[slot] = e[u].y;
            placed++;
            // the entries come in global-id order (sources in rank order, each in file
            // order): slots rising along them mean a group's smallest matched slot is its
            // smallest matched id -- the probe then needs no match flags in d16
            if (nq[u] <= e[u].x) fall = true;
        }
    }
    if (__any(fall) && (threadIdx.x & 63) == 0) atomicOr(notmono, 1u);
    for (int o = 32; o > 0; o >>= 1) {
        fl |= (uint32_t)__shfl_down((int)fl, o, 64);
        placed += __shfl_down(placed, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (fl) atomicOr(flag, fl);
        if (placed) atomicAdd(nplaced, placed);
    }
}

// the rising-keys form's first pairs: each group's smallest matched slot -> its id
__global__ void jx_ent_first_kernel(const uint32_t* __restrict__ gminix, const uint32_t* __restrict__ l32,
                                    const uint32_t* __restrict__ notmono, uint32_t* __restrict__ gfirst) {
    if (*notmono) return;
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x) gfirst[k] = gminix[k] != ~0u ? l32[gminix[k]] : ~0u;
}

// partitioned probe over typed entries, pass 1: every probe entry whose slot (q32 -
// qoff) is inside the build range, as {slot, payload} into its key partition's segment
// (slot >> psh) of this block -- the layout jx_part_probe_kernel (pass 2: each XCD's
// blocks look one 2 MiB d16 slice up at a time, in its L2) reads.  An entry past its
// segment's capacity sets flag 128 (the caller reruns unpartitioned).  Entries are
// read in block-contiguous runs, so a block's segments fill in entry order.
__global__ __launch_bounds__(1024) void jx_ent_part_kernel(const uint2* __restrict__ ent, uint64_t n, uint32_t qoff,
                                                           uint64_t range, uint32_t np, uint32_t pcap, uint32_t psh,
                                                           unsigned long long* __restrict__ pent,
                                                           uint32_t* __restrict__ pcnt, unsigned int* __restrict__ flag) {
    extern __shared__ uint32_t pcl[];                // per partition: this block's entries so far
    for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pcl[k] = 0;
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n, lo + per);
    unsigned long long* seg = pent + (size_t)blockIdx.x * np * pcap;
    bool over = false;
    constexpr int U = 4;                             // entries in flight per thread
    for (uint64_t i = lo + threadIdx.x; i < hi; i += U * blockDim.x) {
        uint2 e[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const unsigned long long v =
                i + u * blockDim.x < hi ? __builtin_nontemporal_load((const unsigned long long*)ent + i + u * blockDim.x) : 0ull;
            e[u] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t slot = e[u].x - qoff;
            if (i + u * blockDim.x >= hi || e[u].x < qoff || (uint64_t)slot >= range) continue;
            const uint32_t pr = slot >> psh;
            const uint32_t at = atomicAdd(&pcl[pr], 1u);
            if (at < pcap) seg[(size_t)pr * pcap + at] = (unsigned long long)slot | ((unsigned long long)e[u].y << 32);
            else over = true;
        }
    }
    if (__any(over) && (threadIdx.x & 63) == 0) atomicOr(flag, 128u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pcnt[(size_t)blockIdx.x * np + k] = min(pcl[k], pcap);
}

// probe: every entry's slot looked up in d16 (bit 15 set on a first match, for
// jx_star_first_kernel), its pair added to the block's per-group LDS sums, then the
// sums into gsum; npairs: the pairs found
__global__ __launch_bounds__(1024) void jx_ent_probe_kernel(const uint2* __restrict__ ent, uint64_t n, uint32_t qoff,
                                                            uint64_t range, uint16_t* __restrict__ d16,
                                                            unsigned long long* __restrict__ gsum,
                                                            unsigned long long* __restrict__ npairs,
                                                            const uint32_t* __restrict__ notmono,
                                                            uint32_t* __restrict__ gminix) {
    __shared__ unsigned long long sfix[JX_G];
    __shared__ uint32_t scnt[JX_G], snum[JX_G], smix[JX_G];
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x) { sfix[k] = 0; scnt[k] = 0; snum[k] = 0; smix[k] = ~0u; }
    // rising build keys (jx_ent_build_kernel): the smallest matched slot per group in
    // LDS instead of the d16 match flags
    const bool mono = __builtin_amdgcn_readfirstlane(*notmono) == 0u;
    __syncthreads();
    unsigned long long pairs = 0;
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    constexpr int U = 4;                              // entries in flight per thread
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += U * nt) {
        uint2 e[U];
        uint32_t gv[U];
        uint64_t slot[U];
#pragma unroll
        for (int u = 0; u < U; u++) e[u] = i + u * nt < n ? ent[i + u * nt] : make_uint2(0xFFFFFFFFu, 0u);
#pragma unroll
        for (int u = 0; u < U; u++) {
            slot[u] = (uint64_t)(uint32_t)(e[u].x - qoff);
#if PROBE_EXP == 2
            slot[u] = (i + u * nt) % range;
#endif
            const bool in = e[u].x >= qoff && slot[u] < range;
            gv[u] = in ? (uint32_t)d16[slot[u]] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (!gv[u]) continue;
            const uint32_t gi = (gv[u] & 0x7FFFu) - 1u;
#if !defined(PROBE_EXP) || PROBE_EXP == 0
            if (mono) {
                if ((uint32_t)slot[u] < smix[gi]) atomicMin(&smix[gi], (uint32_t)slot[u]);
            } else if (!(gv[u] & 0x8000u)) {
                d16[slot[u]] = (uint16_t)(gv[u] | 0x8000u);   // (every writer: the same value)
            }
#endif
            atomicAdd(&scnt[gi], 1u);
            if (e[u].y != JX_PNULL) {
                atomicAdd(&sfix[gi], (unsigned long long)(long long)(int32_t)e[u].y);
                atomicAdd(&snum[gi], 1u);
            }
            pairs++;
        }
    }
    for (int o = 32; o > 0; o >>= 1) pairs += __shfl_down(pairs, o, 64);
    if ((threadIdx.x & 63) == 0 && pairs) atomicAdd(npairs, pairs);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < JX_G; k += blockDim.x) {
        if (!scnt[k]) continue;
        if (mono) atomicMin(&gminix[k], smix[k]);
        atomicAdd(&gsum[3 * k], (unsigned long long)scnt[k]);
        if (snum[k]) {
            atomicAdd(&gsum[3 * k + 1], sfix[k]);
            atomicAdd(&gsum[3 * k + 2], (unsigned long long)snum[k]);
        }
    }
}

// ------------------------------------------------------------------ fused join: build, probe + aggregate
// The build side's keys into an open-addressing table of 16-byte entries (stored key
// + 2, so 0 is free; the build record's index), every record its own entry (equal keys
// occupy consecutive probes: many-to-many pairs are all found).
struct JxEntry {
    unsigned long long k;
    uint32_t idx, pad;
};
__device__ __forceinline__ uint64_t jx_hash(unsigned long long k) {
    uint64_t x = k * 0x9E3779B97F4A7C15ull;
    return x ^ (x >> 29);
}
__global__ void jx_build_kernel(const unsigned long long* __restrict__ key, uint32_t n, JxEntry* __restrict__ T,
                                uint64_t mask, unsigned int* __restrict__ flag) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const unsigned long long k = key[i], sk = k + 2ull;
        uint64_t h = jx_hash(k) & mask;
        for (uint64_t probes = 0;; probes++) {
            if (probes > mask) { atomicOr(flag, 2u); break; }
            const unsigned long long old = atomicCAS(&T[h].k, 0ull, sk);
            if (old == 0ull) { T[h].idx = i; break; }
            h = (h + 1) & mask;
        }
    }
}

// Build keys of a dense range (the usual primary key): entry D[key - kmin] holds the
// build record's payload and byte offset, so a probe reads one 16-byte entry.  A NULL
// key or a repeated key (flag 8) sends the caller to the hash table.
struct JxDirect {
    unsigned long long pay;
    uint32_t off, used;
};
__global__ void jx_build_direct_kernel(const unsigned long long* __restrict__ key,
                                       const unsigned long long* __restrict__ pay, const uint32_t* __restrict__ off,
                                       uint32_t n, unsigned long long kmin, unsigned long long range,
                                       JxDirect* __restrict__ D, unsigned int* __restrict__ flag) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const unsigned long long k = key[i];
        if (k == JX_NULLKEY || k - kmin >= range) { atomicOr(flag, 8u); continue; }
        JxDirect& e = D[k - kmin];
        if (atomicCAS(&e.used, 0u, 1u) != 0u) { atomicOr(flag, 8u); continue; }
        e.pay = pay[i];
        e.off = off[i];
    }
}

// Probe side records: every pair (build record l, probe record r) with equal keys,
// in any order, aggregated per GROUP BY raw tag (the build record's payload) into a
// block-local LDS table: COUNT, the SUM argument's fixed-point sum and count (the
// probe record's payload), and the first pair in (l, r) order as the key
// (l byte offset << 32) | r byte offset.  Flushed into the HBM raw-key table, which
// raw_merge_kernel canonicalises (GROUP BY typing) like fast_kernel's.
constexpr uint32_t JX_SLOTS = 2048;
template <bool GROUPED, bool VALUE, bool DIRECT>
__global__ __launch_bounds__(1024) void jx_probe_kernel(const unsigned long long* __restrict__ pkey,
                                                        const unsigned long long* __restrict__ ppay,
                                                        const uint32_t* __restrict__ poff,
                                                        uint32_t n, unsigned long long kmin,
                                                        const JxEntry* __restrict__ T, uint64_t mask,
                                                        const unsigned long long* __restrict__ bpay,
                                                        const uint32_t* __restrict__ boff, GroupTable rt, int nacc,
                                                        ScanStats* __restrict__ stats, unsigned int* __restrict__ flag) {
    __shared__ unsigned long long stag[JX_SLOTS], sfix[JX_SLOTS], sfirst[JX_SLOTS];
    __shared__ uint32_t scnt[JX_SLOTS], snum[JX_SLOTS];
    constexpr uint32_t NS = GROUPED ? JX_SLOTS : 1;
    for (uint32_t s = threadIdx.x; s < NS; s += blockDim.x) {
        stag[s] = 0; sfix[s] = 0; sfirst[s] = ~0ull; scnt[s] = 0; snum[s] = 0;
    }
    __syncthreads();
    bool full = false;
    unsigned long long npairs = 0;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        const unsigned long long k = pkey[r], sk = k + 2ull;
        const unsigned long long v = VALUE ? ppay[r] : 0ull;
        const uint32_t ro = poff[r];
        uint64_t h = DIRECT ? k - kmin : jx_hash(k) & mask;
        for (uint64_t probes = 0; probes <= mask; probes++) {
            uint32_t l = 0;
            bool hit;
            unsigned long long btag = 0;
            uint32_t boffv = 0;
            if (DIRECT) {                    // one entry per key: T is the JxDirect array D
                if (k != JX_NULLKEY && h <= mask) {
                    const JxDirect e = ((const JxDirect*)T)[h];
                    hit = e.used != 0u;
                    btag = e.pay;
                    boffv = e.off;
                } else {
                    hit = false;
                }
            } else {
                const JxEntry e = T[h];
                if (e.k == 0ull) break;
                hit = e.k == sk;
                l = e.idx;
            }
            if (hit) {
                if (!DIRECT) {
                    btag = GROUPED ? bpay[l] : 0ull;
                    boffv = boff[l];
                }
                const unsigned long long pk = ((unsigned long long)boffv << 32) | ro;
                uint32_t s = 0;
                if (GROUPED) {
                    const unsigned long long tag = btag;
                    s = fast_key_hash((uint32_t)tag, (uint32_t)(tag >> 32)) & (JX_SLOTS - 1);
                    for (uint32_t q = 0;; q++) {
                        if (q == JX_SLOTS) { full = true; break; }
                        const unsigned long long t = stag[s];
                        if (t == tag) break;
                        if (t == 0ull) {
                            const unsigned long long old = atomicCAS(&stag[s], 0ull, tag);
                            if (old == 0ull || old == tag) break;
                        }
                        s = (s + 1) & (JX_SLOTS - 1);
                    }
                    if (full) break;
                }
                atomicAdd(&scnt[s], 1u);
                if (pk < sfirst[s]) atomicMin(&sfirst[s], pk);   // (the first pair is found early)
                if (VALUE && v != JX_NOVAL) {
                    atomicAdd(&sfix[s], v);
                    atomicAdd(&snum[s], 1u);
                }
                npairs++;
            }
            if (DIRECT) break;
            h = (h + 1) & mask;
        }
    }
    if (full) atomicOr(flag, 4u);
    for (int o = 32; o > 0; o >>= 1) npairs += __shfl_down(npairs, o, 64);
    if ((threadIdx.x & 63) == 0 && npairs) atomicAdd(&stats->passed, npairs);
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < NS; s += blockDim.x) {
        if (!scnt[s]) continue;
        GKey kk;
        if (GROUPED) {
            const unsigned long long w0 = stag[s];
            const uint32_t kl = key_len8(w0);
            kk = raw_key(kl, kl ? w0 : 0ull);
        } else {
            kk.cls = GK_ALL; kk.len = 0; kk.w0 = 0; kk.w1 = 0;
        }
        const int gi = g_insert(rt, kk, GROUPED ? gk_hash(kk) : 0x12345678ULL, stats);
        if (gi < 0) continue;
        atomicAdd(&rt.cnt[gi], (unsigned long long)scnt[s]);
        atomicMin(&rt.first[gi], sfirst[s]);
        if (VALUE && snum[s]) {                 // every accumulator sums the one probe-side argument
            for (int a = 0; a < nacc; a++) {
                atomicAdd(&rt.sum[a][gi], (double)(long long)sfix[s] / 1000.0);
                atomicAdd(&rt.num[a][gi], (unsigned long long)snum[s]);
            }
        }
    }
}

}  // namespace fast
}  // namespace cq

// ------------------------------------------------------------------ host side
namespace {

using namespace cq;
using fast::FastPlan;

bool fcmp_result(uint32_t op, int c) {
    switch (op) {
        case CMP_EQ: return c == 0;
        case CMP_NE: return c != 0;
        case CMP_LT: return c < 0;
        case CMP_GT: return c > 0;
        case CMP_LE: return c <= 0;
        default: return c >= 0;
    }
}

// A compound WHERE for the WX builds: the post-order program (plan.h OP_*) read as a
// tree of NOT / AND / OR over leaves `column op literal` (either side), `column [NOT]
// IN (literals)` and constants; <= 4 leaves over <= 2 columns, each column's literals
// of one class (NUMBER: INTEGER / DOUBLE, negated by a unary minus or not; STRING: 1-8
// bytes).  The tree becomes a truth table over the leaves' outcomes (every leaf is
// evaluated, as evaluator_conditions.c:76-86 evaluates both sides).  `s`: the stream
// to read STRING literal bytes with (launch time), null at plan time.  wslot: the need
// slots of the WHERE columns.
namespace {
// the fixed-point field values V (exact 10^-3, < 10^7: <= 4-byte numerals) whose double
// RN(V / 1000) -- the strtod value parse_value gives the field -- compares >= (gt:
// >) the literal's double: the smallest such V (10^7 + 1: none)
uint32_t wx_first_v(double l, bool gt) {
    uint32_t lo = 0, hi = 10000001u;              // answer in [lo, hi]
    while (lo < hi) {
        const uint32_t m = lo + (hi - lo) / 2;
        const double v = (double)m / 1000.0;
        if (gt ? v > l : v >= l) hi = m;
        else lo = m + 1;
    }
    return lo;
}
bool wx_word(const Cell& L, hipStream_t s, uint64_t* w) {
    if (L.kind != K_STR || L.len < 1 || L.len > 8) return false;
    if (!s) { *w = 0; return true; }
    uint8_t b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyAsync(b, (const void*)(uintptr_t)L.bits, L.len, hipMemcpyDeviceToHost, s) != hipSuccess) return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    bool nul = false;
    uint64_t x = 0;
    for (int i = 0; i < 8; i++) {                 // strcmp stops at a NUL
        nul = nul || b[i] == 0;
        x = (x << 8) | (nul ? 0u : b[i]);
    }
    *w = x;
    return true;
}
}  // namespace

bool wx_compile(const ScanPlan* P, FastPlan* fp, int wslot[2], int* nwc, hipStream_t s) {
    if (getenv("CQGPU_NO_FAST_WX")) return false;
    struct It { int kind; int v; bool neg; };      // kind 0 column (v slot), 1 literal (v const), 2 tree (v table)
    It st[16];
    int sp = 0, nleaf = 0;
    *nwc = 0;
    int ccls[2] = {-1, -1};                        // per WHERE column: 0 NUMBER, 1 STRING
    auto colx = [&](int slot) -> int {
        for (int c = 0; c < *nwc; c++)
            if (wslot[c] == slot) return c;
        if (*nwc == 2) return -1;
        wslot[*nwc] = slot;
        return (*nwc)++;
    };
    auto leaf_table = [](int j) {
        uint32_t t = 0;
        for (uint32_t i = 0; i < 16; i++) t |= ((i >> j) & 1u) << i;
        return t;
    };
    auto number = [&](const It& x, double* v) {
        const Cell& L = P->consts[x.v];
        if (L.kind == K_INT) *v = (double)(int64_t)L.bits;
        else if (L.kind == K_DBL) memcpy(v, &L.bits, 8);
        else return false;
        if (x.neg) *v = -*v;
        return std::isfinite(*v);
    };
    for (int pc = 0; pc < P->nprog; pc++) {
        const Insn& in = P->prog[pc];
        if (sp >= 14) return false;
        switch (in.op) {
            case OP_COL: st[sp++] = It{0, (int)in.a, false}; break;
            case OP_CONST: st[sp++] = It{1, (int)in.b, false}; break;
            case OP_NEG:
                if (sp < 1 || st[sp - 1].kind != 1 || st[sp - 1].neg) return false;
                {
                    const Cell& L = P->consts[st[sp - 1].v];
                    if (L.kind != K_INT && L.kind != K_DBL) return false;
                    if (L.kind == K_INT && (int64_t)L.bits == INT64_MIN) return false;
                }
                st[sp - 1].neg = true;
                break;
            case OP_BOOL: st[sp++] = It{2, in.a ? 0xFFFF : 0, false}; break;
            case OP_NOT:
                if (sp < 1 || st[sp - 1].kind != 2) return false;
                st[sp - 1].v = ~st[sp - 1].v & 0xFFFF;
                break;
            case OP_AND: case OP_OR: {
                if (sp < 2 || st[sp - 1].kind != 2 || st[sp - 2].kind != 2) return false;
                const int r = st[--sp].v;
                st[sp - 1].v = in.op == OP_AND ? (st[sp - 1].v & r) : (st[sp - 1].v | r);
                break;
            }
            case OP_CMP: {
                if (sp < 2 || nleaf == 4) return false;
                It l = st[sp - 2], r = st[sp - 1];
                sp -= 2;
                uint32_t op = in.a;
                if (l.kind == 1 && r.kind == 0) {          // literal op column: mirror the operator
                    std::swap(l, r);
                    op = op == CMP_LT ? CMP_GT : op == CMP_GT ? CMP_LT : op == CMP_LE ? CMP_GE : op == CMP_GE ? CMP_LE : op;
                }
                if (l.kind != 0 || r.kind != 1) return false;
                const int c = colx(l.v);
                if (c < 0) return false;
                const int j = nleaf++;
                fp->lx_col[j] = (uint32_t)c;
                fp->lx_null[j] = fcmp_result(op, -1) ? 1u : 0u;     // NULL < any non-NULL
                uint64_t w;
                if (wx_word(P->consts[r.v], s, &w)) {
                    if (r.neg || ccls[c] == 0) return false;
                    ccls[c] = 1;
                    fp->lx_kind[j] = fast::LX_STR;
                    fp->lx_lit[j] = w;
                    fp->lx_tt[j] = (fcmp_result(op, -1) ? 1u : 0u) | (fcmp_result(op, 0) ? 2u : 0u) |
                                   (fcmp_result(op, 1) ? 4u : 0u);
                } else {
                    double lv;
                    if (!number(r, &lv) || ccls[c] == 1) return false;
                    ccls[c] = 0;
                    // V < Vlt <=> RN(V/1000) < l;  V < Vle <=> RN(V/1000) <= l
                    const int64_t vlt = wx_first_v(lv, false), vle = wx_first_v(lv, true);
                    const bool lt = fcmp_result(op, -1), eq = fcmp_result(op, 0), gt = fcmp_result(op, 1);
                    int64_t A, B;
                    fp->lx_kind[j] = fast::LX_NUM;
                    fp->lx_neg[j] = 0;
                    if (lt && !eq && gt) { fp->lx_neg[j] = 1; A = vlt; B = vle - 1; }
                    else if (!lt && !eq && !gt) { A = 1; B = 0; }
                    else {
                        A = lt ? 0 : (eq ? vlt : vle);
                        B = gt ? 10000000 : (eq ? vle - 1 : vlt - 1);
                    }
                    if (A > B) { fp->lx_a[j] = 0xFFFFFFFFu; fp->lx_w[j] = 0; }   // empty (V + 1 > 0)
                    else { fp->lx_a[j] = (uint32_t)A; fp->lx_w[j] = (uint32_t)(B - A); }
                }
                st[sp++] = It{2, (int)leaf_table(j), false};
                break;
            }
            case OP_IN: {
                const int k = in.b;
                if (k < 1 || k > 8 || sp < k + 1 || nleaf == 4) return false;
                const It l = st[sp - k - 1];
                if (l.kind != 0) return false;
                const int c = colx(l.v);
                if (c < 0) return false;
                const int j = nleaf++;
                fp->lx_col[j] = (uint32_t)c;
                fp->lx_neg[j] = in.a ? 1u : 0u;
                fp->lx_null[j] = in.a ? 1u : 0u;           // NULL matches no item: IN false, NOT IN true
                fp->lx_nin[j] = (uint32_t)k;
                for (int t = 0; t < k; t++) {
                    const It x = st[sp - k + t];
                    if (x.kind != 1) return false;
                    uint64_t w;
                    if (!x.neg && wx_word(P->consts[x.v], s, &w)) {
                        if (ccls[c] == 0) return false;
                        ccls[c] = 1;
                        fp->lx_in[j][t] = w;
                    } else {
                        double lv;
                        if (!number(x, &lv) || ccls[c] == 1) return false;
                        ccls[c] = 0;
                        const uint32_t vlt = wx_first_v(lv, false), vle = wx_first_v(lv, true);
                        fp->lx_in[j][t] = vlt < vle ? vlt : 0xFFFFFFFFu;     // the one V equal to it, or none
                    }
                }
                fp->lx_kind[j] = ccls[c] == 1 ? fast::LX_SIN : fast::LX_NIN;
                sp -= k + 1;
                st[sp++] = It{2, (int)leaf_table(j), false};
                break;
            }
            default:
                return false;
        }
    }
    if (sp != 1 || st[0].kind != 2 || nleaf == 0 || *nwc == 0) return false;
    fp->wx_nleaf = (uint32_t)nleaf;
    fp->wx_tt = (uint32_t)st[0].v;
    fp->wx_str = (ccls[0] == 1 ? 1u : 0u) | (ccls[1] == 1 ? 2u : 0u);
    // leaves beyond nleaf never run; the table ignores their bits (they read as 0)
    return true;
}

// fast_kernel's plan shape (see the file comment); fills the FastPlan fields that
// depend on the plan only
bool fast_shape(const ScanPlan* P, int grouped, FastPlan* fp, int* ns, bool* where, bool* canonical,
                bool* wide_num = nullptr, int* ext_out = nullptr, int* wx_out = nullptr, hipStream_t wx_s = nullptr) {
    if (P->nacc > MAX_ACC || P->ngpart > 0) return false;
    const uint32_t d = P->delim;
    if ((d - '0') < 10u || d == '.' || ((d | 32) >= 'a' && (d | 32) <= 'z') || d == '+' || d == '-') return false;
    if (d == '\n' || d == '\r' || d <= ' ') return false;
    if (P->quote == d || P->quote == '\n' || P->quote == '\r') return false;
    *fp = FastPlan{};
    fp->delim = d;
    fp->quote = P->quote;
    fp->nacc = P->nacc;
    int sslot[2] = {-1, -1};
    *ns = 0;
    // at most one MIN / MAX, over the one numeric argument of the plan (EXT builds)
    int ext = 0, ext_slot = -1;
    fp->ext_acc = -1;
    for (int a = 0; a < P->nacc; a++) {
        if (P->acc[a].kind == ACC_MIN || P->acc[a].kind == ACC_MAX) {
            if (ext || getenv("CQGPU_NO_FAST_EXT")) return false;
            ext = P->acc[a].kind == ACC_MIN ? 1 : 2;
            fp->ext_acc = a;
            ext_slot = P->acc[a].slot;
            continue;
        }
        if (P->acc[a].kind != ACC_SUM) return false;
        fp->sum_mask |= 1u << a;
        const int slot = P->acc[a].slot;
        int j = 0;
        while (j < *ns && sslot[j] != slot) j++;
        if (j == *ns) {
            if (*ns == 2) return false;
            sslot[(*ns)++] = slot;
        }
        if (j) fp->acc1 |= 1u << a;
    }
    if (ext) {
        if (*ns == 0) sslot[(*ns)++] = ext_slot;
        if (*ns != 1 || sslot[0] != ext_slot) return false;
        fp->ext_col = (uint32_t)P->need_col[ext_slot];
    }
    if (ext_out) *ext_out = ext;
    int wcol = -1, wcol1 = -1, wx = 0;
    if (P->nprog == 0) {
        *where = false;
    } else if (P->nprog == 3 && P->prog[0].op == OP_COL && P->prog[1].op == OP_CONST && P->prog[2].op == OP_CMP) {
        const Cell& L = P->consts[P->prog[1].b];
        const bool slit = L.kind == K_STR && L.len >= 1 && L.len <= 8;
        if (L.kind != K_INT && L.kind != K_DBL && !slit) return false;
        *where = true;
        wcol = P->need_col[P->prog[0].a];
        const uint32_t op = P->prog[2].a;
        fp->wtt = (fcmp_result(op, -1) ? 1u : 0u) | (fcmp_result(op, 0) ? 2u : 0u) | (fcmp_result(op, 1) ? 4u : 0u);
        fp->pass_null = fcmp_result(op, -1) ? 1u : 0u;             // NULL < any non-NULL
        if (slit) {   // (the literal's bytes: cq_launch_fast; ',' / '"' canonical narrow builds only)
            fp->wstr_lit = 1;
            if (ext || d != ',' || P->quote != '"') return false;
        }
    } else {
        int wslot[2] = {-1, -1};
        if (ext || d != ',' || P->quote != '"' || !wx_compile(P, fp, wslot, &wx, wx_s)) return false;
        *where = true;
        wcol = P->need_col[wslot[0]];
        wcol1 = wx == 2 ? P->need_col[wslot[1]] : -1;
    }
    if (wx_out) *wx_out = wx;
    if (*where && !fp->wstr_lit && !wx) {   // numeric literal: the thresholds
        const Cell& L = P->consts[P->prog[1].b];
        double lv;
        if (L.kind == K_INT) lv = (double)(int64_t)L.bits;
        else memcpy(&lv, &L.bits, 8);
        if (!std::isfinite(lv)) return false;
        fp->wl = lv;
        const double c = std::ceil(lv), f = std::floor(lv);
        fp->wlo = c >= 2147483647.0 ? 2147483647 : (c <= -2147483648.0 ? (-2147483647 - 1) : (int32_t)c);
        fp->whi = f >= 2147483647.0 ? 2147483647 : (f <= -2147483648.0 ? (-2147483647 - 1) : (int32_t)f);
        // the outcome over M in [0, 9999] (num4's INTEGER range) as one interval test:
        // the parts M < L, M == L, M > L are consecutive intervals, so any selection of
        // them is an interval or (< and > without ==) the complement of one
        const bool lt = fp->wtt & 1, eq = fp->wtt & 2, gt = fp->wtt & 4;
        const int64_t lo_eq = fp->wlo, hi_eq = fp->whi;
        int64_t A, B;
        fp->wneg = 0;
        if (lt && !eq && gt) { fp->wneg = 1; A = lo_eq; B = hi_eq; }
        else if (!lt && !eq && !gt) { A = 1; B = 0; }
        else {
            A = lt ? INT64_MIN : (eq ? lo_eq : hi_eq + 1);
            B = gt ? INT64_MAX : (eq ? hi_eq : lo_eq - 1);
        }
        A = A < 0 ? 0 : A;
        B = B > 9999 ? 9999 : B;
        if (A > B) { fp->wa = 0xFFFFFFFFu; fp->ww = 0; }     // empty: M - wa = M + 1 > 0
        else { fp->wa = (uint32_t)A; fp->ww = (uint32_t)(B - A); }
    }
    if (grouped && (P->group_slot < 0 || P->lean_k16)) return false;
    // the roles' fields in column order (equal columns share a field; ties keep the
    // role order WHERE, SUM 0, SUM 1, GROUP BY)
    int cols[5], roles[5], nr = 0;
    if (*where) { cols[nr] = wcol; roles[nr++] = 0; }
    if (wx == 2) { cols[nr] = wcol1; roles[nr++] = 4; }
    for (int j = 0; j < *ns; j++) { cols[nr] = P->need_col[sslot[j]]; roles[nr++] = 1 + j; }
    if (grouped) { cols[nr] = P->need_col[P->group_slot]; roles[nr++] = 3; }
    for (int a = 1; a < nr; a++)
        for (int b = a; b > 0 && cols[b - 1] > cols[b]; b--) {
            std::swap(cols[b - 1], cols[b]);
            std::swap(roles[b - 1], roles[b]);
        }
    bool canon = true;
    for (int k = 0; k < nr; k++) {
        if (cols[k] < 0) return false;
        fp->skip[k] = (uint32_t)(k ? cols[k] - cols[k - 1] : cols[k]);
        fp->rank[roles[k]] = (uint32_t)k;
        // compile-time ranks: WHERE 0, WHERE column 1 (WX == 2) 1, SUM j (WHERE ? 1 : 0) +
        // (WX == 2 ? 1 : 0) + j, GROUP BY the last
        const int sbase = (*where ? 1 : 0) + (wx == 2 ? 1 : 0);
        const int want = roles[k] == 0 ? 0 : roles[k] == 4 ? 1 : (roles[k] == 3 ? nr - 1 : sbase + roles[k] - 1);
        canon = canon && k == want;
    }
    *canonical = canon;
    if (wide_num || ext || fp->wstr_lit || wx) {   // a WHERE / SUM column whose sampled fields exceed 4 bytes
        bool wn = false;
        for (int k = 0; k < nr; k++) {    // (a STRING-literal WHERE reads up to 8 bytes itself)
            if (roles[k] == 3 || (roles[k] == 0 && fp->wstr_lit)) continue;
            if (wx && (roles[k] == 0 || roles[k] == 4) && ((fp->wx_str >> (roles[k] == 0 ? 0 : 1)) & 1)) continue;
            wn = wn || ((P->fast_wide_cols >> (cols[k] < 63 ? cols[k] : 63)) & 1);
        }
        wn = wn || getenv("CQGPU_FAST_WN") != nullptr;
        if (wide_num) *wide_num = wn;
        // MIN / MAX: the narrow-numeral ',' / '"' builds only (fixed point, no doubles)
        if (ext && (wn || d != ',' || P->quote != '"' || P->n >= (1ull << fast::EXT_POS_BITS))) return false;
        if (fp->wstr_lit && (wn || !canon)) return false;   // (the STRING-literal builds: narrow, canonical)
        if (wx && wn) return false;                         // (the compound builds: narrow numerals)
    }
    return true;
}

typedef void (*fast_fn_t)(const uint8_t*, ScanStats*, unsigned long long*, unsigned long long, const FastPlan,
                          const GroupTable*);

// rp3: three records per lane pass (records shorter than ~33 bytes: a lane's 64
// bytes usually hold three starts, and a two-record pass would run a second pass
// for the few lanes with a third); ungrouped plans only, the grouped kernels keep
// two (register budget of the lookup and atomics)
template <bool G, bool WH, bool COMMA, bool CANON, bool WN>
fast_fn_t pick_ns(int ns, bool rp3) {
    if constexpr (!G) {
        if (rp3) {
            if (ns == 0) return fast::fast_kernel<G, WH, 0, COMMA, CANON, 3, WN>;
            return ns == 1 ? fast::fast_kernel<G, WH, 1, COMMA, CANON, 3, WN> : fast::fast_kernel<G, WH, 2, COMMA, CANON, 3, WN>;
        }
    }
    if (ns == 0) return fast::fast_kernel<G, WH, 0, COMMA, CANON, 2, WN>;
    return ns == 1 ? fast::fast_kernel<G, WH, 1, COMMA, CANON, 2, WN> : fast::fast_kernel<G, WH, 2, COMMA, CANON, 2, WN>;
}
// (the narrow-numeral kernels for the ',' / '"' canonical plans only: the others keep
// the side path)
template <bool G, bool CANON>
fast_fn_t pick_wc(bool where, int ns, bool comma, bool rp3, bool wn) {
    if (where) {
        if (!comma) return pick_ns<G, true, false, CANON, true>(ns, rp3);
        return (CANON && !wn) ? pick_ns<G, true, true, CANON, false>(ns, rp3) : pick_ns<G, true, true, CANON, true>(ns, rp3);
    }
    if (!comma) return pick_ns<G, false, false, CANON, true>(ns, rp3);
    return (CANON && !wn) ? pick_ns<G, false, true, CANON, false>(ns, rp3) : pick_ns<G, false, true, CANON, true>(ns, rp3);
}
// the compound-WHERE builds (fast_shape: ',' / '"', narrow numerals, two records a pass)
template <bool G, int WXN>
fast_fn_t pick_wx(int ns, bool canon) {
    if (canon) {
        if (ns == 0) return fast::fast_kernel<G, true, 0, true, true, 2, false, 0, false, WXN>;
        return ns == 1 ? fast::fast_kernel<G, true, 1, true, true, 2, false, 0, false, WXN>
                       : fast::fast_kernel<G, true, 2, true, true, 2, false, 0, false, WXN>;
    }
    if (ns == 0) return fast::fast_kernel<G, true, 0, true, false, 2, false, 0, false, WXN>;
    return ns == 1 ? fast::fast_kernel<G, true, 1, true, false, 2, false, 0, false, WXN>
                   : fast::fast_kernel<G, true, 2, true, false, 2, false, 0, false, WXN>;
}
template <bool G>
fast_fn_t pick_fast(bool where, int ns, bool comma, bool canon, bool rp3, bool wn, int ext = 0, bool wstr = false,
                    int wx = 0) {
    if (wx) return wx == 1 ? pick_wx<G, 1>(ns, canon) : pick_wx<G, 2>(ns, canon);
    if (wstr) {    // (fast_shape: ',' / '"', canonical roles, narrow numerals, no MIN / MAX)
        if (ns == 0) return fast::fast_kernel<G, true, 0, true, true, 2, false, 0, true>;
        return ns == 1 ? fast::fast_kernel<G, true, 1, true, true, 2, false, 0, true>
                       : fast::fast_kernel<G, true, 2, true, true, 2, false, 0, true>;
    }
    if (ext) {     // (fast_shape: one argument, ',' / '"', narrow numerals)
        if (canon) {
            if (where) return ext == 1 ? fast::fast_kernel<G, true, 1, true, true, 2, false, 1>
                                       : fast::fast_kernel<G, true, 1, true, true, 2, false, 2>;
            return ext == 1 ? fast::fast_kernel<G, false, 1, true, true, 2, false, 1>
                            : fast::fast_kernel<G, false, 1, true, true, 2, false, 2>;
        }
        if (where) return ext == 1 ? fast::fast_kernel<G, true, 1, true, false, 2, false, 1>
                                   : fast::fast_kernel<G, true, 1, true, false, 2, false, 2>;
        return ext == 1 ? fast::fast_kernel<G, false, 1, true, false, 2, false, 1>
                        : fast::fast_kernel<G, false, 1, true, false, 2, false, 2>;
    }
    return canon ? pick_wc<G, true>(where, ns, comma, rp3, wn) : pick_wc<G, false>(where, ns, comma, rp3, wn);
}

// the window range and the key / payload field walk of a join side (jx_extract_kernel)
bool jx_plan(const uint8_t* g, uint64_t lo, uint64_t hi, uint32_t ws, uint32_t delim, uint32_t quote, int kcol,
             int pcol, fast::JxPlan* jp) {
    if (((uintptr_t)g & 255) != 0 || kcol < 0 || ws > (uint32_t)fast::WS || ws % 128 || ws == 0) return false;
    memset(jp, 0, sizeof *jp);
    jp->ws = ws;
    jp->delim = delim;
    jp->quote = quote;
    if (hi > lo) {
        const uint64_t wl = lo / ws, wh = (hi - 1) / ws;
        if (wh - wl + 1 >= (1ull << 31)) return false;
        jp->first_win = wl;
        jp->nwin = (uint32_t)(wh - wl + 1);
        jp->lo_s = (uint32_t)(lo - wl * ws);
        jp->hi_s = (uint32_t)(hi - wh * ws);
    }
    if (pcol < 0) {
        jp->skip[0] = (uint32_t)kcol;
        jp->rank_key = 0;
    } else {
        const int c0 = std::min(kcol, pcol), c1 = std::max(kcol, pcol);
        jp->skip[0] = (uint32_t)c0;
        jp->skip[1] = (uint32_t)(c1 - c0);
        jp->rank_key = kcol <= pcol ? 0u : 1u;
    }
    return true;
}

size_t fast_lds(int grouped, int ns, int wx = 0) {
    const size_t t = !grouped ? 0 : (ns == 0 ? fast::table_bytes<0>(true) : (ns == 1 ? fast::table_bytes<1>(true)
                                                                                     : fast::table_bytes<2>(true)));
    return fast::fixed_bytes() + t + 256 + (wx ? 4 * fast::LX_WORDS * 4 : 0);
}

}  // namespace

extern "C" {

// 1 when fast_kernel handles this plan (grouped: GROUP BY one column; want_rows:
// the launch must also emit matching record offsets, which fast_kernel does not)
int cq_fast_eligible(const cq::ScanPlan* P, int grouped, int want_rows) {
    if (want_rows) return 0;
    FastPlan fp;
    int ns = 0;
    bool where = false, canon = false;
    int wx = 0;
    if (!fast_shape(P, grouped, &fp, &ns, &where, &canon, nullptr, nullptr, &wx)) return 0;
    return fast_lds(grouped, ns, wx) <= 160 * 1024 ? 1 : 0;
}
// 1 when the plan has a MIN / MAX that fast_kernel takes (an EXT build): the
// executor gives such plans a raw-key table with extreme cells
int cq_fast_ext_plan(const cq::ScanPlan* P, int grouped) {
    FastPlan fp;
    int ns = 0, ext = 0;
    bool where = false, canon = false;
    return fast_shape(P, grouped, &fp, &ns, &where, &canon, nullptr, &ext) && ext ? 1 : 0;
}

// the scan (the caller runs slow_kernel over slow_list, then raw_merge_kernel)
hipError_t cq_launch_fast(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          const cq::GroupTable* rt, cq::ScanStats* stats, int grouped, int grid, hipStream_t s,
                          unsigned long long* slow_list, unsigned long long slow_cap) {
    FastPlan fp;
    int ns = 0;
    bool where = false, canon = false;
    bool wn = true;
    int ext = 0, wx = 0;
    if (!fast_shape(P, grouped, &fp, &ns, &where, &canon, &wn, &ext, &wx, s)) return hipErrorInvalidValue;
    if (((uintptr_t)g & 255) != 0) return hipErrorInvalidValue;
    const uint64_t hi = P->range_end < P->n ? P->range_end : P->n;
    const uint64_t lo = P->data_begin > P->range_begin ? P->data_begin : P->range_begin;
    fp.ws = P->lean_ws ? P->lean_ws : (uint32_t)fast::WS;
    if (fp.ws > (uint32_t)fast::WS || fp.ws % 128) return hipErrorInvalidValue;
    // the sampled stride is 120 records' worth (lean_kernel's choice): below the
    // largest stride the records average under 33 bytes -> the three-record pass,
    // over windows of the largest stride (test knob CQGPU_FAST_RP2: keep two)
    const bool rp3 = !grouped && !ext && !fp.wstr_lit && !wx && fp.ws < (uint32_t)fast::WS && !getenv("CQGPU_FAST_RP2");
    if (rp3) fp.ws = (uint32_t)fast::WS;
    if (hi > lo) {
        const uint64_t wl = lo / fp.ws, wh = (hi - 1) / fp.ws;
        if (wh - wl + 1 >= (1ull << 31)) return hipErrorInvalidValue;
        fp.first_win = wl;
        fp.nwin = (uint32_t)(wh - wl + 1);
        fp.lo_s = (uint32_t)(lo - wl * fp.ws);
        fp.hi_s = (uint32_t)(hi - wh * fp.ws);
    }
    fp.seed = grouped ? (const unsigned long long*)(uintptr_t)P->fast_seed : nullptr;
    // the launch's table pair in device memory of this thread and device (one pair
    // per thread: concurrent callers never share it)
    thread_local GroupTable* tabs_dev[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (!tabs_dev[dev & 63]) {
        hipError_t e = hipMalloc((void**)&tabs_dev[dev & 63], 2 * sizeof(GroupTable));
        if (e != hipSuccess) return e;
    }
    GroupTable tabs[2];
    tabs[0] = *gt;
    if (rt) tabs[1] = *rt;
    else memset(&tabs[1], 0, sizeof tabs[1]);
    hipError_t e = cq::upload_buffer(tabs_dev[dev & 63], tabs, sizeof tabs, s);
    if (e != hipSuccess) return e;
    if (fp.wstr_lit) {   // the literal's bytes (a STRING cell points at device memory); strcmp stops at a NUL
        const Cell& L = P->consts[P->prog[1].b];
        uint8_t b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        hipError_t e = hipMemcpyAsync(b, (const void*)(uintptr_t)L.bits, L.len, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        bool nul = false;
        uint64_t x = 0;
        for (int i = 0; i < 8; i++) {
            nul = nul || b[i] == 0;
            x = (x << 8) | (nul ? 0u : b[i]);
        }
        fp.wstr = x;
    }
    const bool comma = P->delim == ',' && P->quote == '"';
    // (EXT builds: the packed extreme keys go to the raw table's extpos words)
    if (ext && (!rt || !rt->extpos[fp.ext_acc] || rt->cap < 1)) return hipErrorInvalidValue;
    const bool wstr = fp.wstr_lit != 0;
    const fast_fn_t fn = grouped ? pick_fast<true>(where, ns, comma, canon, false, wn, ext, wstr, wx)
                                 : pick_fast<false>(where, ns, comma, canon, rp3, wn, ext, wstr, wx);
    const size_t lds = fast_lds(grouped, ns, wx);
    cq::set_max_lds((const void*)fn, (int)lds);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(fast::LT), lds, s, g, stats, slow_list, slow_cap, fp,
                       (const GroupTable*)tabs_dev[dev & 63]);
    return hipGetLastError();
}

int cq_fast_waves_per_block() { return fast::NWV; }

// one-group MIN / MAX build: the packed key the waves left in the raw table's word 0,
// typed from its record and merged into the group (the canonical table's GK_ALL key)
__global__ void fast_ext_final_kernel(const uint8_t* __restrict__ g, const GroupTable gt, const GroupTable rt, int a,
                                      uint32_t col, uint32_t delim, uint8_t kind, ScanStats* __restrict__ stats) {
    const unsigned long long x = rt.extpos[a][0];
    int gi = -1;
    Cell cc = cell_null();
    uint64_t pos = NOPOS;
    if (threadIdx.x == 0 && x != ~0ull) {
        GKey k;
        k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
        gi = g_insert(gt, k, 0x12345678ULL, stats);       // (fast_kernel's one-group key and hash)
        pos = x & ((1ull << fast::EXT_POS_BITS) - 1);
        cc = field_cell(g, pos, col, delim);
    }
    g_ext_update(gi >= 0 && cc.kind != K_NULL, gt, a, kind, gi >= 0 ? (uint32_t)gi : 0u, cc, pos, stats);
    if (threadIdx.x == 0) rt.extpos[a][0] = ~0ull;     // consumed (a chunked rescan adds its own)
}
// the MIN / MAX accumulator and its column of a fast_kernel EXT build (-1: none)
int cq_fast_ext_info(const cq::ScanPlan* P, int grouped, uint32_t* col) {
    FastPlan fp;
    int ns = 0, ext = 0;
    bool where = false, canon = false;
    if (!fast_shape(P, grouped, &fp, &ns, &where, &canon, nullptr, &ext) || !ext) return -1;
    *col = fp.ext_col;
    return fp.ext_acc;
}
hipError_t cq_fast_ext_final(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt, const cq::GroupTable* rt,
                             cq::ScanStats* stats, hipStream_t s) {
    uint32_t col = 0;
    const int a = cq_fast_ext_info(P, 0, &col);
    if (a < 0 || !rt || !rt->extpos[a]) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fast_ext_final_kernel, dim3(1), dim3(64), 0, s, g, *gt, *rt, a, col, (uint32_t)P->delim,
                       (uint8_t)P->acc[a].kind, stats);
    return hipGetLastError();
}

// ---- fused aggregate join (executor.hip run_fast_join)
// windows of the table's bytes [lo, hi) at stride ws
uint64_t cq_jx_windows(uint64_t lo, uint64_t hi, uint32_t ws) { return hi > lo ? (hi - 1) / ws - lo / ws + 1 : 0; }
// extraction of one side, records of the table's bytes [lo, hi) (lo at a record start);
// kcol the ON key's column, pcol the payload's (-1: none); build: the payload is the
// GROUP BY field's raw bytes, else the SUM argument.  pass 0 counts each window's
// records into wcount; pass 1 emits every record at wbase[window] + its rank (file order)
hipError_t cq_jx_extract(const uint8_t* g, uint64_t lo, uint64_t hi, uint32_t ws, uint32_t delim, uint32_t quote,
                         int kcol, int pcol, int build, int pass, unsigned long long* key, unsigned long long* pay,
                         uint32_t* off, unsigned int* wcount, const unsigned int* wbase, unsigned int cap,
                         unsigned int* flag, unsigned long long* krange, int grid, hipStream_t s) {
    using namespace cq::fast;
    JxPlan jp;
    if (!jx_plan(g, lo, hi, ws, delim, quote, kcol, pcol, &jp)) return hipErrorInvalidValue;
    const int nr = pcol >= 0 ? 2 : 1;
    const bool comma = delim == ',' && quote == '"';
    typedef void (*xfn_t)(const uint8_t*, const JxPlan, const JxOut);
    static const xfn_t tab[2][2][2][2] = {
        {{{jx_extract_kernel<false, false, 1, false>, jx_extract_kernel<false, false, 1, true>},
          {jx_extract_kernel<false, false, 2, false>, jx_extract_kernel<false, false, 2, true>}},
         {{jx_extract_kernel<false, true, 1, false>, jx_extract_kernel<false, true, 1, true>},
          {jx_extract_kernel<false, true, 2, false>, jx_extract_kernel<false, true, 2, true>}}},
        {{{jx_extract_kernel<true, false, 1, false>, jx_extract_kernel<true, false, 1, true>},
          {jx_extract_kernel<true, false, 2, false>, jx_extract_kernel<true, false, 2, true>}},
         {{jx_extract_kernel<true, true, 1, false>, jx_extract_kernel<true, true, 1, true>},
          {jx_extract_kernel<true, true, 2, false>, jx_extract_kernel<true, true, 2, true>}}}};
    const xfn_t fn = tab[build ? 1 : 0][comma ? 1 : 0][nr - 1][pass == 0 ? 1 : 0];
    JxOut jo;
    memset(&jo, 0, sizeof jo);
    jo.key = key; jo.pay = pay; jo.off = off; jo.wcount = wcount; jo.wbase = wbase; jo.cap = cap; jo.flag = flag;
    jo.krange = krange;
    const size_t lds = sizeof(WaveLds) * NWV;
    cq::set_max_lds((const void*)fn, (int)lds);
    if (jp.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(LT), lds, s, g, jp, jo);
    return hipGetLastError();
}

// STAR join passes (jx_extract_kernel<..., STAR>): build -- every record's key straight
// into d16 / l32 at key - kmin, its GROUP BY tag's id through ttab; probe -- every
// record's key looked up in d16, m8 set, COUNT / SUM per group id into gsum.
// counter: build records placed (build) / pairs (probe).
hipError_t cq_jx_star_extract(const uint8_t* g, uint64_t lo, uint64_t hi, uint32_t ws, uint32_t delim, uint32_t quote,
                              int kcol, int pcol, int build, unsigned long long kmin, unsigned long long range,
                              uint32_t stride, uint16_t* d16, uint32_t* l32, unsigned long long* ttab,
                              unsigned long long* gsum, unsigned long long* counter, unsigned int* flag,
                              unsigned long long* krange, uint32_t* notmono, unsigned long long* wfl,
                              uint32_t* gminix, int rp, int grid, hipStream_t s, unsigned long long* pent,
                              uint32_t* pcnt, uint32_t np, uint32_t pcap, uint32_t psh) {
    using namespace cq::fast;
    JxPlan jp;
    if (!jx_plan(g, lo, hi, ws, delim, quote, kcol, pcol, &jp)) return hipErrorInvalidValue;
    const int nr = pcol >= 0 ? 2 : 1;
    const bool comma = delim == ',' && quote == '"';
    typedef void (*xfn_t)(const uint8_t*, const JxPlan, const JxOut);
    const bool part = pent != nullptr;
    if (part && (build || np == 0 || np > JX_PMAX || pcap == 0 || ((unsigned long long)np << psh) < range))
        return hipErrorInvalidValue;
    // partitioned probe, pass 1: [comma][roles - 1][three records per pass]
    static const xfn_t ptab[2][2][2] = {
        {{jx_extract_kernel<false, false, 1, false, true, 2, true>, jx_extract_kernel<false, false, 1, false, true, 3, true>},
         {jx_extract_kernel<false, false, 2, false, true, 2, true>, jx_extract_kernel<false, false, 2, false, true, 3, true>}},
        {{jx_extract_kernel<false, true, 1, false, true, 2, true>, jx_extract_kernel<false, true, 1, false, true, 3, true>},
         {jx_extract_kernel<false, true, 2, false, true, 2, true>, jx_extract_kernel<false, true, 2, false, true, 3, true>}}};
    // [build][comma][roles - 1][three records per pass: records under ~33 bytes, where
    // two per pass leave a second, mostly idle pass for the lanes holding a third start]
    static const xfn_t tab[2][2][2][2] = {
        {{{jx_extract_kernel<false, false, 1, false, true>, jx_extract_kernel<false, false, 1, false, true, 3>},
          {jx_extract_kernel<false, false, 2, false, true>, jx_extract_kernel<false, false, 2, false, true, 3>}},
         {{jx_extract_kernel<false, true, 1, false, true>, jx_extract_kernel<false, true, 1, false, true, 3>},
          {jx_extract_kernel<false, true, 2, false, true>, jx_extract_kernel<false, true, 2, false, true, 3>}}},
        {{{jx_extract_kernel<true, false, 1, false, true>, jx_extract_kernel<true, false, 1, false, true, 3>},
          {jx_extract_kernel<true, false, 2, false, true>, jx_extract_kernel<true, false, 2, false, true, 3>}},
         {{jx_extract_kernel<true, true, 1, false, true>, jx_extract_kernel<true, true, 1, false, true, 3>},
          {jx_extract_kernel<true, true, 2, false, true>, jx_extract_kernel<true, true, 2, false, true, 3>}}}};
    const xfn_t fn = part ? ptab[comma ? 1 : 0][nr - 1][rp == 3 ? 1 : 0]
                          : tab[build ? 1 : 0][comma ? 1 : 0][nr - 1][rp == 3 ? 1 : 0];
    JxOut jo;
    memset(&jo, 0, sizeof jo);
    jo.pent = pent;
    jo.pcnt = pcnt;
    jo.np = np;
    jo.pcap = pcap;
    jo.psh = psh;
    jo.flag = flag;
    jo.krange = krange;
    jo.kmin = kmin;
    jo.range = range;
    if (stride == 0 || (unsigned long long)stride * range >= (1ull << 32)) return hipErrorInvalidValue;
    jo.sshift = (uint32_t)__builtin_ctz(stride);
    jo.smask = (1u << jo.sshift) - 1u;
    jo.stride = stride;
    {
        const uint32_t m = stride >> jo.sshift;     // odd: Newton's iteration for m^-1 mod 2^32
        uint32_t inv = m;                           // (correct to 3 bits; each step doubles them)
        for (int k = 0; k < 4; k++) inv *= 2u - m * inv;
        jo.sinv = inv;
    }
    jo.d16 = d16;
    jo.l32 = l32;
    jo.ttab = ttab;
    jo.gsum = gsum;
    jo.nbuilt = counter;
    jo.notmono = notmono;
    jo.wfl = wfl;
    jo.gminix = gminix;
    const size_t lds = sizeof(WaveLds) * NWV +
                       (part ? (size_t)np * 4 : build ? (nr == 2 ? (size_t)JX_G * 8 : 0) : (size_t)JX_G * 20);
    cq::set_max_lds((const void*)fn, (int)lds);
    if (jp.nwin == 0) {
        if (part) return hipMemsetAsync(pcnt, 0, (size_t)grid * np * 4, s);
        return hipSuccess;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(LT), lds, s, g, jp, jo);
    return hipGetLastError();
}
// partitioned STAR probe, pass 2 (jx_part_probe_kernel): `grid` a multiple of 8
hipError_t cq_jx_part_probe(const unsigned long long* pent, const uint32_t* pcnt, uint32_t nsrc, uint32_t np,
                            uint32_t pcap, unsigned long long range, uint16_t* d16, const uint32_t* notmono,
                            unsigned long long* gsum, uint32_t* gminix, unsigned long long* npairs, int grid,
                            hipStream_t s) {
    if (grid < 8 || grid % 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cq::fast::jx_part_probe_kernel, dim3(grid), dim3(1024), 0, s, pent, pcnt, nsrc, np, pcap,
                       (uint64_t)range, d16, notmono, gsum, gminix, npairs);
    return hipGetLastError();
}
hipError_t cq_jx_star_order(const unsigned long long* wfl, unsigned long long nwin, uint32_t* notmono, hipStream_t s) {
    if (nwin < 2) return hipSuccess;
    hipLaunchKernelGGL(cq::fast::jx_star_order_kernel, dim3((unsigned)std::min<unsigned long long>((nwin + 255) / 256, 1024)),
                       dim3(256), 0, s, wfl, (uint64_t)nwin, notmono);
    return hipGetLastError();
}
hipError_t cq_jx_star_init(void* d16, size_t d16_bytes, void* small, size_t small_bytes, uint32_t ff0, uint32_t ff1,
                           uint32_t ffw, const void* seed, size_t seed_bytes, int grid, hipStream_t s) {
    if (((uintptr_t)d16 | (uintptr_t)small | (uintptr_t)seed | d16_bytes | small_bytes | seed_bytes | ffw) & 7 ||
        ((uintptr_t)d16 | (uintptr_t)small | (uintptr_t)seed | d16_bytes | small_bytes | seed_bytes | ff0 | ff1) & 15)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(cq::fast::jx_star_init_kernel, dim3(grid), dim3(1024), 0, s, (uint4*)d16, (uint64_t)(d16_bytes / 16),
                       (uint4*)small, (uint32_t)(small_bytes / 16), ff0, ff1, ffw, (const uint4*)seed,
                       (uint32_t)(seed_bytes / 16));
    return hipGetLastError();
}
hipError_t cq_jx_star_first(const uint16_t* d16, const uint32_t* l32, unsigned long long range, const uint32_t* notmono,
                            uint32_t* gfirst, unsigned long long* nocc, int grid, hipStream_t s) {
    if (((uintptr_t)d16 & 15) || ((uintptr_t)l32 & 15)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cq::fast::jx_star_first_kernel, dim3(grid), dim3(1024), 0, s, d16, l32, (uint64_t)range, notmono,
                       gfirst, nocc);
    return hipGetLastError();
}
hipError_t cq_jx_star_flush(int grouped, int value, const unsigned long long* ttab, const unsigned long long* gsum,
                            const uint32_t* gfirst, const uint32_t* gminix, const uint32_t* l32, const uint32_t* notmono,
                            const unsigned long long* cnts, const cq::GroupTable* rt, int nacc, cq::ScanStats* stats,
                            unsigned int* flag, hipStream_t s) {
    using namespace cq::fast;
    typedef void (*ffn_t)(const unsigned long long*, const unsigned long long*, const uint32_t*, const uint32_t*,
                          const uint32_t*, const uint32_t*, const unsigned long long*, GroupTable, int, ScanStats*,
                          unsigned int*);
    static const ffn_t tab[2][2] = {{jx_star_flush_kernel<false, false>, jx_star_flush_kernel<false, true>},
                                    {jx_star_flush_kernel<true, false>, jx_star_flush_kernel<true, true>}};
    hipLaunchKernelGGL(tab[grouped ? 1 : 0][value ? 1 : 0], dim3(1), dim3(1024), 0, s, ttab, gsum, gfirst, gminix, l32,
                       notmono, cnts, *rt, nacc, stats, flag);
    return hipGetLastError();
}
uint32_t cq_jx_star_groups() { return cq::fast::JX_G; }
uint32_t cq_jx_rchunk() { return cq::fast::JX_RCHUNK; }

// the typed exchange's sender passes over one side (jx_extract_kernel ROUTE):
//   pass 1  per window i and destination d the entries into rcnt[d * nwin + i] (build:
//           the window's records into wcount); pcol is ignored (the key field only)
//   pass 2  the entries at roffs[d * nwin + i] + their rank (roffs: rcnt's exclusive
//           scan, destination-major); build: 16-byte {q32, gid, tag} (wbase: wcount's
//           exclusive scan), probe 8-byte {q32, pay}
//   pass 3  (probe, nranks <= 8) the entries in one pass: destination d's in chunks of
//           [d * cap, (d + 1) * cap) of rent, reserved from the cursors rcnt[64 d] (zeroed)
hipError_t cq_jx_route(const uint8_t* g, uint64_t lo, uint64_t hi, uint32_t ws, uint32_t delim, uint32_t quote,
                       int kcol, int pcol, int build, int rp, int pass, uint32_t nranks, unsigned long long qbase,
                       unsigned long long gbase, unsigned int* rcnt, unsigned int* wcount, const unsigned int* roffs,
                       const unsigned int* wbase, void* rent, uint32_t cap, unsigned int* flag,
                       unsigned long long* krange, int grid, hipStream_t s) {
    using namespace cq::fast;
    JxPlan jp;
    if (pass == 1) pcol = -1;
    if (!jx_plan(g, lo, hi, ws, delim, quote, kcol, pcol, &jp)) return hipErrorInvalidValue;
    if (nranks < 1 || nranks > 64) return hipErrorInvalidValue;
    if (pass == 3 ? (build || nranks > 8 || !rcnt || !rent || !cap)
                  : pass == 1 ? (!rcnt || (build && !wcount)) : (!roffs || !rent || (build && !wbase)))
        return hipErrorInvalidValue;
    const int nr = pcol >= 0 ? 2 : 1;
    if (delim != ',' || quote != '"') return hipErrorInvalidValue;      // (the ',' / '"' builds)
    typedef void (*xfn_t)(const uint8_t*, const JxPlan, const JxOut);
    // count: [build][three records per pass]; emit: [build][roles - 1][three records per pass]
    static const xfn_t ctab[2][2] = {
        {jx_extract_kernel<false, true, 1, false, false, 2, false, 1>, jx_extract_kernel<false, true, 1, false, false, 3, false, 1>},
        {jx_extract_kernel<true, true, 1, false, false, 2, false, 1>, jx_extract_kernel<true, true, 1, false, false, 3, false, 1>}};
    static const xfn_t etab[2][2][2] = {
        {{jx_extract_kernel<false, true, 1, false, false, 2, false, 2>, jx_extract_kernel<false, true, 1, false, false, 3, false, 2>},
         {jx_extract_kernel<false, true, 2, false, false, 2, false, 2>, jx_extract_kernel<false, true, 2, false, false, 3, false, 2>}},
        {{jx_extract_kernel<true, true, 1, false, false, 2, false, 2>, jx_extract_kernel<true, true, 1, false, false, 3, false, 2>},
         {jx_extract_kernel<true, true, 2, false, false, 2, false, 2>, jx_extract_kernel<true, true, 2, false, false, 3, false, 2>}}};
    static const xfn_t otab[2][2] = {
        {jx_extract_kernel<false, true, 1, false, false, 2, false, 3>, jx_extract_kernel<false, true, 1, false, false, 3, false, 3>},
        {jx_extract_kernel<false, true, 2, false, false, 2, false, 3>, jx_extract_kernel<false, true, 2, false, false, 3, false, 3>}};
    const xfn_t fn = pass == 1   ? ctab[build ? 1 : 0][rp == 3 ? 1 : 0]
                     : pass == 3 ? otab[nr - 1][rp == 3 ? 1 : 0]
                                 : etab[build ? 1 : 0][nr - 1][rp == 3 ? 1 : 0];
    JxOut jo;
    memset(&jo, 0, sizeof jo);
    jo.wbase = wbase;
    jo.wcount = wcount;
    jo.flag = flag;
    jo.krange = krange;
    jo.rent = rent;
    jo.rcnt = rcnt;
    jo.roffs = roffs;
    jo.rn = nranks;
    jo.cap = cap;
    // ceil(2^64 / n): key / n = mulhi(key, magic) for keys below 2^64 / n (canonical keys < 10^15)
    jo.rmagic = nranks > 1 ? (unsigned long long)(((unsigned __int128)1 << 64) / nranks) + 1ull : 0ull;
    if (nranks > 1 && (nranks & (nranks - 1)) == 0) jo.rmagic = 1ull << (64 - __builtin_ctz(nranks));
    jo.qbase = qbase;
    jo.gbase = gbase;
    const size_t lds = sizeof(WaveLds) * NWV;
    cq::set_max_lds((const void*)fn, (int)lds);
    if (jp.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(LT), lds, s, g, jp, jo);
    return hipGetLastError();
}
// the receiving rank's STAR over the entries (jx_ent_build_kernel, jx_ent_probe_kernel)
hipError_t cq_jx_ent_build(const void* ent, unsigned long long n, uint32_t qoff, unsigned long long range, uint16_t* d16,
                           uint32_t* l32, unsigned long long* ttab, unsigned long long* nplaced, unsigned int* flag,
                           int grid, hipStream_t s, int ungrouped, uint32_t* notmono) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::fast::jx_ent_build_kernel, dim3(grid), dim3(1024), 0, s, (const uint4*)ent, (uint64_t)n, qoff,
                       (uint64_t)range, d16, l32, ttab, nplaced, flag, (uint32_t)(ungrouped != 0), notmono);
    return hipGetLastError();
}
hipError_t cq_jx_ent_first(const uint32_t* gminix, const uint32_t* l32, const uint32_t* notmono, uint32_t* gfirst,
                           hipStream_t s) {
    hipLaunchKernelGGL(cq::fast::jx_ent_first_kernel, dim3(1), dim3(1024), 0, s, gminix, l32, notmono, gfirst);
    return hipGetLastError();
}
hipError_t cq_jx_ent_part(const void* ent, unsigned long long n, uint32_t qoff, unsigned long long range, uint32_t np,
                          uint32_t pcap, uint32_t psh, unsigned long long* pent, uint32_t* pcnt, unsigned int* flag,
                          int grid, hipStream_t s) {
    if (np == 0 || np > cq::fast::JX_PMAX || ((unsigned long long)np << psh) < range) return hipErrorInvalidValue;
    const size_t lds = (size_t)np * 4;
    cq::set_max_lds((const void*)cq::fast::jx_ent_part_kernel, (int)lds);
    hipLaunchKernelGGL(cq::fast::jx_ent_part_kernel, dim3(grid), dim3(1024), lds, s, (const uint2*)ent, (uint64_t)n, qoff,
                       (uint64_t)range, np, pcap, psh, pent, pcnt, flag);
    return hipGetLastError();
}
hipError_t cq_jx_ent_probe(const void* ent, unsigned long long n, uint32_t qoff, unsigned long long range, uint16_t* d16,
                           unsigned long long* gsum, unsigned long long* npairs, int grid, hipStream_t s,
                           const uint32_t* notmono, uint32_t* gminix) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::fast::jx_ent_probe_kernel, dim3(grid), dim3(1024), 0, s, (const uint2*)ent, (uint64_t)n, qoff,
                       (uint64_t)range, d16, gsum, npairs, notmono, gminix);
    return hipGetLastError();
}

hipError_t cq_jx_build(const unsigned long long* key, uint32_t n, void* table, uint64_t tcap, unsigned int* flag,
                       int grid, hipStream_t s) {
    if (tcap & (tcap - 1)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cq::fast::jx_build_kernel, dim3(grid), dim3(256), 0, s, key, n, (cq::fast::JxEntry*)table,
                       tcap - 1, flag);
    return hipGetLastError();
}
size_t cq_jx_entry_bytes() { return sizeof(cq::fast::JxEntry); }
hipError_t cq_jx_build_direct(const unsigned long long* key, const unsigned long long* pay, const uint32_t* off,
                              uint32_t n, unsigned long long kmin, unsigned long long range, void* D,
                              unsigned int* flag, int grid, hipStream_t s) {
    hipLaunchKernelGGL(cq::fast::jx_build_direct_kernel, dim3(grid), dim3(256), 0, s, key, pay, off, n, kmin, range,
                       (cq::fast::JxDirect*)D, flag);
    return hipGetLastError();
}
size_t cq_jx_direct_bytes() { return sizeof(cq::fast::JxDirect); }
// direct: table is jx_build_direct's D of `tcap` entries (keys kmin ..), else the hash
// table of tcap (a power of two) entries
hipError_t cq_jx_probe(int grouped, int value, int direct, const unsigned long long* pkey,
                       const unsigned long long* ppay, const uint32_t* poff, uint32_t n, unsigned long long kmin,
                       const void* table, uint64_t tcap, const unsigned long long* bpay, const uint32_t* boff,
                       const cq::GroupTable* rt, int nacc, cq::ScanStats* stats, unsigned int* flag, int grid,
                       hipStream_t s) {
    using namespace cq::fast;
    typedef void (*pfn_t)(const unsigned long long*, const unsigned long long*, const uint32_t*, uint32_t,
                          unsigned long long, const JxEntry*, uint64_t, const unsigned long long*, const uint32_t*,
                          GroupTable, int, ScanStats*, unsigned int*);
    static const pfn_t tab[2][2][2] = {
        {{jx_probe_kernel<false, false, false>, jx_probe_kernel<false, false, true>},
         {jx_probe_kernel<false, true, false>, jx_probe_kernel<false, true, true>}},
        {{jx_probe_kernel<true, false, false>, jx_probe_kernel<true, false, true>},
         {jx_probe_kernel<true, true, false>, jx_probe_kernel<true, true, true>}}};
    const pfn_t fn = tab[grouped ? 1 : 0][value ? 1 : 0][direct ? 1 : 0];
    hipLaunchKernelGGL(fn, dim3(grid), dim3(1024), 0, s, pkey, ppay, poff, n, kmin, (const JxEntry*)table, tcap - 1,
                       bpay, boff, *rt, nacc, stats, flag);
    return hipGetLastError();
}

// The LDS table seed of a GROUP BY column: the distinct raw keys of the sampled
// records (records split on '\n' / '\r' runs, fields on the delimiter, quote-blind;
// records holding a quote skipped), placed into the 1024 two-slot buckets by cuckoo
// insertion with fast_key_hash's two bucket choices.  tags: TSLOTS words (0: free).
// Returns the number of keys placed (keys that do not fit are left to the kernel's
// own insertion).
uint32_t cq_fast_seed(const uint8_t* data, uint64_t n, uint32_t delim, uint32_t quote, uint32_t col,
                      unsigned long long* tags) {
    using fast::TSLOTS;
    using fast::TBUCKETS;
    memset(tags, 0, TSLOTS * sizeof(unsigned long long));
    std::unordered_set<unsigned long long> keys;
    uint64_t i = 0;
    while (i < n && keys.size() < TSLOTS) {
        while (i < n && (data[i] == '\n' || data[i] == '\r')) i++;
        const uint64_t rs = i;
        while (i < n && data[i] != '\n' && data[i] != '\r') i++;
        if (i >= n) break;                               // the sample's last record may be cut
        const uint8_t* r = data + rs;
        const uint64_t rl = i - rs;
        if (memchr(r, (int)quote, rl)) continue;
        uint32_t c = 0;
        uint64_t fs = 0;
        bool found = false;
        uint64_t kf = 0, kl = 0;
        for (uint64_t j = 0; j <= rl; j++) {
            if (j == rl || r[j] == delim) {
                if (c == col) { kf = fs; kl = j - fs; found = true; break; }
                c++;
                fs = j + 1;
            }
        }
        if (!found || kl > 8) continue;
        bool ok = true;
        unsigned long long t = 0;
        for (uint64_t j = 0; j < kl; j++) {
            if (r[kf + j] <= ' ') ok = false;
            t |= (unsigned long long)r[kf + j] << (8 * j);
        }
        if (!ok) continue;
        keys.insert(kl ? t : (1ull << 32));
    }
    uint32_t placed = 0;
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    for (unsigned long long k : keys) {
        unsigned long long cur = k;
        bool done = false;
        for (int kick = 0; kick < 512 && !done; kick++) {
            const uint32_t h = fast_key_hash((uint32_t)cur, (uint32_t)(cur >> 32));
            const uint32_t b[2] = {h & (TBUCKETS - 1), (h >> 16) & (TBUCKETS - 1)};
            for (int x = 0; x < 2 && !done; x++)
                for (int y = 0; y < 2 && !done; y++)
                    if (!tags[2 * b[x] + y]) { tags[2 * b[x] + y] = cur; done = true; }
            if (done) break;
            rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
            const uint32_t v = 2 * b[(rng >> 1) & 1] + (uint32_t)(rng & 1);
            std::swap(cur, tags[v]);
        }
        if (done) placed++;                              // else the carried key is left out
    }
    return placed;
}

size_t cq_fast_seed_slots() { return fast::TSLOTS; }

}  // extern "C"
