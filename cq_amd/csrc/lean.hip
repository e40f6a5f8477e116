// lean.hip -- the wave-autonomous CSV scan for the common SELECT plan shapes.
//
// Same job as scan_kernel (scan.hip) -- csv_load + filter_rows + create_groups +
// evaluate_aggregate in one pass over the HBM-resident bytes (reference
// csv_reader.c:375-465, evaluator_utils.c:986, evaluator_aggregates.c:108-414) --
// for plans whose WHERE is absent or `column op literal` and whose aggregates are
// COUNT / SUM / AVG (at most 4 parsed columns, 2 distinct SUM arguments).
//
// Every wave works on its own windows with no block barrier in the loop, so one
// wave's byte classification overlaps another's record work on the same SIMD:
//
//   load      a window is 2 KiB, lane l holds bytes [32l, 32l + 32) in registers
//             (two 16-byte non-temporal loads, issued one window ahead); windows
//             start WS = 1920 bytes apart and own the records starting in their
//             first WS bytes, so the last 128 bytes only serve the record views
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
//   values    parse_value (csv_reader.c:195-240) is a pure function of the field
//             bytes, so its result is memoised: per WHERE / SUM column a 512-entry
//             LDS table maps the raw bytes of a field (<= 8 bytes) to the WHERE
//             outcome or the SUM addend; only a miss runs the exact field typers
//             (scanlib.h) and fills the entry.  A wave stops consulting a column's
//             table once most lookups miss (high-cardinality column)
//   group     the block's LDS open-addressing table is keyed by the RAW bytes of
//             the GROUP BY field (<= 16 bytes): a raw key partitions the rows at
//             least as finely as the reference's printf-canonical key.  Blocks
//             flush (and a full LDS table spills) into an HBM table of raw keys;
//             raw_merge_kernel then types every distinct raw key once with the
//             general parser (parse_cell + group_key) and merges it into the
//             canonical HBM table -- so "1.5" and "1.50" still meet there
//   aggregate COUNT and SUM are fire-and-forget LDS atomics; the block flushes once
#include <hip/hip_runtime.h>
#include <cstring>
#include "plan.h"
#include "scanlib.h"

namespace cq {
namespace lean {

constexpr int LT = 1024;                  // threads per block
constexpr int NWV = LT / 64;              // waves per block
constexpr int LB = 32;                    // staged bytes per lane
constexpr int WB = 64 * LB;               // staged window bytes (2 KiB)
constexpr int WS = WB - 128;              // window stride: records starting in [ws, ws + WS) are owned
constexpr int NMW = WB / 32;              // 32-bit bitmap words per window
constexpr int WBYTES = WB + 32;           // staged bytes + slack for 16-byte field loads
constexpr int RSN = 64;                   // record slots per pass
constexpr int MAXS = 2;                   // distinct SUM arguments
constexpr int PROBES = 32;                // LDS probe window before spilling to HBM
constexpr int MEMO_N = 512;               // memo entries per WHERE / SUM column
constexpr uint32_t NOFIRST = 0xFFFFFFFFu;
static_assert(WS + 64 + 16 <= WB, "a record view (64 bytes) plus a 16-byte field load stays in the window");

// memo values (SUM: IEEE bits of the addend; NaN payloads never come out of a parse)
constexpr uint64_t MV_NOTNUM = 0x7FF80000000000A1ULL;   // not INTEGER / DOUBLE: SUM skips it
constexpr uint64_t MV_SLOW = 0x7FF80000000000A2ULL;     // only the general parser can type it

// per-wave LDS area
struct WaveLds {
    uint8_t bytes[WBYTES];
    uint2 bm[NMW + 2];          // {separator bits, terminator bits} per 32 window bytes
    uint32_t qt[NMW + 4];       // quote bits (written only when the window holds a quote)
    uint16_t rs[RSN];           // record starts of the current pass (window offsets)
};
static_assert(sizeof(WaveLds) % 16 == 0, "16-byte aligned wave areas");

// what the lean kernel needs beyond the ScanPlan
struct LeanPlan {
    int32_t ns;                  // distinct SUM argument slots
    int32_t sum_slot[MAXS];      // need slot of each
    int32_t acc_sidx[MAX_ACC];   // accumulator -> SUM index
    int32_t wslot;               // W_SIMPLE: need slot compared
    uint32_t wop;                // CMP_*
    int32_t wconst;              // consts index of the literal
};

__constant__ ScanPlan c_plan;
__constant__ GroupTable c_gt;        // canonical keys (shared with slow_kernel)
__constant__ GroupTable c_rt;        // raw-byte keys (GK_RAW): block flushes and LDS spills
__constant__ LeanPlan c_lp;

constexpr uint32_t GK_RAW = 6;       // raw field bytes as key (cell.h GK_* never produce 6)
__device__ __forceinline__ GKey raw_key(uint32_t len, uint64_t w0, uint64_t w1) {
    GKey k;
    k.cls = GK_RAW; k.len = len; k.w0 = w0; k.w1 = w1;
    return k;
}

struct Win {            // one window in flight
    v4u a, b;           // bytes [32l, 32l + 32)
    uint32_t prev;      // byte before the window (lane 0)
};

__device__ __forceinline__ void load_win(const uint8_t* g, uint64_t w, Win& x) {
    const uint64_t ws = w * WS;
    const v4u* src = (const v4u*)(g + ws);
    const int lane = threadIdx.x & 63;
    x.a = __builtin_nontemporal_load(src + 2 * lane);
    x.b = __builtin_nontemporal_load(src + 2 * lane + 1);
    x.prev = lane == 0 ? (uint32_t)g[ws - 1] : 0u;   // g has 64 padding bytes before byte 0
}

// separator / terminator bits of 32 bytes (bit i = byte i)
__device__ __forceinline__ void classify(const v4u a, const v4u b, uint32_t rep_d, uint32_t& sep, uint32_t& nl) {
    uint32_t s = 0, n = 0;
#pragma unroll
    for (int v = 0; v < 2; v++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t x = v ? b[j] : a[j];
            const uint32_t nl_inv = nonzero_bytes(x ^ 0x0A0A0A0Au) & nonzero_bytes(x ^ 0x0D0D0D0Du);
            const uint32_t sp_inv = nl_inv & nonzero_bytes(x ^ rep_d);
            // 0x80 flags -> nibbles: separators in bits 0-3, terminators in bits 4-7
            const uint32_t c = ((~sp_inv & 0x80808080u) >> 7) | ((~nl_inv & 0x80808080u) >> 3);
            uint32_t t = c | (c >> 7);
            t = t | (t >> 14);
            const int sh = (v * 4 + j) * 4;
            s |= (t & 0xFu) << sh;
            n |= ((t >> 4) & 0xFu) << sh;
        }
    }
    sep = s;
    nl = n;
}
__device__ __forceinline__ bool any_byte(const v4u a, const v4u b, uint32_t rep) {
    uint32_t acc = 0x80808080u;
#pragma unroll
    for (int j = 0; j < 4; j++) acc &= nonzero_bytes(a[j] ^ rep) & nonzero_bytes(b[j] ^ rep);
    return acc != 0x80808080u;
}
__device__ __forceinline__ uint32_t byte_bits(const v4u a, const v4u b, uint32_t rep) {
    uint32_t m = 0;
#pragma unroll
    for (int v = 0; v < 2; v++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t x = v ? b[j] : a[j];
            const uint32_t f = ~nonzero_bytes(x ^ rep) & 0x80808080u;
            uint32_t t = (f >> 7);
            t = t | (t >> 7);
            t = t | (t >> 14);
            m |= (t & 0xFu) << ((v * 4 + j) * 4);
        }
    }
    return m;
}

// same-wave LDS hand-off: DS operations of one wave complete in order, so only
// the compiler must not move accesses across this point
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t ctz64(uint64_t x) { return (uint32_t)__builtin_ctzg(x, 64); }
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t fmix(uint32_t x) {      // murmur3 finaliser
    x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
    return x;
}

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

// raw bytes of a field of `len` <= 8 at window offset o, zero padded; false when
// a byte <= ' ' (blank, control, NUL) is inside: those need the general parser
__device__ __forceinline__ bool raw8(const uint8_t* bytes, uint32_t o, uint32_t len, uint64_t& w) {
    uint32_t d0, d1;
    load8(bytes, o, d0, d1);
    const uint64_t k = len >= 8 ? ~0ULL : ((1ULL << (8 * len)) - 1);
    w = ((uint64_t)d0 | ((uint64_t)d1 << 32)) & k;
    return lt64(w | ~k, 0x21 * B01) == 0;
}

// exact typing of a field (infer_type + parse_value); false: only the general
// parser can tell (dates, signs, long numerals, blanks ...)
__device__ __forceinline__ bool type_field(const uint8_t* bytes, uint32_t o, uint32_t len, bool num_ok, Cell& c) {
    if (len == 0) { c = cell_null(); return true; }
    uint64_t kw;
    if (lean_field(bytes, o, len, num_ok, c, kw)) return true;
    GKey unused;
    return fast_field(bytes, o, len, num_ok, false, c, unused) == FF_OK;
}

// LDS group table (structure of arrays carved from dynamic LDS), raw-byte keys
struct LTab {
    uint32_t H;
    v4u* A;               // {header, first-row code, key bytes 0-3, key bytes 4-7}
    uint2* B;             // key bytes 8-15
    uint32_t* cnt;
    double* sum[MAXS];
    uint32_t* miss[MAXS]; // SUM arguments that were not numeric
};

// find or insert raw key (len, w0, w1) with hash h; -1 when the probe window is
// full.  `a` returns the slot's first 16 bytes as read (first-row code in a.y).
__device__ __forceinline__ int lt_find(const LTab& t, uint32_t len, uint64_t w0, uint64_t w1, uint32_t h, v4u& a) {
    const uint32_t hd = 0x80000000u | (h & 0x7FF80000u) | len;
    const uint32_t k0 = (uint32_t)w0, k1 = (uint32_t)(w0 >> 32);
    const bool wide = len > 8;
    for (uint32_t probe = 0; probe < PROBES; probe++) {
        const uint32_t i = (h + probe) & (t.H - 1);
        uint32_t* ap = (uint32_t*)(t.A + i);
        a = t.A[i];
        if (a.x == hd && a.z == k0 && a.w == k1) {
            if (!wide) return (int)i;
            const uint2 b = t.B[i];
            if (b.x == (uint32_t)w1 && b.y == (uint32_t)(w1 >> 32)) return (int)i;
        }
        uint32_t cur = a.x;
        if (cur == 0) {
            const uint32_t old = atomicCAS(ap, 0u, 1u);
            if (old == 0) {
                ap[2] = k0;
                ap[3] = k1;
                t.B[i] = make_uint2((uint32_t)w1, (uint32_t)(w1 >> 32));
                __hip_atomic_store(ap, hd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                a.x = hd;
                a.y = NOFIRST;
                return (int)i;
            }
            cur = old;
        }
        for (uint32_t spin = 0; cur == 1; spin++) {
            if (spin > (1u << 20)) return -1;             // the HBM table takes the record
            cur = __hip_atomic_load(ap, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (cur == hd) {                                   // published meanwhile: re-read the key
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            a = t.A[i];
            if (a.z == k0 && a.w == k1) {
                if (!wide) return (int)i;
                const uint2 b = t.B[i];
                if (b.x == (uint32_t)w1 && b.y == (uint32_t)(w1 >> 32)) return (int)i;
            }
        }
    }
    return -1;
}

__device__ __forceinline__ uint32_t key_hash(uint32_t len, uint64_t w0, uint64_t w1) {
    return fmix((uint32_t)w0 ^ rotl((uint32_t)(w0 >> 32), 11) ^ rotl((uint32_t)w1, 19) ^
                rotl((uint32_t)(w1 >> 32), 27) ^ (len << 26));
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

// GROUPED: GROUP BY (else one group); WM: W_NONE / W_SIMPLE; NS: distinct SUM arguments
template <bool GROUPED, int WM, int NS>
__global__ __launch_bounds__(LT) void lean_kernel(const uint8_t* __restrict__ g, ScanStats* __restrict__ stats,
                                                  unsigned long long* __restrict__ row_out,
                                                  unsigned long long row_cap, uint32_t lds_h,
                                                  unsigned long long* __restrict__ slow_list,
                                                  unsigned long long slow_cap) {
    constexpr int KN = 4;
    constexpr int NR = 1 + NS;                         // memo roles: 0 WHERE, 1 + j SUM j
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    const GroupTable& rt = c_rt;
    const LeanPlan& LP = c_lp;
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t* q = smem;
    WaveLds* waves = (WaveLds*)carve(q, sizeof(WaveLds) * NWV);
    v4u* memo = (v4u*)carve(q, sizeof(v4u) * MEMO_N * NR);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    WaveLds& W = waves[wv];
    LTab lt;
    lt.H = lds_h;
    lt.A = nullptr; lt.B = nullptr; lt.cnt = nullptr;
#pragma unroll
    for (int s = 0; s < MAXS; s++) { lt.sum[s] = nullptr; lt.miss[s] = nullptr; }
    if (GROUPED) {
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
    }
    for (uint32_t i = tid; i < (uint32_t)(MEMO_N * NR); i += LT) memo[i] = v4u{0u, 0u, 0u, 0u};   // raw 0: empty
    __syncthreads();

    // uniform plan facts
    const int nneed = P.nneed;
    const int gslot = GROUPED ? P.group_slot : -1;
    const Cell wconst = WM == W_SIMPLE ? P.consts[LP.wconst] : cell_null();
    const uint32_t wop = WM == W_SIMPLE ? LP.wop : 0u;
    const bool pass_null = WM == W_SIMPLE ? cmp_result(wop, compare(cell_null(), wconst)) : true;
    int rslot[NR];                                     // need slot of each memo role (-1: none)
    rslot[0] = WM == W_SIMPLE ? LP.wslot : -1;
#pragma unroll
    for (int j = 0; j < NS; j++) rslot[1 + j] = j < LP.ns ? LP.sum_slot[j] : -1;
    const uint32_t rep_d = P.delim * 0x01010101u, rep_q = P.quote * 0x01010101u;
    const bool num_ok = true;                          // the host admits plans whose delimiter no numeral parse consumes
    const uint64_t lo_ok = P.data_begin > P.range_begin ? P.data_begin : P.range_begin;
    const uint64_t hi_ok = P.range_end < P.n ? P.range_end : P.n;
    const uint64_t first_win = P.range_begin / WS;
    const uint64_t last_win = (hi_ok + WS - 1) / WS;
    const uint64_t tile_g = (uint64_t)(uintptr_t)W.bytes;

    // per-lane single-group partials and per-wave statistics
    uint32_t my_cnt = 0;
    unsigned long long my_first = ~0ULL;
    double my_sum[MAXS] = {0.0, 0.0};
    uint32_t my_num[MAXS] = {0u, 0u};
    unsigned long long n_rec = 0, n_pass = 0, n_spill = 0;
    uint32_t m_look[NR], m_miss[NR];                   // memo statistics (wave-uniform)
    bool m_on[NR];
#pragma unroll
    for (int r = 0; r < NR; r++) { m_look[r] = 0; m_miss[r] = 0; m_on[r] = true; }

    Win nx;
    uint64_t w = first_win + (uint64_t)blockIdx.x * NWV + wv;
    if (w < last_win) load_win(g, w, nx);
    for (uint32_t round = 0; w < last_win; round++, w += (uint64_t)gridDim.x * NWV) {
        const uint64_t ws = w * WS;
        const Win cur = nx;
        if (w + (uint64_t)gridDim.x * NWV < last_win) load_win(g, w + (uint64_t)gridDim.x * NWV, nx);

        // ---- stage and classify
        ((v4u*)W.bytes)[2 * lane] = cur.a;
        ((v4u*)W.bytes)[2 * lane + 1] = cur.b;
#if defined(LEAN_PROF) && LEAN_PROF == 0   // profiling build: loads + staging only
        if (lane == 0) n_rec += W.bytes[w & 2047];
        continue;
#endif
        uint32_t sep, nl;
        classify(cur.a, cur.b, rep_d, sep, nl);
        W.bm[lane] = make_uint2(sep, nl);
        const bool wq = __ballot(any_byte(cur.a, cur.b, rep_q)) != 0;   // window holds a quote (uniform)
        if (wq) W.qt[lane] = byte_bits(cur.a, cur.b, rep_q);

        // ---- record starts owned by this window: [ws, ws + WS) within [lo_ok, hi_ok)
        const uint32_t prevnl = (uint32_t)__builtin_amdgcn_update_dpp((int)(cur.prev == '\n' || cur.prev == '\r'),
                                                                      (int)(nl >> 31), 0x138, 0xf, 0xf, false);
        uint32_t starts = ~nl & ((nl << 1) | prevnl);
        {
            const uint64_t base = ws + (uint64_t)lane * LB;
            const uint64_t lo = lo_ok > ws ? lo_ok : ws;
            const uint64_t hi = hi_ok < ws + WS ? hi_ok : ws + WS;
            if (base + LB <= lo || base >= hi) {
                starts = 0;
            } else {
                if (base < lo) starts &= ~0u << (lo - base);
                if (base + LB > hi) starts &= (1u << (hi - base)) - 1;
            }
        }
        const uint32_t nst = (uint32_t)__popc(starts);
        const uint32_t incl = wave_incl_scan(nst);
        const uint32_t rbase = incl - nst;
        const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);

#if defined(LEAN_PROF) && LEAN_PROF == 1   // profiling build: + classify, bitmaps, record numbering
        n_rec += R;
        continue;
#endif
        for (uint32_t pass = 0; pass < R; pass += RSN) {
            // this pass's record starts -> W.rs
            {
                uint32_t m = starts, r = rbase;
                while (m) {
                    const uint32_t b = (uint32_t)__builtin_ctz(m);
                    m &= m - 1;
                    if (r >= pass && r < pass + RSN) W.rs[r - pass] = (uint16_t)(lane * LB + b);
                    r++;
                }
            }
            wave_sync();
            const bool valid = pass + lane < R;
            const uint32_t p = valid ? W.rs[lane] : 0u;

            // ---- field bounds of the need slots (separator bits only, unrolled)
            uint64_t sv, nv;
            views(W, p, sv, nv);
            const uint32_t e = ctz64(nv);                  // record end (64: beyond the view)
            uint64_t s = sv;
            uint32_t col = 0, fstart = 0, lastpos = 0;
            bool fail = !valid, gone = false;
            uint32_t fpos[KN], flen[KN];
            bool fex[KN];
#pragma unroll
            for (int k = 0; k < KN; k++) {
                fpos[k] = 0; flen[k] = 0; fex[k] = false;
                if (k >= nneed) break;
                const uint32_t c = (uint32_t)P.need_col[k];
                for (; col < c; col++) {                   // skip to column c (uniform trip count)
                    fstart = ctz64(s) + 1;
                    s &= s - 1;
                }
                if (!gone && fstart > e) {                 // the record ended before column c
                    gone = true;
                    if (e == 64) fail = true;              // ... or we cannot see where: general path
                    lastpos = e;
                }
                if (!gone) {
                    const uint32_t fe = ctz64(s);
                    if (fe == 64) fail = true;             // field runs past the view
                    fpos[k] = p + fstart;
                    flen[k] = fe - fstart;
                    fex[k] = true;
                    lastpos = fe;
                    s &= s - 1;
                    col = c + 1;
                    fstart = fe + 1;
                }
            }
            // a quote at or before the last byte examined may hide separators
            if (wq && valid && (qview(W, p) & ((2ULL << (lastpos < 63 ? lastpos : 63)) - 1))) fail = true;

#if defined(LEAN_PROF) && LEAN_PROF == 2   // profiling build: + record list and field walk
            n_rec += __popcll(__ballot(fail || ((fpos[0] + flen[KN - 1]) & 1)));
            wave_sync();
            continue;
#endif
            // ---- WHERE outcome and SUM addends: memo lookups (unrolled over roles)
            uint64_t val[NR], raw[NR];
            uint32_t midx[NR];
            uint32_t todo = 0;                             // roles this lane must type (bit r), memo fill (bit 8 + r)
#pragma unroll
            for (int r = 0; r < NR; r++) {
                val[r] = r == 0 ? (uint64_t)pass_null : MV_NOTNUM;   // missing column / empty field: NULL
                raw[r] = 0;
                midx[r] = 0;
                const int slot = rslot[r];
                if (slot < 0) continue;                    // uniform
                uint32_t fp = fpos[0], fl = flen[0];
                bool ex = fex[0];
#pragma unroll
                for (int k = 1; k < KN; k++)
                    if (k == slot) { fp = fpos[k]; fl = flen[k]; ex = fex[k]; }
                if (fail || !ex || fl == 0) continue;
                bool memo_ok = false;
                if (fl <= 8 && m_on[r]) {
                    uint64_t x;
                    if (raw8(W.bytes, fp, fl, x)) {
                        const uint32_t mi = fmix((uint32_t)x ^ rotl((uint32_t)(x >> 32), 16)) & (MEMO_N - 1);
                        const v4u m = memo[r * MEMO_N + mi];
                        raw[r] = x;
                        midx[r] = mi;
                        memo_ok = true;
                        if (m.x == (uint32_t)x && m.y == (uint32_t)(x >> 32)) {
                            val[r] = (uint64_t)m.z | ((uint64_t)m.w << 32);
                            continue;
                        }
                    }
                }
                todo |= (1u << r) | (memo_ok ? (0x100u << r) : 0u);
            }
#pragma unroll
            for (int r = 0; r < NR; r++) {                 // memo hit statistics, per wave
                if (rslot[r] < 0 || !m_on[r]) continue;
                const uint32_t looked = (uint32_t)__popcll(__ballot(raw[r] != 0));
                const uint32_t missed = (uint32_t)__popcll(__ballot(((todo >> (8 + r)) & 1) != 0));
                m_look[r] += looked;
                m_miss[r] += missed;
            }
            if (__any(todo & 0xFF)) {                      // misses: the exact typers, one site
#pragma unroll 1
                for (int r = 0; r < NR; r++) {
                    if (!__any((todo >> r) & 1)) continue;
                    const int slot = rslot[r];
                    uint32_t fp = fpos[0], fl = flen[0];
#pragma unroll
                    for (int k = 1; k < KN; k++)
                        if (k == slot) { fp = fpos[k]; fl = flen[k]; }
                    if ((todo >> r) & 1) {
                        Cell c;
                        uint64_t v;
                        if (!type_field(W.bytes, fp, fl, num_ok, c)) {
                            v = MV_SLOW;
                        } else {
                            if (c.kind == K_STR) c.bits = tile_g + fp;
                            if (r == 0) v = cmp_result(wop, compare(c, wconst)) ? 1u : 0u;
                            else v = is_num(c) ? dbl_bits(num_of(c)) : MV_NOTNUM;
                        }
                        uint64_t x = raw[0];
                        uint32_t mi = midx[0];
#pragma unroll
                        for (int j = 1; j < NR; j++)
                            if (j == r) { x = raw[j]; mi = midx[j]; }
                        if ((todo >> (8 + r)) & 1)
                            memo[r * MEMO_N + mi] = v4u{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)v, (uint32_t)(v >> 32)};
#pragma unroll
                        for (int j = 0; j < NR; j++)
                            if (j == r) val[j] = v;
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < NR; r++)
                if (val[r] == MV_SLOW) fail = true;

            // ---- GROUP BY key: the raw field bytes (<= 16, no byte <= ' ')
            uint32_t klen = 0;
            uint64_t kw0 = 0, kw1 = 0;
            if (GROUPED && !fail) {
                uint32_t fp = fpos[0], fl = flen[0];
                bool ex = fex[0];
#pragma unroll
                for (int k = 1; k < KN; k++)
                    if (k == gslot) { fp = fpos[k]; fl = flen[k]; ex = fex[k]; }
                if (ex && fl > 0) {
                    klen = fl;
                    if (fl <= 8) {
                        if (!raw8(W.bytes, fp, fl, kw0)) fail = true;
                    } else if (fl <= 16) {
                        if (!raw8(W.bytes, fp, 8, kw0) || !raw8(W.bytes, fp + 8, fl - 8, kw1)) fail = true;
                    } else {
                        fail = true;
                    }
                }
            }

            // ---- declined records go whole to slow_kernel
            const uint64_t rec = ws + p;
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
            const bool ok = valid && !fail;
            const bool pass_ = ok && (WM == W_NONE || val[0] == 1);
            n_rec += (unsigned long long)__popcll(__ballot(ok));
            n_pass += (unsigned long long)__popcll(__ballot(pass_));
            if (row_out) {
                const unsigned long long slot = wave_slot(pass_, &stats->rows_emitted);
                if (pass_ && slot < row_cap) row_out[slot] = rec;
            }
#if defined(LEAN_PROF) && LEAN_PROF == 3   // profiling build: + values, filter, keys
            n_rec += __popcll(__ballot((kw0 ^ val[NR - 1]) & 1));
            wave_sync();
            continue;
#endif

            // ---- aggregate
            if (!GROUPED) {
                if (pass_) {
                    my_cnt++;
                    if (rec < my_first) my_first = rec;
#pragma unroll
                    for (int j = 0; j < NS; j++)
                        if (val[1 + j] != MV_NOTNUM) { my_sum[j] += as_dbl(val[1 + j]); my_num[j]++; }
                }
            } else {
                int slot = -1;
                const uint32_t h = key_hash(klen, kw0, kw1);
                if (pass_) {
                    v4u a;
                    slot = lt_find(lt, klen, kw0, kw1, h, a);
                    if (slot >= 0) {
                        const uint32_t fc = (round << 15) | ((uint32_t)wv << 11) | p;
                        atomicAdd(&lt.cnt[slot], 1u);
                        if (fc < a.y) atomicMin((uint32_t*)(lt.A + slot) + 1, fc);
#pragma unroll
                        for (int j = 0; j < NS; j++) {
                            if (val[1 + j] != MV_NOTNUM) atomicAdd(&lt.sum[j][slot], as_dbl(val[1 + j]));
                            else atomicAdd(&lt.miss[j][slot], 1u);
                        }
                    }
                }
                const bool spill = pass_ && slot < 0;
                if (__any(spill)) {                        // LDS table full: straight to the HBM raw table
                    n_spill += (unsigned long long)__popcll(__ballot(spill));
                    if (spill) {
                        const GKey k = raw_key(klen, kw0, kw1);
                        const int gi = g_insert(rt, k, gk_hash(k), stats);
                        if (gi >= 0) {
                            atomicAdd(&rt.cnt[gi], 1ULL);
                            atomicMin(&rt.first[gi], (unsigned long long)rec);
                            for (int a = 0; a < P.nacc; a++) {
                                const uint64_t v = LP.acc_sidx[a] == 0 ? val[1] : val[NR - 1];
                                if (v != MV_NOTNUM) {
                                    atomicAdd(&rt.sum[a][gi], as_dbl(v));
                                    atomicAdd(&rt.num[a][gi], 1ULL);
                                }
                            }
                        }
                    }
                }
            }
            wave_sync();                                   // W.rs is rewritten by the next pass
        }
        // a column whose memo misses more than half the time stops consulting it
#pragma unroll
        for (int r = 0; r < NR; r++)
            if (m_on[r] && m_look[r] >= 512 && 2 * m_miss[r] > m_look[r]) m_on[r] = false;
    }

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
            GKey k;
            k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
            const int gi = g_insert(gt, k, 0x12345678ULL, stats);
            if (gi >= 0) {
                if (c) atomicAdd(&gt.cnt[gi], c);
                if (f != ~0ULL) atomicMin(&gt.first[gi], f);
                for (int a = 0; a < P.nacc; a++) {
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
            const uint64_t fw = first_win + ((uint64_t)(a.y >> 15) * gridDim.x + blockIdx.x) * NWV + ((a.y >> 11) & 15);
            atomicMin(&rt.first[gi], (unsigned long long)(fw * WS + (a.y & 2047)));
        }
        for (int acc = 0; acc < P.nacc; acc++) {
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
__global__ __launch_bounds__(256) void raw_merge_kernel(ScanStats* __restrict__ stats) {
    const GroupTable& gt = c_gt;
    const GroupTable& rt = c_rt;
    const ScanPlan& P = c_plan;
    __shared__ __align__(16) uint8_t buf[256 * 32];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= rt.cap || rt.tag[i] < 2) return;
    const GKey k = canonical_key(buf + threadIdx.x * 32, rt.clslen[i] & 0xFFFF, rt.w0[i], rt.w1[i]);
    const int gi = g_insert(gt, k, gk_hash(k), stats);
    if (gi < 0) return;
    atomicAdd(&gt.cnt[gi], rt.cnt[i]);
    atomicMin(&gt.first[gi], rt.first[i]);
    for (int a = 0; a < P.nacc; a++) {
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

bool lean_shape(const ScanPlan* P, LeanPlan* lp, int* wm) {
    if (P->nneed > 4 || P->nacc > MAX_ACC) return false;
    // numeral parses (strtod / strtoll) must stop at the delimiter
    const uint32_t d = P->delim;
    if ((d - '0') < 10u || d == '.' || ((d | 32) >= 'a' && (d | 32) <= 'z') || d == '+' || d == '-') return false;
    if (d == '\n' || d == '\r' || d <= ' ') return false;
    *lp = LeanPlan{};
    lp->wslot = -1;
    for (int a = 0; a < P->nacc; a++) {
        if (P->acc[a].kind != ACC_SUM) return false;
        const int slot = P->acc[a].slot;
        int j = 0;
        while (j < lp->ns && lp->sum_slot[j] != slot) j++;
        if (j == lp->ns) {
            if (lp->ns == lean::MAXS) return false;
            lp->sum_slot[lp->ns++] = slot;
        }
        lp->acc_sidx[a] = j;
    }
    if (P->nprog == 0) {
        *wm = W_NONE;
    } else if (P->nprog == 3 && P->prog[0].op == OP_COL && P->prog[1].op == OP_CONST && P->prog[2].op == OP_CMP) {
        *wm = W_SIMPLE;
        lp->wslot = P->prog[0].a;
        lp->wconst = P->prog[1].b;
        lp->wop = P->prog[2].a;
    } else {
        return false;
    }
    return true;
}

int ns_of(const LeanPlan& lp) { return lp.ns > 1 ? 2 : 1; }
size_t lean_slot_bytes(int ns) { return 16 + 8 + 4 + (size_t)ns * 12; }
size_t lean_fixed_bytes(int ns) {
    return sizeof(lean::WaveLds) * lean::NWV + sizeof(v4u) * lean::MEMO_N * (1 + ns);
}

uint32_t lean_slots(int ns, int grouped) {
    if (!grouped) return 0;
    uint32_t h = 2048;
    while (h > 64 && lean_fixed_bytes(ns) + (size_t)h * lean_slot_bytes(ns) + 256 > (size_t)(160 * 1024)) h >>= 1;
    return h;
}
size_t lean_lds(int ns, int grouped) {
    return lean_fixed_bytes(ns) + (size_t)lean_slots(ns, grouped) * lean_slot_bytes(ns) + 256;
}

typedef void (*lean_fn_t)(const uint8_t*, ScanStats*, unsigned long long*, unsigned long long, uint32_t,
                          unsigned long long*, unsigned long long);

template <bool G>
lean_fn_t pick(int wm, int ns) {
    if (wm == W_NONE) return ns <= 1 ? lean::lean_kernel<G, W_NONE, 1> : lean::lean_kernel<G, W_NONE, 2>;
    return ns <= 1 ? lean::lean_kernel<G, W_SIMPLE, 1> : lean::lean_kernel<G, W_SIMPLE, 2>;
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
uint64_t cq_lean_windows(uint64_t begin, uint64_t end) {
    return (end + lean::WS - 1) / lean::WS - begin / lean::WS;
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
    const int ns = ns_of(lp);
    const uint32_t h = lean_slots(ns, grouped);
    const size_t lds = lean_lds(ns, grouped);
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(lean::c_plan), P, sizeof *P, 0, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyToSymbolAsync(HIP_SYMBOL(lean::c_gt), gt, sizeof *gt, 0, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyToSymbolAsync(HIP_SYMBOL(lean::c_lp), &lp, sizeof lp, 0, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && rt)
        e = hipMemcpyToSymbolAsync(HIP_SYMBOL(lean::c_rt), rt, sizeof *rt, 0, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    const lean_fn_t fn = grouped ? pick<true>(wm, ns) : pick<false>(wm, ns);
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(lean::LT), lds, s, g, stats, row_out, row_cap, h, slow_list, slow_cap);
    return hipGetLastError();
}

// raw-key table -> canonical table (after cq_launch_lean of a grouped plan)
hipError_t cq_launch_raw_merge(const cq::GroupTable* rt, cq::ScanStats* stats, hipStream_t s) {
    hipLaunchKernelGGL(lean::raw_merge_kernel, dim3((rt->cap + 255) / 256), dim3(256), 0, s, stats);
    return hipGetLastError();
}

}  // extern "C"
