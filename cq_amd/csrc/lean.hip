// lean.hip -- the wave-autonomous CSV scan for the common SELECT plan shapes.
//
// Same job as scan_kernel (scan.hip) -- csv_load + filter_rows + create_groups +
// evaluate_aggregate in one pass over the HBM-resident bytes (reference
// csv_reader.c:375-465, evaluator_utils.c:986, evaluator_aggregates.c:108-414) --
// for plans whose WHERE is absent or `column op literal` and whose aggregates are
// COUNT / SUM / AVG (at most 4 parsed columns, 2 distinct SUM arguments).
//
// Every wave works on its own 2 KiB window with no block barrier in the loop, so
// one wave's byte classification overlaps another's record typing and hash
// updates on the same SIMD (scan_kernel's block-wide phases serialise them):
//
//   load      lane l holds window bytes [32l, 32l + 32) in registers (two 16-byte
//             non-temporal loads, issued one window ahead), lanes 0-3 also the
//             128-byte tail after the window; staged to the wave's LDS area
//   classify  per lane two 32-bit masks -- separators (delimiter and record
//             terminators '\n' '\r') and terminators -- plus a quote mask when
//             the window holds a quote; stored as the window's LDS bitmaps
//   starts    record starts owned by the window (previous byte a terminator);
//             one DPP wave scan numbers them, 64 per pass go to an LDS list
//   fields    one lane per record: a funnel shift gives the 64 separator and
//             terminator bits from the record start, field c ends at the c-th
//             set separator bit; the needed fields are typed from LDS by the
//             fast field typers (scanlib.h).  A record the fast path cannot
//             prove identical to parse_line + parse_value (a quote before its
//             last needed field, a needed field past its first 64 bytes,
//             blanks, control bytes, date-shaped or long numerals) goes whole to
//             the slow list and slow_kernel (scan.hip)
//   filter    direct `cell op literal` (value_compare, csv_reader.c:98-130)
//   group     block-shared LDS open-addressing table: one 16-byte read brings
//             the slot header, its first-row code and the key's first 8 bytes;
//             COUNT and SUM are fire-and-forget LDS atomics; flushed once per
//             block into the HBM table shared with slow_kernel
#include <hip/hip_runtime.h>
#include <cstring>
#include "plan.h"
#include "scanlib.h"

namespace cq {
namespace lean {

constexpr int LT = 1024;                  // threads per block
constexpr int NWV = LT / 64;              // waves per block
constexpr int LB = 32;                    // window bytes per lane
constexpr int WB = 64 * LB;               // window bytes (2 KiB)
constexpr int TB = 128;                   // tail bytes staged after the window
constexpr int NTL = TB / LB;              // lanes loading the tail (4)
constexpr int NMW = (WB + TB) / 32;       // 32-bit bitmap words per window (68)
constexpr int WBYTES = WB + TB + 32;      // staged bytes + slack for 16-byte field loads
constexpr int RSN = 64;                   // record slots per pass
constexpr int MAXS = 2;                   // distinct SUM arguments
constexpr int PROBES = 32;                // LDS probe window before spilling to HBM
constexpr uint32_t NOFIRST = 0xFFFFFFFFu;

// per-wave LDS area
struct WaveLds {
    uint8_t bytes[WBYTES];
    uint2 bm[NMW + 4];          // {separator bits, terminator bits} per 32 window bytes
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
__constant__ GroupTable c_gt;
__constant__ LeanPlan c_lp;

struct Win {            // one window in flight
    v4u a, b;           // bytes [32l, 32l + 32)
    v4u ta, tb;         // tail bytes (lanes < NTL)
    uint32_t prev;      // byte before the window (lane 0)
};

__device__ __forceinline__ void load_win(const uint8_t* g, uint64_t w, Win& x) {
    const uint64_t ws = w * WB;
    const v4u* src = (const v4u*)(g + ws);
    const int lane = threadIdx.x & 63;
    x.a = __builtin_nontemporal_load(src + 2 * lane);
    x.b = __builtin_nontemporal_load(src + 2 * lane + 1);
    if (lane < NTL) {
        x.ta = src[WB / 16 + 2 * lane];
        x.tb = src[WB / 16 + 2 * lane + 1];
    }
    x.prev = lane == 0 ? (uint32_t)g[ws - 1] : 0u;   // g has 64 padding bytes before byte 0
}

// separator / terminator / quote bits of 32 bytes (bit i = byte i)
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

// LDS group table (structure of arrays carved from dynamic LDS)
struct LTab {
    uint32_t H;
    v4u* A;               // {header, first-row code, key w0 lo, key w0 hi}
    uint2* B;             // key w1
    uint32_t* cnt;
    double* sum[MAXS];
    uint32_t* miss[MAXS]; // SUM arguments that were not numeric
};

// find or insert key k (hash h, LDS header hd); -1 when the probe window is full.
// `a` returns the slot's first 16 bytes as read (first-row code in a.y).
__device__ __forceinline__ int lt_find(const LTab& t, const GKey& k, uint64_t h, uint32_t hd, v4u& a) {
    const uint32_t k0 = (uint32_t)k.w0, k1 = (uint32_t)(k.w0 >> 32);
    const bool wide = k.cls == GK_STR && k.len > 8;    // the only keys with w1 != 0
    for (uint32_t probe = 0; probe < PROBES; probe++) {
        const uint32_t i = (uint32_t)(h + probe) & (t.H - 1);
        a = t.A[i];
        if (a.x == hd && a.z == k0 && a.w == k1) {
            if (!wide) return (int)i;
            const uint2 b = t.B[i];
            if (b.x == (uint32_t)k.w1 && b.y == (uint32_t)(k.w1 >> 32)) return (int)i;
        }
        uint32_t cur = a.x;
        if (cur == 0) {
            const uint32_t old = atomicCAS((uint32_t*)(t.A + i), 0u, 1u);
            if (old == 0) {
                ((uint32_t*)(t.A + i))[2] = k0;
                ((uint32_t*)(t.A + i))[3] = k1;
                t.B[i] = make_uint2((uint32_t)k.w1, (uint32_t)(k.w1 >> 32));
                __hip_atomic_store((uint32_t*)(t.A + i), hd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                a.x = hd;
                a.y = NOFIRST;
                return (int)i;
            }
            cur = old;
        }
        for (uint32_t spin = 0; cur == 1; spin++) {
            if (spin > (1u << 20)) return -1;             // the HBM table takes the record
            cur = __hip_atomic_load((uint32_t*)(t.A + i), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (cur == hd) {                                   // published meanwhile: re-read the key
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            a = t.A[i];
            if (a.z == k0 && a.w == k1) {
                if (!wide) return (int)i;
                const uint2 b = t.B[i];
                if (b.x == (uint32_t)k.w1 && b.y == (uint32_t)(k.w1 >> 32)) return (int)i;
            }
        }
    }
    return -1;
}

// group key of a non-string cell (INT / DOUBLE from the fast typers), out of line
__device__ __noinline__ GKey gkey_num(const Cell c) { return group_key(c); }

__device__ __forceinline__ uint8_t* carve(uint8_t*& q, size_t bytes) {
    uint8_t* r = q;
    q += (bytes + 15) & ~(size_t)15;
    return r;
}

// GROUPED: GROUP BY (else one group); WM: W_NONE / W_SIMPLE (scan.hip enum values);
// KN: need slots (<= 4); NS: distinct SUM arguments.
template <bool GROUPED, int WM, int NS>
__global__ __launch_bounds__(LT) void lean_kernel(const uint8_t* __restrict__ g, ScanStats* __restrict__ stats,
                                                  unsigned long long* __restrict__ row_out,
                                                  unsigned long long row_cap, uint32_t lds_h,
                                                  unsigned long long* __restrict__ slow_list,
                                                  unsigned long long slow_cap) {
    constexpr int KN = 4;
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    const LeanPlan& LP = c_lp;
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t* q = smem;
    WaveLds* waves = (WaveLds*)carve(q, sizeof(WaveLds) * NWV);
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
        __syncthreads();
    }

    // uniform plan facts
    const int nneed = P.nneed;
    const int gslot = GROUPED ? P.group_slot : -1;
    const int wslot = WM == W_SIMPLE ? LP.wslot : -1;
    const uint32_t wop = WM == W_SIMPLE ? LP.wop : 0u;
    const Cell wconst = WM == W_SIMPLE ? P.consts[LP.wconst] : cell_null();
    const bool wnum = is_num(wconst);
    const double wval = wnum ? num_of(wconst) : 0.0;
    int sslot[MAXS];
#pragma unroll
    for (int s = 0; s < MAXS; s++) sslot[s] = (s < NS && s < LP.ns) ? LP.sum_slot[s] : -1;
    const GKey null_key = group_key(cell_null());
    const uint32_t rep_d = P.delim * 0x01010101u, rep_q = P.quote * 0x01010101u;
    const bool num_ok = !(is_digit(P.delim) || P.delim == '.' || ((P.delim | 32) >= 'a' && (P.delim | 32) <= 'z'));
    const uint64_t lo_ok = P.data_begin > P.range_begin ? P.data_begin : P.range_begin;
    const uint64_t hi_ok = P.range_end < P.n ? P.range_end : P.n;
    const uint64_t first_win = P.range_begin / WB;
    const uint64_t last_win = (hi_ok + WB - 1) / WB;
    const uint64_t tile_g = (uint64_t)(uintptr_t)W.bytes;

    // per-lane single-group partials and per-wave statistics
    uint32_t my_cnt = 0;
    unsigned long long my_first = ~0ULL;
    double my_sum[MAXS] = {0.0, 0.0};
    uint32_t my_num[MAXS] = {0u, 0u};
    unsigned long long n_rec = 0, n_pass = 0, n_spill = 0;

    Win nx;
    uint64_t w = first_win + (uint64_t)blockIdx.x * NWV + wv;
    if (w < last_win) load_win(g, w, nx);
    for (uint32_t round = 0; w < last_win; round++, w += (uint64_t)gridDim.x * NWV) {
        const uint64_t ws = w * WB;
        const Win cur = nx;
        if (w + (uint64_t)gridDim.x * NWV < last_win) load_win(g, w + (uint64_t)gridDim.x * NWV, nx);

        // ---- stage and classify
        ((v4u*)W.bytes)[2 * lane] = cur.a;
        ((v4u*)W.bytes)[2 * lane + 1] = cur.b;
        uint32_t sep, nl;
        classify(cur.a, cur.b, rep_d, sep, nl);
        W.bm[lane] = make_uint2(sep, nl);
        bool hq = any_byte(cur.a, cur.b, rep_q);
        if (lane < NTL) {
            ((v4u*)W.bytes)[WB / 16 + 2 * lane] = cur.ta;
            ((v4u*)W.bytes)[WB / 16 + 2 * lane + 1] = cur.tb;
            uint32_t ts, tn;
            classify(cur.ta, cur.tb, rep_d, ts, tn);
            W.bm[64 + lane] = make_uint2(ts, tn);
            hq = hq || any_byte(cur.ta, cur.tb, rep_q);
        }
        const bool wq = __ballot(hq) != 0;                 // window holds a quote (uniform)
        if (wq) {
            W.qt[lane] = byte_bits(cur.a, cur.b, rep_q);
            if (lane < NTL) W.qt[64 + lane] = byte_bits(cur.ta, cur.tb, rep_q);
        }

        // ---- record starts owned by this window
        const uint32_t prevnl = (uint32_t)__builtin_amdgcn_update_dpp((int)(cur.prev == '\n' || cur.prev == '\r'),
                                                                      (int)(nl >> 31), 0x138, 0xf, 0xf, false);
        uint32_t starts = ~nl & ((nl << 1) | prevnl);
        if (ws < lo_ok || ws + WB > hi_ok) {               // first / last window of the range
            const uint64_t base = ws + (uint64_t)lane * LB;
            if (base + LB <= lo_ok || base >= hi_ok) {
                starts = 0;
            } else {
                if (base < lo_ok) starts &= ~0u << (lo_ok - base);
                if (base + LB > hi_ok) starts &= (1u << (hi_ok - base)) - 1;
            }
        }
        const uint32_t nst = (uint32_t)__popc(starts);
        const uint32_t incl = wave_incl_scan(nst);
        const uint32_t rbase = incl - nst;
        const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);

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
            // ---- type the fields the plan uses, one typing site (role loop, not unrolled):
            //      role 0 the WHERE column, 1 the GROUP BY column, 2.. the SUM arguments
            Cell wc = cell_null();
            Cell sc[MAXS];
#pragma unroll
            for (int j = 0; j < MAXS; j++) sc[j] = cell_null();
            GKey key = null_key;
#pragma unroll 1
            for (int r = 0; r < 2 + NS; r++) {
                const int slot = r == 0 ? wslot : (r == 1 ? gslot : sslot[r - 2 < MAXS ? r - 2 : 0]);
                if (slot < 0) continue;                    // uniform
                uint32_t fp = fpos[0], fl = flen[0];
                bool ex = fex[0];
#pragma unroll
                for (int k = 1; k < KN; k++)
                    if (k == slot) { fp = fpos[k]; fl = flen[k]; ex = fex[k]; }
                Cell cell = cell_null();
                GKey kk = null_key;
                if (ex && !fail) {
                    uint64_t kw = 0;
                    if (lean_field(W.bytes, fp, fl, num_ok, cell, kw)) {
                        if (r == 1) {
                            if (cell.kind == K_STR) { kk.cls = GK_STR; kk.len = fl; kk.w0 = kw; kk.w1 = 0; }
                            else kk = gkey_num(cell);
                        }
                    } else {
                        fail = fast_field(W.bytes, fp, fl, num_ok, r == 1, cell, kk) != FF_OK;
                    }
                    if (cell.kind == K_STR) cell.bits = tile_g + fp;
                }
                if (r == 0) wc = cell;
                if (r == 1) key = kk;
#pragma unroll
                for (int j = 0; j < MAXS; j++)
                    if (r == 2 + j) sc[j] = cell;
            }
            // a quote at or before the last byte examined may hide separators
            if (wq && valid && (qview(W, p) & ((2ULL << (lastpos < 63 ? lastpos : 63)) - 1))) fail = true;

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
            bool pass_ = false;
            if (ok) {
                if (WM == W_NONE) pass_ = true;
                else if (wnum && is_num(wc)) {
                    const double x = num_of(wc);
                    pass_ = cmp_result(wop, x < wval ? -1 : (x > wval ? 1 : 0));
                } else {
                    pass_ = cmp_result(wop, compare(wc, wconst));
                }
            }
            n_rec += (unsigned long long)__popcll(__ballot(ok));
            n_pass += (unsigned long long)__popcll(__ballot(pass_));
            if (row_out) {
                const unsigned long long slot = wave_slot(pass_, &stats->rows_emitted);
                if (pass_ && slot < row_cap) row_out[slot] = rec;
            }

            // ---- aggregate
            if (!GROUPED) {
                if (pass_) {
                    my_cnt++;
                    if (rec < my_first) my_first = rec;
#pragma unroll
                    for (int j = 0; j < NS; j++)
                        if (is_num(sc[j])) { my_sum[j] += num_of(sc[j]); my_num[j]++; }
                }
            } else {
                int slot = -1;
                uint64_t h = 0;
                if (pass_) {
                    h = gk_hash(key);
                    v4u a;
                    slot = lt_find(lt, key, h, lds_hdr(key, h), a);
                    if (slot >= 0) {
                        const uint32_t fc = (round << 15) | ((uint32_t)wv << 11) | p;
                        atomicAdd(&lt.cnt[slot], 1u);
                        if (fc < a.y) atomicMin((uint32_t*)(lt.A + slot) + 1, fc);
#pragma unroll
                        for (int j = 0; j < NS; j++) {
                            if (is_num(sc[j])) atomicAdd(&lt.sum[j][slot], num_of(sc[j]));
                            else atomicAdd(&lt.miss[j][slot], 1u);
                        }
                    }
                }
                const bool spill = pass_ && slot < 0;
                if (__any(spill)) {                        // LDS table full: straight to the HBM table
                    n_spill += (unsigned long long)__popcll(__ballot(spill));
                    if (spill) {
                        const int gi = g_insert(gt, key, h, stats);
                        if (gi >= 0) {
                            atomicAdd(&gt.cnt[gi], 1ULL);
                            atomicMin(&gt.first[gi], (unsigned long long)rec);
                            for (int a = 0; a < P.nacc; a++) {
                                const int j = LP.acc_sidx[a];
                                const Cell c = j == 0 ? sc[0] : sc[MAXS - 1];
                                if (is_num(c)) {
                                    atomicAdd(&gt.sum[a][gi], num_of(c));
                                    atomicAdd(&gt.num[a][gi], 1ULL);
                                }
                            }
                        }
                    }
                }
            }
            wave_sync();                                   // W.rs is rewritten by the next pass
        }
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

    // ---- flush the block's LDS table into the HBM table
    __syncthreads();
    for (uint32_t i = tid; i < lds_h; i += LT) {
        const v4u a = lt.A[i];
        if (a.x < 2) continue;
        GKey k;
        k.cls = (a.x >> 16) & 7;
        k.len = a.x & 0xFFFF;
        k.w0 = (uint64_t)a.z | ((uint64_t)a.w << 32);
        const uint2 b = lt.B[i];
        k.w1 = (uint64_t)b.x | ((uint64_t)b.y << 32);
        const int gi = g_insert(gt, k, gk_hash(k), stats);
        if (gi < 0) continue;
        const uint32_t n = lt.cnt[i];
        if (n) atomicAdd(&gt.cnt[gi], (unsigned long long)n);
        if (a.y != NOFIRST) {
            const uint64_t fw = first_win + ((uint64_t)(a.y >> 15) * gridDim.x + blockIdx.x) * NWV + ((a.y >> 11) & 15);
            atomicMin(&gt.first[gi], (unsigned long long)(fw * WB + (a.y & 2047)));
        }
        for (int acc = 0; acc < P.nacc; acc++) {
            const int j = LP.acc_sidx[acc];
            const double sa = j == 0 ? lt.sum[0][i] : lt.sum[MAXS - 1][i];
            const uint32_t ms = j == 0 ? lt.miss[0][i] : lt.miss[MAXS - 1][i];
            const uint32_t num = n - ms;
            if (num) {
                atomicAdd(&gt.sum[acc][gi], sa);
                atomicAdd(&gt.num[acc][gi], (unsigned long long)num);
            }
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
    if (P->max_col >= 64) return false;
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

size_t lean_slot_bytes(int ns) { return 16 + 8 + 4 + (size_t)ns * 12; }
size_t lean_fixed_bytes() { return sizeof(lean::WaveLds) * lean::NWV; }

uint32_t lean_slots(int ns, int grouped) {
    if (!grouped) return 0;
    uint32_t h = 2048;
    while (h > 64 && lean_fixed_bytes() + (size_t)h * lean_slot_bytes(ns) + 256 > (size_t)(160 * 1024)) h >>= 1;
    return h;
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

uint64_t cq_lean_windows(uint64_t bytes) { return (bytes + lean::WB - 1) / lean::WB; }
int cq_lean_waves_per_block() { return lean::NWV; }

size_t cq_lean_lds_bytes(const cq::ScanPlan* P, int grouped) {
    LeanPlan lp;
    int wm = 0;
    if (!lean_shape(P, &lp, &wm)) return 0;
    const uint32_t h = lean_slots(lp.ns > 0 ? lp.ns : 1, grouped);
    return lean_fixed_bytes() + (size_t)h * lean_slot_bytes(lp.ns > 0 ? lp.ns : 1) + 256;
}

// the lean scan (the caller runs slow_kernel over slow_list afterwards)
hipError_t cq_launch_lean(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt, cq::ScanStats* stats,
                          unsigned long long* row_out, unsigned long long row_cap, int grouped, int grid,
                          hipStream_t s, unsigned long long* slow_list, unsigned long long slow_cap) {
    LeanPlan lp;
    int wm = 0;
    if (!lean_shape(P, &lp, &wm)) return hipErrorInvalidValue;
    const int ns = lp.ns > 0 ? lp.ns : 1;
    const uint32_t h = lean_slots(ns, grouped);
    const size_t lds = lean_fixed_bytes() + (size_t)h * lean_slot_bytes(ns) + 256;
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(lean::c_plan), P, sizeof *P, 0, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyToSymbolAsync(HIP_SYMBOL(lean::c_gt), gt, sizeof *gt, 0, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyToSymbolAsync(HIP_SYMBOL(lean::c_lp), &lp, sizeof lp, 0, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    const lean_fn_t fn = grouped ? pick<true>(wm, ns) : pick<false>(wm, ns);
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(lean::LT), lds, s, g, stats, row_out, row_cap, h, slow_list, slow_cap);
    return hipGetLastError();
}

}  // extern "C"
