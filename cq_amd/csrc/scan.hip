// scan.hip -- the fused CSV scan for cq's SELECT hot path on gfx950.
//
// One pass over the CSV bytes resident in HBM does what the reference spreads
// over csv_load (csv_reader.c:375-465), filter_rows (evaluator_utils.c:986),
// create_groups (evaluator_aggregates.c:108) and evaluate_aggregate (:263).
// Per 32 KiB window, one 512-thread block:
//
//   stage     the window (+16 B before, +2 KiB after) is copied from registers
//             into LDS; the next window's 16 B/lane loads are already in flight
//   classify  each lane turns 64 window bytes into three 64-bit masks in LDS:
//             record terminators ('\n' '\r'), separators (terminators + the
//             delimiter) and "bad" bytes (every other byte below '-': quotes,
//             whitespace, NUL, '+', ...), with exact SWAR byte tests
//   split     record starts come from the terminator mask; a block-wide scan
//             gives every record an LDS slot
//   parse     one lane per record walks its fields with find-first-set on the
//             separator mask and types the needed cells with specialised int /
//             decimal / string parsers reading LDS; any field the fast parsers
//             cannot prove identical to infer_type/parse_value (quotes,
//             whitespace, date-shaped numbers, >15 significant digits ...) goes
//             through the general parser in cell.h -- same semantics, slower
//   filter    WHERE bytecode (plan.h OP_*), or a direct compare for col-op-const
//   group     LDS open-addressing table, 16-byte inline keys, COUNT / SUM / AVG /
//             MIN / MAX accumulators; flushed once per block into the HBM table
//             (per-thread registers when the query has no GROUP BY)
//
// Records are owned by the window holding their first byte, so every byte range
// [range_begin, range_end) can be scanned independently: that is also how the
// multi-GPU path shards a file.
#include <hip/hip_runtime.h>
#include "plan.h"

namespace cq {

constexpr int SCAN_T = 512;                  // threads per block (8 waves)
constexpr int WIN = 32768;                   // window bytes (64 per lane)
constexpr int PRE = 16;                      // bytes staged before the window
constexpr int MARGIN = 2048;                 // bytes staged after the window
constexpr int TILE = PRE + WIN + MARGIN;     // 34832
constexpr int TILE16 = TILE / 16;            // 2177 uint4 per tile
constexpr int NMW = (WIN + MARGIN) / 64;     // mask words covering [ws, ws + WIN + MARGIN)
constexpr int RSMAX = 2048;                  // record slots per pass
constexpr int LDS_BUDGET = 160 * 1024;       // LDS bytes per CU
constexpr int PF = (TILE16 + SCAN_T - 1) / SCAN_T;   // prefetch registers per lane (5)
constexpr uint64_t NOPOS = ~0ULL;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));   // one 16-byte load

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ bool is_nl(uint32_t c) { return c == '\n' || c == '\r'; }

// LDS-only barrier: waits for this wave's LDS traffic, not for in-flight global
// loads (the next window's prefetch must stay in flight across it)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// exact per-byte tests on a dword: 0x80 in every byte that matches
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t eq_bytes(uint32_t x, uint32_t rep) { return zero_bytes(x ^ rep); }
// 0x80 in every byte < n, for 0 < n <= 0x80 (rep_n = n * 0x01010101): no borrows
// cross bytes because every byte of (x | 0x80..) is >= 0x80 >= n
__device__ __forceinline__ uint32_t lt_bytes(uint32_t x, uint32_t rep_n) {
    return ~((x | 0x80808080u) - rep_n) & ~x & 0x80808080u;
}
__device__ __forceinline__ uint32_t pack4(uint32_t m) {   // 0x80 flags -> 4 bits
    return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}

// block-wide exclusive scan of one value per thread (SCAN_T threads)
__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    lds_barrier();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_T / 64; w++) {
        uint32_t s = wsum[w];
        if (w < wid) base += s;
        tot += s;
    }
    *total = tot;
    lds_barrier();
    return base + x - v;
}

// ------------------------------------------------------------------ general record parse
// parse_line (csv_reader.c:278-338) restricted to the needed columns, reading
// global memory: the exact path for records the fast walk declines, and for the
// representative-row gather.  Fills cells[0..nneed) (NULL for columns the
// record is too short to have); false when the record is short.
__device__ bool parse_record_global(const uint8_t* rec, const ScanPlan& P, Cell* cells) {
    if (P.nneed == 0) return true;
    const uint32_t delim = P.delim, quote = P.quote;
    uint32_t i = 0;
    int col = 0, k = 0;
    int want = P.need_col[0];
    while (true) {
        uint32_t c = rec[i];
        while (c == ' ' || c == '\t' || c == 0x0b || c == 0x0c) { i = i + 1; c = rec[i]; }
        if (is_nl(c)) break;                       // trailing empty field dropped
        uint32_t fs, flen;
        if (c == quote) {                          // quoted field (:294-317)
            i = i + 1;
            fs = i;
            uint32_t acc = 0;
            bool closed = false;
            flen = 0;
            while (true) {
                c = rec[i];
                if (is_nl(c)) break;
                if (c == quote) {
                    if (rec[i + 1] == quote) { i = i + 2; acc += 2; }
                    else { flen = i - fs; i = i + 1; closed = true; break; }
                } else {
                    i = i + 1;
                }
            }
            if (!closed) flen = acc;
            c = rec[i];
            while (c != delim && !is_nl(c)) { i = i + 1; c = rec[i]; }
        } else {                                   // unquoted field (:318-324)
            fs = i;
            while (c != delim && !is_nl(c)) { i = i + 1; c = rec[i]; }
            flen = i - fs;
        }
        if (col == want) {
            cells[k] = parse_cell(rec + fs, flen);
            if (++k == P.nneed) return true;
            want = P.need_col[k];
        }
        col++;
        if (c != delim) break;
        i = i + 1;
    }
    for (; k < P.nneed; k++) cells[k] = cell_null();
    return false;
}

// ------------------------------------------------------------------ predicate VM
struct Stack {
    Cell s0, s1, s2, s3, s4, s5, s6, s7;
    __device__ __forceinline__ Cell get(int i) const {
        switch (i) {
            case 0: return s0; case 1: return s1; case 2: return s2; case 3: return s3;
            case 4: return s4; case 5: return s5; case 6: return s6; default: return s7;
        }
    }
    __device__ __forceinline__ void set(int i, const Cell& v) {
        switch (i) {
            case 0: s0 = v; break; case 1: s1 = v; break; case 2: s2 = v; break;
            case 3: s3 = v; break; case 4: s4 = v; break; case 5: s5 = v; break;
            case 6: s6 = v; break; default: s7 = v; break;
        }
    }
};

__device__ __forceinline__ Cell cell_at(const Cell* cells, int k) {
    switch (k) {
        case 0: return cells[0]; case 1: return cells[1]; case 2: return cells[2];
        case 3: return cells[3]; case 4: return cells[4]; case 5: return cells[5];
        case 6: return cells[6]; default: return cells[7];
    }
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

// evaluate_condition (evaluator_conditions.c:62-164) over the flattened WHERE tree
__device__ bool eval_where(const ScanPlan& P, const Cell* cells) {
    if (P.nprog == 3 && P.prog[0].op == OP_COL && P.prog[1].op == OP_CONST && P.prog[2].op == OP_CMP)
        return cmp_result(P.prog[2].a, compare(cell_at(cells, P.prog[0].a), P.consts[P.prog[1].b]));
    Stack st;
    int sp = 0;
    uint32_t bs = 0;   // bool stack, top = bit 0
    for (int pc = 0; pc < P.nprog; pc++) {
        const Insn in = P.prog[pc];
        switch (in.op) {
            case OP_COL: st.set(sp++, cell_at(cells, in.a)); break;
            case OP_CONST: st.set(sp++, P.consts[in.b]); break;
            case OP_NULLV: st.set(sp++, cell_null()); break;
            case OP_ARITH: {
                Cell r = st.get(--sp), l = st.get(--sp);
                st.set(sp++, arith(in.a, l, r));
                break;
            }
            case OP_NEG: { Cell x = st.get(--sp); st.set(sp++, negate(x)); break; }
            case OP_CMP: {
                Cell r = st.get(--sp), l = st.get(--sp);
                bs = (bs << 1) | (cmp_result(in.a, compare(l, r)) ? 1u : 0u);
                break;
            }
            case OP_IN: {
                int n = in.b;
                Cell l = st.get(sp - n - 1);
                bool found = false;
                for (int j = 0; j < n; j++)
                    if (!found && compare(l, st.get(sp - n + j)) == 0) found = true;
                sp -= n + 1;
                bool b = in.a ? !found : found;
                bs = (bs << 1) | (b ? 1u : 0u);
                break;
            }
            case OP_LIKE: {
                Cell r = st.get(--sp), l = st.get(--sp);
                bool b = l.kind == K_STR && r.kind == K_STR &&
                         like(str_ptr(l), l.len, str_ptr(r), r.len, in.a != 0);
                bs = (bs << 1) | (b ? 1u : 0u);
                break;
            }
            case OP_NOT: bs ^= 1u; break;
            case OP_AND: { uint32_t r = bs & 1u; bs >>= 1; bs = (bs & ~1u) | ((bs & 1u) & r); break; }
            case OP_OR: { uint32_t r = bs & 1u; bs >>= 1; bs = bs | r; break; }
            case OP_BOOL: bs = (bs << 1) | (uint32_t)(in.a & 1); break;
            default: break;
        }
    }
    return (bs & 1u) != 0;
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

// ------------------------------------------------------------------ global table
__device__ __forceinline__ uint32_t tag_of(uint64_t h) {
    uint32_t t = (uint32_t)(h >> 32);
    return t < 2 ? t + 2 : t;
}

__device__ int g_insert(const GroupTable& gt, const GKey& k, uint64_t h, ScanStats* st) {
    const uint32_t tg = tag_of(h);
    const uint32_t mask = gt.cap - 1;
    const uint32_t cl = gk_clslen(k);
    for (uint32_t probe = 0; probe < gt.cap; probe++) {
        uint32_t i = (uint32_t)(h + probe) & mask;
        uint32_t t = __hip_atomic_load(&gt.tag[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0) {
            uint32_t old = atomicCAS(&gt.tag[i], 0u, 1u);
            if (old == 0) {
                __hip_atomic_store(&gt.clslen[i], cl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&gt.w0[i], k.w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&gt.w1[i], k.w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint32_t used = atomicAdd(gt.used, 1u) + 1;
                if (used * 2 > gt.cap) atomicExch(&st->overflow, 1ULL);
                __hip_atomic_store(&gt.tag[i], tg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                return (int)i;
            }
            t = old;
        }
        for (uint32_t spin = 0; t == 1; spin++) {
            if (spin > (1u << 24)) { atomicExch(&st->overflow, 2ULL); return -1; }   // never hang
            t = __hip_atomic_load(&gt.tag[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
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

// MIN/MAX merges take a per-slot lock.  A lock loop written per lane deadlocks
// on SIMT hardware (the compiler may park the lane that won the lock until every
// lane of the wave has won it), so every lock loop here is wave-uniform: the loop
// runs while ANY lane of the wave still needs the lock, and a lane that takes the
// lock releases it in the same trip.  Callers must reach these with the whole
// wave (uniform control flow), passing `need` = false for idle lanes.
__device__ void g_ext_update(bool need, const GroupTable& gt, int a, uint8_t kind, uint32_t i,
                             const Cell& c, uint64_t pos, ScanStats* st) {
    if (pos == NOPOS) need = false;
    uint32_t trips = 0;
    while (__any(need)) {
        if (need) {
            uint32_t* lk = &gt.lock[a][i];
            if (atomicCAS(lk, 0u, 1u) == 0u) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                Cell* ec = &gt.ext[a][i];
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
                __hip_atomic_store(lk, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                need = false;
            }
        }
        if (++trips > (1u << 24)) {                    // never hang: report and give up
            if (need) atomicExch(&st->overflow, 2ULL);
            break;
        }
    }
}

// ------------------------------------------------------------------ LDS table
// structure of arrays carved from dynamic LDS; capacity H (power of two) is
// chosen by the host so that the window tile and every accumulator fit
struct LdsTable {
    uint32_t H;
    uint32_t* tag;
    uint32_t* clslen;
    uint64_t* w0;
    uint64_t* w1;
    uint32_t* cnt;
    unsigned long long* first;
};
struct LdsAcc {            // ACC_SUM
    double* sum;
    uint32_t* num;
};
struct ExtLds {            // ACC_MIN / ACC_MAX
    Cell* c;
    unsigned long long* pos;
    uint32_t* lock;
};

__device__ int l_insert(const LdsTable& t, const GKey& k, uint64_t h) {
    const uint32_t tg = tag_of(h);
    const uint32_t cl = gk_clslen(k);
    for (uint32_t probe = 0; probe < 64; probe++) {
        uint32_t i = (uint32_t)(h + probe) & (t.H - 1);
        uint32_t cur = __hip_atomic_load(&t.tag[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
            uint32_t old = atomicCAS(&t.tag[i], 0u, 1u);
            if (old == 0) {
                t.clslen[i] = cl;
                t.w0[i] = k.w0;
                t.w1[i] = k.w1;
                __hip_atomic_store(&t.tag[i], tg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                return (int)i;
            }
            cur = old;
        }
        for (uint32_t spin = 0; cur == 1; spin++) {
            if (spin > (1u << 24)) return -1;          // the HBM table takes the record
            cur = __hip_atomic_load(&t.tag[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (cur == tg && t.clslen[i] == cl && t.w1[i] == k.w1) {
            const uint64_t ow0 = t.w0[i];
            if (ow0 == k.w0) return (int)i;
            if (k.cls == GK_LONG) {
                GKey o;
                o.cls = GK_LONG; o.len = k.len; o.w0 = ow0; o.w1 = k.w1;
                if (gk_equal(o, k)) return (int)i;
            }
        }
    }
    return -1;
}

// wave-uniform LDS MIN/MAX update (see g_ext_update)
__device__ void lds_ext_update(bool need, const ExtLds& e, uint32_t s, uint8_t kind, const Cell& c,
                               uint64_t pos) {
    while (__any(need)) {
        if (need) {
            if (atomicCAS(&e.lock[s], 0u, 1u) == 0u) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (ext_better(kind, c, pos, e.c[s], e.pos[s])) {
                    e.c[s] = c;
                    e.pos[s] = pos;
                }
                __hip_atomic_store(&e.lock[s], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                need = false;
            }
        }
    }
}

// ------------------------------------------------------------------ fast field parsers
// 16 bytes of the tile starting at byte offset `o` (any alignment), little-endian
__device__ __forceinline__ void load16(const uint8_t* tile, uint32_t o, uint64_t& w0, uint64_t& w1) {
    const uint32_t* t32 = (const uint32_t*)tile;
    const uint32_t a = o >> 2, sh = (o & 3) * 8;
    const uint32_t d0 = t32[a], d1 = t32[a + 1], d2 = t32[a + 2], d3 = t32[a + 3], d4 = t32[a + 4];
    const uint32_t e0 = (uint32_t)((((uint64_t)d1 << 32) | d0) >> sh);
    const uint32_t e1 = (uint32_t)((((uint64_t)d2 << 32) | d1) >> sh);
    const uint32_t e2 = (uint32_t)((((uint64_t)d3 << 32) | d2) >> sh);
    const uint32_t e3 = (uint32_t)((((uint64_t)d4 << 32) | d3) >> sh);
    w0 = (uint64_t)e0 | ((uint64_t)e1 << 32);
    w1 = (uint64_t)e2 | ((uint64_t)e3 << 32);
}

__device__ __forceinline__ uint32_t byte_of(uint64_t w0, uint64_t w1, uint32_t i) {
    return (uint32_t)((i < 8 ? w0 >> (8 * i) : w1 >> (8 * (i - 8))) & 0xff);
}

__device__ __forceinline__ double pow10_exact(uint32_t e) {   // 10^e, e <= 22, exact in double
    double r = 1.0, b = 10.0;
    while (e) { if (e & 1) r *= b; b *= b; e >>= 1; }   // every partial product is exact
    return r;
}

// Type one field of `len` bytes at tile offset `o` that holds no bad byte (no
// whitespace, quote, NUL, '+').  Returns false when the exact general parser
// must decide: date-shaped fields (parse_date may accept them), numerals past
// the exact fast cases, fields over 16 bytes, or a delimiter strtod/strtoll
// could read across (`num_ok` false).  `want_key`: also produce the group key.
__device__ __forceinline__ bool fast_cell(const uint8_t* tile, uint32_t o, uint32_t len,
                                          const uint8_t* gfield, bool num_ok, Cell& out,
                                          bool want_key, GKey& key) {
    if (len == 0) {
        out = cell_null();
        if (want_key) key = group_key(out);
        return true;
    }
    if (len > 16) return false;
    uint64_t w0, w1;
    load16(tile, o, w0, w1);
    if (len <= 8) {
        if (len < 8) w0 &= (1ULL << (8 * len)) - 1;
        w1 = 0;
    } else if (len < 16) {
        w1 &= (1ULL << (8 * (len - 8))) - 1;
    }
    const uint32_t c0 = (uint32_t)(w0 & 0xff);
    const bool lead_num = is_digit(c0) || c0 == '-' || c0 == '.';
    if (len >= 8 && len <= 10 && lead_num) return false;     // parse_date may accept it
    // infer_type's numeric shape ([+-] digits with at most one '.', at least one digit)
    bool numeric = lead_num, dot = false, dig = false;
    uint64_t w = 0;
    uint32_t nsig = 0, frac = 0;
    if (numeric) {
        for (uint32_t i = (c0 == '-') ? 1u : 0u; i < len; i++) {
            const uint32_t b = byte_of(w0, w1, i);
            if (is_digit(b)) {
                dig = true;
                if (nsig || b != '0') { w = w * 10 + (b - '0'); nsig++; }
                if (dot) frac++;
            } else if (b == '.' && !dot) {
                dot = true;
            } else {
                numeric = false;
                break;
            }
        }
        numeric = numeric && dig;
    }
    if (numeric) {
        if (!num_ok) return false;
        const bool neg = c0 == '-';
        if (!dot) {
            if (nsig > 18) return false;                       // strtoll range: general path
            out = cell_int(neg ? -(int64_t)w : (int64_t)w);
        } else {
            if (nsig > 15 || frac > 22) return false;          // Clinger's exact case only
            double v = (double)w;                              // exact: w < 10^15
            if (frac) v = v / pow10_exact(frac);               // one correctly rounded division
            out = cell_dbl(neg ? -v : v);
        }
        if (want_key) key = group_key(out);
        return true;
    }
    // STRING without whitespace or NUL: already what trim_whitespace returns
    out.kind = K_STR;
    out.len = len;
    out.bits = (uint64_t)(uintptr_t)gfield;
    if (want_key) {
        key.cls = GK_STR;
        key.len = len;
        key.w0 = w0;
        key.w1 = w1;
    }
    return true;
}

// any set bit of the per-64-byte masks `m` in [a, b)
__device__ __forceinline__ bool any_bits(const uint64_t* m, uint32_t a, uint32_t b) {
    if (a >= b) return false;
    const uint32_t wa = a >> 6, wb = (b - 1) >> 6;
    const uint64_t lo = ~0ULL << (a & 63);
    const uint64_t hi = ((b & 63) == 0) ? ~0ULL : ((1ULL << (b & 63)) - 1);
    if (wa == wb) return (m[wa] & lo & hi) != 0;
    if (m[wa] & lo) return true;
    for (uint32_t w = wa + 1; w < wb; w++)
        if (m[w]) return true;
    return (m[wb] & hi) != 0;
}

// Walk the record at window offset r with the separator mask.  Returns false if
// the record must take the general path: a field starting with a bad byte
// (quote, leading whitespace), or a record running past the staged bytes.
// Fills cells (NULL where the record is short) and the group key.
__device__ __forceinline__ bool fast_record(const uint8_t* tile, const uint64_t* sepw, const uint64_t* nlw,
                                            const uint64_t* badw, uint32_t r, const uint8_t* grec,
                                            const ScanPlan& P, bool num_ok, Cell* cells, GKey& key,
                                            bool& short_row) {
    short_row = false;
    if (P.nneed == 0) return true;
    uint32_t pos = r;
    int col = 0, k = 0;
    int want = P.need_col[0];
    while (true) {
        const uint32_t wi = pos >> 6;
        if (wi >= (uint32_t)NMW) return false;
        if ((badw[wi] >> (pos & 63)) & 1ULL) return false;
        const uint64_t m = sepw[wi] >> (pos & 63);
        uint32_t e;
        if (m) {
            e = pos + (uint32_t)__ffsll((long long)m) - 1;
        } else {
            uint32_t w = wi + 1;
            while (w < (uint32_t)NMW && sepw[w] == 0) w++;
            if (w >= (uint32_t)NMW) return false;
            e = w * 64 + (uint32_t)__ffsll((long long)sepw[w]) - 1;
        }
        const bool at_nl = (nlw[e >> 6] >> (e & 63)) & 1ULL;
        if (e == pos && at_nl) break;                  // empty trailing field: dropped
        if (col == want) {
            const uint32_t len = e - pos;
            const bool gkey = k == P.group_slot;
            Cell c;
            const bool ok = !any_bits(badw, pos, e) &&
                            fast_cell(tile, PRE + pos, len, grec + (pos - r), num_ok, c, gkey, key);
            if (!ok) {
                c = parse_cell(grec + (pos - r), len);
                if (gkey) key = group_key(c);
            }
            cells[k] = c;
            if (++k == P.nneed) return true;
            want = P.need_col[k];
        }
        col++;
        if (at_nl) break;
        pos = e + 1;
    }
    for (; k < P.nneed; k++) {
        cells[k] = cell_null();
        if (k == P.group_slot) key = group_key(cells[k]);
    }
    short_row = true;
    return true;
}

// ------------------------------------------------------------------ the scan kernel
// dynamic LDS: [tile][nl/sep/bad masks][rs][scan scratch][group table][accumulators]
__device__ __forceinline__ uint8_t* carve(uint8_t*& q, size_t bytes) {
    uint8_t* r = q;
    q += (bytes + 15) & ~(size_t)15;
    return r;
}

__device__ __forceinline__ void prefetch(const uint8_t* g, uint64_t ws, v4u* pf) {
    const v4u* src = (const v4u*)(g + ws - PRE);
#pragma unroll
    for (int j = 0; j < PF; j++) {
        const int i = threadIdx.x + j * SCAN_T;
        if (i < TILE16) pf[j] = __builtin_nontemporal_load(src + i);
    }
}

// The plan and the table descriptor live in constant memory (written on the
// launch stream before each launch): passed by value they would be copied to
// per-lane scratch, because the kernel indexes their arrays at run time.
__constant__ ScanPlan c_plan;
__constant__ GroupTable c_gt;

template <bool GROUPED>
__global__ __launch_bounds__(SCAN_T) void scan_kernel(const uint8_t* __restrict__ g,
                                                      ScanStats* __restrict__ stats,
                                                      unsigned long long* __restrict__ row_out,
                                                      unsigned long long row_cap, uint32_t lds_h,
                                                      Cell* __restrict__ cells_out) {
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t* q = smem;
    uint8_t* tile = carve(q, TILE);
    uint64_t* nlw = (uint64_t*)carve(q, NMW * 8);
    uint64_t* sepw = (uint64_t*)carve(q, NMW * 8);
    uint64_t* badw = (uint64_t*)carve(q, NMW * 8);
    uint32_t* rs = (uint32_t*)carve(q, RSMAX * 4);
    uint32_t* wsum = (uint32_t*)carve(q, 64);
    LdsTable lt;
    LdsAcc la[MAX_ACC];
    ExtLds le[MAX_ACC];
    const uint32_t H = lds_h;
    lt.H = H;
    lt.tag = nullptr; lt.clslen = nullptr; lt.w0 = nullptr; lt.w1 = nullptr; lt.cnt = nullptr; lt.first = nullptr;
    if (GROUPED) {
        lt.tag = (uint32_t*)carve(q, H * 4);
        lt.clslen = (uint32_t*)carve(q, H * 4);
        lt.w0 = (uint64_t*)carve(q, H * 8);
        lt.w1 = (uint64_t*)carve(q, H * 8);
        lt.cnt = (uint32_t*)carve(q, H * 4);
        lt.first = (unsigned long long*)carve(q, H * 8);
    }
#pragma unroll
    for (int a = 0; a < MAX_ACC; a++) {
        la[a].sum = nullptr; la[a].num = nullptr;
        le[a].c = nullptr; le[a].pos = nullptr; le[a].lock = nullptr;
        if (!GROUPED || a >= P.nacc) continue;
        if (P.acc[a].kind == ACC_SUM) {
            la[a].sum = (double*)carve(q, H * 8);
            la[a].num = (uint32_t*)carve(q, H * 4);
        } else {
            le[a].c = (Cell*)carve(q, H * sizeof(Cell));
            le[a].pos = (unsigned long long*)carve(q, H * 8);
            le[a].lock = (uint32_t*)carve(q, H * 4);
        }
    }
    const int tid = threadIdx.x;

    if (GROUPED) {
        for (uint32_t i = tid; i < H; i += SCAN_T) {
            lt.tag[i] = 0; lt.cnt[i] = 0; lt.first[i] = NOPOS;
#pragma unroll
            for (int a = 0; a < MAX_ACC; a++) {
                if (la[a].sum) { la[a].sum[i] = 0.0; la[a].num[i] = 0; }
                if (le[a].c) { le[a].pos[i] = NOPOS; le[a].lock[i] = 0; le[a].c[i] = cell_null(); }
            }
        }
    }
    // per-thread partials (single-group mode) and statistics
    unsigned long long my_cnt = 0, my_first = NOPOS, my_records = 0, my_short = 0, my_spill = 0,
                       my_slow = 0, my_pass = 0;
    double my_sum[MAX_ACC];
    unsigned long long my_num[MAX_ACC];
    Cell my_ext[MAX_ACC];
    unsigned long long my_pos[MAX_ACC];
    uint32_t my_cls[MAX_ACC];
#pragma unroll
    for (int a = 0; a < MAX_ACC; a++) {
        my_sum[a] = 0.0; my_num[a] = 0; my_ext[a] = cell_null(); my_pos[a] = NOPOS; my_cls[a] = 0;
    }

    const uint64_t lo_ok = P.data_begin > P.range_begin ? P.data_begin : P.range_begin;
    const uint64_t hi_ok = P.range_end < P.n ? P.range_end : P.n;
    const uint64_t first_win = P.range_begin / WIN;
    const uint64_t last_win = (hi_ok + WIN - 1) / WIN;
    const uint32_t delim = P.delim, quote = P.quote;
    const uint32_t rep_d = delim * 0x01010101u, rep_q = quote * 0x01010101u;
    // strtoll/strtod read past the field end: a delimiter they could consume
    // (digit, '.', letter) disables the fast numeric parsers
    const bool num_ok = !(is_digit(delim) || delim == '.' || ((delim | 32) >= 'a' && (delim | 32) <= 'z'));

    v4u pf[PF];
    uint64_t w = first_win + blockIdx.x;
    if (w < last_win) prefetch(g, w * WIN, pf);

    for (; w < last_win; w += gridDim.x) {
        const uint64_t ws = w * WIN;
        lds_barrier();                                   // previous window fully consumed
#pragma unroll
        for (int j = 0; j < PF; j++) {
            const int i = tid + j * SCAN_T;
            if (i < TILE16) ((v4u*)tile)[i] = pf[j];
        }
        lds_barrier();
        if (w + gridDim.x < last_win) prefetch(g, (w + gridDim.x) * WIN, pf);   // in flight meanwhile

        // ---- classify: lane t -> mask word t (lanes 0..31 also the margin words)
        for (int wi = tid; wi < NMW; wi += SCAN_T) {
            const v4u* src = (const v4u*)(tile + PRE + wi * 64);
            uint64_t nlm = 0, sepm = 0, badm = 0;
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const v4u x4 = src[v];
                const uint32_t xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t x = xs[j];
                    uint32_t special = lt_bytes(x, 0x2D2D2D2Du);
                    if (delim >= 0x2D) special |= eq_bytes(x, rep_d);
                    if (quote >= 0x2D) special |= eq_bytes(x, rep_q);
                    if (special) {
                        const uint32_t nl = eq_bytes(x, 0x0A0A0A0Au) | eq_bytes(x, 0x0D0D0D0Du);
                        const uint32_t dl = eq_bytes(x, rep_d) & ~nl;
                        const uint32_t bd = special & ~nl & ~dl;
                        const int sh = v * 16 + j * 4;
                        nlm |= (uint64_t)pack4(nl) << sh;
                        sepm |= (uint64_t)pack4(nl | dl) << sh;
                        badm |= (uint64_t)pack4(bd) << sh;
                    }
                }
            }
            nlw[wi] = nlm;
            sepw[wi] = sepm;
            badw[wi] = badm;
        }
        lds_barrier();
        // ---- record starts in this lane's 64 window bytes
        uint64_t starts;
        {
            const uint64_t nlm = nlw[tid];
            const uint64_t prev_nl = (tid == 0) ? (is_nl(tile[PRE - 1]) ? 1ULL : 0ULL) : (nlw[tid - 1] >> 63);
            starts = ~nlm & ((nlm << 1) | prev_nl);
            const uint64_t base = ws + (uint64_t)tid * 64;
            if (base + 64 <= lo_ok || base >= hi_ok) {
                starts = 0;
            } else {
                if (base < lo_ok) starts &= ~0ULL << (lo_ok - base);
                if (base + 64 > hi_ok) starts &= (1ULL << (hi_ok - base)) - 1;
            }
        }
        const uint32_t cnt = (uint32_t)__popcll(starts);
        uint32_t total;
        const uint32_t idx = block_excl_scan(cnt, wsum, &total);
        for (uint32_t chunk = 0; chunk < total; chunk += RSMAX) {
            {
                uint64_t m = starts;
                uint32_t ri = idx;
                while (m) {
                    const int b = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    if (ri >= chunk && ri < chunk + RSMAX) rs[ri - chunk] = tid * 64 + b;
                    ri++;
                }
            }
            lds_barrier();
            const uint32_t nrec = min((uint32_t)RSMAX, total - chunk);
            for (uint32_t base0 = 0; base0 < nrec; base0 += SCAN_T) {
                // trip count is block-uniform: every lane of a wave runs every trip
                const uint32_t ri = base0 + tid;
                const bool valid = ri < nrec;
                const uint32_t r = valid ? rs[ri] : 0;
                const uint64_t rec = ws + r;
                Cell cells[MAX_NEED];
#pragma unroll
                for (int k = 0; k < MAX_NEED; k++) cells[k] = cell_null();
                GKey key;
                key.cls = 0; key.len = 0; key.w0 = 0; key.w1 = 0;
                bool pass = false;
                if (valid) {
                    bool short_row = false;
                    if (!fast_record(tile, sepw, nlw, badw, r, g + rec, P, num_ok, cells, key, short_row)) {
                        my_slow++;
                        short_row = !parse_record_global(g + rec, P, cells);
                        if (GROUPED) key = group_key(cell_at(cells, P.group_slot));
                    }
                    my_records++;
                    if (short_row) my_short++;
                    pass = P.nprog == 0 || eval_where(P, cells);
                    if (pass) my_pass++;
                }
                if (pass && row_out) {
                    const unsigned long long slot = atomicAdd(&stats->rows_emitted, 1ULL);
                    if (slot < row_cap) {
                        row_out[slot] = rec;
                        if (cells_out)   // debug: the cells this kernel parsed
                            for (int k = 0; k < P.nneed; k++) cells_out[slot * P.nneed + k] = cell_at(cells, k);
                    }
                }
                if (pass) {
#pragma unroll
                    for (int a = 0; a < MAX_ACC; a++)
                        if (a < P.nacc) my_cls[a] |= class_bit(cell_at(cells, P.acc[a].slot));
                }
                if (!GROUPED) {
                    if (pass) {
                        my_cnt++;
                        if (rec < my_first) my_first = rec;
#pragma unroll
                        for (int a = 0; a < MAX_ACC; a++) {
                            if (a >= P.nacc) continue;
                            const Cell c = cell_at(cells, P.acc[a].slot);
                            if (P.acc[a].kind == ACC_SUM) {
                                if (is_num(c)) { my_sum[a] += num_of(c); my_num[a]++; }
                            } else if (c.kind != K_NULL && ext_better(P.acc[a].kind, c, rec, my_ext[a], my_pos[a])) {
                                my_ext[a] = c;
                                my_pos[a] = rec;
                            }
                        }
                    }
                } else {
                    uint64_t h = 0;
                    int s = -1;
                    if (pass) {
                        h = gk_hash(key);
                        s = l_insert(lt, key, h);
                    }
                    const bool in_lds = pass && s >= 0;
                    const bool spill = pass && s < 0;
                    if (in_lds) {
                        atomicAdd(&lt.cnt[s], 1u);
                        if (rec < lt.first[s]) atomicMin(&lt.first[s], (unsigned long long)rec);
#pragma unroll
                        for (int a = 0; a < MAX_ACC; a++) {
                            if (a >= P.nacc || !la[a].sum) continue;
                            const Cell c = cell_at(cells, P.acc[a].slot);
                            if (is_num(c)) {
                                atomicAdd(&la[a].sum[s], num_of(c));
                                atomicAdd(&la[a].num[s], 1u);
                            }
                        }
                    }
#pragma unroll
                    for (int a = 0; a < MAX_ACC; a++) {
                        if (a >= P.nacc || !le[a].c) continue;   // uniform
                        const Cell c = cell_at(cells, P.acc[a].slot);
                        lds_ext_update(in_lds && c.kind != K_NULL, le[a], in_lds ? (uint32_t)s : 0u,
                                       P.acc[a].kind, c, rec);
                    }
                    if (__any(spill)) {
                        // LDS table full: this record goes straight to the HBM table
                        int gi = -1;
                        if (spill) {
                            my_spill++;
                            gi = g_insert(gt, key, h, stats);
                            if (gi >= 0) {
                                atomicAdd(&gt.cnt[gi], 1ULL);
                                atomicMin(&gt.first[gi], (unsigned long long)rec);
                                for (int a = 0; a < P.nacc; a++) {
                                    const Cell c = cell_at(cells, P.acc[a].slot);
                                    if (P.acc[a].kind == ACC_SUM && is_num(c)) {
                                        atomicAdd(&gt.sum[a][gi], num_of(c));
                                        atomicAdd(&gt.num[a][gi], 1ULL);
                                    }
                                }
                            }
                        }
                        for (int a = 0; a < P.nacc; a++) {
                            if (P.acc[a].kind == ACC_SUM) continue;   // uniform
                            const Cell c = cell_at(cells, P.acc[a].slot);
                            g_ext_update(spill && gi >= 0 && c.kind != K_NULL, gt, a, P.acc[a].kind,
                                         gi >= 0 ? (uint32_t)gi : 0u, c, rec, stats);
                        }
                    }
                }
            }
            lds_barrier();
        }
    }
    __syncthreads();

    // ---- statistics and value-class masks
    {
        unsigned long long r = my_records, s = my_short, sp = my_spill, sl = my_slow, ps = my_pass;
        for (int o = 32; o > 0; o >>= 1) {
            r += __shfl_down(r, o, 64);
            s += __shfl_down(s, o, 64);
            sp += __shfl_down(sp, o, 64);
            sl += __shfl_down(sl, o, 64);
            ps += __shfl_down(ps, o, 64);
        }
        if ((tid & 63) == 0) {
            if (r) atomicAdd(&stats->records, r);
            if (s) atomicAdd(&stats->short_rows, s);
            if (sp) atomicAdd(&stats->lds_spills, sp);
            if (sl) atomicAdd(&stats->slow_records, sl);
            if (ps) atomicAdd(&stats->passed, ps);
        }
    }
    for (int a = 0; a < P.nacc; a++) {
        uint32_t m = my_cls[a];
        for (int o = 32; o > 0; o >>= 1) m |= __shfl_down(m, o, 64);
        if ((tid & 63) == 0 && m) atomicOr(&stats->acc_classes[a], m);
    }

    if (!GROUPED) {
        // ---- wave-reduce the single group, then one global update per wave
        unsigned long long c = my_cnt, f = my_first;
        for (int o = 32; o > 0; o >>= 1) {
            c += __shfl_down(c, o, 64);
            const unsigned long long ff = __shfl_down(f, o, 64);
            f = ff < f ? ff : f;
        }
        double sm[MAX_ACC];
        unsigned long long nm[MAX_ACC];
#pragma unroll
        for (int a = 0; a < MAX_ACC; a++) {
            sm[a] = my_sum[a];
            nm[a] = my_num[a];
            for (int o = 32; o > 0; o >>= 1) {
                sm[a] += __shfl_down(sm[a], o, 64);
                nm[a] += __shfl_down(nm[a], o, 64);
            }
        }
        GKey k;
        k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
        int gi = -1;
        if ((tid & 63) == 0) {
            gi = g_insert(gt, k, 0x12345678ULL, stats);
            if (gi >= 0) {
                if (c) atomicAdd(&gt.cnt[gi], c);
                if (f != NOPOS) atomicMin(&gt.first[gi], f);
                for (int a = 0; a < P.nacc; a++)
                    if (P.acc[a].kind == ACC_SUM && nm[a]) {
                        atomicAdd(&gt.sum[a][gi], sm[a]);
                        atomicAdd(&gt.num[a][gi], nm[a]);
                    }
            }
        }
        gi = __shfl(gi, 0, 64);
        for (int a = 0; a < P.nacc; a++) {
            if (P.acc[a].kind == ACC_SUM) continue;
            g_ext_update(gi >= 0 && my_pos[a] != NOPOS, gt, a, P.acc[a].kind, gi >= 0 ? (uint32_t)gi : 0u,
                         my_ext[a], my_pos[a], stats);
        }
        return;
    }

    // ---- flush the LDS table into the global table (wave-uniform trips)
    for (uint32_t b0 = 0; b0 < H; b0 += SCAN_T) {
        const uint32_t i = b0 + tid;
        const bool act = i < H && lt.tag[i] >= 2;
        int gi = -1;
        if (act) {
            GKey k;
            k.cls = lt.clslen[i] >> 16;
            k.len = lt.clslen[i] & 0xffff;
            k.w0 = lt.w0[i];
            k.w1 = lt.w1[i];
            gi = g_insert(gt, k, gk_hash(k), stats);
            if (gi >= 0) {
                atomicAdd(&gt.cnt[gi], (unsigned long long)lt.cnt[i]);
                atomicMin(&gt.first[gi], lt.first[i]);
                for (int a = 0; a < P.nacc; a++) {
                    if (la[a].sum && la[a].num[i]) {
                        atomicAdd(&gt.sum[a][gi], la[a].sum[i]);
                        atomicAdd(&gt.num[a][gi], (unsigned long long)la[a].num[i]);
                    }
                }
            }
        }
        for (int a = 0; a < P.nacc; a++) {
            if (!le[a].c) continue;                     // uniform
            const bool ok = act && gi >= 0;
            const Cell c = ok ? le[a].c[i] : cell_null();
            const uint64_t pos = ok ? le[a].pos[i] : NOPOS;
            g_ext_update(ok, gt, a, P.acc[a].kind, ok ? (uint32_t)gi : 0u, c, pos, stats);
        }
    }
}

// ------------------------------------------------------------------ compaction
__global__ void compact_kernel(int nacc, GroupOut* out, unsigned int* count,
                               unsigned int cap_out) {
    const GroupTable& gt = c_gt;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= gt.cap) return;
    if (gt.tag[i] < 2) return;
    const unsigned int o = atomicAdd(count, 1u);
    if (o >= cap_out) return;
    GroupOut r;
    r.clslen = gt.clslen[i];
    r.pad = 0;
    r.w0 = gt.w0[i];
    r.w1 = gt.w1[i];
    r.cnt = gt.cnt[i];
    r.first = gt.first[i];
    for (int a = 0; a < MAX_ACC; a++) {
        r.sum[a] = (a < nacc && gt.sum[a]) ? gt.sum[a][i] : 0.0;
        r.num[a] = (a < nacc && gt.num[a]) ? gt.num[a][i] : 0ULL;
        r.ext[a] = (a < nacc && gt.ext[a]) ? gt.ext[a][i] : cell_null();
        r.extpos[a] = (a < nacc && gt.extpos[a]) ? gt.extpos[a][i] : NOPOS;
    }
    out[o] = r;
}

// ------------------------------------------------------------------ gather cells
// representative / projected cells of given records (build_aggregated_result
// uses the group's first row, evaluator_aggregates.c:679-689)
__global__ void gather_kernel(const uint8_t* __restrict__ g,
                              const unsigned long long* __restrict__ recs, uint32_t nrec,
                              Cell* __restrict__ out) {
    const ScanPlan& P = c_plan;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    Cell cells[MAX_NEED];
    parse_record_global(g + recs[i], P, cells);
    for (int k = 0; k < P.nneed; k++) out[(uint64_t)i * P.nneed + k] = cells[k];
}

// string bytes of cells -> packed host-visible buffer
__global__ void copy_strings_kernel(const Cell* __restrict__ cells, uint32_t n,
                                    const unsigned long long* __restrict__ offs,
                                    uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const Cell c = cells[i];
    if (c.kind != K_STR) return;
    const uint8_t* s = (const uint8_t*)(uintptr_t)c.bits;
    for (uint32_t j = threadIdx.x; j < c.len; j += blockDim.x) out[offs[i] + j] = s[j];
}

// literal texts -> cells (parse_value on LITERAL nodes, evaluator_expressions.c:30-31)
__global__ void parse_literals_kernel(const uint8_t* __restrict__ text,
                                      const unsigned int* __restrict__ offs,
                                      const unsigned int* __restrict__ lens, uint32_t n,
                                      Cell* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = parse_cell(text + offs[i], lens[i]);
}

}  // namespace cq

// ------------------------------------------------------------------ host wrappers
extern "C" {
static size_t lds_slot_bytes(const cq::ScanPlan* P) {
    size_t b = 4 + 4 + 8 + 8 + 4 + 8;   // tag, clslen, w0, w1, cnt, first
    for (int a = 0; a < P->nacc; a++) b += P->acc[a].kind == cq::ACC_SUM ? 12 : sizeof(cq::Cell) + 12;
    return b;
}
static size_t lds_fixed_bytes() {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    return r16(cq::TILE) + 3 * r16(cq::NMW * 8) + r16(cq::RSMAX * 4) + r16(64);
}

// group-table capacity: the largest power of two <= 2048 that fits the budget
// (each carved array is rounded to 16 bytes: 16 arrays at most -> 256 bytes slack)
uint32_t cq_scan_lds_slots(const cq::ScanPlan* P, int grouped) {
    if (!grouped) return 0;
    const size_t per = lds_slot_bytes(P);
    uint32_t h = 2048;
    while (h > 64 && lds_fixed_bytes() + (size_t)h * per + 512 > (size_t)cq::LDS_BUDGET) h >>= 1;
    return h;
}

size_t cq_scan_lds_bytes(const cq::ScanPlan* P, int grouped) {
    size_t b = lds_fixed_bytes();
    if (grouped) b += (size_t)cq_scan_lds_slots(P, grouped) * lds_slot_bytes(P) + 512;
    return b;
}

hipError_t cq_launch_scan(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          cq::ScanStats* stats, unsigned long long* row_out,
                          unsigned long long row_cap, int grouped, int grid, hipStream_t s,
                          cq::Cell* cells_out) {
    const size_t lds = cq_scan_lds_bytes(P, grouped);
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(cq::c_plan), P, sizeof *P, 0, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyToSymbolAsync(HIP_SYMBOL(cq::c_gt), gt, sizeof *gt, 0, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    if (grouped) {
        (void)hipFuncSetAttribute((const void*)cq::scan_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(cq::scan_kernel<true>, dim3(grid), dim3(cq::SCAN_T), lds, s, g,
                           stats, row_out, row_cap, cq_scan_lds_slots(P, grouped), cells_out);
    } else {
        (void)hipFuncSetAttribute((const void*)cq::scan_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(cq::scan_kernel<false>, dim3(grid), dim3(cq::SCAN_T), lds, s, g,
                           stats, row_out, row_cap, 0u, cells_out);
    }
    return hipGetLastError();
}

int cq_scan_occupancy(const cq::ScanPlan* P, int grouped) {
    const size_t lds = cq_scan_lds_bytes(P, grouped);
    int blocks = 0;
    const void* fn = grouped ? (const void*)cq::scan_kernel<true> : (const void*)cq::scan_kernel<false>;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, cq::SCAN_T, lds) != hipSuccess) return 1;
    return blocks > 0 ? blocks : 1;
}

hipError_t cq_launch_compact(const cq::GroupTable* gt, int nacc, cq::GroupOut* out,
                             unsigned int* count, unsigned int cap_out, hipStream_t s) {
    const dim3 grid((gt->cap + 255) / 256);
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(cq::c_gt), gt, sizeof *gt, 0, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cq::compact_kernel, grid, dim3(256), 0, s, nacc, out, count, cap_out);
    return hipGetLastError();
}

hipError_t cq_launch_gather(const uint8_t* g, const cq::ScanPlan* P, const unsigned long long* recs,
                            uint32_t nrec, cq::Cell* out, hipStream_t s) {
    if (!nrec) return hipSuccess;
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(cq::c_plan), P, sizeof *P, 0, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cq::gather_kernel, dim3((nrec + 127) / 128), dim3(128), 0, s, g, recs, nrec, out);
    return hipGetLastError();
}

hipError_t cq_launch_copy_strings(const cq::Cell* cells, uint32_t n, const unsigned long long* offs,
                                  uint8_t* out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::copy_strings_kernel, dim3(n), dim3(64), 0, s, cells, n, offs, out);
    return hipGetLastError();
}

hipError_t cq_launch_parse_literals(const uint8_t* text, const unsigned int* offs,
                                    const unsigned int* lens, uint32_t n, cq::Cell* out,
                                    hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::parse_literals_kernel, dim3((n + 63) / 64), dim3(64), 0, s, text, offs,
                       lens, n, out);
    return hipGetLastError();
}
}
