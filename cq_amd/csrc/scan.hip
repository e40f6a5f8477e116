// scan.hip -- the fused CSV scan for cq's SELECT hot path on gfx950.
//
// One pass over the CSV bytes resident in HBM does what the reference spreads
// over csv_load (csv_reader.c:375-465), filter_rows (evaluator_utils.c:986),
// create_groups (evaluator_aggregates.c:108) and evaluate_aggregate (:263).
// Per 32 KiB window, one 512-thread block:
//
//   stage     the window (+16 B before, +2 KiB after) is copied from registers
//             into LDS; the next window's 16 B/lane loads are already in flight
//   classify  each lane turns 64 window bytes into two 64-bit masks in LDS --
//             record terminators ('\n' '\r') and separators (terminators and
//             the delimiter) -- plus a "has a quote byte" flag, branch-free SWAR
//   split     record starts come from the terminator mask; a block-wide scan
//             gives every record an LDS slot
//   parse     one lane per record takes a 128-bit view of both masks at its
//             start and pops separators up to the last needed column (the
//             column walk is uniform across the wave); needed fields are typed
//             by specialised int / decimal / string parsers reading LDS.  A
//             field the fast parsers cannot prove identical to infer_type /
//             parse_value (date-shaped, long numerals) goes through the general
//             cell parser; a record with quotes, control or blank bytes in a
//             needed field, or longer than the view, goes through the general
//             parse_line cursor (csv_reader.c:278-338) -- same semantics, slower
//   filter    WHERE bytecode (plan.h OP_*), or a direct compare for col-op-const
//   group     LDS open-addressing table, 16-byte inline keys, COUNT / SUM / AVG /
//             MIN / MAX accumulators; flushed once per block into the HBM table
//             (per-thread registers when the query has no GROUP BY)
//
// Every per-record array (cells, accumulator pointers) is indexed with
// compile-time indices only, so it lives in registers: a run-time index would
// move it to scratch memory, which costs more than the whole parse.
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
constexpr int TILE16 = TILE / 16;            // 2177 16-byte loads per tile
constexpr int NMW = (WIN + MARGIN) / 64;     // mask words covering [ws, ws + WIN + MARGIN)
constexpr int RSMAX = 2048;                  // record slots per pass
constexpr int LDS_BUDGET = 160 * 1024;       // LDS bytes per CU
constexpr int PF = (TILE16 + SCAN_T - 1) / SCAN_T;   // prefetch registers per lane (5)
constexpr uint64_t NOPOS = ~0ULL;
constexpr uint32_t NONE = 255;               // "no separator in the 128-bit view"
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

// ------------------------------------------------------------------ per-record cells
// cells of one record in registers: callers index them with unrolled loops only
struct Cells {
    Cell c[MAX_NEED];
};

// cells.c[a] for a uniform run-time slot `a`, without a run-time index
// (field-wise selects: a branch per slot would let the optimiser merge the
// copies into one load through a computed address, i.e. back into memory)
__device__ __forceinline__ Cell sel_cell(bool t, const Cell& x, const Cell& y) {
    Cell r;
    r.kind = t ? x.kind : y.kind;
    r.len = t ? x.len : y.len;
    r.bits = t ? x.bits : y.bits;
    return r;
}
__device__ __forceinline__ Cell get_cell(const Cells& cs, int a, int n = MAX_NEED) {
    Cell r = cs.c[0];
#pragma unroll
    for (int k = 1; k < MAX_NEED; k++) {
        if (k >= n) break;                        // n is uniform: a scalar branch
        r = sel_cell(k == a, cs.c[k], r);
    }
    return r;
}

// the general cell parser (cell.h parse_cell) kept out of line: it carries the
// date test and the big-number strtod fallback, which the fast paths rarely need
__device__ __noinline__ Cell parse_cell_slow(const uint8_t* f, uint32_t len) { return parse_cell(f, len); }
__device__ __noinline__ GKey group_key_slow(const Cell c) { return group_key(c); }

// ------------------------------------------------------------------ general record parse
// One field of parse_line (csv_reader.c:278-338) at rec[i]: leading blanks are
// skipped; returns false if the record ends there (a trailing field of blanks
// is dropped).  On return [fs, fs + flen) is the field's value (a quoted field
// without its quotes, `""` kept as two bytes; an unclosed quoted field has the
// length of its `""` pairs) and i is at the terminator (delimiter or newline).
__device__ __forceinline__ bool g_field(const uint8_t* rec, uint32_t& i, uint32_t delim, uint32_t quote,
                                        uint32_t& fs, uint32_t& flen) {
    uint32_t c = rec[i];
    while (is_blank(c)) { i = i + 1; c = rec[i]; }
    if (is_nl(c)) return false;
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
    return true;
}

// parse_line restricted to the needed columns, into registers (unrolled over
// the need slots).  Returns true when the record is too short for a needed column.
__device__ __forceinline__ bool parse_record_regs(const uint8_t* rec, const ScanPlan& P, Cells& cs) {
    const uint32_t delim = P.delim, quote = P.quote;
    uint32_t i = 0, fs = 0, flen = 0;
    int col = 0;
    bool ended = false;
#pragma unroll
    for (int k = 0; k < MAX_NEED; k++) {
        if (k >= P.nneed) break;
        const int want = P.need_col[k];
        Cell c = cell_null();
        while (!ended && col < want) {
            if (!g_field(rec, i, delim, quote, fs, flen) || rec[i] != delim) ended = true;
            else { i = i + 1; col++; }
        }
        if (!ended) {
            if (!g_field(rec, i, delim, quote, fs, flen)) {
                ended = true;
            } else {
                c = parse_cell_slow(rec + fs, flen);
                if (rec[i] == delim) { i = i + 1; col++; }
                else ended = true;                  // later columns do not exist
            }
        }
        cs.c[k] = c;
    }
    return ended;
}

// the same into a global array (representative-row gather)
__device__ void parse_record_out(const uint8_t* rec, const ScanPlan& P, Cell* out) {
    const uint32_t delim = P.delim, quote = P.quote;
    uint32_t i = 0, fs = 0, flen = 0;
    int col = 0;
    bool ended = false;
    for (int k = 0; k < P.nneed; k++) {
        const int want = P.need_col[k];
        Cell c = cell_null();
        while (!ended && col < want) {
            if (!g_field(rec, i, delim, quote, fs, flen) || rec[i] != delim) ended = true;
            else { i = i + 1; col++; }
        }
        if (!ended) {
            if (!g_field(rec, i, delim, quote, fs, flen)) {
                ended = true;
            } else {
                c = parse_cell(rec + fs, flen);
                if (rec[i] == delim) { i = i + 1; col++; }
                else ended = true;
            }
        }
        out[k] = c;
    }
}

// ------------------------------------------------------------------ predicate VM
// value stack in registers: select-based access (no run-time array index)
struct Stack {
    Cell s[8];
    __device__ __forceinline__ Cell get(int i) const {
        Cell r = s[0];
#pragma unroll
        for (int j = 1; j < 8; j++) r = sel_cell(j == i, s[j], r);
        return r;
    }
    __device__ __forceinline__ void set(int i, const Cell& v) {
#pragma unroll
        for (int j = 0; j < 8; j++) s[j] = sel_cell(j == i, v, s[j]);
    }
};

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
__device__ __forceinline__ bool eval_where_vm(const ScanPlan& P, const Cells& cs) {
    Stack st;
#pragma unroll
    for (int j = 0; j < 8; j++) st.s[j] = cell_null();
    int sp = 0;
    uint32_t bs = 0;   // bool stack, top = bit 0
    for (int pc = 0; pc < P.nprog; pc++) {
        const Insn in = P.prog[pc];
        switch (in.op) {
            case OP_COL: st.set(sp++, get_cell(cs, in.a)); break;
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

__device__ int g_insert(const GroupTable& gt, const GKey k, uint64_t h, ScanStats* st) {
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
                             const Cell c, uint64_t pos, ScanStats* st) {
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

__device__ __forceinline__ int l_insert(const LdsTable& t, const GKey k, uint64_t h) {
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
__device__ __forceinline__ void lds_ext_update(bool need, const ExtLds& e, uint32_t s, uint8_t kind,
                                               const Cell c, uint64_t pos) {
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

// ------------------------------------------------------------------ fast field path
// 128-bit view of a per-64-byte mask starting at window offset 64*wi + o
struct View {
    uint64_t lo, hi;
};
__device__ __forceinline__ View view128(const uint64_t* m, uint32_t wi, uint32_t o) {
    const uint64_t a0 = m[wi], a1 = m[wi + 1];
    View v;
    v.lo = o ? (a0 >> o) | (a1 << (64 - o)) : a0;
    v.hi = a1 >> o;
    return v;
}
__device__ __forceinline__ uint32_t first128(const View& v) {
    return v.lo ? (uint32_t)__builtin_ctzll(v.lo) : (v.hi ? 64u + (uint32_t)__builtin_ctzll(v.hi) : NONE);
}
__device__ __forceinline__ void pop128(View& v) {
    const bool l = v.lo != 0;
    const uint64_t hi2 = v.hi & (v.hi - 1);
    v.lo = v.lo & (v.lo - 1);
    v.hi = l ? v.hi : hi2;
}

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

// Type a field of `len` bytes at tile offset `to` whose bytes hold no record
// terminator, delimiter or quote (infer_type + parse_value, csv_reader.c:
// 136-240).  FF_OK: `out` (and `key` when want_key) are final; FF_SLOW: the
// general record path decides -- a byte <= ' ' (blank, control, NUL: leading
// blanks move the field start and a blank-only last field is dropped), a date
// shaped field, a leading '+', a numeral past the exact fast cases, a field over
// 16 bytes, or a delimiter strtod/strtoll could read across (num_ok false).
// Control flow depends only on the field's shape, which is normally the same
// for every record of a column, so the wave rarely diverges here.
__device__ __forceinline__ int fast_field(const uint8_t* tile, uint32_t to, uint32_t len, bool num_ok,
                                          bool want_key, Cell& out, GKey& key) {
    out = cell_null();
    if (len == 0) {
        if (want_key) key = group_key(out);
        return FF_OK;
    }
    if (len > 16) return FF_SLOW;
    uint32_t d0, d1, d2, d3;
    load16(tile, to, d0, d1, d2, d3);
    const uint32_t m0 = len_mask(len, 0), m1 = len_mask(len, 1), m2 = len_mask(len, 2), m3 = len_mask(len, 3);
    const uint32_t low = lt_bytes(d0 | ~m0, 0x21212121u) | lt_bytes(d1 | ~m1, 0x21212121u) |
                         lt_bytes(d2 | ~m2, 0x21212121u) | lt_bytes(d3 | ~m3, 0x21212121u);
    const uint32_t c0 = d0 & 0xffu;
    if (low || c0 == '+') return FF_SLOW;
    d0 &= m0; d1 &= m1; d2 &= m2; d3 &= m3;
    const bool neg = c0 == '-';
    // infer_type's numeric shape: [-] digits with at most one '.', at least one digit
    const uint32_t f0 = m0 & 0x80808080u, f1 = m1 & 0x80808080u, f2 = m2 & 0x80808080u, f3 = m3 & 0x80808080u;
    const uint32_t g0 = digit_bytes(d0) & f0, g1 = digit_bytes(d1) & f1, g2 = digit_bytes(d2) & f2,
                   g3 = digit_bytes(d3) & f3;
    const uint32_t p0 = ~nonzero_bytes(d0 ^ 0x2E2E2E2Eu) & f0, p1 = ~nonzero_bytes(d1 ^ 0x2E2E2E2Eu) & f1,
                   p2 = ~nonzero_bytes(d2 ^ 0x2E2E2E2Eu) & f2, p3 = ~nonzero_bytes(d3 ^ 0x2E2E2E2Eu) & f3;
    const uint32_t other = ((f0 & ~g0 & ~p0) & ~(neg ? 0x80u : 0u)) | (f1 & ~g1 & ~p1) | (f2 & ~g2 & ~p2) |
                           (f3 & ~g3 & ~p3);
    const uint32_t ndig = __popc(g0) + __popc(g1) + __popc(g2) + __popc(g3);
    const uint32_t ndot = __popc(p0) + __popc(p1) + __popc(p2) + __popc(p3);
    const uint64_t w0 = (uint64_t)d0 | ((uint64_t)d1 << 32), w1 = (uint64_t)d2 | ((uint64_t)d3 << 32);
    if (len >= 8 && len <= 10 && (is_digit(c0) || c0 == '-')) return FF_SLOW;   // parse_date may accept it
    if (other == 0 && ndig != 0 && ndot <= 1) {
        if (!num_ok) return FF_SLOW;
        // digit values (sign and dot bytes -> 0), dot removed, right-aligned in 16 bytes
        uint64_t v0 = (w0 ^ 0x3030303030303030ULL) &
                      ((uint64_t)spread(g0) | ((uint64_t)spread(g1) << 32));
        uint64_t v1 = (w1 ^ 0x3030303030303030ULL) &
                      ((uint64_t)spread(g2) | ((uint64_t)spread(g3) << 32));
        const uint64_t dotm0 = (uint64_t)p0 | ((uint64_t)p1 << 32), dotm1 = (uint64_t)p2 | ((uint64_t)p3 << 32);
        const uint32_t pb = dotm0 ? (uint32_t)__builtin_ctzll(dotm0) : (dotm1 ? 64u + (uint32_t)__builtin_ctzll(dotm1) : 128u);
        const uint32_t p = pb >> 3;                                // dot byte index (16: none)
        if (ndot) {
            const uint64_t k0 = p >= 8 ? ~0ULL : ((1ULL << (8 * p)) - 1);
            const uint64_t k1 = p >= 8 ? ((1ULL << (8 * (p - 8))) - 1) : 0ULL;
            const uint64_t s0 = (v0 >> 8) | (v1 << 56), s1 = v1 >> 8;
            v0 = (v0 & k0) | (s0 & ~k0);
            v1 = (v1 & k1) | (s1 & ~k1);
        }
        const uint32_t lc = len - ndot;                            // digit positions (sign counted as 0)
        const uint32_t sh = 8 * (16 - lc);                         // 0..120
        uint64_t a0, a1;
        if (sh >= 64) {
            a1 = v0 << (sh - 64);
            a0 = 0;
        } else {
            a1 = sh ? (v1 << sh) | (v0 >> (64 - sh)) : v1;
            a0 = v0 << sh;
        }
        const uint64_t W = (uint64_t)dig8(a0) * 100000000ULL + dig8(a1);
        if (!ndot) {
            out = cell_int(neg ? -(int64_t)W : (int64_t)W);
        } else {
            if (W > (1ULL << 53)) return FF_SLOW;                  // Clinger's exact case only
            const double v = (double)W / pow10_exact(len - 1 - p);   // one correctly rounded division
            out = cell_dbl(neg ? -v : v);
        }
        if (want_key) key = group_key(out);
        return FF_OK;
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

// ------------------------------------------------------------------ the scan kernel
// dynamic LDS: [tile][nl/sep masks][quote flags][rs][scan scratch][group table][accumulators]
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

// classify 64 staged bytes: terminator and separator masks, quote presence
__device__ __forceinline__ void classify64(const uint8_t* p, uint32_t rep_d, uint32_t rep_q, uint64_t& nlm,
                                           uint64_t& sepm, bool& has_q) {
    const v4u* src = (const v4u*)p;
    uint32_t nl_lo = 0, nl_hi = 0, sp_lo = 0, sp_hi = 0, qacc = 0x80808080u;
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const v4u x4 = src[v];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t x = x4[j];
            const uint32_t nl_inv = nonzero_bytes(x ^ 0x0A0A0A0Au) & nonzero_bytes(x ^ 0x0D0D0D0Du);
            const uint32_t sp_inv = nl_inv & nonzero_bytes(x ^ rep_d);
            qacc &= nonzero_bytes(x ^ rep_q);
            // 0x80 flags -> nibbles: separators in bits 0-3, terminators in bits 4-7
            const uint32_t c = ((~sp_inv & 0x80808080u) >> 7) | ((~nl_inv & 0x80808080u) >> 3);
            uint32_t t = c | (c >> 7);
            t = t | (t >> 14);
            const int d = v * 4 + j, sh = (d & 7) * 4;
            if (d < 8) {
                sp_lo |= (t & 0xFu) << sh;
                nl_lo |= ((t >> 4) & 0xFu) << sh;
            } else {
                sp_hi |= (t & 0xFu) << sh;
                nl_hi |= ((t >> 4) & 0xFu) << sh;
            }
        }
    }
    nlm = (uint64_t)nl_lo | ((uint64_t)nl_hi << 32);
    sepm = (uint64_t)sp_lo | ((uint64_t)sp_hi << 32);
    has_q = qacc != 0x80808080u;
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
    uint8_t* qfl = carve(q, NMW);
    uint16_t* rs = (uint16_t*)carve(q, RSMAX * 2);
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

    // uniform plan facts
    const int nneed = P.nneed;
    const int gslot = GROUPED ? P.group_slot : -1;
    const bool simple = P.nprog == 3 && P.prog[0].op == OP_COL && P.prog[1].op == OP_CONST && P.prog[2].op == OP_CMP;
    const int wslot = simple ? P.prog[0].a : 0;
    const uint32_t wop = simple ? P.prog[2].a : 0;
    const Cell wconst = simple ? P.consts[P.prog[1].b] : cell_null();
    const GKey null_key = group_key(cell_null());

    const uint64_t lo_ok = P.data_begin > P.range_begin ? P.data_begin : P.range_begin;
    const uint64_t hi_ok = P.range_end < P.n ? P.range_end : P.n;
    const uint64_t first_win = P.range_begin / WIN;
    const uint64_t last_win = (hi_ok + WIN - 1) / WIN;
    const uint32_t delim = P.delim, quote = P.quote;
    const uint32_t rep_d = delim * 0x01010101u, rep_q = quote * 0x01010101u;
    // strtoll/strtod read past the field end: a delimiter they could consume
    // (digit, '.', letter) sends numerals to the general cell parser
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
        uint64_t my_nl;
        {
            uint64_t sepm;
            bool hq;
            classify64(tile + PRE + tid * 64, rep_d, rep_q, my_nl, sepm, hq);
            nlw[tid] = my_nl;
            sepw[tid] = sepm;
            qfl[tid] = hq;
            if (tid < NMW - SCAN_T) {
                uint64_t n2;
                classify64(tile + PRE + (SCAN_T + tid) * 64, rep_d, rep_q, n2, sepm, hq);
                nlw[SCAN_T + tid] = n2;
                sepw[SCAN_T + tid] = sepm;
                qfl[SCAN_T + tid] = hq;
            }
        }
        lds_barrier();
        // ---- record starts in this lane's 64 window bytes
        uint64_t starts;
        {
            const uint64_t prev_nl = (tid == 0) ? (is_nl(tile[PRE - 1]) ? 1ULL : 0ULL) : (nlw[tid - 1] >> 63);
            starts = ~my_nl & ((my_nl << 1) | prev_nl);
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
                    if (ri >= chunk && ri < chunk + RSMAX) rs[ri - chunk] = (uint16_t)(tid * 64 + b);
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
                Cells cs;
#pragma unroll
                for (int k = 0; k < MAX_NEED; k++) cs.c[k] = cell_null();
                GKey key = null_key;
                bool pass = false;
                if (valid) {
                    // -- fast walk over the 128-bit mask views at the record start
                    const uint32_t wi = r >> 6, o = r & 63;
                    View S = view128(sepw, wi, o);
                    const uint32_t rend = first128(view128(nlw, wi, o));
                    bool fail = (qfl[wi] | qfl[wi + 1]) != 0;
                    bool ended = false;
                    uint32_t fs = 0;
                    int col = 0;
#pragma unroll
                    for (int k = 0; k < MAX_NEED; k++) {
                        if (k >= nneed) break;
                        const int want = P.need_col[k];
                        for (; col < want; col++) {            // uniform trip count, no branches
                            const uint32_t e = first128(S);
                            fail = fail || (e == NONE && !ended);
                            ended = ended || e == rend;
                            fs = e + 1;
                            pop128(S);
                        }
                        const uint32_t e = first128(S);
                        fail = fail || (e == NONE && !ended);
                        Cell c = cell_null();
                        if (!ended && !fail) {                 // uniform unless the record is short
                            fail = fast_field(tile, PRE + r + fs, e - fs, num_ok, k == gslot, c, key) != FF_OK;
                            if (c.kind == K_STR) c.bits = (uint64_t)(uintptr_t)(g + rec + fs);
                        }
                        cs.c[k] = c;
                    }
                    bool short_row = ended;
                    if (fail) {
                        // -- the general parse_line cursor over global memory
                        my_slow++;
                        short_row = parse_record_regs(g + rec, P, cs);
                        if (GROUPED) key = group_key_slow(get_cell(cs, gslot, nneed));
                    }
                    my_records++;
                    if (short_row) my_short++;
                    if (P.nprog == 0) pass = true;
                    else if (simple) pass = cmp_result(wop, compare(get_cell(cs, wslot, nneed), wconst));
                    else pass = eval_where_vm(P, cs);
                    if (pass) my_pass++;
                }
                if (pass && row_out) {
                    const unsigned long long slot = atomicAdd(&stats->rows_emitted, 1ULL);
                    if (slot < row_cap) {
                        row_out[slot] = rec;
                        if (cells_out) {   // debug: the cells this kernel parsed
#pragma unroll
                            for (int k = 0; k < MAX_NEED; k++)
                                if (k < nneed) cells_out[slot * nneed + k] = cs.c[k];
                        }
                    }
                }
                if (pass) {
#pragma unroll
                    for (int a = 0; a < MAX_ACC; a++)
                        if (a < P.nacc && P.acc[a].kind != ACC_SUM)
                            my_cls[a] |= class_bit(get_cell(cs, P.acc[a].slot, nneed));
                }
                if (!GROUPED) {
                    if (pass) {
                        my_cnt++;
                        if (rec < my_first) my_first = rec;
#pragma unroll
                        for (int a = 0; a < MAX_ACC; a++) {
                            if (a >= P.nacc) break;
                            const Cell c = get_cell(cs, P.acc[a].slot, nneed);
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
                            if (a >= P.nacc) break;
                            if (!la[a].sum) continue;
                            const Cell c = get_cell(cs, P.acc[a].slot, nneed);
                            if (is_num(c)) {
                                atomicAdd(&la[a].sum[s], num_of(c));
                                atomicAdd(&la[a].num[s], 1u);
                            }
                        }
                    }
#pragma unroll
                    for (int a = 0; a < MAX_ACC; a++) {
                        if (a >= P.nacc) break;
                        if (!le[a].c) continue;                  // uniform
                        const Cell c = get_cell(cs, P.acc[a].slot, nneed);
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
#pragma unroll
                                for (int a = 0; a < MAX_ACC; a++) {
                                    if (a >= P.nacc) break;
                                    const Cell c = get_cell(cs, P.acc[a].slot, nneed);
                                    if (P.acc[a].kind == ACC_SUM && is_num(c)) {
                                        atomicAdd(&gt.sum[a][gi], num_of(c));
                                        atomicAdd(&gt.num[a][gi], 1ULL);
                                    }
                                }
                            }
                        }
#pragma unroll
                        for (int a = 0; a < MAX_ACC; a++) {
                            if (a >= P.nacc) break;
                            if (P.acc[a].kind == ACC_SUM) continue;   // uniform
                            const Cell c = get_cell(cs, P.acc[a].slot, nneed);
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
#pragma unroll
    for (int a = 0; a < MAX_ACC; a++) {
        if (a >= P.nacc) break;
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
#pragma unroll
                for (int a = 0; a < MAX_ACC; a++)
                    if (a < P.nacc && P.acc[a].kind == ACC_SUM && nm[a]) {
                        atomicAdd(&gt.sum[a][gi], sm[a]);
                        atomicAdd(&gt.num[a][gi], nm[a]);
                    }
            }
        }
        gi = __shfl(gi, 0, 64);
#pragma unroll
        for (int a = 0; a < MAX_ACC; a++) {
            if (a >= P.nacc) break;
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
#pragma unroll
                for (int a = 0; a < MAX_ACC; a++) {
                    if (a >= P.nacc) break;
                    if (la[a].sum && la[a].num[i]) {
                        atomicAdd(&gt.sum[a][gi], la[a].sum[i]);
                        atomicAdd(&gt.num[a][gi], (unsigned long long)la[a].num[i]);
                    }
                }
            }
        }
#pragma unroll
        for (int a = 0; a < MAX_ACC; a++) {
            if (a >= P.nacc) break;
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
    parse_record_out(g + recs[i], P, out + (uint64_t)i * P.nneed);
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
    return r16(cq::TILE) + 2 * r16(cq::NMW * 8) + r16(cq::NMW) + r16(cq::RSMAX * 2) + r16(64);
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
