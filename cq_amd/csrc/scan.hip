// scan.hip -- the fused CSV scan for cq's SELECT hot path on gfx950.
//
// One pass over the CSV bytes resident in HBM does what the reference spreads
// over csv_load (csv_reader.c:375-465), filter_rows (evaluator_utils.c:986),
// create_groups (evaluator_aggregates.c:108) and evaluate_aggregate (:263):
//
//   stage   32 KiB window -> LDS with coalesced 16 B/lane loads
//   split   each lane classifies 64 window bytes (SWAR '\n'/'\r' tests), marks
//           record starts, and a block-wide scan hands every record an LDS slot
//   parse   one lane per record walks its fields (quote-aware, parse_line
//           csv_reader.c:278-338) up to the last column the plan needs and types
//           those cells (infer_type/parse_value, cell.h)
//   filter  the WHERE bytecode runs per record in registers (plan.h OP_*)
//   group   LDS open-addressing table keyed by the printf-canonical key identity,
//           COUNT/SUM/AVG/MIN/MAX accumulators; flushed once per block into the
//           HBM table with agent-scope atomics (or per-thread registers when the
//           query has no GROUP BY)
//
// Records are owned by the window holding their first byte, so every byte range
// [range_begin, range_end) can be scanned independently: that is also how the
// multi-GPU path shards a file.
#include <hip/hip_runtime.h>
#include "plan.h"

namespace cq {

constexpr int SCAN_T = 512;        // threads per block (8 waves)
constexpr int WIN = 32768;         // window bytes (64 per lane)
constexpr int PRE = 16;            // bytes staged before the window
constexpr int MARGIN = 2048;       // bytes staged after the window
constexpr int TILE = PRE + WIN + MARGIN;
constexpr int RSMAX = 2048;        // record slots per pass
constexpr int LDS_BUDGET = 160 * 1024; // LDS bytes per CU
constexpr uint64_t NOPOS = ~0ULL;
constexpr uint32_t GK_ALL = 7;     // key class of the single group (no GROUP BY)

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    // 0x80 in each byte of v that is zero (exact, no borrow propagation)
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t nl4(uint32_t x) {
    uint32_t m = zero_bytes(x ^ 0x0A0A0A0Au) | zero_bytes(x ^ 0x0D0D0D0Du);
    return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}
__device__ __forceinline__ bool is_nl(uint32_t c) { return c == '\n' || c == '\r'; }

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
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_T / 64; w++) {
        uint32_t s = wsum[w];
        if (w < wid) base += s;
        tot += s;
    }
    *total = tot;
    __syncthreads();
    return base + x - v;
}

// ------------------------------------------------------------------ record parse
// Byte sources addressed relative to the record start.  WinSrc reads the staged
// LDS window while the offset is inside it and global memory past its end;
// GlobSrc always reads global memory.
struct WinSrc {
    const uint8_t* l;      // LDS copy of the record start
    const uint8_t* g;      // global copy of the record start
    uint32_t lim;          // bytes of the record available in LDS
    __device__ __forceinline__ uint32_t at(uint32_t i) const { return i < lim ? (uint32_t)l[i] : (uint32_t)g[i]; }
};
struct GlobSrc {
    const uint8_t* g;
    __device__ __forceinline__ uint32_t at(uint32_t i) const { return (uint32_t)g[i]; }
};

// parse_line (csv_reader.c:278-338) restricted to the needed columns: fills
// cells[0..nneed) (NULL for columns the record is too short to have).
// `gbase` is the record start in global memory (cells point into it).
template <class Src>
__device__ __forceinline__ bool parse_record(const Src& S, const uint8_t* gbase, const ScanPlan& P,
                                             Cell* cells) {
    if (P.nneed == 0) return true;
    const uint32_t delim = P.delim, quote = P.quote;
    uint32_t i = 0;
    int col = 0, k = 0;
    int want = P.need_col[0];
    while (true) {
        uint32_t c = S.at(i);
        while (c == ' ' || c == '\t' || c == 0x0b || c == 0x0c) {
            i = i + 1;
            c = S.at(i);
        }
        if (is_nl(c)) break;                       // trailing empty field dropped
        uint32_t fs, flen;
        if (c == quote) {                          // quoted field (:294-317)
            i = i + 1;
            fs = i;
            uint32_t acc = 0;
            bool closed = false;
            flen = 0;
            while (true) {
                c = S.at(i);
                if (is_nl(c)) break;
                if (c == quote) {
                    if (S.at(i + 1) == quote) { i = i + 2; acc += 2; }
                    else { flen = i - fs; i = i + 1; closed = true; break; }
                } else {
                    i = i + 1;
                }
            }
            if (!closed) flen = acc;
            c = S.at(i);
            while (c != delim && !is_nl(c)) { i = i + 1; c = S.at(i); }
        } else {                                   // unquoted field (:318-324)
            fs = i;
            while (c != delim && !is_nl(c)) { i = i + 1; c = S.at(i); }
            flen = i - fs;
        }
        if (col == want) {
            cells[k] = parse_cell(gbase + fs, flen);
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

// evaluate_condition over the flattened WHERE tree
__device__ bool eval_where(const ScanPlan& P, const Cell* cells) {
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
                int c = compare(l, r);
                bool b;
                switch (in.a) {
                    case CMP_EQ: b = c == 0; break;
                    case CMP_NE: b = c != 0; break;
                    case CMP_LT: b = c < 0; break;
                    case CMP_GT: b = c > 0; break;
                    case CMP_LE: b = c <= 0; break;
                    default: b = c >= 0; break;
                }
                bs = (bs << 1) | (b ? 1u : 0u);
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
    for (uint32_t probe = 0; probe < gt.cap; probe++) {
        uint32_t i = (uint32_t)(h + probe) & mask;
        uint32_t t = __hip_atomic_load(&gt.tag[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0) {
            uint32_t old = atomicCAS(&gt.tag[i], 0u, 1u);
            if (old == 0) {
                __hip_atomic_store(&gt.kcls[i], k.cls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&gt.klen[i], k.len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&gt.kv[i], k.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
            o.cls = __hip_atomic_load(&gt.kcls[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o.len = __hip_atomic_load(&gt.klen[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o.v = __hip_atomic_load(&gt.kv[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    uint32_t* cnt;
    unsigned long long* first;
    uint32_t* kcls;
    uint32_t* klen;
    uint64_t* kv;
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
    for (uint32_t probe = 0; probe < 64; probe++) {
        uint32_t i = (uint32_t)(h + probe) & (t.H - 1);
        uint32_t cur = __hip_atomic_load(&t.tag[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
            uint32_t old = atomicCAS(&t.tag[i], 0u, 1u);
            if (old == 0) {
                t.kcls[i] = k.cls;
                t.klen[i] = k.len;
                t.kv[i] = k.v;
                __hip_atomic_store(&t.tag[i], tg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                return (int)i;
            }
            cur = old;
        }
        for (uint32_t spin = 0; cur == 1; spin++) {
            if (spin > (1u << 24)) return -1;          // the HBM table takes the record
            cur = __hip_atomic_load(&t.tag[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (cur == tg) {
            GKey o;
            o.cls = t.kcls[i];
            o.len = t.klen[i];
            o.v = t.kv[i];
            if (gk_equal(o, k)) return (int)i;
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

// ------------------------------------------------------------------ the scan kernel
// dynamic LDS: [tile TILE][rs RSMAX*4][scan scratch][group table][accumulators]
__device__ __forceinline__ uint8_t* carve(uint8_t*& q, size_t bytes) {
    uint8_t* r = q;
    q += (bytes + 15) & ~(size_t)15;
    return r;
}

template <bool GROUPED>
__global__ __launch_bounds__(SCAN_T) void scan_kernel(const uint8_t* __restrict__ g, ScanPlan P,
                                                      GroupTable gt, ScanStats* __restrict__ stats,
                                                      unsigned long long* __restrict__ row_out,
                                                      unsigned long long row_cap, uint32_t lds_h,
                                                      Cell* __restrict__ cells_out) {
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t* tile = smem;
    uint32_t* rs = (uint32_t*)(smem + TILE);
    uint32_t* wsum = rs + RSMAX;                       // 16 words of scan scratch
    uint8_t* q = (uint8_t*)(wsum + 16);
    LdsTable lt;
    LdsAcc la[MAX_ACC];
    ExtLds le[MAX_ACC];
    const uint32_t H = lds_h;
    lt.H = H;
    if (GROUPED) {
        lt.tag = (uint32_t*)carve(q, H * 4);
        lt.cnt = (uint32_t*)carve(q, H * 4);
        lt.first = (unsigned long long*)carve(q, H * 8);
        lt.kcls = (uint32_t*)carve(q, H * 4);
        lt.klen = (uint32_t*)carve(q, H * 4);
        lt.kv = (uint64_t*)carve(q, H * 8);
    }
    _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) {
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
            _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
                if (la[a].sum) { la[a].sum[i] = 0.0; la[a].num[i] = 0; }
                if (le[a].c) { le[a].pos[i] = NOPOS; le[a].lock[i] = 0; }
            }
        }
    }
    // per-thread partials (single-group mode) and statistics
    unsigned long long my_cnt = 0, my_first = NOPOS, my_records = 0, my_short = 0, my_spill = 0;
    double my_sum[MAX_ACC];
    unsigned long long my_num[MAX_ACC];
    Cell my_ext[MAX_ACC];
    unsigned long long my_pos[MAX_ACC];
    uint32_t my_cls[MAX_ACC];
    for (int a = 0; a < MAX_ACC; a++) {
        my_sum[a] = 0.0; my_num[a] = 0; my_ext[a] = cell_null(); my_pos[a] = NOPOS; my_cls[a] = 0;
    }

    const uint64_t lo_ok = P.data_begin > P.range_begin ? P.data_begin : P.range_begin;
    const uint64_t hi_ok = P.range_end < P.n ? P.range_end : P.n;
    const uint64_t first_win = P.range_begin / WIN;
    const uint64_t last_win = (hi_ok + WIN - 1) / WIN;

    for (uint64_t w = first_win + blockIdx.x; w < last_win; w += gridDim.x) {
        const uint64_t ws = w * WIN;
        __syncthreads();
        // ---- stage the window (+PRE before, +MARGIN after) into LDS, 16 B per lane
        const uint4* src = (const uint4*)(g + ws - PRE);
        for (int i = tid; i < TILE / 16; i += SCAN_T) ((uint4*)tile)[i] = src[i];
        __syncthreads();
        // ---- record starts in this lane's 64 bytes
        const uint32_t off = PRE + tid * 64;
        uint64_t nlm = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            uint32_t x = *(const uint32_t*)(tile + off + 4 * j);
            nlm |= (uint64_t)nl4(x) << (4 * j);
        }
        uint64_t prev_nl = is_nl(tile[off - 1]) ? 1ULL : 0ULL;
        uint64_t starts = ~nlm & ((nlm << 1) | prev_nl);
        const uint64_t base = ws + (uint64_t)tid * 64;
        // keep starts in [lo_ok, hi_ok)
        if (base + 64 <= lo_ok || base >= hi_ok) starts = 0;
        else {
            if (base < lo_ok) starts &= ~0ULL << (lo_ok - base);
            if (base + 64 > hi_ok) starts &= (hi_ok - base >= 64) ? ~0ULL : ((1ULL << (hi_ok - base)) - 1);
        }
        uint32_t cnt = (uint32_t)__popcll(starts);
        uint32_t total;
        uint32_t idx = block_excl_scan(cnt, wsum, &total);
        for (uint32_t chunk = 0; chunk < total; chunk += RSMAX) {
            // ---- scatter this chunk's record starts into LDS slots
            {
                uint64_t m = starts;
                uint32_t r = idx;
                while (m) {
                    int b = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    if (r >= chunk && r < chunk + RSMAX) rs[r - chunk] = tid * 64 + b;
                    r++;
                }
            }
            __syncthreads();
            const uint32_t nrec = min((uint32_t)RSMAX, total - chunk);
            for (uint32_t base0 = 0; base0 < nrec; base0 += SCAN_T) {
                // trip count is block-uniform: every lane of a wave runs every trip
                const uint32_t ri = base0 + tid;
                const bool valid = ri < nrec;
                const uint64_t rec = valid ? ws + rs[ri] : 0;
                Cell cells[MAX_NEED];
                _Pragma("unroll") for (int k = 0; k < MAX_NEED; k++) cells[k] = cell_null();
                bool pass = false;
                if (valid) {
                    WinSrc S;
                    S.l = tile + (rec - (ws - PRE));
                    S.g = g + rec;
                    S.lim = (uint32_t)(ws + WIN + MARGIN - rec);
                    bool complete = parse_record(S, g + rec, P, cells);
                    my_records++;
                    if (!complete) my_short++;
                    pass = P.nprog == 0 || eval_where(P, cells);
                }
                if (pass && row_out) {
                    unsigned long long slot = atomicAdd(&stats->rows_emitted, 1ULL);
                    if (slot < row_cap) {
                        row_out[slot] = rec;
                        if (cells_out)   // debug: the cells this kernel parsed
                            for (int k = 0; k < P.nneed; k++) cells_out[slot * P.nneed + k] = cell_at(cells, k);
                    }
                }
                if (pass)
                    _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) my_cls[a] |= class_bit(cell_at(cells, P.acc[a].slot));
                if (!GROUPED) {
                    if (pass) {
                        my_cnt++;
                        if (rec < my_first) my_first = rec;
                        _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
                            Cell c = cell_at(cells, P.acc[a].slot);
                            if (P.acc[a].kind == ACC_SUM) {
                                if (is_num(c)) { my_sum[a] += num_of(c); my_num[a]++; }
                            } else if (c.kind != K_NULL && ext_better(P.acc[a].kind, c, rec, my_ext[a], my_pos[a])) {
                                my_ext[a] = c; my_pos[a] = rec;
                            }
                        }
                    }
                } else {
                    GKey k;
                    k.cls = 0; k.len = 0; k.v = 0;
                    uint64_t h = 0;
                    int s = -1;
                    if (pass) {
                        k = group_key(cell_at(cells, P.group_slot));
                        h = gk_hash(k);
                        s = l_insert(lt, k, h);
                    }
                    const bool in_lds = pass && s >= 0;
                    const bool spill = pass && s < 0;
                    if (in_lds) {
                        atomicAdd(&lt.cnt[s], 1u);
                        atomicMin(&lt.first[s], (unsigned long long)rec);
                        _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
                            Cell c = cell_at(cells, P.acc[a].slot);
                            if (la[a].sum && is_num(c)) {
                                atomicAdd(&la[a].sum[s], num_of(c));
                                atomicAdd(&la[a].num[s], 1u);
                            }
                        }
                    }
                    _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
                        if (!le[a].c) continue;                 // uniform
                        Cell c = cell_at(cells, P.acc[a].slot);
                        lds_ext_update(in_lds && c.kind != K_NULL, le[a], in_lds ? (uint32_t)s : 0u,
                                       P.acc[a].kind, c, rec);
                    }
                    if (__any(spill)) {
                        // LDS table full: this record goes straight to the HBM table
                        int gi = -1;
                        if (spill) {
                            my_spill++;
                            gi = g_insert(gt, k, h, stats);
                            if (gi >= 0) {
                                atomicAdd(&gt.cnt[gi], 1ULL);
                                atomicMin(&gt.first[gi], (unsigned long long)rec);
                                _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
                                    Cell c = cell_at(cells, P.acc[a].slot);
                                    if (P.acc[a].kind == ACC_SUM && is_num(c)) {
                                        atomicAdd(&gt.sum[a][gi], num_of(c));
                                        atomicAdd(&gt.num[a][gi], 1ULL);
                                    }
                                }
                            }
                        }
                        _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
                            if (P.acc[a].kind == ACC_SUM) continue;   // uniform
                            Cell c = cell_at(cells, P.acc[a].slot);
                            g_ext_update(spill && gi >= 0 && c.kind != K_NULL, gt, a, P.acc[a].kind,
                                         gi >= 0 ? (uint32_t)gi : 0u, c, rec, stats);
                        }
                    }
                }
            }
            __syncthreads();
        }
    }
    __syncthreads();

    // ---- statistics and value-class masks
    {
        unsigned long long r = my_records, s = my_short, sp = my_spill;
        for (int o = 32; o > 0; o >>= 1) {
            r += __shfl_down(r, o, 64);
            s += __shfl_down(s, o, 64);
            sp += __shfl_down(sp, o, 64);
        }
        if ((tid & 63) == 0) {
            if (r) atomicAdd(&stats->records, r);
            if (s) atomicAdd(&stats->short_rows, s);
            if (sp) atomicAdd(&stats->lds_spills, sp);
        }
    }
    unsigned int* clsmask = stats->acc_classes;
    _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
        uint32_t m = my_cls[a];
        for (int o = 32; o > 0; o >>= 1) m |= __shfl_down(m, o, 64);
        if ((tid & 63) == 0 && m) atomicOr(&clsmask[a], m);
    }

    if (!GROUPED) {
        // ---- block-reduce the single group, then one global update per block
        unsigned long long c = my_cnt, f = my_first;
        for (int o = 32; o > 0; o >>= 1) {
            c += __shfl_down(c, o, 64);
            unsigned long long ff = __shfl_down(f, o, 64);
            f = ff < f ? ff : f;
        }
        double sm[MAX_ACC];
        unsigned long long nm[MAX_ACC];
        for (int a = 0; a < MAX_ACC; a++) {
            sm[a] = my_sum[a]; nm[a] = my_num[a];
            for (int o = 32; o > 0; o >>= 1) {
                sm[a] += __shfl_down(sm[a], o, 64);
                nm[a] += __shfl_down(nm[a], o, 64);
            }
        }
        GKey k;
        k.cls = GK_ALL; k.len = 0; k.v = 0;
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
        // MIN/MAX: every lane with a candidate merges under the slot's lock
        _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
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
            k.cls = lt.kcls[i]; k.len = lt.klen[i]; k.v = lt.kv[i];
            gi = g_insert(gt, k, gk_hash(k), stats);
            if (gi >= 0) {
                atomicAdd(&gt.cnt[gi], (unsigned long long)lt.cnt[i]);
                atomicMin(&gt.first[gi], lt.first[i]);
                _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
                    if (la[a].sum && la[a].num[i]) {
                        atomicAdd(&gt.sum[a][gi], la[a].sum[i]);
                        atomicAdd(&gt.num[a][gi], (unsigned long long)la[a].num[i]);
                    }
                }
            }
        }
        _Pragma("unroll") for (int a = 0; a < MAX_ACC; a++) if (a < P.nacc) {
            if (!le[a].c) continue;                     // uniform
            const bool ok = act && gi >= 0;
            Cell c = ok ? le[a].c[i] : cell_null();
            uint64_t pos = ok ? le[a].pos[i] : NOPOS;
            g_ext_update(ok, gt, a, P.acc[a].kind, ok ? (uint32_t)gi : 0u, c, pos, stats);
        }
    }
}

// ------------------------------------------------------------------ compaction
__global__ void compact_kernel(GroupTable gt, int nacc, GroupOut* out, unsigned int* count,
                               unsigned int cap_out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= gt.cap) return;
    if (gt.tag[i] < 2) return;
    unsigned int o = atomicAdd(count, 1u);
    if (o >= cap_out) return;
    GroupOut r;
    r.kcls = gt.kcls[i]; r.klen = gt.klen[i]; r.kv = gt.kv[i];
    r.cnt = gt.cnt[i]; r.first = gt.first[i];
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
__global__ void gather_kernel(const uint8_t* __restrict__ g, ScanPlan P,
                              const unsigned long long* __restrict__ recs, uint32_t nrec,
                              Cell* __restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    GlobSrc S;
    S.g = g + recs[i];
    Cell cells[MAX_NEED];
    parse_record(S, g + recs[i], P, cells);
    for (int k = 0; k < P.nneed; k++) out[(uint64_t)i * P.nneed + k] = cells[k];
}

// string bytes of cells -> packed host-visible buffer
__global__ void copy_strings_kernel(const Cell* __restrict__ cells, uint32_t n,
                                    const unsigned long long* __restrict__ offs,
                                    uint8_t* __restrict__ out) {
    uint32_t i = blockIdx.x;
    if (i >= n) return;
    Cell c = cells[i];
    if (c.kind != K_STR) return;
    const uint8_t* s = (const uint8_t*)(uintptr_t)c.bits;
    for (uint32_t j = threadIdx.x; j < c.len; j += blockDim.x) out[offs[i] + j] = s[j];
}

// literal texts -> cells (parse_value on LITERAL nodes, evaluator_expressions.c:30-31)
__global__ void parse_literals_kernel(const uint8_t* __restrict__ text,
                                      const unsigned int* __restrict__ offs,
                                      const unsigned int* __restrict__ lens, uint32_t n,
                                      Cell* __restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = parse_cell(text + offs[i], lens[i]);
}

}  // namespace cq

// explicit instantiations with C linkage wrappers for the host executor
extern "C" {
static size_t lds_slot_bytes(const cq::ScanPlan* P) {
    size_t b = 4 + 4 + 8 + 4 + 4 + 8;
    for (int a = 0; a < P->nacc; a++) b += P->acc[a].kind == cq::ACC_SUM ? 12 : sizeof(cq::Cell) + 12;
    return b;
}
static size_t lds_fixed_bytes() { return cq::TILE + cq::RSMAX * 4 + 64; }

// group-table capacity: the largest power of two <= 2048 that fits the budget
uint32_t cq_scan_lds_slots(const cq::ScanPlan* P, int grouped) {
    if (!grouped) return 0;
    size_t per = lds_slot_bytes(P);
    uint32_t h = 2048;
    while (h > 64 && lds_fixed_bytes() + (size_t)h * per + 16 * 16 > (size_t)cq::LDS_BUDGET) h >>= 1;
    return h;
}

size_t cq_scan_lds_bytes(const cq::ScanPlan* P, int grouped) {
    size_t b = lds_fixed_bytes();
    if (grouped) b += (size_t)cq_scan_lds_slots(P, grouped) * lds_slot_bytes(P) + 16 * 16;
    return b;
}

hipError_t cq_launch_scan(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          cq::ScanStats* stats, unsigned long long* row_out,
                          unsigned long long row_cap, int grouped, int grid, hipStream_t s,
                          cq::Cell* cells_out) {
    size_t lds = cq_scan_lds_bytes(P, grouped);
    if (grouped) {
        (void)hipFuncSetAttribute((const void*)cq::scan_kernel<true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(cq::scan_kernel<true>, dim3(grid), dim3(cq::SCAN_T), lds, s, g, *P, *gt,
                           stats, row_out, row_cap, cq_scan_lds_slots(P, grouped), cells_out);
    } else {
        (void)hipFuncSetAttribute((const void*)cq::scan_kernel<false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(cq::scan_kernel<false>, dim3(grid), dim3(cq::SCAN_T), lds, s, g, *P, *gt,
                           stats, row_out, row_cap, 0u, cells_out);
    }
    return hipGetLastError();
}

int cq_scan_occupancy(const cq::ScanPlan* P, int grouped) {
    size_t lds = cq_scan_lds_bytes(P, grouped);
    int blocks = 0;
    const void* fn = grouped ? (const void*)cq::scan_kernel<true> : (const void*)cq::scan_kernel<false>;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, cq::SCAN_T, lds) != hipSuccess) return 1;
    return blocks > 0 ? blocks : 1;
}

hipError_t cq_launch_compact(const cq::GroupTable* gt, int nacc, cq::GroupOut* out,
                             unsigned int* count, unsigned int cap_out, hipStream_t s) {
    dim3 grid((gt->cap + 255) / 256);
    hipLaunchKernelGGL(cq::compact_kernel, grid, dim3(256), 0, s, *gt, nacc, out, count, cap_out);
    return hipGetLastError();
}

hipError_t cq_launch_gather(const uint8_t* g, const cq::ScanPlan* P, const unsigned long long* recs,
                            uint32_t nrec, cq::Cell* out, hipStream_t s) {
    if (!nrec) return hipSuccess;
    hipLaunchKernelGGL(cq::gather_kernel, dim3((nrec + 127) / 128), dim3(128), 0, s, g, *P, recs,
                       nrec, out);
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
