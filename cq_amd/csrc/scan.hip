// scan.hip -- the fused CSV scan for cq's SELECT hot path on gfx950.
//
// One pass over the CSV bytes resident in HBM does what the reference spreads
// over csv_load (csv_reader.c:375-465), filter_rows (evaluator_utils.c:986),
// create_groups (evaluator_aggregates.c:108) and evaluate_aggregate (:263).
// One 512-thread block per window; consecutive windows start WSTRIDE bytes apart
// and each stages 32 KiB -- 64 bytes before its start and 1 KiB of overlap with
// the next window after its end -- so every lane owns one 64-byte mask word:
//
//   stage     the tile is copied from registers into LDS; the next window's
//             16 B/lane loads are already in flight
//   classify  each lane turns its 64 bytes into two 64-bit masks -- record
//             terminators ('\n' '\r') and separators (terminators and the
//             delimiter) -- and a quote-presence flag, branch-free SWAR
//   index     one block-wide scan numbers the separators, terminators and record
//             starts; every lane writes the tile positions of its separators
//             (the separator list), the separator index of its terminators, and
//             one slot per record start: so field c of a record is simply the
//             bytes between separators j0+c-1 and j0+c
//   parse     one lane per record types its needed fields with specialised int /
//             decimal / string parsers reading LDS.  A record with a quote in
//             front of its last needed field, a blank or control byte or a date
//             or long numeral in a needed field, or running past the tile, goes
//             through the general parse_line cursor (csv_reader.c:278-338) and
//             cell parser -- same semantics, slower; both read the LDS copy
//   filter    WHERE bytecode (plan.h OP_*), or a direct compare for col-op-const
//   group     LDS open-addressing table with 16-byte inline keys and fire-and-
//             forget LDS atomics for COUNT / SUM / AVG / first-row order, lock-
//             protected MIN / MAX; flushed once per block into the HBM table
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
#include <type_traits>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include "plan.h"
#include "scanlib.h"
#include "upload.h"

namespace cq {

constexpr int SCAN_T = 1024;                 // threads per block (16 waves, 4 per SIMD)
constexpr int TILE = 32768;                  // bytes staged per window (64 per lane)
constexpr int PREB = 64;                     // staged bytes before the window start
constexpr int WSTRIDE = 31680;               // window stride: 1 KiB of the tile overlaps the next window
constexpr int TILE_PAD = 32;                 // LDS slack after the tile for 16-byte field loads
constexpr int LB = TILE / SCAN_T;            // bytes classified per lane (32)
constexpr int NW = TILE / LB;                // mask words per tile (one per lane)
constexpr int TILE16 = TILE / 16;            // 16-byte loads per tile
constexpr int PF = TILE16 / SCAN_T;          // prefetch registers per lane (2)
constexpr int ECAP = 8192;                   // separator positions kept per tile
constexpr int NLCAP = 4096;                  // terminator indices kept per tile
constexpr int RSMAX = 2048;                  // record slots per pass
constexpr int KSTR = 1024;                   // LDS bytes for string literals
constexpr int LDS_BUDGET = 160 * 1024;       // LDS bytes per CU

static_assert(TILE16 % SCAN_T == 0, "tile loads split evenly over the block");
static_assert(PF == 2, "a lane stages exactly the 32 bytes it classifies");
static_assert(NW == SCAN_T, "one mask word per lane");

// The plan and the table descriptor live in constant memory (written on the
// launch stream before each launch): passed by value they would be copied to
// per-lane scratch, because the kernel indexes their arrays at run time.
__constant__ ScanPlan c_plan;
__constant__ GroupTable c_gt;
// slow_kernel's grid: the slow list's length is only known on the device and is 0
// on well-formed data, where a 256-block launch of this register- and
// scratch-heavy kernel costs ~15 us for nothing; 64 blocks (16 K lanes, grid-stride)
// cost ~4 us and still drain a full 1 Mi-record list
#ifndef SLOW_GRID
#define SLOW_GRID 64
#endif
__device__ __forceinline__ const ScanPlan& c_plan_ref() { return c_plan; }


// block-wide exclusive scan of two values per thread (SCAN_T threads)
__device__ __forceinline__ void block_excl_scan2(uint32_t a, uint32_t b, uint32_t* wsum, uint32_t& ea,
                                                 uint32_t& eb, uint32_t& ta, uint32_t& tb) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t x = wave_incl_scan(a), y = wave_incl_scan(b);
    if (lane == 63) { wsum[wid] = x; wsum[16 + wid] = y; }
    lds_barrier();
    uint32_t ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
    for (int w = 0; w < SCAN_T / 64; w++) {
        const uint32_t p = wsum[w], q = wsum[16 + w];
        if (w < wid) { ba += p; bb += q; }
        sa += p;
        sb += q;
    }
    ea = ba + x - a;
    eb = bb + y - b;
    ta = sa;
    tb = sb;
}

// ------------------------------------------------------------------ per-record cells
// cells of one record in registers: callers index them with unrolled loops only
template <int N>
struct CellsT {
    Cell c[N];
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
template <int N>
__device__ __forceinline__ Cell get_cell(const CellsT<N>& cs, int a, int n = N) {
    Cell r = cs.c[0];
#pragma unroll
    for (int k = 1; k < N; k++) {
        if (k >= n) break;                        // n is uniform: a scalar branch
        r = sel_cell(k == a, cs.c[k], r);
    }
    return r;
}

// A joined (or identity) pair's cells read in place from the sides' parsed cell
// tables: plans over more than MAX_NEED columns ("wide") keep no register copy;
// need slot a lives on side M->side[a] at cell M->col[a] of its row
constexpr uint32_t JOIN_NONE = 0xFFFFFFFFu;      // pair side absent (outer joins): NULL cells
struct PairView {
    const JoinMap* M;
    const Cell* L;
    const Cell* R;
    uint2 pr;
};
__device__ __forceinline__ Cell get_cell(const PairView& v, int a, int = 0) {
    const bool right = v.M->side[a] != 0;
    const uint32_t row = right ? v.pr.y : v.pr.x;
    if (row == JOIN_NONE) return cell_null();
    return right ? v.R[(uint64_t)row * v.M->rstride + v.M->col[a]] : v.L[(uint64_t)row * v.M->lstride + v.M->col[a]];
}

// the general cell parser (cell.h parse_cell) kept out of line: it carries the
// date test and the big-number strtod fallback, which the fast paths rarely need
__device__ __noinline__ Cell parse_cell_slow(const uint8_t* f, uint32_t len) { return parse_cell(f, len); }
__device__ __noinline__ GKey group_key_slow(const Cell c) { return group_key(c); }

// ------------------------------------------------------------------ general record parse
// Byte source of the general parser: the staged tile while the record lasts in
// it, HBM after.  Cells point at the tile copy when the field (plus the bytes
// strtod/strtoll may read past it) is staged, at HBM otherwise.
struct Src {
    const uint8_t* t;   // record start in the tile (LDS); unused when lim == 0
    const uint8_t* g;   // record start in HBM
    uint32_t lim;       // bytes of the record inside the tile
    bool lds_cells;     // cells may point into the tile (false: the delimiter could extend a numeral)
    __device__ __forceinline__ uint32_t at(uint32_t i) const { return i < lim ? (uint32_t)t[i] : (uint32_t)g[i]; }
    __device__ __forceinline__ const uint8_t* ptr(uint32_t i, uint32_t n) const {
        return (lds_cells && i + n + 48 <= lim) ? t + i : g + i;
    }
};

// One field of parse_line (csv_reader.c:278-338) at byte i: leading blanks are
// skipped; returns false if the record ends there (a trailing field of blanks
// is dropped).  On return [fs, fs + flen) is the field's value (a quoted field
// without its quotes, `""` kept as two bytes; an unclosed quoted field has the
// length of its `""` pairs) and i is at the terminator (delimiter or newline).
__device__ __forceinline__ bool g_field(const Src& S, uint32_t& i, uint32_t delim, uint32_t quote,
                                        uint32_t& fs, uint32_t& flen) {
    uint32_t c = S.at(i);
    while (is_blank(c)) { i = i + 1; c = S.at(i); }
    if (is_nl(c)) return false;
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
    return true;
}

// parse_line restricted to the needed columns, into registers (unrolled over
// the need slots).  Returns true when the record is too short for a needed column.
template <int N>
__device__ __forceinline__ bool parse_record_regs(const Src& S, const ScanPlan& P, CellsT<N>& cs) {
    const uint32_t delim = P.delim, quote = P.quote;
    uint32_t i = 0, fs = 0, flen = 0;
    int col = 0;
    bool ended = false;
#pragma unroll
    for (int k = 0; k < N; k++) {
        if (k >= P.nneed) break;
        const int want = P.need_col[k];
        Cell c = cell_null();
        while (!ended && col < want) {
            if (!g_field(S, i, delim, quote, fs, flen) || S.at(i) != delim) ended = true;
            else { i = i + 1; col++; }
        }
        if (!ended) {
            if (!g_field(S, i, delim, quote, fs, flen)) {
                ended = true;
            } else {
                c = parse_cell_slow(S.ptr(fs, flen), flen);
                if (S.at(i) == delim) { i = i + 1; col++; }
                else ended = true;                  // later columns do not exist
            }
        }
        cs.c[k] = c;
    }
    return ended;
}

// parse_line restricted to an ascending column list, from HBM into a global
// array (representative-row gather, projection); out[k * stride] = column cols[k]
__device__ void parse_cols_out(const uint8_t* rec, const int16_t* cols, int ncols, uint32_t delim,
                               uint32_t quote, Cell* out, uint64_t stride) {
    const Src S{rec, rec, 0, false};
    uint32_t i = 0, fs = 0, flen = 0;
    int col = 0;
    bool ended = false;
    for (int k = 0; k < ncols; k++) {
        const int want = cols[k];
        Cell c = cell_null();
        while (!ended && col < want) {
            if (!g_field(S, i, delim, quote, fs, flen) || S.at(i) != delim) ended = true;
            else { i = i + 1; col++; }
        }
        if (!ended && col == want) {
            if (!g_field(S, i, delim, quote, fs, flen)) {
                ended = true;
            } else {
                c = parse_cell(rec + fs, flen);
                if (S.at(i) == delim) { i = i + 1; col++; }
                else ended = true;
            }
        }
        out[k * stride] = c;
    }
}

// the same from a staged copy: the record's first `lim` bytes in `tile` (LDS), the
// rest (and every cell's bytes) in HBM at `rec`
__device__ void parse_cols_out_staged(const uint8_t* tile, uint32_t lim, const uint8_t* rec, const int16_t* cols,
                                      int ncols, uint32_t delim, uint32_t quote, Cell* out) {
    const Src S{tile, rec, lim, false};
    uint32_t i = 0, fs = 0, flen = 0;
    int col = 0;
    bool ended = false;
    for (int k = 0; k < ncols; k++) {
        const int want = cols[k];
        Cell c = cell_null();
        while (!ended && col < want) {
            if (!g_field(S, i, delim, quote, fs, flen) || S.at(i) != delim) ended = true;
            else { i = i + 1; col++; }
        }
        if (!ended && col == want) {
            if (!g_field(S, i, delim, quote, fs, flen)) {
                ended = true;
            } else {
                // typed from the staged copy when the field and the byte after it are
                // staged (the number scans stop there); a STRING keeps its HBM address
                const bool st = fs + flen < lim;
                c = parse_cell(st ? tile + fs : rec + fs, flen);
                if (st && c.kind == K_STR) c.bits = c.bits - (uint64_t)(uintptr_t)tile + (uint64_t)(uintptr_t)rec;
                if (S.at(i) == delim) { i = i + 1; col++; }
                else ended = true;
            }
        }
        out[k] = c;
    }
}

__device__ void parse_record_out(const uint8_t* rec, const ScanPlan& P, Cell* out) {
    parse_cols_out(rec, P.need_col, P.nneed, P.delim, P.quote, out, 1);
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


// evaluate_condition (evaluator_conditions.c:62-164) over the flattened WHERE tree;
// kc: the literal cells (LDS copy, string bytes staged in LDS)
template <class CS>
__device__ __forceinline__ bool eval_where_vm(const ScanPlan& P, const Cell* kc, const CS& cs) {
    Stack st;
#pragma unroll
    for (int j = 0; j < 8; j++) st.s[j] = cell_null();
    int sp = 0;
    uint32_t bs = 0;   // bool stack, top = bit 0
    for (int pc = 0; pc < P.nprog; pc++) {
        const Insn in = P.prog[pc];
        switch (in.op) {
            case OP_COL: st.set(sp++, get_cell(cs, in.a)); break;
            case OP_CONST: st.set(sp++, kc[in.b]); break;
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

// Out-of-line entry points for the rare paths, so the hot loop stays small in
// the instruction cache.  Cells travel by value (a by-reference argument would
// force the caller's register-resident cells into scratch memory).
// (ext_better, class_bit and g_ext_update: scanlib.h, shared with fast_kernel)

// Publish candidate `idx` (already written to gt.cand[a][idx]) as the group's
// extreme if it is better than the current one: a lock-free pointer swing.  Most
// candidates lose the first comparison and never write, so even a group every
// block touches sees few atomics; no lane ever waits on another.
__device__ void g_ext_swing(const GroupTable& gt, int a, uint8_t kind, uint32_t gi, uint64_t idx) {
    unsigned long long* slot = &gt.extref[a][gi];
    const ExtCand mine = gt.cand[a][idx];
    unsigned long long cur = __hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        if (cur != NOPOS) {
            const ExtCand o = gt.cand[a][cur];
            if (!ext_better(kind, mine.c, mine.pos, o.c, o.pos)) return;
        }
        const unsigned long long prev = atomicCAS(slot, cur, (unsigned long long)idx);
        if (prev == cur) return;
        cur = prev;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
}

// ------------------------------------------------------------------ LDS table
// Structure of arrays carved from dynamic LDS; capacity H (power of two) is
// chosen by the host so that the tile, the indexes and every accumulator fit.
struct LdsTable {
    uint32_t H;
    uint32_t* hdr;      // 0 empty, 1 being written, else 0x80000000 | hash tag << 19 | key class/length
    v4u* key;           // key words w0, w1
    uint32_t* cnt;      // COUNT(*) of the block's records in the group
    uint32_t* first;    // min over them of (window iteration << 15 | tile position)
};
struct LdsAcc {         // ACC_SUM
    double* sum;        // sum of numeric cells
    uint32_t* miss;     // cells that were not numeric (numeric count = cnt - miss)
};
struct ExtLds {         // ACC_MIN / ACC_MAX
    Cell* c;
    uint32_t* pos;      // the extreme's row as LdsTable.first codes it (~0u: none)
    uint32_t* lock;
};


// find or insert the slot of key k (hash h) for the lanes with `need`; -1 if the
// probe window is full (the HBM table takes the record).  Wave-uniform (the rule
// above): a slot another lane has claimed but not yet published is retried on
// the next trip instead of spun on, so a lane never waits on a lane of its own
// wave -- a per-lane spin here could run its full bound whenever the compiler
// schedules the waiting lanes before the claiming one.  A claimer publishes in
// the trip it claims, so every pending lane advances within a few trips; the
// trip bound only turns a kernel bug into spilled records, never into a hang.
__device__ __forceinline__ int l_insert(bool need, const LdsTable& t, const GKey& k, uint64_t h) {
    const uint32_t hd = lds_hdr(k, h);
    const v4u kk = key_words(k);
    // H need not be a power of two (the host fits as many slots as LDS holds): the
    // window starts at the hash's low 24 bits (gk_hash's best mixed) scaled into [0, H)
    uint32_t i = __umulhi((uint32_t)h << 8, t.H);
    uint32_t probe = 0;
    int s = -1;
    for (uint32_t trip = 0; __any(need); trip++) {
        if (need) {
            uint32_t cur = __hip_atomic_load(&t.hdr[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (cur == 0) {
                const uint32_t old = atomicCAS(&t.hdr[i], 0u, 1u);
                if (old == 0) {
                    t.key[i] = kk;
                    __hip_atomic_store(&t.hdr[i], hd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    s = (int)i;
                    need = false;
                }
                cur = old;
            }
            if (need && cur != 1) {                     // a published key: compare
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (cur == hd && key_match(k, kk, t.key[i])) {
                    s = (int)i;
                    need = false;
                } else if (++probe >= 32) {
                    need = false;                       // window full: s stays -1
                } else {
                    i = i + 1 == t.H ? 0u : i + 1;
                }
            }
        }
        if (trip > (1u << 20)) break;                   // never hang: pending lanes spill
    }
    return s;
}

// wave-uniform LDS MIN/MAX update (see g_ext_update).  The slot's lock word is a
// sequence number: even = free, odd = held, +2 per update.  A candidate first
// compares against a consistent snapshot (the same even number read before and
// after the cell) and drops out without the lock when it cannot win -- the extreme
// only ever improves, so most candidates lose against any snapshot, and only the
// few that improve it serialise.  The fences order LDS only: a workgroup fence
// over every address space would also wait for the window prefetch in flight.
__device__ __forceinline__ uint64_t lds_pos(uint32_t code) { return code == 0xFFFFFFFFu ? NOPOS : code; }
__device__ __forceinline__ void lds_ext_update(bool need, const ExtLds& e, uint32_t s, uint8_t kind,
                                               const Cell c, uint32_t pos, ScanStats* st) {
#ifdef CQ_AB_EXT_SKIP   // A/B build: no MIN/MAX update at all (results wrong)
    return;
#endif
    uint32_t* lk = &e.lock[s];
#ifndef CQ_AB_EXT_NOSNAP
    if (need) {
        const uint32_t v1 = __hip_atomic_load(lk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        const Cell cur = e.c[s];
        const uint64_t cp = lds_pos(e.pos[s]);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup", "local");
        const uint32_t v2 = __hip_atomic_load(lk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (!(v1 & 1u) && v1 == v2 && !ext_better(kind, c, pos, cur, cp)) need = false;
    }
#endif
    // a lane holds the lock only inside the trip that took it, so a trip never
    // waits on a holder that cannot run; the bound turns a lock word left odd (a
    // kernel bug) into a reported error (overflow 2: the query fails loudly)
    // instead of a hang
    for (uint32_t trips = 0; __any(need); trips++) {
        if (need) {
            const uint32_t v = __hip_atomic_load(lk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (!(v & 1u) && atomicCAS(lk, v, v + 1u) == v) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                if (ext_better(kind, c, pos, e.c[s], lds_pos(e.pos[s]))) {
                    e.c[s] = c;
                    e.pos[s] = pos;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                __hip_atomic_store(lk, v + 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                need = false;
            }
        }
        if (trips > (1u << 20)) {
            if (need) atomicExch(&st->overflow, 2ULL);
            break;
        }
    }
}


// ------------------------------------------------------------------ the scan kernel
__device__ __forceinline__ uint8_t* carve(uint8_t*& q, size_t bytes) {
    uint8_t* r = q;
    q += (bytes + 15) & ~(size_t)15;
    return r;
}

// the tile of the window starting at ws: bytes [ws - PREB, ws - PREB + TILE)
__device__ __forceinline__ void prefetch(const uint8_t* g, uint64_t ws, v4u* pf) {
    const v4u* src = (const v4u*)(g + ws - PREB);
#pragma unroll
    for (int j = 0; j < PF; j++) {   // lane t: the 32 bytes it classifies, [32t, 32t + 32)
#ifdef CQ_PLAIN_LOADS
        pf[j] = src[PF * threadIdx.x + j];
#else
        pf[j] = __builtin_nontemporal_load(src + PF * threadIdx.x + j);
#endif
    }
}

// classify LB = 32 staged bytes: terminator and separator masks, quote presence
__device__ __forceinline__ void classify32(const v4u a, const v4u b, uint32_t rep_d, uint32_t rep_q, uint32_t& nlm,
                                           uint32_t& sepm, bool& has_q) {
    uint32_t nl = 0, sp = 0, qacc = 0x80808080u;
#pragma unroll
    for (int v = 0; v < 2; v++) {
        const v4u x4 = v ? b : a;
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
            const int sh = (v * 4 + j) * 4;
            sp |= (t & 0xFu) << sh;
            nl |= ((t >> 4) & 0xFu) << sh;
        }
    }
    nlm = nl;
    sepm = sp;
    has_q = qacc != 0x80808080u;
}

// bits of m below bit b


// Profiling builds (-DCQ_CLOCKS): per-phase shader cycles, summed over waves
#ifdef CQ_CLOCKS
#define CLK_DECL uint64_t clk_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; uint64_t clk_t = clock64();
#define CLK(i) { const uint64_t n_ = clock64(); clk_acc[i] += n_ - clk_t; clk_t = n_; }
#define CLK_FLUSH(st) if ((threadIdx.x & 63) == 0) { for (int i_ = 0; i_ < 8; i_++) atomicAdd(&(st)->clk[i_], clk_acc[i_]); }
#else
#define CLK_DECL
#define CLK(i)
#define CLK_FLUSH(st)
#endif


// Fast scan kernel, specialised on the plan's shape: GROUPED (GROUP BY key or
// one group), KN need slots and KA accumulators at most, the WHERE shape WM and
// whether any MIN/MAX accumulator exists (EXT).  It has no general-parser code:
// a record the fast field path cannot type exactly is appended to `slow_list`
// and handled completely (filter, rows, aggregation) by slow_kernel.
template <bool GROUPED, int KN, int KA, int WM, bool EXT>
__global__ __launch_bounds__(SCAN_T) void scan_kernel(const uint8_t* __restrict__ g,
                                                      ScanStats* __restrict__ stats,
                                                      unsigned long long* __restrict__ row_out,
                                                      unsigned long long row_cap, uint32_t lds_h,
                                                      Cell* __restrict__ cells_out,
                                                      unsigned long long* __restrict__ slow_list,
                                                      unsigned long long slow_cap) {
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t* q = smem;
    uint8_t* tile = carve(q, TILE + TILE_PAD);
    uint16_t* E = (uint16_t*)carve(q, ECAP * 2);         // tile positions of separators
    uint16_t* NLI = (uint16_t*)carve(q, NLCAP * 2);      // separator index of each terminator
    uint16_t* QP = (uint16_t*)carve(q, (NW + 1) * 2);    // quote words before each mask word
    uint64_t* rs = (uint64_t*)carve(q, RSMAX * 8);       // record: tile position | first separator << 16
                                                         //         | terminators before it << 32
    uint32_t* wsum = (uint32_t*)carve(q, 32 * 4);
    Cell* kc = (Cell*)carve(q, MAX_CONST * sizeof(Cell)); // literal cells, strings staged in LDS
    uint8_t* kstr = carve(q, KSTR);
    LdsTable lt;
    LdsAcc la[KA];
    ExtLds le[KA];
    const uint32_t H = lds_h;
    lt.H = H;
    lt.hdr = nullptr; lt.key = nullptr; lt.cnt = nullptr; lt.first = nullptr;
    if (GROUPED) {
        lt.key = (v4u*)carve(q, H * 16);
        lt.hdr = (uint32_t*)carve(q, H * 4);
        lt.cnt = (uint32_t*)carve(q, H * 4);
        lt.first = (uint32_t*)carve(q, H * 4);
    }
#pragma unroll
    for (int a = 0; a < KA; a++) {
        la[a].sum = nullptr; la[a].miss = nullptr;
        le[a].c = nullptr; le[a].pos = nullptr; le[a].lock = nullptr;
        if (!GROUPED || a >= P.nacc) continue;
        if (P.acc[a].kind == ACC_SUM) {
            la[a].sum = (double*)carve(q, H * 8);
            la[a].miss = (uint32_t*)carve(q, H * 4);
        } else {
            le[a].c = (Cell*)carve(q, H * sizeof(Cell));
            le[a].pos = (uint32_t*)carve(q, H * 4);
            le[a].lock = (uint32_t*)carve(q, H * 4);
        }
    }
    const int tid = threadIdx.x;

    if (GROUPED) {
        for (uint32_t i = tid; i < H; i += SCAN_T) {
            lt.hdr[i] = 0; lt.cnt[i] = 0; lt.first[i] = 0xFFFFFFFFu;
#pragma unroll
            for (int a = 0; a < KA; a++) {
                if (a >= P.nacc) break;
                if (la[a].sum) { la[a].sum[i] = 0.0; la[a].miss[i] = 0; }
                if (EXT && le[a].c) { le[a].pos[i] = 0xFFFFFFFFu; le[a].lock[i] = 0; le[a].c[i] = cell_null(); }
            }
        }
    }
    if (tid == 0) {                                      // literals: string bytes into LDS
        uint32_t used = 0;
        for (int i = 0; i < P.nconst; i++) {
            Cell c = P.consts[i];
            if (c.kind == K_STR && c.len <= KSTR - used) {
                const uint8_t* s = str_ptr(c);
                for (uint32_t j = 0; j < c.len; j++) kstr[used + j] = s[j];
                c.bits = (uint64_t)(uintptr_t)(kstr + used);
                used += c.len;
            }
            kc[i] = c;
        }
    }
    __syncthreads();

    // per-thread partials (single-group mode) and statistics
    unsigned long long my_cnt = 0, my_first = NOPOS, my_records = 0, my_short = 0, my_spill = 0, my_pass = 0;
    double my_sum[KA];
    unsigned long long my_num[KA];
    Cell my_ext[KA];
    unsigned long long my_pos[KA];
    uint32_t my_cls[KA];
#pragma unroll
    for (int a = 0; a < KA; a++) {
        my_sum[a] = 0.0; my_num[a] = 0; my_ext[a] = cell_null(); my_pos[a] = NOPOS; my_cls[a] = 0;
    }

    // uniform plan facts
    const int nneed = P.nneed;
    const int nacc = P.nacc;
    const int gslot = GROUPED ? P.group_slot : -1;
    const int wslot = WM == W_SIMPLE ? P.prog[0].a : -1;
    const uint32_t wop = WM == W_SIMPLE ? P.prog[2].a : 0;
    const Cell wconst = WM == W_SIMPLE ? kc[P.prog[1].b] : cell_null();
    const GKey null_key = group_key(cell_null());
    const int clast = nneed > 0 ? P.need_col[nneed - 1] : 0;

    const uint64_t lo_ok = P.data_begin > P.range_begin ? P.data_begin : P.range_begin;
    const uint64_t hi_ok = P.range_end < P.n ? P.range_end : P.n;
    const uint64_t first_win = P.range_begin / WSTRIDE;
    const uint64_t last_win = (hi_ok + WSTRIDE - 1) / WSTRIDE;
    const uint32_t delim = P.delim, quote = P.quote;
    const uint32_t rep_d = delim * 0x01010101u, rep_q = quote * 0x01010101u;
    // strtoll/strtod read past the field end: a delimiter they could consume
    // (digit, '.', letter) sends numerals to the general cell parser
    const bool num_ok = !(is_digit(delim) || delim == '.' || ((delim | 32) >= 'a' && (delim | 32) <= 'z'));
    const uint64_t tile_g = (uint64_t)(uintptr_t)tile;

    v4u pf[PF];
    uint64_t w = first_win + blockIdx.x;
    if (w < last_win) prefetch(g, w * WSTRIDE, pf);
    CLK_DECL

    for (uint32_t iter = 0; w < last_win; w += gridDim.x, iter++) {
        const uint64_t ws = w * WSTRIDE;
        const uint64_t gt0 = (uint64_t)(uintptr_t)(g + ws - PREB);   // HBM address of tile byte 0
        // (no barrier here: the previous window's last reads of the tile and its
        //  indexes are behind its end-of-chunk barrier or its scan barrier)
        CLK(0)
#pragma unroll
        for (int j = 0; j < PF; j++) ((v4u*)tile)[PF * tid + j] = pf[j];
        const v4u own0 = pf[0], own1 = pf[1];            // this lane's 32 bytes, still in registers
        lds_barrier();
#ifdef CQ_NO_MEM   // profiling build: re-read the block's first tile (L2-resident), results wrong
        if (w + gridDim.x < last_win) prefetch(g, (first_win + blockIdx.x) * WSTRIDE, pf);
#else
        if (w + gridDim.x < last_win) prefetch(g, (w + gridDim.x) * WSTRIDE, pf);   // in flight meanwhile
#endif
        CLK(1)

#if defined(CQ_PROF_STAGE) && CQ_PROF_STAGE == 0   // profiling build: staging only
        if (tid == 0) my_records += ((const uint32_t*)tile)[w & 1023];
        continue;
#endif
        // ---- classify this lane's LB bytes
        uint32_t nlm, sepm;
        bool hq;
        classify32(own0, own1, rep_d, rep_q, nlm, sepm, hq);
        // ---- record starts owned by this window: [ws, ws + WSTRIDE) within [lo_ok, hi_ok)
        uint32_t starts = 0;
        if (tid > 0) {
            const uint32_t prev_nl = is_nl(tile[tid * LB - 1]) ? 1u : 0u;
            starts = ~nlm & ((nlm << 1) | prev_nl);
            const uint64_t base = ws - PREB + (uint64_t)tid * LB;       // file offset of bit 0
            const uint64_t lo = lo_ok > ws ? lo_ok : ws;
            const uint64_t hi = hi_ok < ws + WSTRIDE ? hi_ok : ws + WSTRIDE;
            if (base + LB <= lo || base >= hi) {
                starts = 0;
            } else {
                if (base < lo) starts &= ~0u << (lo - base);
                if (base + LB > hi) starts &= (1u << (hi - base)) - 1;
            }
        }
        CLK(2)
        // ---- number separators, terminators, records and quote words
        const uint32_t nsep = (uint32_t)__popc(sepm), nnl = (uint32_t)__popc(nlm);
        const uint32_t nrs = (uint32_t)__popc(starts);
        uint32_t e_sn, e_rq, t_sn, t_rq;
        block_excl_scan2(nsep | (nnl << 16), nrs | ((hq ? 1u : 0u) << 16), wsum, e_sn, e_rq, t_sn, t_rq);
        const uint32_t sep_base = e_sn & 0xFFFF, nl_base = e_sn >> 16, rec_base = e_rq & 0xFFFF;
        const uint32_t nsep_tot = min(t_sn & 0xFFFF, (uint32_t)ECAP), nnl_tot = min(t_sn >> 16, (uint32_t)NLCAP);
        const uint32_t total = t_rq & 0xFFFF;
        QP[tid] = (uint16_t)(e_rq >> 16);
        if (tid == SCAN_T - 1) QP[NW] = (uint16_t)(t_rq >> 16);
#ifndef CQ_NO_INDEX
        {
            uint32_t m = sepm;
            uint32_t j = sep_base;
            while (m) {
                const uint32_t b = (uint32_t)__builtin_ctzg(m, 32);
                m &= m - 1;
                if (j < ECAP) E[j] = (uint16_t)(tid * LB + b);
                j++;
            }
            m = nlm;
            j = nl_base;
            while (m) {
                const uint32_t b = (uint32_t)__builtin_ctzg(m, 32);
                m &= m - 1;
                if (j < NLCAP) NLI[j] = (uint16_t)(sep_base + popc_below(sepm, b));
                j++;
            }
        }
#endif
        CLK(3)
        for (uint32_t chunk = 0; chunk < total; chunk += RSMAX) {
            {
                uint32_t m = starts;
                uint32_t ri = rec_base;
                while (m) {
                    const uint32_t b = (uint32_t)__builtin_ctzg(m, 32);
                    m &= m - 1;
                    if (ri >= chunk && ri < chunk + RSMAX) {
                        rs[ri - chunk] = (uint64_t)((tid * LB + b) | ((sep_base + popc_below(sepm, b)) << 16)) |
                                         ((uint64_t)(nl_base + popc_below(nlm, b)) << 32);
                    }
                    ri++;
                }
            }
            lds_barrier();
#if defined(CQ_PROF_STAGE) && CQ_PROF_STAGE == 1   // profiling build: split + classify only
            const uint32_t nrec = 0;
            if (tid == 0) my_records += min((uint32_t)RSMAX, total - chunk);
#else
            const uint32_t nrec = min((uint32_t)RSMAX, total - chunk);
#endif
            for (uint32_t base0 = 0; base0 < nrec; base0 += SCAN_T) {
                // trip count is block-uniform: every lane of a wave runs every trip
                const uint32_t ri = base0 + tid;
                const bool valid = ri < nrec;
                const uint64_t ent = valid ? rs[ri] : 0;
                const uint32_t pos = (uint32_t)ent & 0xFFFF, j0 = ((uint32_t)ent) >> 16;
                const uint32_t qi = (uint32_t)(ent >> 32);
                const uint64_t rec = ws - PREB + pos;
                CellsT<KN> cs;
                Cell wc = cell_null();
                Cell av[KA];
                GKey key = null_key;
                // -- fields from the separator list: field c = (E[j0+c-1], E[j0+c])
                bool fail = !valid || qi >= nnl_tot;
                const uint32_t jn = fail ? 0u : NLI[qi];            // the record's terminator
                fail = fail || jn >= nsep_tot;
                uint32_t fend = pos;                                // end of the last field typed
#pragma unroll
                for (int k = 0; k < KN; k++) {
                    if (k >= nneed) break;
                    const uint32_t c = (uint32_t)P.need_col[k];
                    Cell cell = cell_null();
                    if (!fail && j0 + c <= jn) {                   // the record has column c
                        const uint32_t fs = c ? (uint32_t)E[j0 + c - 1] + 1 : pos;
                        const uint32_t fe = E[j0 + c];
                        uint64_t kw;
                        if (lean_field(tile, fs, fe - fs, num_ok, cell, kw)) {
                            if (k == gslot) {
                                if (cell.kind == K_STR) { key.cls = GK_STR; key.len = cell.len; key.w0 = kw; key.w1 = 0; }
                                else key = group_key(cell);
                            }
                        } else {
                            fail = fast_field(tile, fs, fe - fs, num_ok, k == gslot, cell, key) != FF_OK;
                        }
                        if (cell.kind == K_STR) cell.bits = tile_g + fs;
                        fend = fe;
                    }
                    cs.c[k] = cell;
                    if (WM == W_SIMPLE && k == wslot) wc = cell;
#pragma unroll
                    for (int a = 0; a < KA; a++)
                        if (a < nacc && P.acc[a].slot == k) av[a] = cell;
                }
                // a quote before the end of the last typed field may hide separators
                fail = fail || QP[fend / LB + 1] != QP[pos / LB];
                CLK(4)
                // -- records the fast path declines go to slow_kernel, whole
                const bool slow = valid && fail;
                const uint64_t sb = __ballot(slow);
                if (sb) {
                    unsigned long long base = 0;
                    if ((tid & 63) == 0) base = atomicAdd(&stats->slow_records, (unsigned long long)__popcll(sb));
                    base = __shfl(base, 0, 64);
                    if (slow) {
                        const unsigned long long i = base + __popcll(sb & ((1ULL << (tid & 63)) - 1));
                        if (i < slow_cap) slow_list[i] = rec;
                    }
                }
                bool pass = false;
                if (valid && !fail) {
                    if (key.cls == GK_LONG) key.w0 = key.w0 - tile_g + gt0;
                    my_records++;
                    if (j0 + (uint32_t)clast > jn) my_short++;
                    if (WM == W_NONE) pass = true;
                    else if (WM == W_SIMPLE) pass = cmp_result(wop, compare(wc, wconst));
                    else pass = P.nprog == 0 || eval_where_vm(P, kc, cs);
                    if (pass) my_pass++;
                }
                if (row_out) {
                    const unsigned long long slot = wave_slot(pass, &stats->rows_emitted);
                    if (pass && slot < row_cap) {
                        row_out[slot] = rec;
                        if (cells_out) {   // debug: the cells this kernel parsed
#pragma unroll
                            for (int k = 0; k < KN; k++) {
                                if (k >= nneed) break;
                                Cell c = cs.c[k];
                                if (c.kind == K_STR) c.bits = c.bits - tile_g + gt0;
                                cells_out[slot * nneed + k] = c;
                            }
                        }
                    }
                }
                if (EXT && pass) {
#pragma unroll
                    for (int a = 0; a < KA; a++)
                        if (a < nacc && P.acc[a].kind != ACC_SUM) my_cls[a] |= class_bit(av[a]);
                }
                if (!GROUPED) {
                    if (pass) {
                        my_cnt++;
                        if (rec < my_first) my_first = rec;
#pragma unroll
                        for (int a = 0; a < KA; a++) {
                            if (a >= nacc) break;
                            Cell c = av[a];
                            if (P.acc[a].kind == ACC_SUM) {
                                if (is_num(c)) { my_sum[a] += num_of(c); my_num[a]++; }
                            } else if (EXT && c.kind != K_NULL && ext_better(P.acc[a].kind, c, rec, my_ext[a], my_pos[a])) {
                                if (c.kind == K_STR) c.bits = c.bits - tile_g + gt0;
                                my_ext[a] = c;
                                my_pos[a] = rec;
                            }
                        }
                    }
                } else {
                    const uint64_t h = pass ? gk_hash(key) : 0;
#ifdef CQ_NO_INSERT   // profiling build: direct-mapped slot, results wrong
                    const int s = pass ? (int)__umulhi((uint32_t)h << 8, H) : -1;
#else
                    const int s = l_insert(pass, lt, key, h);    // the whole wave (uniform loop)
#endif
                    const bool in_lds = pass && s >= 0;
                    const bool spill = pass && s < 0;
                    if (in_lds) {
                        atomicAdd(&lt.cnt[s], 1u);
                        atomicMin(&lt.first[s], (iter << 15) | pos);
#pragma unroll
                        for (int a = 0; a < KA; a++) {
                            if (a >= nacc) break;
                            if (!la[a].sum) continue;
                            const Cell c = av[a];
                            if (is_num(c)) atomicAdd(&la[a].sum[s], num_of(c));
                            else atomicAdd(&la[a].miss[s], 1u);
                        }
                    }
                    if (EXT) {
#pragma unroll
                        for (int a = 0; a < KA; a++) {
                            if (a >= nacc) break;
                            if (!le[a].c) continue;              // uniform
                            Cell c = av[a];
                            if (c.kind == K_STR) c.bits = c.bits - tile_g + gt0;
                            lds_ext_update(in_lds && c.kind != K_NULL, le[a], in_lds ? (uint32_t)s : 0u,
                                           P.acc[a].kind, c, (iter << 15) | pos, stats);
                        }
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
                                for (int a = 0; a < KA; a++) {
                                    if (a >= nacc) break;
                                    const Cell c = av[a];
                                    if (P.acc[a].kind == ACC_SUM && is_num(c)) {
                                        atomicAdd(&gt.sum[a][gi], num_of(c));
                                        atomicAdd(&gt.num[a][gi], 1ULL);
                                    }
                                }
                            }
                        }
                        if (EXT) {
#pragma unroll
                            for (int a = 0; a < KA; a++) {
                                if (a >= nacc) break;
                                if (P.acc[a].kind == ACC_SUM) continue;   // uniform
                                Cell c = av[a];
                                if (c.kind == K_STR) c.bits = c.bits - tile_g + gt0;
                                g_ext_update(spill && gi >= 0 && c.kind != K_NULL, gt, a, P.acc[a].kind,
                                             gi >= 0 ? (uint32_t)gi : 0u, c, rec, stats);
                            }
                        }
                    }
                }
                CLK(5)
            }
            lds_barrier();
            CLK(6)
        }
    }
    __syncthreads();
    CLK_FLUSH(stats)

    // ---- statistics and value-class masks
    {
        unsigned long long r = my_records, s = my_short, sp = my_spill, ps = my_pass;
        for (int o = 32; o > 0; o >>= 1) {
            r += __shfl_down(r, o, 64);
            s += __shfl_down(s, o, 64);
            sp += __shfl_down(sp, o, 64);
            ps += __shfl_down(ps, o, 64);
        }
        if ((tid & 63) == 0) {
            if (r) atomicAdd(&stats->records, r);
            if (s) atomicAdd(&stats->short_rows, s);
            if (sp) atomicAdd(&stats->lds_spills, sp);
            if (ps) atomicAdd(&stats->passed, ps);
        }
    }
    if (EXT) {
#pragma unroll
        for (int a = 0; a < KA; a++) {
            if (a >= nacc) break;
            uint32_t m = my_cls[a];
            for (int o = 32; o > 0; o >>= 1) m |= __shfl_down(m, o, 64);
            if ((tid & 63) == 0 && m) atomicOr(&stats->acc_classes[a], m);
        }
    }

    if (!GROUPED) {
        // ---- wave-reduce the single group, then one global update per wave
        unsigned long long c = my_cnt, f = my_first;
        for (int o = 32; o > 0; o >>= 1) {
            c += __shfl_down(c, o, 64);
            const unsigned long long ff = __shfl_down(f, o, 64);
            f = ff < f ? ff : f;
        }
        double sm[KA];
        unsigned long long nm[KA];
#pragma unroll
        for (int a = 0; a < KA; a++) {
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
                for (int a = 0; a < KA; a++)
                    if (a < nacc && P.acc[a].kind == ACC_SUM && nm[a]) {
                        atomicAdd(&gt.sum[a][gi], sm[a]);
                        atomicAdd(&gt.num[a][gi], nm[a]);
                    }
            }
        }
        gi = __shfl(gi, 0, 64);
        if (EXT) {
#pragma unroll
            for (int a = 0; a < KA; a++) {
                if (a >= nacc) break;
                if (P.acc[a].kind == ACC_SUM) continue;
                // wave-reduce the extreme first: one published candidate per wave
                Cell e = my_ext[a];
                unsigned long long ep = my_pos[a];
                for (int o = 32; o > 0; o >>= 1) {
                    Cell x;
                    x.kind = __shfl_down(e.kind, o, 64);
                    x.len = __shfl_down(e.len, o, 64);
                    x.bits = __shfl_down(e.bits, o, 64);
                    const unsigned long long xp = __shfl_down(ep, o, 64);
                    if (xp != NOPOS && ext_better(P.acc[a].kind, x, xp, e, ep)) { e = x; ep = xp; }
                }
                if ((tid & 63) == 0 && gi >= 0 && ep != NOPOS) {
                    const uint64_t idx = (uint64_t)blockIdx.x * gt.cand_stride + (tid >> 6);
                    ExtCand ec;
                    ec.c = e; ec.pos = ep; ec.pad = 0;
                    gt.cand[a][idx] = ec;
                    __threadfence();
                    g_ext_swing(gt, a, P.acc[a].kind, (uint32_t)gi, idx);
                }
            }
        }
        return;
    }

    // ---- flush the LDS table into the global table
    for (uint32_t b0 = 0; b0 < H; b0 += SCAN_T) {
        const uint32_t i = b0 + tid;
        const bool act = i < H && lt.hdr[i] >= 2;
        int gi = -1;
        if (act) {
            const uint32_t hd = lt.hdr[i];
            const v4u kw = lt.key[i];
            GKey k;
            k.cls = (hd >> 16) & 7;
            k.len = hd & 0xFFFF;
            k.w0 = (uint64_t)kw.x | ((uint64_t)kw.y << 32);
            k.w1 = (uint64_t)kw.z | ((uint64_t)kw.w << 32);
            gi = g_insert(gt, k, gk_hash(k), stats);
            if (gi >= 0) {
                const uint32_t n = lt.cnt[i];
                const uint32_t f = lt.first[i];
                const uint64_t fw = first_win + blockIdx.x + (uint64_t)(f >> 15) * gridDim.x;
                atomicAdd(&gt.cnt[gi], (unsigned long long)n);
                atomicMin(&gt.first[gi], (unsigned long long)(fw * WSTRIDE - PREB + (f & 0x7FFF)));
#pragma unroll
                for (int a = 0; a < KA; a++) {
                    if (a >= nacc) break;
                    if (!la[a].sum) continue;
                    const uint32_t num = n - la[a].miss[i];
                    if (num) {
                        atomicAdd(&gt.sum[a][gi], la[a].sum[i]);
                        atomicAdd(&gt.num[a][gi], (unsigned long long)num);
                    }
                }
            }
        }
        if (EXT && act && gi >= 0) {
#pragma unroll
            for (int a = 0; a < KA; a++) {
                if (a >= nacc) break;
                if (!le[a].c || le[a].pos[i] == 0xFFFFFFFFu) continue;
                const uint64_t idx = (uint64_t)blockIdx.x * gt.cand_stride + i;
                ExtCand ec;
                const uint32_t pc = le[a].pos[i];
                const uint64_t pw = first_win + blockIdx.x + (uint64_t)(pc >> 15) * gridDim.x;
                ec.c = le[a].c[i]; ec.pos = pw * WSTRIDE - PREB + (pc & 0x7FFF); ec.pad = 0;
                gt.cand[a][idx] = ec;
                __threadfence();
                g_ext_swing(gt, a, P.acc[a].kind, (uint32_t)gi, idx);
            }
        }
    }
}

// The records scan_kernel declined (quotes before a needed field, blanks or
// control bytes in one, date-shaped or long fields, records past the tile):
// general parse_line + parse_value from HBM, WHERE bytecode, aggregation straight
// into the HBM table.  Grid-stride with block-uniform trips (the MIN/MAX lock
// loops need whole waves).
template <bool GROUPED>
__global__ __launch_bounds__(256) void slow_kernel(const uint8_t* __restrict__ g, ScanStats* __restrict__ stats,
                                                   unsigned long long* __restrict__ row_out,
                                                   unsigned long long row_cap, Cell* __restrict__ cells_out,
                                                   const unsigned long long* __restrict__ slow_list,
                                                   unsigned long long slow_cap) {
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    const unsigned long long listed = __hip_atomic_load(&stats->slow_records, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long n = listed < slow_cap ? listed : slow_cap;
    const int nneed = P.nneed, nacc = P.nacc;
    unsigned long long my_records = 0, my_short = 0, my_pass = 0;
    for (unsigned long long b0 = (unsigned long long)blockIdx.x * blockDim.x; b0 < n;
         b0 += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long i = b0 + threadIdx.x;
        const bool valid = i < n;
        const uint64_t rec = valid ? slow_list[i] : 0;
        CellsT<MAX_NEED> cs;
#pragma unroll
        for (int k = 0; k < MAX_NEED; k++) cs.c[k] = cell_null();
        bool pass = false;
        if (valid) {
            const Src S{g + rec, g + rec, 0, false};
            const bool short_row = parse_record_regs(S, P, cs);
            my_records++;
            if (short_row) my_short++;
            pass = P.nprog == 0 || eval_where_vm(P, P.consts, cs);
            if (pass) my_pass++;
        }
        if (row_out) {
            const unsigned long long slot = wave_slot(pass, &stats->rows_emitted);
            if (pass && slot < row_cap) {
                row_out[slot] = rec;
                if (cells_out)
                    for (int k = 0; k < nneed; k++) cells_out[slot * nneed + k] = get_cell(cs, k, nneed);
            }
        }
        if (pass) {
            for (int a = 0; a < nacc; a++)
                if (P.acc[a].kind != ACC_SUM) {
                    const uint32_t m = class_bit(get_cell(cs, P.acc[a].slot, nneed));
                    if (m) atomicOr(&stats->acc_classes[a], m);
                }
        }
        GKey key;
        key.cls = GK_ALL; key.len = 0; key.w0 = 0; key.w1 = 0;
        uint64_t h = 0x12345678ULL;
        if (GROUPED && pass) {
            key = group_key(get_cell(cs, P.group_slot, nneed));
            h = gk_hash(key);
        }
        int gi = -1;
        if (pass) {
            gi = g_insert(gt, key, h, stats);
            if (gi >= 0) {
                atomicAdd(&gt.cnt[gi], 1ULL);
                atomicMin(&gt.first[gi], (unsigned long long)rec);
                for (int a = 0; a < nacc; a++) {
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
            if (a >= nacc) break;
            if (P.acc[a].kind == ACC_SUM) continue;      // uniform
            const Cell c = get_cell(cs, P.acc[a].slot, nneed);
            g_ext_update(pass && gi >= 0 && c.kind != K_NULL, gt, a, P.acc[a].kind, gi >= 0 ? (uint32_t)gi : 0u,
                         c, rec, stats);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        my_records += __shfl_down(my_records, o, 64);
        my_short += __shfl_down(my_short, o, 64);
        my_pass += __shfl_down(my_pass, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (my_records) atomicAdd(&stats->records, my_records);
        if (my_short) atomicAdd(&stats->short_rows, my_short);
        if (my_pass) atomicAdd(&stats->passed, my_pass);
    }
}

// ------------------------------------------------------------------ compaction
__global__ void compact_kernel(const GroupTable gt, int nacc, uint32_t kinds, GroupOut* out, unsigned int* count,
                               unsigned int cap_out, unsigned long long* ofirst) {
    uint8_t kind_of[MAX_ACC];
#pragma unroll
    for (int a = 0; a < MAX_ACC; a++) kind_of[a] = (uint8_t)((kinds >> (2 * a)) & 3);
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
        if (a < nacc && gt.extref[a] && gt.extref[a][i] != NOPOS) {   // the swung candidate
            const ExtCand o = gt.cand[a][gt.extref[a][i]];
            if (ext_better(kind_of[a], o.c, o.pos, r.ext[a], r.extpos[a])) { r.ext[a] = o.c; r.extpos[a] = o.pos; }
        }
    }
    out[o] = r;
    if (ofirst) ofirst[o] = r.first;                   // (finish_pack_kernel's dense order keys)
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

// ------------------------------------------------------------------ composite key texts
// One record's parsed need cells (gather_kernel's rows) as a cell view
struct RowView {
    const Cell* c;
};
__device__ __forceinline__ Cell get_cell(const RowView& v, int a, int = 0) { return v.c[a]; }
// joined-text sink with a byte cap (n keeps counting past it: the caller sees the overflow)
struct TextSink {
    uint8_t* p;
    uint32_t cap, n;
    __device__ void byte(uint8_t c) {
        if (n < cap) p[n] = c;
        n++;
    }
    __device__ void bytes(const uint8_t* q, uint32_t k) { for (uint32_t i = 0; i < k; i++) byte(q[i]); }
    __device__ void dec(uint64_t v, int mind) {
        uint8_t t[20];
        int k = 0;
        do { t[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
        while (k < mind) t[k++] = '0';
        while (k) byte(t[--k]);
    }
};


// slots: a composite / expression GROUP BY part, prog[b, e)
template <class CS>
__device__ Cell eval_expr_vm(const ScanPlan& P, const Cell* kc, const CS& cs, uint32_t b, uint32_t e) {
    Stack st;
#pragma unroll
    for (int j = 0; j < 8; j++) st.s[j] = cell_null();
    int sp = 0;
    for (uint32_t pc = b; pc < e; pc++) {
        const Insn in = P.prog[pc];
        switch (in.op) {
            case OP_COL: st.set(sp++, get_cell(cs, in.a)); break;
            case OP_CONST: st.set(sp++, kc[in.b]); break;
            case OP_ARITH: {
                Cell r = st.get(--sp), l = st.get(--sp);
                st.set(sp++, arith(in.a, l, r));
                break;
            }
            case OP_NEG: { Cell x = st.get(--sp); st.set(sp++, negate(x)); break; }
            default: st.set(sp++, cell_null()); break;
        }
    }
    return sp > 0 ? st.get(sp - 1) : cell_null();
}

// the group key of a record: the GROUP BY column's canonical key, one expression's
// (create_groups_by_expression), or the composite digest of several parts (cell.h
// CompKey); a part list with a tab inside a text part keys on its joined text
// (cell.h joined_text_key).  `tab`: such a list held a DOUBLE part the joined
// text cannot render (the plan is refused)
template <class CS>
__device__ Cell plan_group_part(const ScanPlan& P, const Cell* kc, const CS& cs, int nneed, int k) {
    const int s = P.gpart_slot[k];
    return s >= 0 ? get_cell(cs, s, nneed)
                  : (s == -1 ? eval_expr_vm(P, kc, cs, P.gcode_off[k], P.gcode_off[k + 1]) : cell_null());
}
template <class CS>
__device__ GKey plan_group_key(const ScanPlan& P, const Cell* kc, const CS& cs, int nneed, bool& tab) {
    if (P.ngpart == 0) return group_key(get_cell(cs, P.group_slot, nneed));
    CompKey ck;
    bool has_tab = false;
    for (int k = 0; k < MAX_GPART; k++) {
        if (k >= P.ngpart) break;
        const Cell c = plan_group_part(P, kc, cs, nneed, k);
        const GKey pk = group_key(c);
        if (P.ngpart == 1) return pk;
        has_tab = has_tab || text_has_tab(c);
        ck.add(pk);
    }
    if (has_tab) {                                      // rare: the joined text
        TextHash h;
        bool ok = true;
        for (int k = 0; k < MAX_GPART; k++) {
            if (k >= P.ngpart) break;
            ok = joined_text_add(h, plan_group_part(P, kc, cs, nneed, k), k == 0) && ok;
        }
        tab = tab || !ok;
        GKey k = joined_text_key(h, (uint32_t)P.ngpart);
        if (P.test_digest_bits) {                      // test knob: force collisions
            k.w0 &= (1ULL << P.test_digest_bits) - 1;
            k.w1 = 0;
        }
        return k;
    }
    GKey k = comp_key(ck, (uint32_t)P.ngpart);
    if (P.test_digest_bits) {                          // test knob: force digest collisions
        k.w0 &= (1ULL << P.test_digest_bits) - 1;
        k.w1 = 0;
    }
    return k;
}

// A composite GROUP BY group's key as create_groups builds it (evaluator.c:113-212):
// every part's key text (NULL, %lld, %.6f, %04d-%02d-%02d, the string) joined with
// '\t', rendered from the group's first record (its need cells, gather_kernel).
// Range partials carry this text instead of the 128-bit part digest, so the merges
// across ranks group composite keys byte for byte, as the reference does.
// lens[i] = ~0: longer than cap.
__global__ void comp_text_kernel(const Cell* __restrict__ cells, uint32_t n, uint32_t cap, uint8_t* __restrict__ out,
                                 uint32_t* __restrict__ lens) {
    const ScanPlan& P = c_plan;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const RowView v{cells + (uint64_t)i * P.nneed};
    TextSink sk{out + (size_t)i * cap, cap, 0};
    bool ok = true;
    for (int k = 0; k < MAX_GPART; k++) {
        if (k >= P.ngpart) break;
        ok = joined_text_add(sk, plan_group_part(P, P.consts, v, P.nneed, k), k == 0) && ok;
    }
    lens[i] = ok && sk.n <= cap ? sk.n : 0xFFFFFFFFu;
}

// ------------------------------------------------------------------ projection
// evaluate_expression (evaluator_expressions.c:23-263) for one SELECT item of a
// row-returning query (build_result, evaluator_utils.c:249-549): the program's
// OP_COL operand b indexes the parsed columns of this record (cells[b * cstride])
__device__ Cell eval_value(const Insn* code, uint32_t b, uint32_t e, const Cell* cells, uint64_t cstride,
                           const Cell* consts) {
    Stack st;
#pragma unroll
    for (int j = 0; j < 8; j++) st.s[j] = cell_null();
    int sp = 0;
    for (uint32_t pc = b; pc < e; pc++) {
        const Insn in = code[pc];
        switch (in.op) {
            case OP_COL: st.set(sp++, cells[(uint64_t)in.b * cstride]); break;
            case OP_CONST: st.set(sp++, consts[in.b]); break;
            case OP_ARITH: {
                Cell r = st.get(--sp), l = st.get(--sp);
                st.set(sp++, arith(in.a, l, r));
                break;
            }
            case OP_NEG: { Cell x = st.get(--sp); st.set(sp++, negate(x)); break; }
            default: st.set(sp++, cell_null()); break;
        }
    }
    return sp > 0 ? st.get(sp - 1) : cell_null();
}

// one thread per matching record: parse the referenced columns (column-major
// scratch), then evaluate every output program into out[row * nout + o]
__global__ __launch_bounds__(256) void project_kernel(const uint8_t* __restrict__ g,
                                                      const unsigned long long* __restrict__ recs, uint32_t nrec,
                                                      ProjDesc D, Cell* __restrict__ scratch,
                                                      Cell* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    Cell* mine = scratch + i;
    if (D.ncols) parse_cols_out(g + recs[i], D.cols, D.ncols, D.delim, D.quote, mine, nrec);
    Cell* o = out + (uint64_t)i * D.nout;
    for (int k = 0; k < D.nout; k++) {
        const uint32_t b = D.off[k], e = D.off[k + 1];
        const Insn first = D.code[b];
        Cell v;
        if (e == b + 1 && first.op == OP_COL) v = mine[(uint64_t)first.b * nrec];
        else if (e == b + 1 && first.op == OP_CONST) v = D.consts[first.b];
        else v = eval_value(D.code, b, e, mine, nrec, D.consts);
        o[k] = v;
    }
}

// string bytes of cells -> packed host-visible buffer
// After compaction, per group: the representative cells of its first row
// (build_aggregated_result's non-aggregate columns, evaluator_aggregates.c:679-689),
// its MIN/MAX cells and its long-key text, with the first `sb` bytes of every
// STRING inline -- so the host fetches a whole aggregate result in one copy.
constexpr int FINISH_T = 128;
__global__ __launch_bounds__(FINISH_T) void finish_kernel(const uint8_t* __restrict__ g, uint64_t n, const GroupOut* __restrict__ out,
                              const unsigned int* __restrict__ count, unsigned int cap_out, FinishDesc D,
                              Cell* __restrict__ cells, uint8_t* __restrict__ bytes) {
    const uint32_t ncell = (uint32_t)(D.ncols + D.nacc + 1);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ng = *count < cap_out ? *count : cap_out;
    // the column list through LDS (a pointer into the by-value descriptor would put
    // the whole descriptor in every lane's scratch)
    __shared__ int16_t scols[MAX_WIDE];
    for (int k = threadIdx.x; k < D.ncols; k += blockDim.x) scols[k] = D.cols[k];
    __syncthreads();
    if (i >= ng) return;
    Cell* cs = cells + (size_t)i * ncell;
    const unsigned long long first = out[i].first == NOPOS ? NOPOS : out[i].first >> D.first_shift;
    if (D.ncols) {
        if (first != NOPOS && first < n) {
            // the record's first 128 bytes staged in LDS by nine independent 16-byte
            // loads (the byte walk from HBM was one dependent load per byte; the
            // table's tail padding covers the over-read)
            __shared__ uint4 stage[FINISH_T][9];
            const uint8_t* rec = g + first;
            const uint4* src = (const uint4*)((uintptr_t)rec & ~(uintptr_t)15);
            uint4 v[9];
#pragma unroll
            for (int w = 0; w < 9; w++) v[w] = src[w];
#pragma unroll
            for (int w = 0; w < 9; w++) stage[threadIdx.x][w] = v[w];
            const uint8_t* tile = (const uint8_t*)stage[threadIdx.x] + ((uintptr_t)rec & 15);
            parse_cols_out_staged(tile, 128, rec, scols, D.ncols, D.delim, D.quote, cs);
        } else {
            for (int k = 0; k < D.ncols; k++) cs[k] = cell_null();
        }
    }
    for (int a = 0; a < D.nacc; a++) cs[D.ncols + a] = out[i].ext[a];
    Cell kc = cell_null();
    const uint32_t cl = out[i].clslen;
    if ((cl >> 16) == GK_LONG) { kc.kind = K_STR; kc.len = cl & 0xffff; kc.bits = out[i].w0; }
    cs[D.ncols + D.nacc] = kc;
    for (uint32_t k = 0; k < ncell; k++) {
        const Cell c = cs[k];
        if (c.kind != K_STR) continue;
        const uint8_t* src = (const uint8_t*)(uintptr_t)c.bits;
        uint8_t* dst = bytes + ((size_t)i * ncell + k) * D.sb;
        const uint32_t m = c.len < D.sb ? c.len : D.sb;
        for (uint32_t j = 0; j < m; j++) dst[j] = src[j];
    }
}

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

// ------------------------------------------------------------------ JOIN
// perform_join (evaluator_joins.c:63-181) as a hash join on the device: the
// right side's keys are built into a hash table (hash_build_kernel) with the
// rows of each key kept in row order, every left row probes it for its run, and
// the (l, r) pairs come out in the reference's nested-loop order (left rows
// ascending, then right rows).  value_compare (csv_reader.c:98-130) equality is
// what "matches" means: numbers compare as doubles, strings by strcmp, dates by
// (y, m, d), NULL = NULL, and keys of different non-NULL classes compare "equal".

// The columns of one side, parsed per record (parse_line + parse_value).  A block
// takes 256 consecutive records: their bytes (one contiguous span of the table,
// the records being in file order) are staged into LDS with coalesced 16-byte
// loads, and each thread then walks its record there; STRING cells are rebased to
// their HBM bytes.  A span too long for the buffer walks the record in HBM.
// 0x80 flags of a dword -> 4 bits (bit i = byte i)
__device__ __forceinline__ uint32_t flag_nib(uint32_t f) {
    uint32_t t = f >> 7;
    t |= t >> 7;
    t |= t >> 14;
    return t & 0xFu;
}
constexpr uint32_t CELLS_T = 256;
constexpr uint32_t CELLS_SPAN = 16384;
__global__ __launch_bounds__(CELLS_T) void cells_kernel(const uint8_t* __restrict__ g, uint64_t tn,
                                                        const unsigned long long* __restrict__ recs, uint32_t n,
                                                        ColsDesc D, Cell* __restrict__ out) {
    __shared__ __align__(16) uint8_t buf[CELLS_SPAN + 64];
    const uint32_t first = blockIdx.x * CELLS_T;
    const uint32_t last = first + CELLS_T < n ? first + CELLS_T : n;
    const uint64_t lo = recs[first] & ~15ull;
    const uint64_t hi = last < n ? recs[last] : tn + 16;    // the table has '\n' padding after byte tn
    const uint64_t span = hi - lo + 48;                     // + strtod look-ahead past the last field
    const bool staged = span <= CELLS_SPAN;
    if (staged) {
        const uint32_t nch = (uint32_t)((span + 15) / 16);
        const v4u* src = (const v4u*)(g + lo);
        for (uint32_t c = threadIdx.x; c < nch; c += CELLS_T) ((v4u*)buf)[c] = __builtin_nontemporal_load(src + c);
    }
    __syncthreads();
    const uint32_t i = first + threadIdx.x;
    if (i >= n) return;
    const uint64_t r = recs[i];
    Cell* o = out + (uint64_t)i * D.ncols;
    if (!staged || r < lo || r - lo >= span - 48) {      // (record lists out of file order stay correct)
        parse_cols_out(g + r, D.cols, D.ncols, D.delim, D.quote, o, 1);
        return;
    }
    const uint32_t off = (uint32_t)(r - lo);
    const Src S{buf + off, g + r, (uint32_t)span - off, true};
    // fast path (delimiter above ' ', so blank skipping never meets a delimiter):
    // the record's first 64 bytes from LDS as separator / terminator / quote masks,
    // fields found by clearing separator bits, each field typed from its exact bytes
    // -- short numerals and plain strings in registers, anything else by parse_cell.
    // A quote before the terminator, no terminator in the view, or a needed field
    // starting with a blank falls back to the byte walk below.
    if (D.delim > 0x20u) {
        const uint32_t* b32 = (const uint32_t*)buf;
        const uint32_t a = off >> 2, sh = off & 3;
        const uint32_t rep_d = D.delim * 0x01010101u, rep_q = D.quote * 0x01010101u;
        uint64_t sv = 0, nv = 0, qv = 0;
        uint32_t prev = b32[a];
#pragma unroll
        for (int jj = 0; jj < 16; jj++) {
            const uint32_t nx = b32[a + jj + 1];
            const uint32_t x = __builtin_amdgcn_alignbyte(nx, prev, sh);
            prev = nx;
            const uint32_t fn = (~nonzero_bytes(x ^ 0x0A0A0A0Au) | ~nonzero_bytes(x ^ 0x0D0D0D0Du)) & 0x80808080u;
            const uint32_t fd = ~nonzero_bytes(x ^ rep_d) & 0x80808080u;
            const uint32_t fq = ~nonzero_bytes(x ^ rep_q) & 0x80808080u;
            sv |= (uint64_t)flag_nib(fd | fn) << (4 * jj);
            nv |= (uint64_t)flag_nib(fn) << (4 * jj);
            qv |= (uint64_t)flag_nib(fq) << (4 * jj);
        }
        const uint32_t e = nv ? (uint32_t)__builtin_ctzll(nv) : 64u;
        bool ok = e < 64 && (qv & ((2ull << e) - 1)) == 0;
        if (ok) {
            uint64_t sm = sv;
            uint32_t start = 0;
            int col = 0;
            bool gone = false;
            for (int k = 0; k < D.ncols && ok; k++) {
                const int want = D.cols[k];
                while (!gone && col < want) {
                    const uint32_t b = (uint32_t)__builtin_ctzll(sm);       // sm holds the terminator bit e
                    if (b >= e) gone = true;
                    else { start = b + 1; sm &= sm - 1; col++; }
                }
                Cell c = cell_null();
                if (!gone) {
                    const uint32_t end = (uint32_t)__builtin_ctzll(sm), fl = end - start;
                    if (fl) {
                        uint32_t e0, e1, e2, e3;
                        load16(buf, off + start, e0, e1, e2, e3);
                        const uint32_t c0 = e0 & 0xFFu;
                        if (c0 <= 0x20u) { ok = false; break; }            // leading blank: the byte walk
                        bool done = false;
                        if (fl <= 16) {
                            const uint32_t m0 = len_mask(fl, 0), m1 = len_mask(fl, 1), m2 = len_mask(fl, 2),
                                           m3 = len_mask(fl, 3);
                            const uint32_t low = lt_bytes(e0 | ~m0, 0x21212121u) | lt_bytes(e1 | ~m1, 0x21212121u) |
                                                 lt_bytes(e2 | ~m2, 0x21212121u) | lt_bytes(e3 | ~m3, 0x21212121u);
                            if (!low) {
                                const uint32_t f0 = m0 & 0x80808080u, f1 = m1 & 0x80808080u, f2 = m2 & 0x80808080u,
                                               f3 = m3 & 0x80808080u;
                                const uint32_t g0 = digit_bytes(e0) & f0, g1 = digit_bytes(e1) & f1,
                                               g2 = digit_bytes(e2) & f2, g3 = digit_bytes(e3) & f3;
                                const uint32_t t0 = ~nonzero_bytes(e0 ^ 0x2E2E2E2Eu) & f0,
                                               t1 = ~nonzero_bytes(e1 ^ 0x2E2E2E2Eu) & f1,
                                               t2 = ~nonzero_bytes(e2 ^ 0x2E2E2E2Eu) & f2,
                                               t3 = ~nonzero_bytes(e3 ^ 0x2E2E2E2Eu) & f3;
                                const uint32_t ndot = __popc(t0) + __popc(t1) + __popc(t2) + __popc(t3);
                                const bool allnum = (g0 | t0) == f0 && (g1 | t1) == f1 && (g2 | t2) == f2 &&
                                                    (g3 | t3) == f3;
                                // digits with at most one dot, not 8-10 bytes (parse_date's lengths),
                                // at most 15 digits: INTEGER exactly, DOUBLE = RN(M / 10^k)
                                if (allnum && ndot <= 1 && fl - ndot >= 1 && fl - ndot <= 15 && (fl < 8 || fl > 10)) {
                                    const uint32_t w[4] = {e0, e1, e2, e3};
                                    unsigned long long M = 0;
                                    uint32_t kd = 0;
                                    bool seen = false;
#pragma unroll
                                    for (uint32_t bi = 0; bi < 16; bi++) {
                                        const uint32_t ch = (w[bi >> 2] >> (8 * (bi & 3))) & 0xFFu;
                                        if (bi < fl) {
                                            if (ch == '.') seen = true;
                                            else { M = M * 10 + (ch - '0'); kd += seen ? 1u : 0u; }
                                        }
                                    }
                                    c = ndot ? cell_dbl((double)M / pow10_exact(kd)) : cell_int((int64_t)M);
                                    done = true;
                                } else if (!is_digit(c0) && c0 != '+' && c0 != '-' && c0 != '.') {
                                    c.kind = K_STR;                             // a plain string (never a date)
                                    c.len = fl;
                                    c.bits = (uint64_t)(uintptr_t)(g + r + start);
                                    done = true;
                                }
                            }
                        }
                        if (!done) {
                            c = parse_cell(S.ptr(start, fl), fl);
                            if (c.kind == K_STR) {
                                const uint8_t* p = (const uint8_t*)(uintptr_t)c.bits;
                                if (p >= S.t && p < S.t + S.lim) c.bits = (uint64_t)(uintptr_t)(S.g + (p - S.t));
                            }
                        }
                    }
                }
                o[k] = c;
            }
            if (ok) return;
        }
    }
    uint32_t j = 0, fs = 0, flen = 0;
    int col = 0;
    bool ended = false;
    for (int k = 0; k < D.ncols; k++) {
        const int want = D.cols[k];
        Cell c = cell_null();
        while (!ended && col < want) {
            if (!g_field(S, j, D.delim, D.quote, fs, flen) || S.at(j) != D.delim) ended = true;
            else { j = j + 1; col++; }
        }
        if (!ended && col == want) {
            if (!g_field(S, j, D.delim, D.quote, fs, flen)) {
                ended = true;
            } else {
                c = parse_cell(S.ptr(fs, flen), flen);
                if (c.kind == K_STR) {                      // point at the HBM copy of the bytes
                    const uint8_t* p = (const uint8_t*)(uintptr_t)c.bits;
                    if (p >= S.t && p < S.t + S.lim) c.bits = (uint64_t)(uintptr_t)(S.g + (p - S.t));
                }
                if (S.at(j) == D.delim) { j = j + 1; col++; }
                else ended = true;
            }
        }
        o[k] = c;
    }
}

// value class of a key under value_compare: 0 NULL, 1 number, 2 string, 3 date.
// Keys of different non-NULL classes compare "equal" (csv_reader.c:128): a left
// key matches the equal keys of its own class plus EVERY non-NULL right key of
// another class; NULL matches only NULL.
__device__ __forceinline__ uint32_t key_class(const Cell& c) {
    return c.kind == K_NULL ? 0u : (c.kind == K_STR ? 2u : (c.kind == K_DATE ? 3u : 1u));
}
__device__ __forceinline__ uint64_t join_code(const Cell& c) {
    if (c.kind == K_NULL) return 0;
    if (c.kind == K_STR) return fnv_bytes(str_ptr(c), c.len);
    if (c.kind == K_DATE) return c.bits;
    double d = num_of(c);
    if (d == 0.0) d = 0.0;                                    // -0 == +0 under value_compare
    return dbl_bits(d);
}

// key code, class and row index of every row; rows per class
__global__ void join_code_kernel(const Cell* __restrict__ cells, uint32_t stride, uint32_t kcol, uint32_t n,
                                 unsigned long long* __restrict__ codes, uint32_t* __restrict__ cls,
                                 uint32_t* __restrict__ idx, unsigned int* __restrict__ per_class) {
    // per-class counts: per-lane counters over a grid-stride loop, one global atomic per
    // class per block (one per block of 256 rows put 2.4*10^5 atomics per class of a
    // 62.5 M-row side on four addresses: 2.8 ms of serialised atomics)
    uint32_t mine[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const Cell c = cells[(uint64_t)i * stride + kcol];
        codes[i] = join_code(c);
        const uint32_t k = key_class(c);
        cls[i] = k;
        if (idx) idx[i] = i;
#pragma unroll
        for (int j = 0; j < 4; j++) mine[j] += k == (uint32_t)j ? 1u : 0u;
    }
    if (!per_class) return;
    __shared__ unsigned int cnt[4];
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint32_t v = mine[j];
        for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&cnt[j], v);
    }
    __syncthreads();
    if (threadIdx.x < 4 && cnt[threadIdx.x]) atomicAdd(&per_class[threadIdx.x], cnt[threadIdx.x]);
}

__global__ void gather_codes_kernel(const unsigned long long* __restrict__ codes, const uint32_t* __restrict__ idx,
                                    uint32_t n, unsigned long long* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = codes[idx[i]];
}

// The right side's build: every distinct key (value class, code) gets one slot of
// an open-addressing hash table in HBM (linear probing, at most half full); the
// rows sorted stably by slot (sidx) put each key's rows together in row order,
// hstart / hcnt delimiting them.  A left row probes the table once for its run;
// STRING codes are hashes, so their candidates are verified byte for byte.  The
// other non-NULL classes' rows, which value_compare calls equal to any key of
// another class (csv_reader.c:128), are the class lists ridx_c.
__device__ __forceinline__ uint64_t hj_hash(unsigned long long code, uint32_t cls) {
    return mix64(code ^ ((uint64_t)cls << 62) ^ 0x243F6A8885A308D3ULL);
}

// value classes present in one column of a cell table (bit k: class k of
// key_class), OR-reduced per wave: what a repartitioned join's rank reports
__global__ void class_mask_kernel(const Cell* __restrict__ cells, uint32_t stride, uint32_t kcol, uint32_t n,
                                  unsigned int* __restrict__ mask) {
    uint32_t m = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        m |= 1u << key_class(cells[(uint64_t)i * stride + kcol]);
    for (int o = 32; o > 0; o >>= 1) m |= (uint32_t)__shfl_xor((int)m, o, 64);
    if ((threadIdx.x & 63) == 0 && m) atomicOr(mask, m);
}

// slot of every right row's key (inserted when new); row counts per slot.  The
// probe loop is wave-uniform (it runs while any lane of the wave still looks for
// its slot, one probe per lane per trip): a lane that finds a slot claimed but
// not yet published retries it on the next trip instead of spinning, so the
// claiming lane -- perhaps in the same wave -- always gets to publish.
__global__ void hash_build_kernel(const unsigned long long* __restrict__ codes, const uint32_t* __restrict__ cls,
                                  uint32_t n, JoinHashW H, uint32_t* __restrict__ sid,
                                  unsigned long long* __restrict__ overflow) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    bool pending = r < n;
    const unsigned long long code = pending ? codes[r] : 0ull;
    const uint32_t k = pending ? cls[r] : 0u;
    const uint32_t mask = H.cap - 1;
    uint32_t i = (uint32_t)hj_hash(code, k) & mask, slot = 0, probes = 0;
    for (uint32_t trip = 0; __any(pending); trip++) {
        if (pending) {
            // relaxed agent-scope atomics (coherent at L2, no cache maintenance); the
            // publisher drains its code store (vmcnt) before the state store, and a
            // reader loads the code only after it has seen the published state
            HSlot& S = H.slot[i];
            uint32_t st = __hip_atomic_load(&S.st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st == 0) {
                const uint32_t old = atomicCAS(&S.st, 0u, 1u);
                if (old == 0) {                          // claimed: the code first, then publish
                    __hip_atomic_store(&S.code, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&S.st, 2u + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    slot = i;
                    pending = false;
                }
                st = old;
            }
            if (pending && st >= 2) {
                if (st == 2u + k && __hip_atomic_load(&S.code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == code) {
                    slot = i;
                    pending = false;
                } else {
                    i = (i + 1) & mask;
                    if (++probes >= H.cap) { atomicExch(overflow, 1ULL); pending = false; }   // full
                }
            }
            // st == 1: claimed, not yet published -- the same slot again next trip
        }
        if (trip > (1u << 24)) {                          // never hang: report and stop
            if (pending) atomicExch(overflow, 3ULL);
            break;
        }
    }
    if (r < n) sid[r] = slot;
}

// each slot's run [start, end) in the rows sorted by slot (ssid: the sorted slots)
__global__ void run_bounds_kernel(const uint32_t* __restrict__ ssid, uint32_t n, HSlot* __restrict__ slots) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t s = ssid[j];
    if (j == 0 || ssid[j - 1] != s) slots[s].start = j;
    if (j + 1 == n || ssid[j + 1] != s) slots[s].end = j + 1;
}

// [lo, hi) in sidx of the right rows whose key has this class and code
__device__ __forceinline__ void eq_run(const JoinRight& J, uint32_t k, unsigned long long code, uint32_t& lo,
                                       uint32_t& hi) {
    lo = hi = 0;
    const uint32_t mask = J.hcap - 1;
    uint32_t i = (uint32_t)hj_hash(code, k) & mask;
    for (uint32_t probe = 0; probe < J.hcap; probe++, i = (i + 1) & mask) {
        const HSlot S = J.hslot[i];
        if (S.st == 0) return;
        if (S.st == 2u + k && S.code == code) {
            lo = S.start;
            hi = S.end;
            return;
        }
    }
}

__global__ void join_count_kernel(const Cell* __restrict__ L, uint32_t ls, uint32_t lk, uint32_t nL, JoinRight J,
                                  int outer_left, uint32_t* __restrict__ lo_out, unsigned long long* __restrict__ cnt) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nL) return;
    const Cell kc = L[(uint64_t)l * ls + lk];
    const uint32_t k = key_class(kc);
    uint32_t lo, hi;
    eq_run(J, k, join_code(kc), lo, hi);
    unsigned long long n = hi - lo;
    if (k == 2) {
        n = 0;
        for (uint32_t j = lo; j < hi; j++) n += compare(kc, J.cells[(uint64_t)J.sidx[j] * J.stride + J.kcol]) == 0;
    }
    if (k != 0)
        for (uint32_t y = 1; y < 4; y++)
            if (y != k) n += J.seg[y + 1] - J.seg[y];
    lo_out[l] = lo;
    cnt[l] = (outer_left && n == 0) ? 1 : n;             // LEFT / FULL: the unmatched row, NULL-padded
}

__global__ void join_emit_kernel(const Cell* __restrict__ L, uint32_t ls, uint32_t lk, uint32_t nL, JoinRight J,
                                 const uint32_t* __restrict__ lo_in, const unsigned long long* __restrict__ cnt,
                                 const unsigned long long* __restrict__ offs, uint2* __restrict__ pairs,
                                 unsigned int* __restrict__ rmatched) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nL) return;
    const unsigned long long want = cnt[l];
    if (!want) return;
    const Cell kc = L[(uint64_t)l * ls + lk];
    const uint32_t k = key_class(kc);
    const unsigned long long code = join_code(kc);
    // three row-ordered streams: the equal run, and the other two non-NULL classes
    uint32_t e, ee;
    eq_run(J, k, code, e, ee);
    (void)lo_in;
    uint32_t ya = 0, yb = 0, za = 0, zb = 0;
    if (k != 0) {
        const uint32_t y = k == 1 ? 2 : 1, z = k == 3 ? 2 : 3;
        ya = J.seg[y]; yb = J.seg[y + 1];
        za = J.seg[z]; zb = J.seg[z + 1];
    }
    const unsigned long long o = offs[l];
    for (unsigned long long m = 0; m < want; m++) {
        // next verified row of the equal run (~0: exhausted)
        uint32_t re = 0xFFFFFFFFu;
        while (e < ee) {
            const uint32_t r = J.sidx[e];
            if (k != 2 || compare(kc, J.cells[(uint64_t)r * J.stride + J.kcol]) == 0) { re = r; break; }
            e++;
        }
        const uint32_t ry = ya < yb ? J.ridx_c[ya] : 0xFFFFFFFFu;
        const uint32_t rz = za < zb ? J.ridx_c[za] : 0xFFFFFFFFu;
        uint32_t r = re;
        int src = 0;
        if (ry < r) { r = ry; src = 1; }
        if (rz < r) { r = rz; src = 2; }
        if (r == 0xFFFFFFFFu) {                               // only an outer join's unmatched left row
            if (m == 0) pairs[o] = make_uint2(l, JOIN_NONE);
            break;
        }
        pairs[o + m] = make_uint2(l, r);
        if (rmatched) rmatched[r] = 0u;                       // rmatched starts 1: "unmatched"
        if (src == 0) e++;
        else if (src == 1) ya++;
        else za++;
    }
}

// a join chain's intermediate table: the cells later levels read of every joined
// row (M: column k from side M.side[k], cell slot M.col[k]; NULL for a missing side)
__global__ void join_gather_kernel(const uint2* __restrict__ pairs, unsigned long long np, JoinMap M,
                                   const Cell* __restrict__ L, const Cell* __restrict__ R, Cell* __restrict__ out) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const uint2 pr = pairs[i];
    for (int k = 0; k < M.n; k++) {
        const uint32_t row = M.side[k] ? pr.y : pr.x;
        Cell c = cell_null();
        if (row != JOIN_NONE)
            c = M.side[k] ? R[(uint64_t)row * M.rstride + M.col[k]] : L[(uint64_t)row * M.lstride + M.col[k]];
        out[i * (uint64_t)M.n + k] = c;
    }
}

// outer joins: pairs for the unmatched right rows (flags: 1 = unmatched; RIGHT / FULL, appended after
// the left-major part in row order), or every row of one side (ON that matches
// nothing: `ident = ident` not resolvable, or another condition shape)
__global__ void join_fill_kernel(const unsigned int* __restrict__ flags, const unsigned int* __restrict__ pos,
                                 uint32_t n, unsigned long long base, int right_side, uint2* __restrict__ pairs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (flags && !flags[i]) return;                           // matched: not appended
    const unsigned long long at = base + (pos ? pos[i] : i);
    pairs[at] = right_side ? make_uint2(JOIN_NONE, i) : make_uint2(i, JOIN_NONE);
}

// JOIN without ON: every (l, r) pair, l-major (the nested loops' order)
__global__ void join_cross_kernel(uint32_t na, uint32_t nb, unsigned long long np, uint2* __restrict__ pairs) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < np;
         i += (unsigned long long)gridDim.x * blockDim.x)
        pairs[i] = make_uint2((uint32_t)(i / nb), (uint32_t)(i % nb));
}

// A repartitioned join whose keys mix value classes (cqgpu_route_plan2's replication):
// every non-NULL key of a class other than `major` was sent to every rank, so a pair
// of two such records is found on every rank; flags[i] = 0 for those pairs (the
// rank that owns them keeps them: not called there), 1 for every other pair.  An
// unmatched side (JOIN_NONE) never occurs: outer joins are refused in this mode.
__global__ void pair_rep_flags_kernel(const uint2* __restrict__ pairs, unsigned long long np,
                                      const Cell* __restrict__ L, uint32_t ls, uint32_t lk,
                                      const Cell* __restrict__ R, uint32_t rs, uint32_t rk, uint32_t major,
                                      unsigned int* __restrict__ flags) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const uint2 p = pairs[i];
    const uint32_t a = key_class(L[(uint64_t)p.x * ls + lk]), b = key_class(R[(uint64_t)p.y * rs + rk]);
    flags[i] = (a != 0u && a != major && b != 0u && b != major) ? 0u : 1u;
}

// the plan's need slots of one joined row: in registers (plans over <= MAX_NEED
// columns), or a view of the cell tables (wide plans)
__device__ __forceinline__ void join_cells(const JoinMap& M, const Cell* L, const Cell* R, uint2 pr,
                                           CellsT<MAX_NEED>& cs) {
#pragma unroll
    for (int k = 0; k < MAX_NEED; k++) {
        cs.c[k] = cell_null();
        if (k < M.n) {
            const uint32_t row = M.side[k] ? pr.y : pr.x;
            if (row != JOIN_NONE)
                cs.c[k] = M.side[k] ? R[(uint64_t)row * M.rstride + M.col[k]] : L[(uint64_t)row * M.lstride + M.col[k]];
        }
    }
}
__device__ __forceinline__ void join_cells(const JoinMap& M, const Cell* L, const Cell* R, uint2 pr, PairView& v) {
    v.M = &M;
    v.L = L;
    v.R = R;
    v.pr = pr;
}
template <bool WIDE>
using PairCells = typename std::conditional<WIDE, PairView, CellsT<MAX_NEED>>::type;

// Exactness of composite GROUP BY keys (evaluator.c:113-212 groups by the parts' key
// texts joined with '\t'; the kernels key such groups by a 128-bit digest of the
// parts).  After the aggregation every passing pair looks its digest up and compares
// its parts, one by one under the canonical key equality, with the parts of its
// group's first pair: a digest shared by two different part lists (a collision)
// sets *bad and the host fails the query instead of merging them.  Joined-text keys
// (a part holding a tab, COMPT_FLAG) compare the two joined texts byte for byte.
static __device__ int g_find(const GroupTable& gt, const GKey k, uint64_t h) {
    const uint32_t tg = tag_of(h), mask = gt.cap - 1;
    for (uint32_t probe = 0; probe < gt.cap; probe++) {
        const uint32_t i = (uint32_t)(h + probe) & mask;
        const uint32_t t = gt.tag[i];
        if (t == 0) return -1;
        if (t != tg) continue;
        GKey o;
        const uint32_t ocl = gt.clslen[i];
        o.cls = ocl >> 16;
        o.len = ocl & 0xffff;
        o.w0 = gt.w0[i];
        o.w1 = gt.w1[i];
        if (gk_equal(o, k)) return (int)i;
    }
    return -1;
}

// two part lists' joined texts (evaluator.c:113-212), compared exactly: lengths, then
// 16-byte windows rendered from the parts again (joined-text keys are rare: a text
// part holding a tab)
template <class CS>
__device__ bool joined_text_equal(const ScanPlan& P, const Cell* kc, const CS& a, const CS& b, int nneed) {
    for (uint64_t lo = 0;; lo += 16) {
        TextWindow x(lo), y(lo);
        for (int k = 0; k < MAX_GPART; k++) {
            if (k >= P.ngpart) break;
            joined_text_add(x, plan_group_part(P, kc, a, nneed, k), k == 0);
            joined_text_add(y, plan_group_part(P, kc, b, nneed, k), k == 0);
        }
        if (x.pos != y.pos || x.w0 != y.w0 || x.w1 != y.w1) return false;
        if (lo + 16 >= x.pos) return true;
    }
}

template <bool WIDE>
__global__ __launch_bounds__(256) void comp_verify_kernel(const uint2* __restrict__ pairs, unsigned long long np,
                                                          JoinMap M, const Cell* __restrict__ L,
                                                          const Cell* __restrict__ R, unsigned int* __restrict__ bad) {
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    const int nneed = P.nneed;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < np;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        PairCells<WIDE> cs;
        join_cells(M, L, R, pairs[i], cs);
        if (P.nprog != 0 && !eval_where_vm(P, P.consts, cs)) continue;
        bool tab = false;
        const GKey key = plan_group_key(P, P.consts, cs, nneed, tab);
        if (key.cls != GK_COMP) continue;
        const int gi = g_find(gt, key, gk_hash(key));
        if (gi < 0) { atomicOr(bad, 2u); continue; }
        const unsigned long long f = gt.first[gi];
        if (f == i) continue;
        if (f >= np) { atomicOr(bad, 2u); continue; }
        PairCells<WIDE> cf;
        join_cells(M, L, R, pairs[f], cf);
        if (key.len & COMPT_FLAG) {                    // the joined text itself
            if (!joined_text_equal(P, P.consts, cs, cf, nneed)) atomicOr(bad, 1u);
            continue;
        }
        bool same = true;
        for (int k = 0; k < MAX_GPART; k++) {
            if (k >= P.ngpart) break;
            const GKey a = group_key(plan_group_part(P, P.consts, cs, nneed, k));
            const GKey b = group_key(plan_group_part(P, P.consts, cf, nneed, k));
            same = same && gk_equal(a, b);
        }
        if (!same) atomicOr(bad, 1u);
    }
}

// WHERE + GROUP BY + aggregates over the joined rows (filter_rows, create_groups,
// evaluate_aggregate over perform_join's table); a group's `first` is its first
// pair's index, i.e. its first row of the joined table
template <bool WIDE>
__global__ __launch_bounds__(256) void join_agg_kernel(const uint2* __restrict__ pairs, unsigned long long np,
                                                       JoinMap M, const Cell* __restrict__ L,
                                                       const Cell* __restrict__ R, ScanStats* __restrict__ stats,
                                                       int grouped) {
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    const int nneed = P.nneed, nacc = P.nacc;
    unsigned long long my_pass = 0;
    uint32_t my_cls[MAX_ACC];             // value classes seen per MIN/MAX argument, flushed once per wave
    // one group (no GROUP BY): MIN/MAX candidates kept per lane, merged per wave at
    // the end, so the group's lock is taken once per wave instead of once per pair
    Cell my_ext[MAX_ACC];
    unsigned long long my_pos[MAX_ACC];
#pragma unroll
    for (int a = 0; a < MAX_ACC; a++) { my_cls[a] = 0; my_ext[a] = cell_null(); my_pos[a] = NOPOS; }
    for (unsigned long long b0 = (unsigned long long)blockIdx.x * blockDim.x; b0 < np;
         b0 += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long i = b0 + threadIdx.x;
        const bool valid = i < np;
        PairCells<WIDE> cs;
        bool pass = false;
        join_cells(M, L, R, valid ? pairs[i] : make_uint2(JOIN_NONE, JOIN_NONE), cs);
        if (valid) pass = P.nprog == 0 || eval_where_vm(P, P.consts, cs);
        if (pass) {
            my_pass++;
#pragma unroll
            for (int a = 0; a < MAX_ACC; a++)
                if (a < nacc && P.acc[a].kind != ACC_SUM) my_cls[a] |= class_bit(get_cell(cs, P.acc[a].slot, nneed));
        }
        GKey key;
        key.cls = GK_ALL; key.len = 0; key.w0 = 0; key.w1 = 0;
        uint64_t h = 0x12345678ULL;
        if (grouped && pass) {
            bool tab = false;
            key = plan_group_key(P, P.consts, cs, nneed, tab);
            if (tab) atomicOr(&stats->key_flags, 2u);
            h = gk_hash(key);
        }
        int gi = -1;
        if (pass) {
            gi = g_insert(gt, key, h, stats);
            if (gi >= 0) {
                atomicAdd(&gt.cnt[gi], 1ULL);
                if (__atomic_load_n(&gt.first[gi], __ATOMIC_RELAXED) > i) atomicMin(&gt.first[gi], i);   // first only decreases
                for (int a = 0; a < nacc; a++) {
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
            if (a >= nacc) break;
            if (P.acc[a].kind == ACC_SUM) continue;      // uniform
            Cell c = get_cell(cs, P.acc[a].slot, nneed);
            const uint32_t cf = P.acc[a].cls;             // class-split MIN/MAX (mixed classes, host fold)
            const bool in_cls = (cf == 0 || (class_bit(c) & cf) != 0) && c.kind != K_NULL;
            if (P.acc[a].pos_only) c = cell_int(0);
            if (!grouped) {
                if (pass && gi >= 0 && in_cls && ext_better(P.acc[a].kind, c, i, my_ext[a], my_pos[a])) {
                    my_ext[a] = c;
                    my_pos[a] = i;
                }
            } else {
                g_ext_update(pass && gi >= 0 && in_cls, gt, a, P.acc[a].kind, gi >= 0 ? (uint32_t)gi : 0u, c, i,
                             stats);
            }
        }
    }
    if (!grouped) {
#pragma unroll
        for (int a = 0; a < MAX_ACC; a++) {
            if (a >= nacc) break;
            if (P.acc[a].kind == ACC_SUM) continue;      // uniform
            Cell c = my_ext[a];
            unsigned long long p = my_pos[a];
            for (int o = 32; o > 0; o >>= 1) {
                Cell oc;
                oc.kind = (uint32_t)__shfl_down((int)c.kind, o, 64);
                oc.len = (uint32_t)__shfl_down((int)c.len, o, 64);
                oc.bits = __shfl_down(c.bits, o, 64);
                const unsigned long long op = __shfl_down(p, o, 64);
                if (op != NOPOS && ext_better(P.acc[a].kind, oc, op, c, p)) { c = oc; p = op; }
            }
            int gi = -1;
            const bool lead = (threadIdx.x & 63) == 0 && p != NOPOS;
            if (lead) {
                GKey k;
                k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
                gi = g_insert(gt, k, 0x12345678ULL, stats);
            }
            g_ext_update(lead && gi >= 0, gt, a, P.acc[a].kind, gi >= 0 ? (uint32_t)gi : 0u, c, p, stats);
        }
    }
    for (int o = 32; o > 0; o >>= 1) my_pass += __shfl_down(my_pass, o, 64);
    if ((threadIdx.x & 63) == 0 && my_pass) atomicAdd(&stats->passed, my_pass);
#pragma unroll
    for (int a = 0; a < MAX_ACC; a++) {
        if (a >= nacc) break;
        uint32_t m = my_cls[a];
        for (int o = 32; o > 0; o >>= 1) m |= (uint32_t)__shfl_xor((int)m, o, 64);
        if ((threadIdx.x & 63) == 0 && m) atomicOr(&stats->acc_classes[a], m);
    }
}

// join_agg_kernel for grouped COUNT / SUM / AVG plans with a block-local LDS
// pre-aggregation: each pair's group is found (or claimed) in the block's LDS
// table of JS_SLOTS keys (linear probing, the key words stored beside the tag,
// a wave-uniform claim loop so a lane never spins on a slot its own wave has yet
// to publish), COUNT / SUM / numeric count / first pair go to LDS atomics, and the
// block's groups are flushed into the HBM table once at the end: one HBM insert
// and a few atomics per (block, group) instead of per pair.  Pairs whose group
// finds no slot within JS_PROBES probes take join_agg_kernel's HBM path.
constexpr uint32_t JS_SLOTS = 1024, JS_PROBES = 64;
template <bool WIDE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void join_sum_kernel(const uint2* __restrict__ pairs, unsigned long long np,
                                                       JoinMap M, const Cell* __restrict__ L,
                                                       const Cell* __restrict__ R, ScanStats* __restrict__ stats) {
    const ScanPlan& P = c_plan;
    const GroupTable& gt = c_gt;
    const int nneed = P.nneed, nacc = P.nacc;
    extern __shared__ __align__(16) uint8_t smem[];
    uint32_t* tag = (uint32_t*)smem;                                  // 0 free, 1 claimed, else lds_hdr
    v4u* kw = (v4u*)(smem + JS_SLOTS * 4);
    uint32_t* cnt = (uint32_t*)(smem + JS_SLOTS * 20);
    unsigned long long* first = (unsigned long long*)(smem + JS_SLOTS * 24);
    double* sum = (double*)(smem + JS_SLOTS * 32);                    // [nacc][JS_SLOTS]
    uint32_t* num = (uint32_t*)(smem + JS_SLOTS * (32 + 8 * (uint32_t)nacc));
    for (uint32_t i = threadIdx.x; i < JS_SLOTS; i += blockDim.x) {
        tag[i] = 0;
        cnt[i] = 0;
        first[i] = ~0ull;
        for (int a = 0; a < nacc; a++) { sum[a * JS_SLOTS + i] = 0.0; num[a * JS_SLOTS + i] = 0; }
    }
    __syncthreads();
    unsigned long long my_pass = 0;
    for (unsigned long long b0 = (unsigned long long)blockIdx.x * blockDim.x; b0 < np;
         b0 += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long i = b0 + threadIdx.x;
        const bool valid = i < np;
        PairCells<WIDE> cs;
        bool pass = false;
        join_cells(M, L, R, valid ? pairs[i] : make_uint2(JOIN_NONE, JOIN_NONE), cs);
        if (valid) pass = P.nprog == 0 || eval_where_vm(P, P.consts, cs);
        GKey key;
        key.cls = GK_ALL; key.len = 0; key.w0 = 0; key.w1 = 0;
        uint64_t h = 0;
        if (pass) {
            my_pass++;
            bool tab = false;
            key = plan_group_key(P, P.consts, cs, nneed, tab);
            if (tab) atomicOr(&stats->key_flags, 2u);
            h = gk_hash(key);
        }
        // the block's slot of the key (wave-uniform loop: claims publish within the trip)
        const uint32_t hd = lds_hdr(key, h);
        const v4u mine = key_words(key);
        uint32_t pos = (uint32_t)h & (JS_SLOTS - 1), probes = 0;
        int s = -1;
        bool pending = pass;
        for (uint32_t trip = 0; __any(pending); trip++) {
            if (pending) {
                uint32_t t = __hip_atomic_load(&tag[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (t == 0) {
                    const uint32_t old = atomicCAS(&tag[pos], 0u, 1u);
                    if (old == 0) {
                        kw[pos] = mine;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __hip_atomic_store(&tag[pos], hd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        s = (int)pos;
                        pending = false;
                    }
                    t = old;
                }
                if (pending && t != 1) {                       // a published key: compare
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    if (t == hd && key_match(key, mine, kw[pos])) {
                        s = (int)pos;
                        pending = false;
                    } else if (++probes >= JS_PROBES) {
                        pending = false;                          // no room: the HBM path
                    } else {
                        pos = (pos + 1) & (JS_SLOTS - 1);
                    }
                }
            }
            if (trip > (1u << 20)) break;                          // never hang (s stays -1)
        }
        if (s >= 0) {
            atomicAdd(&cnt[s], 1u);
            atomicMin(&first[s], i);
            for (int a = 0; a < nacc; a++) {
                const Cell c = get_cell(cs, P.acc[a].slot, nneed);
                if (is_num(c)) {
                    atomicAdd(&sum[a * JS_SLOTS + s], num_of(c));
                    atomicAdd(&num[a * JS_SLOTS + s], 1u);
                }
            }
        } else if (pass) {
            const int gi = g_insert(gt, key, h, stats);
            if (gi >= 0) {
                atomicAdd(&gt.cnt[gi], 1ULL);
                if (__atomic_load_n(&gt.first[gi], __ATOMIC_RELAXED) > i) atomicMin(&gt.first[gi], i);
                for (int a = 0; a < nacc; a++) {
                    const Cell c = get_cell(cs, P.acc[a].slot, nneed);
                    if (is_num(c)) {
                        atomicAdd(&gt.sum[a][gi], num_of(c));
                        atomicAdd(&gt.num[a][gi], 1ULL);
                    }
                }
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) my_pass += __shfl_down(my_pass, o, 64);
    if ((threadIdx.x & 63) == 0 && my_pass) atomicAdd(&stats->passed, my_pass);
    __syncthreads();
    // flush: one HBM insert and a few atomics per group of this block
    for (uint32_t i = threadIdx.x; i < JS_SLOTS; i += blockDim.x) {
        const uint32_t t = tag[i];
        if (t < 0x80000000u || !cnt[i]) continue;
        const v4u w = kw[i];
        GKey k;
        k.cls = (t >> 16) & 7u;
        k.len = t & 0xFFFFu;
        k.w0 = (uint64_t)w.x | ((uint64_t)w.y << 32);
        k.w1 = (uint64_t)w.z | ((uint64_t)w.w << 32);
        const int gi = g_insert(gt, k, gk_hash(k), stats);
        if (gi < 0) continue;
        atomicAdd(&gt.cnt[gi], (unsigned long long)cnt[i]);
        const unsigned long long f = first[i];
        if (__atomic_load_n(&gt.first[gi], __ATOMIC_RELAXED) > f) atomicMin(&gt.first[gi], f);
        for (int a = 0; a < nacc; a++) {
            const uint32_t nn = num[a * JS_SLOTS + i];
            if (nn) {
                atomicAdd(&gt.sum[a][gi], sum[a * JS_SLOTS + i]);
                atomicAdd(&gt.num[a][gi], (unsigned long long)nn);
            }
        }
    }
}

// WHERE over the joined rows of a row-returning query: 1 / 0 per pair
template <bool WIDE>
__global__ void join_filter_kernel(const uint2* __restrict__ pairs, unsigned long long np, JoinMap M,
                                   const Cell* __restrict__ L, const Cell* __restrict__ R,
                                   unsigned int* __restrict__ flags) {
    const ScanPlan& P = c_plan;
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    PairCells<WIDE> cs;
    join_cells(M, L, R, pairs[i], cs);
    flags[i] = (P.nprog == 0 || eval_where_vm(P, P.consts, cs)) ? 1u : 0u;
}

// build_result's projection (evaluator_utils.c:249-549) of the passing joined rows
// whose output index falls in [lo, lo + m): M maps the projection's columns
__global__ void join_project_kernel(const uint2* __restrict__ pairs, unsigned long long np,
                                    const unsigned int* __restrict__ flags, const unsigned int* __restrict__ pos,
                                    unsigned long long lo, uint32_t m, JoinMap M, const Cell* __restrict__ L,
                                    const Cell* __restrict__ R, const Insn* __restrict__ code,
                                    const uint32_t* __restrict__ off, int nout, const Cell* __restrict__ consts,
                                    Cell* __restrict__ scratch, Cell* __restrict__ out) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np || !flags[i]) return;
    const unsigned long long o = pos[i];
    if (o < lo || o >= lo + m) return;
    const uint64_t row = o - lo;
    const uint2 pr = pairs[i];
    Cell* cs = scratch + row * (uint64_t)(M.n ? M.n : 1);
    for (int k = 0; k < M.n; k++) {
        const uint32_t rw = M.side[k] ? pr.y : pr.x;
        cs[k] = rw == JOIN_NONE ? cell_null()
                                : (M.side[k] ? R[(uint64_t)rw * M.rstride + M.col[k]] : L[(uint64_t)rw * M.lstride + M.col[k]]);
    }
    for (int k = 0; k < nout; k++) out[row * nout + k] = eval_value(code, off[k], off[k + 1], cs, 1, consts);
}

// finish_kernel for joined groups: representative cells from the group's first pair
__global__ void join_finish_kernel(const GroupOut* __restrict__ out, const unsigned int* __restrict__ count,
                                   unsigned int cap_out, const uint2* __restrict__ pairs, JoinMap M,
                                   const Cell* __restrict__ L, const Cell* __restrict__ R, int nacc, uint32_t sb,
                                   Cell* __restrict__ cells, uint8_t* __restrict__ bytes) {
    const uint32_t ncell = (uint32_t)(M.n + nacc + 1);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ng = *count < cap_out ? *count : cap_out;
    if (i >= ng) return;
    Cell* cs = cells + (size_t)i * ncell;
    const unsigned long long first = out[i].first;
    for (int k = 0; k < M.n; k++) {
        Cell c = cell_null();
        if (first != NOPOS) {
            const uint2 pr = pairs[first];
            const uint32_t rw = M.side[k] ? pr.y : pr.x;
            if (rw != JOIN_NONE)
                c = M.side[k] ? R[(uint64_t)rw * M.rstride + M.col[k]] : L[(uint64_t)rw * M.lstride + M.col[k]];
        }
        cs[k] = c;
    }
    for (int a = 0; a < nacc; a++) cs[M.n + a] = out[i].ext[a];
    Cell kc = cell_null();
    const uint32_t cl = out[i].clslen;
    if ((cl >> 16) == GK_LONG) { kc.kind = K_STR; kc.len = cl & 0xffff; kc.bits = out[i].w0; }
    cs[M.n + nacc] = kc;
    for (uint32_t k = 0; k < ncell; k++) {
        const Cell c = cs[k];
        if (c.kind != K_STR) continue;
        const uint8_t* src = (const uint8_t*)(uintptr_t)c.bits;
        uint8_t* dst = bytes + ((size_t)i * ncell + k) * sb;
        const uint32_t mm = c.len < sb ? c.len : sb;
        for (uint32_t j = 0; j < mm; j++) dst[j] = src[j];
    }
}

// ------------------------------------------------------------------ STDDEV / MEDIAN
// evaluate_aggregate's value-list aggregates (evaluator_aggregates.c:328-411): the
// numeric values of a column per group, sorted by (group key, value) on the
// device, then one pass per group: population STDDEV (mean first, then the
// squared deviations) and MEDIAN (middle value, or the mean of the middle two).

// per passing record: group key words (GK_LONG keys by content hash) and the
// column's numeric value as an order-preserving 64-bit key; flag 1 when numeric
__global__ void vla_prep_kernel(const Cell* __restrict__ cells, uint32_t n, uint32_t nc, int gslot, uint32_t vslot,
                                unsigned long long* __restrict__ kw0, unsigned long long* __restrict__ kw1,
                                unsigned long long* __restrict__ kcl, unsigned long long* __restrict__ vkey,
                                unsigned int* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    GKey k;
    k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
    if (gslot >= 0) k = group_key(cells[(uint64_t)i * nc + gslot]);
    kw0[i] = k.cls == GK_LONG ? 0ull : k.w0;
    kw1[i] = k.w1;
    kcl[i] = gk_clslen(k);
    const Cell v = cells[(uint64_t)i * nc + vslot];
    const uint64_t b = dbl_bits(num_of(v));
    vkey[i] = (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
    flag[i] = is_num(v) ? 1u : 0u;
}

// the same per (l, r) pair of parsed cells (joins, composite / expression keys
// over identity pairs): WHERE by the plan's VM, the group key as join_agg_kernel
// computes it (plan_group_key), the value from V's one column
template <bool WIDE>
__global__ void vla_pair_prep_kernel(const uint2* __restrict__ pairs, uint32_t n, JoinMap M, JoinMap V,
                                     const Cell* __restrict__ L, const Cell* __restrict__ R, int grouped,
                                     unsigned long long* __restrict__ kw0, unsigned long long* __restrict__ kw1,
                                     unsigned long long* __restrict__ kcl, unsigned long long* __restrict__ vkey,
                                     unsigned int* __restrict__ flag) {
    const ScanPlan& P = c_plan;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2 pr = pairs[i];
    PairCells<WIDE> cs;
    join_cells(M, L, R, pr, cs);
    const bool pass = P.nprog == 0 || eval_where_vm(P, P.consts, cs);
    GKey k;
    k.cls = GK_ALL; k.len = 0; k.w0 = 0; k.w1 = 0;
    if (grouped) {
        bool tab = false;
        k = plan_group_key(P, P.consts, cs, P.nneed, tab);
    }
    kw0[i] = k.cls == GK_LONG ? 0ull : k.w0;
    kw1[i] = k.w1;
    kcl[i] = gk_clslen(k);
    const uint32_t row = V.side[0] ? pr.y : pr.x;
    Cell v = cell_null();
    if (row != JOIN_NONE) v = V.side[0] ? R[(uint64_t)row * V.rstride + V.col[0]] : L[(uint64_t)row * V.lstride + V.col[0]];
    const uint64_t b = dbl_bits(num_of(v));
    vkey[i] = (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
    flag[i] = pass && is_num(v) ? 1u : 0u;
}

__global__ void vla_compact_kernel(const unsigned int* __restrict__ flag, const unsigned int* __restrict__ pos,
                                   uint32_t n, unsigned int* __restrict__ perm) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && flag[i]) perm[pos[i]] = i;
}

__global__ void vla_gather_kernel(const unsigned long long* __restrict__ a, const unsigned int* __restrict__ perm,
                                  uint32_t m, unsigned long long* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i] = a[perm[i]];
}

// 1 where a new group starts in the sorted order
__global__ void vla_heads_kernel(const unsigned long long* __restrict__ kw0, const unsigned long long* __restrict__ kw1,
                                 const unsigned long long* __restrict__ kcl, const unsigned int* __restrict__ perm,
                                 uint32_t m, unsigned int* __restrict__ head) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t p = perm[i];
    bool h = i == 0;
    if (!h) {
        const uint32_t q = perm[i - 1];
        h = kw0[p] != kw0[q] || kw1[p] != kw1[q] || kcl[p] != kcl[q];
    }
    head[i] = h ? 1u : 0u;
}

__global__ void vla_starts_kernel(const unsigned int* __restrict__ head, const unsigned int* __restrict__ sid,
                                  uint32_t m, unsigned int* __restrict__ start) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m && head[i]) start[sid[i]] = i;
}

__device__ __forceinline__ double vla_value(unsigned long long k) {
    const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
    return as_dbl(b);
}

// one thread per group: kind 0 STDDEV (population), 1 MEDIAN
__global__ void vla_reduce_kernel(const unsigned long long* __restrict__ vkey, const unsigned long long* __restrict__ kw0,
                                  const unsigned long long* __restrict__ kw1, const unsigned long long* __restrict__ kcl,
                                  const unsigned int* __restrict__ perm, const unsigned int* __restrict__ start,
                                  uint32_t nseg, uint32_t m, int kind, unsigned long long* __restrict__ out,
                                  double* __restrict__ aux) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    const uint32_t a = start[s], b = s + 1 < nseg ? start[s + 1] : m;
    const uint32_t n = b - a;
    double r;
    if (kind == 2) {          // a partial's STDDEV state: sum (out), squared deviations and count (aux)
        double sum = 0;
        for (uint32_t i = a; i < b; i++) sum += vla_value(vkey[perm[i]]);
        const double mean = sum / n;
        double vs = 0;
        for (uint32_t i = a; i < b; i++) {
            const double d = vla_value(vkey[perm[i]]) - mean;
            vs += d * d;
        }
        r = sum;
        aux[2 * (uint64_t)s] = vs;
        aux[2 * (uint64_t)s + 1] = (double)n;
    } else if (kind == 0) {
        double sum = 0;
        for (uint32_t i = a; i < b; i++) sum += vla_value(vkey[perm[i]]);
        const double mean = sum / n;
        double vs = 0;
        for (uint32_t i = a; i < b; i++) {
            const double d = vla_value(vkey[perm[i]]) - mean;
            vs += d * d;
        }
        r = sqrt(vs / n);
    } else {
        r = (n & 1) ? vla_value(vkey[perm[a + n / 2]])
                    : (vla_value(vkey[perm[a + n / 2 - 1]]) + vla_value(vkey[perm[a + n / 2]])) / 2.0;
    }
    const uint32_t p = perm[a];
    out[4 * (uint64_t)s + 0] = kcl[p];
    out[4 * (uint64_t)s + 1] = kw0[p];
    out[4 * (uint64_t)s + 2] = kw1[p];
    out[4 * (uint64_t)s + 3] = dbl_bits(r);
}

}  // namespace cq

// ------------------------------------------------------------------ host wrappers
extern "C" {
static size_t lds_slot_bytes(const cq::ScanPlan* P) {
    size_t b = 16 + 4 + 4 + 4;   // key, hdr, cnt, first
    for (int a = 0; a < P->nacc; a++) b += P->acc[a].kind == cq::ACC_SUM ? 12 : sizeof(cq::Cell) + 8;
    return b;
}
static size_t lds_fixed_bytes() {
    auto r16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    return r16(cq::TILE + cq::TILE_PAD) + r16(cq::ECAP * 2) + r16(cq::NLCAP * 2) + r16((cq::NW + 1) * 2) +
           r16(cq::RSMAX * 8) + r16(32 * 4) + r16(cq::MAX_CONST * sizeof(cq::Cell)) +
           r16(cq::KSTR);
}

// group-table capacity: the largest multiple of 64 <= 2048 that fits the budget
// (each carved array is rounded to 16 bytes: 16 arrays at most -> 256 bytes slack).
// Not a power of two: a MIN/MAX plan's wider slots would otherwise halve the table
// to 1024 slots, which 1000 groups fill to the point that inserts overflow to HBM.
uint32_t cq_scan_lds_slots(const cq::ScanPlan* P, int grouped) {
    if (!grouped) return 0;
    const size_t per = lds_slot_bytes(P);
    uint32_t h = 2048;
    while (h > 64 && lds_fixed_bytes() + (size_t)h * per + 512 > (size_t)cq::LDS_BUDGET) h -= 64;
    return h;
}

// MIN/MAX candidate slots per block (GroupTable.cand_stride): an LDS slot, or a wave
uint32_t cq_scan_cand_stride(const cq::ScanPlan* P, int grouped) {
    const uint32_t h = cq_scan_lds_slots(P, grouped);
    const uint32_t waves = cq::SCAN_T / 64;
    return h > waves ? h : waves;
}

size_t cq_scan_lds_bytes(const cq::ScanPlan* P, int grouped) {
    size_t b = lds_fixed_bytes();
    if (grouped) b += (size_t)cq_scan_lds_slots(P, grouped) * lds_slot_bytes(P) + 512;
    return b;
}

}  // extern "C"

// plan shape -> kernel instance
static int where_mode(const cq::ScanPlan* P) {
    if (P->nprog == 0) return cq::W_NONE;
    if (P->nprog == 3 && P->prog[0].op == cq::OP_COL && P->prog[1].op == cq::OP_CONST && P->prog[2].op == cq::OP_CMP)
        return cq::W_SIMPLE;
    return cq::W_VM;
}
static bool has_ext(const cq::ScanPlan* P) {
    for (int a = 0; a < P->nacc; a++)
        if (P->acc[a].kind != cq::ACC_SUM) return true;
    return false;
}
static bool small_plan(const cq::ScanPlan* P) { return P->nneed <= 4 && P->nacc <= 2; }

typedef void (*scan_fn_t)(const uint8_t*, cq::ScanStats*, unsigned long long*, unsigned long long, uint32_t,
                          cq::Cell*, unsigned long long*, unsigned long long);
template <bool G>
static scan_fn_t pick_scan(const cq::ScanPlan* P) {
    using namespace cq;
    if (!small_plan(P)) return scan_kernel<G, 8, 8, W_VM, true>;
    const int wm = where_mode(P);
    const bool ext = has_ext(P);
    if (wm == W_NONE) return ext ? scan_kernel<G, 4, 2, W_NONE, true> : scan_kernel<G, 4, 2, W_NONE, false>;
    if (wm == W_SIMPLE) return ext ? scan_kernel<G, 4, 2, W_SIMPLE, true> : scan_kernel<G, 4, 2, W_SIMPLE, false>;
    return ext ? scan_kernel<G, 4, 2, W_VM, true> : scan_kernel<G, 4, 2, W_VM, false>;
}
static scan_fn_t scan_fn(const cq::ScanPlan* P, int grouped) {
    return grouped ? pick_scan<true>(P) : pick_scan<false>(P);
}

extern "C" {
// the fast scan, then the general kernel over the records it declined
int cq_lean_eligible(const cq::ScanPlan* P);
uint64_t cq_lean_windows(uint64_t begin, uint64_t end, uint32_t ws);
int cq_lean_waves_per_block();
hipError_t cq_launch_lean(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          const cq::GroupTable* rt, cq::ScanStats* stats, unsigned long long* row_out,
                          unsigned long long row_cap, int grouped, int grid, hipStream_t s,
                          unsigned long long* slow_list, unsigned long long slow_cap);
int cq_fast_ext_plan(const cq::ScanPlan* P, int grouped);
int cq_fast_ext_info(const cq::ScanPlan* P, int grouped, uint32_t* col);
hipError_t cq_fast_ext_final(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt, const cq::GroupTable* rt,
                             cq::ScanStats* stats, hipStream_t s);
hipError_t cq_launch_raw_merge(const cq::GroupTable* gt, const cq::GroupTable* rt, int nacc, cq::ScanStats* stats,
                               hipStream_t s, uint32_t max_mask = 0, const uint8_t* g = nullptr,
                               int pk_acc = -1, uint32_t pk_col = 0, uint32_t delim = ',');
int cq_fast_eligible(const cq::ScanPlan* P, int grouped, int want_rows);
int cq_fast_waves_per_block();
hipError_t cq_launch_fast(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          const cq::GroupTable* rt, cq::ScanStats* stats, int grouped, int grid, hipStream_t s,
                          unsigned long long* slow_list, unsigned long long slow_cap);

// cqgpu_set_scan_kernel / CQ_SCAN_KERNEL: 0 (default) fast_kernel, else lean_kernel,
// else scan_kernel, by plan shape; 1 ("general"): scan_kernel for every plan; 2
// ("lean"): never fast_kernel (A/B runs, parity tests of every kernel)
static int g_scan_mode = -1;
static int scan_mode() {
    if (g_scan_mode < 0) {
        const char* v = getenv("CQ_SCAN_KERNEL");
        g_scan_mode = (v && strcmp(v, "general") == 0) ? 1 : ((v && strcmp(v, "lean") == 0) ? 2 : 0);
    }
    return g_scan_mode;
}
static bool lean_enabled() { return scan_mode() != 1; }
int cq_set_scan_mode(int mode) {
    const int old = scan_mode();
    g_scan_mode = mode == 1 ? 1 : (mode == 2 ? 2 : 0);
    return old;
}

// 1 when cq_launch_scan runs lean_kernel or fast_kernel for this plan
int cq_scan_uses_lean(const cq::ScanPlan* P, int with_cells) {
    return !with_cells && lean_enabled() && cq_lean_eligible(P);
}
// bit a set: accumulator a is a MAX (raw_merge_kernel's extreme merge)
static uint32_t max_mask(const cq::ScanPlan* P) {
    uint32_t m = 0;
    for (int a = 0; a < P->nacc; a++) m |= (P->acc[a].kind == cq::ACC_MAX ? 1u : 0u) << a;
    return m;
}
// 2 when it runs fast_kernel, 1 lean_kernel, 0 scan_kernel
int cq_scan_kernel_kind(const cq::ScanPlan* P, int grouped, int want_rows, int with_cells) {
    if (with_cells || !lean_enabled()) return 0;
    if (scan_mode() == 0 && cq_fast_eligible(P, grouped, want_rows)) return 2;   // (incl. its MIN / MAX builds)
    return cq_lean_eligible(P) ? 1 : 0;
}

static int device_cus() {
    static int ncu[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (!ncu[dev & 63]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        ncu[dev & 63] = n;
    }
    return ncu[dev & 63];
}

hipError_t cq_launch_scan(const uint8_t* g, const cq::ScanPlan* P, const cq::GroupTable* gt,
                          const cq::GroupTable* rt, cq::ScanStats* stats, unsigned long long* row_out,
                          unsigned long long row_cap, int grouped, int grid, hipStream_t s,
                          cq::Cell* cells_out, unsigned long long* slow_list, unsigned long long slow_cap) {
    // fast_kernel's MIN / MAX builds (cq_fast_ext_plan) take the same route as the
    // lean-eligible plans; any other MIN / MAX plan the general scan_kernel
    const bool fext = scan_mode() == 0 && !cells_out && lean_enabled() && row_out == nullptr &&
                      cq_fast_ext_plan(P, grouped) && cq_fast_eligible(P, grouped, 0);
    // (plans fast_kernel takes that lean_kernel does not: its compound-WHERE builds)
    const bool fonly = scan_mode() == 0 && !cells_out && lean_enabled() && cq_fast_eligible(P, grouped, row_out != nullptr);
    if ((cq_scan_uses_lean(P, cells_out != nullptr) || fext || fonly) && (!grouped || rt)) {
        // slow_kernel reads this file's plan and table symbols
        hipError_t e0 = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
        if (e0 == hipSuccess)
            e0 = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_gt), gt, sizeof *gt, s);
        if (e0 != hipSuccess) return e0;
        // one 16-wave block per CU, each wave streaming its own windows
        const uint64_t hi = P->range_end < P->n ? P->range_end : P->n;
        const uint64_t wins = cq_lean_windows(P->range_begin, hi, P->lean_ws) + 1;
        const bool fast = scan_mode() == 0 && cq_fast_eligible(P, grouped, row_out != nullptr);
        const uint64_t per = (uint64_t)(fast ? cq_fast_waves_per_block() : cq_lean_waves_per_block());
        uint64_t lg = (wins + per - 1) / per;
        if (lg > (uint64_t)device_cus()) lg = (uint64_t)device_cus();
        if (lg < 1) lg = 1;
        if ((wins + lg * per - 1) / (lg * per) < (1u << 16)) {   // first-row codes hold 16 bits of round
            hipError_t e = fast ? cq_launch_fast(g, P, gt, rt, stats, grouped, (int)lg, s, slow_list, slow_cap)
                                : cq_launch_lean(g, P, gt, rt, stats, row_out, row_cap, grouped, (int)lg, s,
                                                 slow_list, slow_cap);
            if (e != hipSuccess) return e;
            if (grouped)
                hipLaunchKernelGGL(cq::slow_kernel<true>, dim3(SLOW_GRID), dim3(256), 0, s, g, stats, row_out, row_cap,
                                   cells_out, slow_list, slow_cap);
            else
                hipLaunchKernelGGL(cq::slow_kernel<false>, dim3(SLOW_GRID), dim3(256), 0, s, g, stats, row_out, row_cap,
                                   cells_out, slow_list, slow_cap);
            e = hipGetLastError();
            uint32_t pk_col = 0;
            const int pk_acc = fext ? cq_fast_ext_info(P, grouped, &pk_col) : -1;
            if (e == hipSuccess && grouped)
                e = cq_launch_raw_merge(gt, rt, P->nacc, stats, s, max_mask(P), g, pk_acc, pk_col, P->delim);
            if (e == hipSuccess && !grouped && pk_acc >= 0) e = cq_fast_ext_final(g, P, gt, rt, stats, s);
            return e;
        }
    }
    const size_t lds = cq_scan_lds_bytes(P, grouped);
    hipError_t e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
    if (e == hipSuccess) e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_gt), gt, sizeof *gt, s);
    if (e != hipSuccess) return e;
    const uint32_t h = cq_scan_lds_slots(P, grouped);
    const scan_fn_t fn = scan_fn(P, grouped);
    cq::set_max_lds((const void*)fn, (int)lds);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(cq::SCAN_T), lds, s, g, stats, row_out, row_cap, h, cells_out,
                       slow_list, slow_cap);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (grouped)
        hipLaunchKernelGGL(cq::slow_kernel<true>, dim3(SLOW_GRID), dim3(256), 0, s, g, stats, row_out, row_cap, cells_out,
                           slow_list, slow_cap);
    else
        hipLaunchKernelGGL(cq::slow_kernel<false>, dim3(SLOW_GRID), dim3(256), 0, s, g, stats, row_out, row_cap, cells_out,
                           slow_list, slow_cap);
    return hipGetLastError();
}

int cq_scan_occupancy(const cq::ScanPlan* P, int grouped) {
    const size_t lds = cq_scan_lds_bytes(P, grouped);
    int blocks = 0;
    const void* fn = (const void*)scan_fn(P, grouped);
    cq::set_max_lds((const void*)fn, (int)lds);
    // (per step otherwise: the occupancy query is a slow runtime call)
    static std::mutex mu;
    static std::map<std::tuple<const void*, size_t, int>, int> memo;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(fn, lds, dev);
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
    }
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, cq::SCAN_T, lds) != hipSuccess) return 1;
    blocks = blocks > 0 ? blocks : 1;
    std::lock_guard<std::mutex> g(mu);
    memo[key] = blocks;
    return blocks;
}

hipError_t cq_launch_compact(const cq::GroupTable* gt, const cq::ScanPlan* P, cq::GroupOut* out,
                             unsigned int* count, unsigned int cap_out, hipStream_t s, unsigned long long* ofirst) {
    const int nacc = P->nacc;
    uint32_t kinds = 0;
    for (int a = 0; a < nacc; a++) kinds |= (uint32_t)P->acc[a].kind << (2 * a);
    const dim3 grid((gt->cap + 255) / 256);
    hipLaunchKernelGGL(cq::compact_kernel, grid, dim3(256), 0, s, *gt, nacc, kinds, out, count, cap_out, ofirst);
    return hipGetLastError();
}

hipError_t cq_launch_gather(const uint8_t* g, const cq::ScanPlan* P, const unsigned long long* recs,
                            uint32_t nrec, cq::Cell* out, hipStream_t s) {
    if (!nrec) return hipSuccess;
    hipError_t e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cq::gather_kernel, dim3((nrec + 127) / 128), dim3(128), 0, s, g, recs, nrec, out);
    return hipGetLastError();
}

// (c_plan: the plan cq_launch_gather uploaded for the same cells)
hipError_t cq_launch_comp_text(const cq::Cell* cells, uint32_t n, uint32_t cap, uint8_t* out, uint32_t* lens,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::comp_text_kernel, dim3((n + 127) / 128), dim3(128), 0, s, cells, n, cap, out, lens);
    return hipGetLastError();
}

hipError_t cq_launch_project(const uint8_t* g, const unsigned long long* recs, uint32_t nrec,
                             const cq::ProjDesc* D, cq::Cell* scratch, cq::Cell* out, hipStream_t s) {
    if (!nrec) return hipSuccess;
    hipLaunchKernelGGL(cq::project_kernel, dim3((nrec + 255) / 256), dim3(256), 0, s, g, recs, nrec, *D, scratch,
                       out);
    return hipGetLastError();
}

namespace cq {
// the aggregate result in one contiguous buffer (host-mapped: no copy, one sync):
// per group its key, COUNT, first row and the plan's accumulators only (40 + 40 *
// nacc bytes instead of the whole GroupOut), then the finish cells, then their
// inline string bytes -- sections laid out by the device's group count.  With
// `order` and at most PACK_ORDER_MAX groups, group i lands at its rank in (first
// row, index) order: create_groups' first-appearance order, so the host does not
// sort.  `hdr` (optional) receives the scan statistics and the group count.
constexpr uint32_t PACK_ORDER_MAX = 8192;
// group i's rank in first-appearance order (by first-row offset, ties by index):
// an LDS-tiled count of the groups before it; every thread of the block calls it
__device__ uint32_t first_rank(const GroupOut* __restrict__ out, uint32_t ng, uint32_t i) {
    __shared__ unsigned long long tile[1024];
    const unsigned long long fi = i < ng ? out[i].first : 0ull;
    uint32_t below = 0;
    for (uint32_t base = 0; base < ng; base += 1024) {
        const uint32_t m = min(1024u, ng - base);
        __syncthreads();
        {   // eight independent loads in flight per thread (GroupOut rows are 360 bytes apart)
            unsigned long long t[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t k = threadIdx.x + u * blockDim.x;
                t[u] = k < m ? out[base + k].first : 0ull;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t k = threadIdx.x + u * blockDim.x;
                if (k < m) tile[k] = t[u];
            }
            for (uint32_t k = threadIdx.x + 8 * blockDim.x; k < m; k += blockDim.x) tile[k] = out[base + k].first;
        }
        __syncthreads();
        if (i < ng) {
            // eight independent LDS reads in flight per trip (a one-at-a-time loop
            // waits out the LDS latency per element: ~30 us for 1,000 groups)
            uint32_t k = 0;
            for (; k + 8 <= m; k += 8) {
                unsigned long long f[8];
#pragma unroll
                for (int u = 0; u < 8; u++) f[u] = tile[k + u];
#pragma unroll
                for (int u = 0; u < 8; u++) below += (f[u] < fi) | ((f[u] == fi) & (base + k + u < i));
            }
            for (; k < m; k++) {
                const unsigned long long f = tile[k];
                below += (f < fi) | ((f == fi) & (base + k < i));
            }
        }
    }
    return below;
}

__global__ void pack_result_kernel(const GroupOut* __restrict__ out, const unsigned int* __restrict__ count,
                                   unsigned int cap_out, int nacc, const Cell* __restrict__ cells,
                                   const uint8_t* __restrict__ bytes, uint32_t ncell, uint32_t sb,
                                   uint8_t* __restrict__ dst, const ScanStats* __restrict__ stats,
                                   uint8_t* __restrict__ hdr, int order) {
    const uint32_t ng = min(*count, cap_out);
    const uint32_t rec = 40u + 40u * (uint32_t)nacc;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (hdr && blockIdx.x == 0) {
        const uint32_t nw = (uint32_t)(sizeof(ScanStats) / 4);
        for (uint32_t k = threadIdx.x; k < nw; k += blockDim.x) ((uint32_t*)hdr)[k] = ((const uint32_t*)stats)[k];
        if (threadIdx.x == 0) *(uint32_t*)(hdr + sizeof(ScanStats)) = ng;
    }
    const uint32_t r = (order && ng <= PACK_ORDER_MAX) ? first_rank(out, ng, i) : i;
    if (i >= ng) return;
    // every load of the group's record first, then the stores (interleaved, each
    // store waited on its load)
    const GroupOut o = out[i];
    uint8_t* rp = dst + (size_t)r * rec;
    ((uint32_t*)rp)[0] = o.clslen;
    ((uint32_t*)rp)[1] = 0;
    ((uint64_t*)rp)[1] = o.w0;
    ((uint64_t*)rp)[2] = o.w1;
    ((unsigned long long*)rp)[3] = o.cnt;
    ((unsigned long long*)rp)[4] = o.first;
    uint64_t* q = (uint64_t*)(rp + 40);
#pragma unroll
    for (int a = 0; a < MAX_ACC; a++) {
        if (a >= nacc) break;
        q[5 * a + 0] = dbl_bits(o.sum[a]);
        q[5 * a + 1] = o.num[a];
        q[5 * a + 2] = ((uint64_t)o.ext[a].len << 32) | o.ext[a].kind;
        q[5 * a + 3] = o.ext[a].bits;
        q[5 * a + 4] = o.extpos[a];
    }
    Cell* dc = (Cell*)(dst + (size_t)ng * rec);
    uint8_t* db = (uint8_t*)(dc + (size_t)ng * ncell);
    for (uint32_t k = 0; k < ncell; k++) {
        const Cell c = cells[(size_t)i * ncell + k];
        dc[(size_t)r * ncell + k] = c;
        // only a STRING's own bytes cross to the host (it reads len <= sb of them)
        const uint32_t nb = c.kind == K_STR ? (min(c.len, sb) + 15u) / 16u : 0u;
        const uint4* sbs = (const uint4*)(bytes + ((size_t)i * ncell + k) * sb);
        uint4* dbs = (uint4*)(db + ((size_t)r * ncell + k) * sb);
        for (uint32_t w = 0; w < nb; w++) dbs[w] = sbs[w];
    }
}
}  // namespace cq

extern "C++" {
namespace cq {
// ---- finish_kernel + pack_result_kernel in one launch: one wave per group.  The
// wave counts the groups ahead of its own in (first row, index) order over
// compact_kernel's dense `ofirst` (8 bytes per group instead of a 360-byte GroupOut
// row each; 64 lanes share the count) -- create_groups' first-appearance order --
// then lane 0 writes the group's packed record, representative / extreme /
// long-key cells and STRING bytes at that rank in pack_result_kernel's layout, into
// HBM (mail_copy_kernel then moves it into the mailbox in coalesced 16-byte stores).
constexpr uint32_t FP_T = 256, FP_W = FP_T / 64, FP_MAX = 1u << 20;
__global__ __launch_bounds__(FP_T) void finish_pack_kernel(const uint8_t* __restrict__ g, uint64_t n,
                                                           const GroupOut* __restrict__ out,
                                                           const unsigned long long* __restrict__ ofirst,
                                                           const unsigned int* __restrict__ count,
                                                           unsigned int cap_out, const FinishDesc D,
                                                           uint8_t* __restrict__ dst,
                                                           const ScanStats* __restrict__ stats,
                                                           uint8_t* __restrict__ hdr) {
    __shared__ uint4 stage[FP_W][9];
    __shared__ int16_t scols[MAX_WIDE];
    __shared__ Cell wcell[FP_W][MAX_WIDE + MAX_ACC + 1];
    const uint32_t ng = min(*count, cap_out);
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    {   // the mailbox header (host memory over PCIe): one store instruction across lanes,
        // not a serial loop of small writes the wave must drain before it ends
        constexpr uint32_t nw = (uint32_t)(sizeof(ScanStats) / 4);
        static_assert(nw + 1 <= 64, "mailbox header in one wave store");
        if (blockIdx.x == 0 && tid <= nw)
            ((uint32_t*)hdr)[tid] = tid < nw ? ((const uint32_t*)stats)[tid] : ng;
    }
    if (blockIdx.x * FP_W >= ng) return;                       // (uniform)
    for (int k = (int)tid; k < D.ncols; k += FP_T) scols[k] = D.cols[k];
    __syncthreads();
    // grid-stride over the groups, one wave each (a bounded grid: every launched wave
    // reserves the kernel's scratch, which the rare exact-strtod path needs)
    for (uint32_t i = blockIdx.x * FP_W + wv; i < ng; i += gridDim.x * FP_W) {
    const unsigned long long fi = ofirst[i];
    uint32_t r = 0;
    for (uint32_t k0 = 0; k0 < ng; k0 += 64 * 8) {      // eight loads in flight per lane
        unsigned long long f[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t k = k0 + 64u * j + lane;
            f[j] = k < ng ? ofirst[k] : ~0ull;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t k = k0 + 64u * j + lane;
            r += (k < ng) & ((f[j] < fi) | ((f[j] == fi) & (k < i)));
        }
    }
    for (int o = 32; o > 0; o >>= 1) r += (uint32_t)__shfl_xor((int)r, o, 64);
    const int nacc = D.nacc;
    const uint32_t rec = 40u + 40u * (uint32_t)nacc;
    const uint32_t ncell = (uint32_t)(D.ncols + nacc + 1);
    // the first record's bytes staged by the wave (lanes 0..8: one 16-byte load each)
    const unsigned long long fr = fi == NOPOS ? NOPOS : fi >> D.first_shift;
    const bool have = D.ncols && fr != NOPOS && fr < n;
    const uint8_t* recp = have ? g + fr : g;
    if (have && lane < 9) stage[wv][lane] = ((const uint4*)((uintptr_t)recp & ~(uintptr_t)15))[lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    Cell* wcs = wcell[wv];
    // lane 1: the row's record, extreme cells and long-key cell; lane 0: the
    // representative cells (a call: nothing of the row's is live across it)
    if (lane == 1) {
        const GroupOut& o = out[i];
        uint64_t* rp = (uint64_t*)(dst + (size_t)r * rec);
        const uint32_t cl = o.clslen;
        const uint64_t w0 = o.w0;
        rp[0] = (uint64_t)cl;
        rp[1] = w0;
        rp[2] = o.w1;
        rp[3] = o.cnt;
        rp[4] = fi;
#pragma unroll
        for (int a = 0; a < MAX_ACC; a++) {
            if (a >= nacc) break;
            const Cell e = o.ext[a];
            rp[5 + 5 * a + 0] = dbl_bits(o.sum[a]);
            rp[5 + 5 * a + 1] = o.num[a];
            rp[5 + 5 * a + 2] = ((uint64_t)e.len << 32) | e.kind;
            rp[5 + 5 * a + 3] = e.bits;
            rp[5 + 5 * a + 4] = o.extpos[a];
            wcs[D.ncols + a] = e;
        }
        Cell kc = cell_null();
        if ((cl >> 16) == GK_LONG) { kc.kind = K_STR; kc.len = cl & 0xffff; kc.bits = w0; }
        wcs[D.ncols + nacc] = kc;
    }
    if (lane == 0 && D.ncols) {
        if (have) {
            const uint8_t* tile = (const uint8_t*)stage[wv] + ((uintptr_t)recp & 15);
            parse_cols_out_staged(tile, 128, recp, scols, D.ncols, D.delim, D.quote, wcs);
        } else {
            for (int c = 0; c < D.ncols; c++) wcs[c] = cell_null();
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    // the wave stores the cells and copies the STRING bytes, one byte per lane
    Cell* cs = (Cell*)(dst + (size_t)ng * rec) + (size_t)r * ncell;
    uint8_t* db = dst + (size_t)ng * rec + (size_t)ng * ncell * sizeof(Cell) + (size_t)r * ncell * D.sb;
    for (uint32_t c = lane; c < ncell; c += 64) cs[c] = wcs[c];
    for (uint32_t c = 0; c < ncell; c++) {
        const Cell x = wcs[c];
        if (x.kind != K_STR) continue;
        const uint8_t* sp = (const uint8_t*)(uintptr_t)x.bits;
        const uint32_t m = x.len < D.sb ? x.len : D.sb;
        for (uint32_t j = lane; j < m; j += 64) db[(size_t)c * D.sb + j] = sp[j];
    }
    __builtin_amdgcn_wave_barrier();
    }
}
}  // namespace cq
}  // extern "C++"
hipError_t cq_launch_finish_pack(const uint8_t* g, uint64_t n, const cq::GroupOut* out, const unsigned long long* ofirst,
                                 const unsigned int* count, unsigned int cap_out, const cq::FinishDesc* D, uint8_t* dst,
                                 const cq::ScanStats* stats, uint8_t* hdr, hipStream_t s) {
    if (cap_out > cq::FP_MAX || D->sb % 16) return hipErrorInvalidValue;
    const unsigned quads = (cap_out + cq::FP_W - 1) / cq::FP_W;
    hipLaunchKernelGGL(cq::finish_pack_kernel, dim3(quads < 512u ? quads : 512u), dim3(cq::FP_T), 0, s, g, n,
                       out, ofirst, count, cap_out, *D, dst, stats, hdr);
    return hipGetLastError();
}
unsigned int cq_finish_pack_max() { return cq::FP_MAX; }

namespace cq {
// the packed result's records and cells, device buffer -> host-mapped mailbox in
// coalesced 16-byte lanes (pack_result_kernel's own writes are one thread per group
// at its rank: scattered 8-byte PCIe writes); the string-byte section follows
// sparsely, only a STRING's own bytes
__global__ void mail_copy_kernel(const uint4* __restrict__ src, const unsigned int* __restrict__ count,
                                 unsigned int cap_out, int nacc, uint32_t ncell, uint32_t sb, uint4* __restrict__ dst) {
    const uint32_t ng = min(*count, cap_out);
    const size_t head = (size_t)ng * (40u + 40u * (uint32_t)nacc + ncell * (uint32_t)sizeof(Cell));
    // rounded up: with an odd group count and an even accumulator count the head ends
    // 8 bytes into a 16-byte unit (the last cell's address word); the extra bytes are
    // the source's own string section, which the sparse copy below writes identically
    const size_t n16 = (head + 15) / 16;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
    const Cell* cells = (const Cell*)((const uint8_t*)src + (size_t)ng * (40u + 40u * (uint32_t)nacc));
    const uint8_t* sbytes = (const uint8_t*)src + head;
    uint8_t* dbytes = (uint8_t*)dst + head;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < (size_t)ng * ncell;
         k += (size_t)gridDim.x * blockDim.x) {
        const Cell c = cells[k];
        const uint32_t nb = c.kind == K_STR ? (min(c.len, sb) + 15u) / 16u : 0u;
        for (uint32_t w = 0; w < nb; w++) ((uint4*)(dbytes + k * sb))[w] = ((const uint4*)(sbytes + k * sb))[w];
    }
}
}  // namespace cq
hipError_t cq_launch_mail_copy(const void* src, const unsigned int* count, unsigned int cap_out, int nacc, uint32_t ncell,
                               uint32_t sb, void* dst, hipStream_t s) {
    hipLaunchKernelGGL(cq::mail_copy_kernel, dim3(64), dim3(256), 0, s, (const uint4*)src, count, cap_out, nacc, ncell,
                       sb, (uint4*)dst);
    return hipGetLastError();
}
size_t cq_pack_result_bytes(unsigned int ng, int nacc, uint32_t ncell, uint32_t sb) {
    return (size_t)ng * (40u + 40u * (uint32_t)nacc + ncell * (uint32_t)sizeof(cq::Cell) + ncell * sb);
}
hipError_t cq_launch_pack_result(const cq::GroupOut* out, const unsigned int* count, unsigned int cap_out, int nacc,
                                 const cq::Cell* cells, const uint8_t* bytes, uint32_t ncell, uint32_t sb,
                                 uint8_t* dst, const cq::ScanStats* stats, uint8_t* hdr, int order, hipStream_t s) {
    if (sb % 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cq::pack_result_kernel, dim3((cap_out + 127) / 128), dim3(128), 0, s, out, count, cap_out, nacc,
                       cells, bytes, ncell, sb, dst, stats, hdr, order);
    return hipGetLastError();
}
unsigned int cq_pack_order_max() { return cq::PACK_ORDER_MAX; }

namespace cq {
// ---- gather-merge (multi-GPU, executor.hip dist_query): this rank's groups in its
// own first-appearance order as self-contained records (no table addresses) for the
// root's merge (merge.hip gm_*).  Send buffer: a 64-byte header, then maxg records
// of gm_rec_bytes(nacc, R) (layout in plan.h GmHdr / GM_* offsets).  A group the
// format cannot carry (more than maxg groups, a representative STRING or long key
// over GM_TEXT bytes) sets the header's status to GM_DECLINE.
__global__ void gm_pack_kernel(const GroupOut* __restrict__ out, const unsigned int* __restrict__ count,
                               unsigned int cap_out, int nacc, uint32_t R, const Cell* __restrict__ cells,
                               const uint8_t* __restrict__ bytes, uint32_t sb, uint32_t maxg, uint8_t* __restrict__ dst,
                               const ScanStats* __restrict__ stats, uint8_t* __restrict__ hdr) {
    const uint32_t ng = min(*count, cap_out);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    GmHdr* H = (GmHdr*)dst;
    if (blockIdx.x == 0) {
        if (hdr) {   // the local mailbox header (statistics and group count, as pack_result)
            const uint32_t nw = (uint32_t)(sizeof(ScanStats) / 4);
            for (uint32_t k = threadIdx.x; k < nw; k += blockDim.x) ((uint32_t*)hdr)[k] = ((const uint32_t*)stats)[k];
            if (threadIdx.x == 0) *(uint32_t*)(hdr + sizeof(ScanStats)) = ng;
        }
        if (threadIdx.x == 0) {
            H->ng = min(ng, maxg);
            H->records = stats->records;
            H->passed = stats->passed;
            H->slow_records = stats->slow_records;
            H->lds_spills = stats->lds_spills;
            if (ng > maxg) atomicMax(&H->status, GM_DECLINE);
        }
    }
    if (ng > maxg) return;
    const uint32_t r = first_rank(out, ng, i);
    if (i >= ng) return;
    const uint32_t ncell = R + (uint32_t)nacc + 1;
    const GroupOut o = out[i];
    uint8_t* rp = dst + GM_HDR + (size_t)r * gm_rec_bytes(nacc, R);
    const bool longk = (o.clslen >> 16) == GK_LONG;
    ((uint32_t*)rp)[0] = o.clslen;
    ((uint32_t*)rp)[1] = 0;
    ((uint64_t*)rp)[1] = longk ? 0ull : o.w0;       // (GK_LONG: w0 is a table address; the text follows)
    ((uint64_t*)rp)[2] = o.w1;
    ((unsigned long long*)rp)[3] = o.cnt;
    ((unsigned long long*)rp)[4] = o.first;
    uint64_t* q = (uint64_t*)(rp + 40);
    for (int a = 0; a < nacc; a++) {
        q[2 * a] = dbl_bits(o.sum[a]);
        q[2 * a + 1] = o.num[a];
    }
    uint8_t* cp = rp + 40 + 16 * (uint32_t)nacc;
    for (uint32_t k = 0; k <= R; k++) {
        // representative cells, then the key text of a long key (finish_kernel's last cell)
        const uint32_t src = k < R ? k : ncell - 1;
        Cell c = cells[(size_t)i * ncell + src];
        if (k == R && !longk) c = cell_null();
        uint8_t* cc = cp + (size_t)k * GM_CELL;
        ((uint32_t*)cc)[0] = c.kind;
        ((uint32_t*)cc)[1] = c.len;
        ((uint64_t*)cc)[1] = c.kind == K_STR ? 0ull : c.bits;
        if (c.kind == K_STR) {
            if (c.len > GM_TEXT || c.len > sb) atomicMax(&H->status, GM_DECLINE);
            const uint8_t* sbs = bytes + ((size_t)i * ncell + src) * sb;
            const uint32_t nb = min(min(c.len, (uint32_t)GM_TEXT), sb);
            for (uint32_t w = 0; w < nb; w++) cc[16 + w] = sbs[w];
        }
    }
}
}  // namespace cq
hipError_t cq_launch_gm_pack(const cq::GroupOut* out, const unsigned int* count, unsigned int cap_out, int nacc,
                             uint32_t R, const cq::Cell* cells, const uint8_t* bytes, uint32_t sb, uint32_t maxg,
                             uint8_t* dst, const cq::ScanStats* stats, uint8_t* hdr, hipStream_t s) {
    hipLaunchKernelGGL(cq::gm_pack_kernel, dim3((cap_out + 127) / 128), dim3(128), 0, s, out, count, cap_out, nacc, R,
                       cells, bytes, sb, maxg, dst, stats, hdr);
    return hipGetLastError();
}
hipError_t cq_launch_finish(const uint8_t* g, uint64_t n, const cq::GroupOut* out, const unsigned int* count,
                            unsigned int cap_out, const cq::FinishDesc* D, cq::Cell* cells, uint8_t* bytes,
                            hipStream_t s) {
    hipLaunchKernelGGL(cq::finish_kernel, dim3((cap_out + cq::FINISH_T - 1) / cq::FINISH_T), dim3(cq::FINISH_T), 0, s,
                       g, n, out, count, cap_out, *D,
                       cells, bytes);
    return hipGetLastError();
}

// ---- INNER JOIN kernels (executor.hip run_join)
static unsigned grid_of(uint64_t n, unsigned b) { return (unsigned)std::max<uint64_t>(1, (n + b - 1) / b); }

hipError_t cq_launch_cells(const uint8_t* g, uint64_t tn, const unsigned long long* recs, uint32_t n,
                           const cq::ColsDesc* D, cq::Cell* out, hipStream_t s) {
    if (!n) return hipSuccess;
    if (((uintptr_t)g & 15) != 0) return hipErrorInvalidValue;     // 16-byte staged loads
    hipLaunchKernelGGL(cq::cells_kernel, dim3((n + cq::CELLS_T - 1) / cq::CELLS_T), dim3(cq::CELLS_T), 0, s, g, tn,
                       recs, n, *D, out);
    return hipGetLastError();
}
hipError_t cq_launch_join_code(const cq::Cell* cells, uint32_t stride, uint32_t kcol, uint32_t n,
                               unsigned long long* codes, uint32_t* cls, uint32_t* idx, unsigned int* per_class,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::join_code_kernel, dim3(std::min(grid_of(n, 256), 8192u)), dim3(256), 0, s, cells, stride,
                       kcol, n, codes,
                       cls, idx, per_class);
    return hipGetLastError();
}
hipError_t cq_launch_gather_codes(const unsigned long long* codes, const uint32_t* idx, uint32_t n,
                                  unsigned long long* out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::gather_codes_kernel, dim3(grid_of(n, 256)), dim3(256), 0, s, codes, idx, n, out);
    return hipGetLastError();
}
hipError_t cq_launch_join_count(const cq::Cell* L, uint32_t ls, uint32_t lk, uint32_t nL, const cq::JoinRight* J,
                                int outer_left, uint32_t* lo, unsigned long long* cnt, hipStream_t s) {
    if (!nL) return hipSuccess;
    hipLaunchKernelGGL(cq::join_count_kernel, dim3(grid_of(nL, 256)), dim3(256), 0, s, L, ls, lk, nL, *J, outer_left,
                       lo, cnt);
    return hipGetLastError();
}
hipError_t cq_launch_join_emit(const cq::Cell* L, uint32_t ls, uint32_t lk, uint32_t nL, const cq::JoinRight* J,
                               const uint32_t* lo, const unsigned long long* cnt, const unsigned long long* offs,
                               uint2* pairs, unsigned int* rmatched, hipStream_t s) {
    if (!nL) return hipSuccess;
    hipLaunchKernelGGL(cq::join_emit_kernel, dim3(grid_of(nL, 256)), dim3(256), 0, s, L, ls, lk, nL, *J, lo, cnt, offs,
                       pairs, rmatched);
    return hipGetLastError();
}
hipError_t cq_launch_join_gather(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                                 const cq::Cell* R, cq::Cell* out, hipStream_t s) {
    const unsigned long long blocks = (np + 255) / 256;
    hipLaunchKernelGGL(cq::join_gather_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, pairs, np, *M, L, R, out);
    return hipGetLastError();
}
hipError_t cq_launch_class_mask(const cq::Cell* cells, uint32_t stride, uint32_t kcol, uint32_t n, unsigned int* mask,
                                hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t grid = std::min<uint32_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(cq::class_mask_kernel, dim3(grid), dim3(256), 0, s, cells, stride, kcol, n, mask);
    return hipGetLastError();
}
hipError_t cq_launch_run_bounds(const uint32_t* ssid, uint32_t n, cq::HSlot* slots, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::run_bounds_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ssid, n, slots);
    return hipGetLastError();
}
hipError_t cq_launch_hash_build(const unsigned long long* codes, const uint32_t* cls, uint32_t n, const cq::JoinHashW* H,
                                uint32_t* sid, unsigned long long* overflow, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::hash_build_kernel, dim3((n + 255) / 256), dim3(256), 0, s, codes, cls, n, *H, sid, overflow);
    return hipGetLastError();
}
hipError_t cq_launch_join_fill(const unsigned int* flags, const unsigned int* pos, uint32_t n, unsigned long long base,
                               int right_side, uint2* pairs, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::join_fill_kernel, dim3(grid_of(n, 256)), dim3(256), 0, s, flags, pos, n, base, right_side,
                       pairs);
    return hipGetLastError();
}
hipError_t cq_launch_pair_rep_flags(const uint2* pairs, unsigned long long np, const cq::Cell* L, uint32_t ls,
                                    uint32_t lk, const cq::Cell* R, uint32_t rs, uint32_t rk, uint32_t major,
                                    unsigned int* flags, hipStream_t s) {
    if (!np) return hipSuccess;
    hipLaunchKernelGGL(cq::pair_rep_flags_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, pairs, np, L, ls,
                       lk, R, rs, rk, major, flags);
    return hipGetLastError();
}
hipError_t cq_launch_join_cross(uint32_t na, uint32_t nb, uint2* pairs, hipStream_t s) {
    const unsigned long long np = (unsigned long long)na * nb;
    if (!np) return hipSuccess;
    const unsigned grid = (unsigned)std::min<unsigned long long>((np + 255) / 256, 8192);
    hipLaunchKernelGGL(cq::join_cross_kernel, dim3(grid), dim3(256), 0, s, na, nb, np, pairs);
    return hipGetLastError();
}
hipError_t cq_launch_join_agg(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                              const cq::Cell* R, const cq::ScanPlan* P, const cq::GroupTable* gt,
                              cq::ScanStats* stats, int grouped, hipStream_t s) {
    hipError_t e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
    if (e == hipSuccess) e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_gt), gt, sizeof *gt, s);
    if (e != hipSuccess || !np) return e;
    const unsigned grid = (unsigned)std::min<uint64_t>(grid_of(np, 256), 4096);
    if (M->n > cq::MAX_NEED)
        hipLaunchKernelGGL(cq::join_agg_kernel<true>, dim3(grid), dim3(256), 0, s, pairs, np, *M, L, R, stats, grouped);
    else
        hipLaunchKernelGGL(cq::join_agg_kernel<false>, dim3(grid), dim3(256), 0, s, pairs, np, *M, L, R, stats, grouped);
    return hipGetLastError();
}
hipError_t cq_launch_comp_verify(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                                 const cq::Cell* R, const cq::ScanPlan* P, const cq::GroupTable* gt, unsigned int* bad,
                                 hipStream_t s) {
    hipError_t e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
    if (e == hipSuccess) e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_gt), gt, sizeof *gt, s);
    if (e != hipSuccess || !np) return e;
    const unsigned grid = (unsigned)std::min<uint64_t>(grid_of(np, 256), 4096);
    if (M->n > cq::MAX_NEED)
        hipLaunchKernelGGL(cq::comp_verify_kernel<true>, dim3(grid), dim3(256), 0, s, pairs, np, *M, L, R, bad);
    else
        hipLaunchKernelGGL(cq::comp_verify_kernel<false>, dim3(grid), dim3(256), 0, s, pairs, np, *M, L, R, bad);
    return hipGetLastError();
}
size_t cq_join_sum_lds(int nacc) { return (size_t)cq::JS_SLOTS * (32 + 12 * (size_t)nacc); }
hipError_t cq_launch_join_sum(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                              const cq::Cell* R, const cq::ScanPlan* P, const cq::GroupTable* gt,
                              cq::ScanStats* stats, int ncu, hipStream_t s) {
    hipError_t e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
    if (e == hipSuccess) e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_gt), gt, sizeof *gt, s);
    if (e != hipSuccess || !np) return e;
    const size_t lds = cq_join_sum_lds(P->nacc);
    const unsigned grid = (unsigned)std::min<uint64_t>(grid_of(np, 512), (uint64_t)std::max(ncu, 1) * 2);
    if (M->n > cq::MAX_NEED)
        hipLaunchKernelGGL(cq::join_sum_kernel<true>, dim3(grid), dim3(512), lds, s, pairs, np, *M, L, R, stats);
    else
        hipLaunchKernelGGL(cq::join_sum_kernel<false>, dim3(grid), dim3(512), lds, s, pairs, np, *M, L, R, stats);
    return hipGetLastError();
}
hipError_t cq_launch_join_filter(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                                 const cq::Cell* R, const cq::ScanPlan* P, unsigned int* flags, hipStream_t s) {
    hipError_t e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
    if (e != hipSuccess || !np) return e;
    if (M->n > cq::MAX_NEED)
        hipLaunchKernelGGL(cq::join_filter_kernel<true>, dim3(grid_of(np, 256)), dim3(256), 0, s, pairs, np, *M, L, R, flags);
    else
        hipLaunchKernelGGL(cq::join_filter_kernel<false>, dim3(grid_of(np, 256)), dim3(256), 0, s, pairs, np, *M, L, R, flags);
    return hipGetLastError();
}
hipError_t cq_launch_join_project(const uint2* pairs, unsigned long long np, const unsigned int* flags,
                                  const unsigned int* pos, unsigned long long lo, uint32_t m, const cq::JoinMap* M,
                                  const cq::Cell* L, const cq::Cell* R, const cq::Insn* code, const uint32_t* off,
                                  int nout, const cq::Cell* consts, cq::Cell* scratch, cq::Cell* out, hipStream_t s) {
    if (!np || !m) return hipSuccess;
    hipLaunchKernelGGL(cq::join_project_kernel, dim3(grid_of(np, 256)), dim3(256), 0, s, pairs, np, flags, pos, lo, m,
                       *M, L, R, code, off, nout, consts, scratch, out);
    return hipGetLastError();
}
hipError_t cq_launch_join_finish(const cq::GroupOut* out, const unsigned int* count, unsigned int cap_out,
                                 const uint2* pairs, const cq::JoinMap* M, const cq::Cell* L, const cq::Cell* R,
                                 int nacc, uint32_t sb, cq::Cell* cells, uint8_t* bytes, hipStream_t s) {
    hipLaunchKernelGGL(cq::join_finish_kernel, dim3(grid_of(cap_out, 128)), dim3(128), 0, s, out, count, cap_out,
                       pairs, *M, L, R, nacc, sb, cells, bytes);
    return hipGetLastError();
}

// ---- STDDEV / MEDIAN kernels (executor.hip compute_vla)
hipError_t cq_launch_vla_pair_prep(const uint2* pairs, uint32_t n, const cq::JoinMap* M, const cq::JoinMap* V,
                                   const cq::Cell* L, const cq::Cell* R, const cq::ScanPlan* P, int grouped,
                                   unsigned long long* kw0, unsigned long long* kw1, unsigned long long* kcl,
                                   unsigned long long* vkey, unsigned int* flag, hipStream_t s) {
    hipError_t e = cq::upload_symbol((const void*)&HIP_SYMBOL(cq::c_plan), P, sizeof *P, s);
    if (e != hipSuccess || !n) return e;
    if (M->n > cq::MAX_NEED)
        hipLaunchKernelGGL(cq::vla_pair_prep_kernel<true>, dim3(grid_of(n, 256)), dim3(256), 0, s, pairs, n, *M, *V, L, R,
                           grouped, kw0, kw1, kcl, vkey, flag);
    else
        hipLaunchKernelGGL(cq::vla_pair_prep_kernel<false>, dim3(grid_of(n, 256)), dim3(256), 0, s, pairs, n, *M, *V, L,
                           R, grouped, kw0, kw1, kcl, vkey, flag);
    return hipGetLastError();
}
hipError_t cq_launch_vla_prep(const cq::Cell* cells, uint32_t n, uint32_t nc, int gslot, uint32_t vslot,
                              unsigned long long* kw0, unsigned long long* kw1, unsigned long long* kcl,
                              unsigned long long* vkey, unsigned int* flag, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::vla_prep_kernel, dim3(grid_of(n, 256)), dim3(256), 0, s, cells, n, nc, gslot, vslot, kw0,
                       kw1, kcl, vkey, flag);
    return hipGetLastError();
}
hipError_t cq_launch_vla_compact(const unsigned int* flag, const unsigned int* pos, uint32_t n, unsigned int* perm,
                                 hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::vla_compact_kernel, dim3(grid_of(n, 256)), dim3(256), 0, s, flag, pos, n, perm);
    return hipGetLastError();
}
hipError_t cq_launch_vla_gather(const unsigned long long* a, const unsigned int* perm, uint32_t m,
                                unsigned long long* out, hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(cq::vla_gather_kernel, dim3(grid_of(m, 256)), dim3(256), 0, s, a, perm, m, out);
    return hipGetLastError();
}
hipError_t cq_launch_vla_heads(const unsigned long long* kw0, const unsigned long long* kw1,
                               const unsigned long long* kcl, const unsigned int* perm, uint32_t m, unsigned int* head,
                               hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(cq::vla_heads_kernel, dim3(grid_of(m, 256)), dim3(256), 0, s, kw0, kw1, kcl, perm, m, head);
    return hipGetLastError();
}
hipError_t cq_launch_vla_starts(const unsigned int* head, const unsigned int* sid, uint32_t m, unsigned int* start,
                                hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(cq::vla_starts_kernel, dim3(grid_of(m, 256)), dim3(256), 0, s, head, sid, m, start);
    return hipGetLastError();
}
hipError_t cq_launch_vla_reduce(const unsigned long long* vkey, const unsigned long long* kw0,
                                const unsigned long long* kw1, const unsigned long long* kcl, const unsigned int* perm,
                                const unsigned int* start, uint32_t nseg, uint32_t m, int kind, unsigned long long* out,
                                double* aux, hipStream_t s) {
    if (!nseg) return hipSuccess;
    hipLaunchKernelGGL(cq::vla_reduce_kernel, dim3(grid_of(nseg, 64)), dim3(64), 0, s, vkey, kw0, kw1, kcl, perm, start,
                       nseg, m, kind, out, aux);
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
