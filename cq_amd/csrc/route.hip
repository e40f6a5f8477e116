// route.hip -- join-key repartition for the multi-GPU JOIN.
//
// Each rank holds a contiguous byte range of both join inputs.  Every record is
// sent to rank (whole number key) mod N or hash(key class, key code) mod N
// (route_dest), so all records whose keys can be
// equal under value_compare (reference csv_reader.c:98-130, evaluator_joins.c:40-60)
// meet on one rank: the code is join_code (scan.hip) -- the double bits for
// INTEGER/DOUBLE (they compare as doubles), the (y, m, d) word for DATE, the FNV
// hash of the bytes for STRING, 0 for NULL.  Cross-class "equal" pairs cannot be
// routed this way; the executor refuses such inputs after the exchange.
//
// The send buffer is the records themselves (bytes up to the terminator, one
// '\n' appended), grouped by destination and in file order within a destination,
// plus one u64 global record id per record.  With a keep mask (the columns the plan
// reads from this side, executor.hip route_keep_mask) every other field is sent
// empty -- its delimiter stays, so every kept field keeps its column -- and the
// record ends after its last kept field: an empty or missing field is NULL, and the
// plan never reads those columns.  Concatenated in source-rank order the
// received records are a file-ordered subsequence of the whole input, so the local
// join's (l, r) nested-loop order is the global one restricted to this rank.
// Work is byte copying: HBM-bound, no MFMA (LDS only to stage the projection).
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {      // splitmix64 finalizer
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// A key's rank.  Numbers that are whole, non-negative and below 2^53 go to
// (value mod N): every rank then holds one residue class of the integer keys, so a
// dense key range (a primary key) stays dense with stride N on every rank and the
// STAR join indexes it directly (cqgpu_table_set_key_stride).  INTEGER 7 and DOUBLE
// 7.0 have the same code (join_code: the double bits), so they still meet.  Every
// other key (strings, dates, fractions, negatives) by a hash of (class, code).
__device__ __forceinline__ uint32_t route_dest(uint64_t code, uint32_t cls, uint32_t nranks) {
    const double v = __longlong_as_double((long long)code);
    if (cls == 1u && v >= 0.0 && v < 9007199254740992.0 && v == __builtin_floor(v))
        return (uint32_t)((uint64_t)v % nranks);
    return (uint32_t)(mix64(code ^ ((uint64_t)cls << 62)) % nranks);
}

__device__ __forceinline__ bool r_nl(uint32_t c) { return c == '\n' || c == '\r'; }
// parse_line's leading isspace skip (csv_reader.c:287) minus the terminators: scanlib.h is_blank
__device__ __forceinline__ bool r_blank(uint32_t c) { return c == ' ' || c == '\t' || c == 0x0b || c == 0x0c; }

// The record at p with only the fields of `mask` (bit c: column c; columns from 63 on
// follow bit 63) and the delimiters before the last kept one; returns its length
// with the closing '\n'; WRITE: into out (out == p allowed: bytes only move
// forward).  Field ends as parse_line finds them (csv_reader.c:278-338, scan.hip
// g_field): a quoted field runs to its closing quote (a doubled quote inside), then
// to the delimiter; a field's raw bytes (blanks, quotes) are copied as they are, so
// the receiver's parser reads the same values.
template <bool WRITE>
__device__ uint32_t project_record(const uint8_t* p, uint64_t mask, uint32_t last_keep, uint32_t delim,
                                   uint32_t quote, uint8_t* out) {
    uint32_t i = 0, o = 0;
    for (uint32_t col = 0;; col++) {
        const uint32_t s = i;
        uint32_t c = p[i];
        while (r_blank(c)) c = p[++i];
        if (!r_nl(c)) {
            if (c == quote) {
                i++;
                for (;;) {
                    c = p[i];
                    if (r_nl(c)) break;
                    if (c == quote) {
                        if (p[i + 1] == quote) { i += 2; continue; }
                        i++;
                        break;
                    }
                    i++;
                }
            }
            c = p[i];
            while (c != delim && !r_nl(c)) c = p[++i];
        }
        const bool keep = (mask >> (col < 63 ? col : 63)) & 1;
        if (keep) {
            if (WRITE)
                for (uint32_t k = s; k < i; k++) out[o + k - s] = p[k];
            o += i - s;
        }
        if (p[i] != delim || col >= last_keep) break;     // the record ends / nothing kept after
        if (WRITE) out[o] = (uint8_t)delim;
        o++;
        i++;
    }
    if (o == 0) {                                          // all kept fields empty: a lone delimiter
        if (WRITE) out[0] = (uint8_t)delim;                // keeps the record a record (an empty
        o = 1;                                             // line is none), its fields NULL
    }
    if (WRITE) out[o] = '\n';
    return o + 1;
}

// record length (through the terminator, which becomes '\n') and destination rank
__global__ void route_len_kernel(const uint8_t* __restrict__ g, const unsigned long long* __restrict__ recs,
                                 uint32_t n, const unsigned long long* __restrict__ codes,
                                 const uint32_t* __restrict__ cls, uint32_t nranks, uint32_t* __restrict__ len,
                                 uint32_t* __restrict__ dest) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // the first terminator at or after the start, 16 aligned bytes at a time (the
    // table is padded with '\n' after its end, and 256-byte aligned)
    const uint64_t st = recs[i];
    uint64_t a = st & ~15ull;
    uint32_t drop = (uint32_t)(st - a);                // bytes before the record in the first chunk
    uint64_t pos = 0;
    for (;;) {
        const uint4 v = *(const uint4*)(g + a);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t x = w[q], t1 = x ^ 0x0A0A0A0Au, t2 = x ^ 0x0D0D0D0Du;
            const uint32_t z = ~((((t1 & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t1) & (((t2 & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t2))
                               & 0x80808080u;              // 0x80 in every terminator byte
            uint32_t nb = z >> 7;
            nb |= nb >> 7;
            nb |= nb >> 14;
            m |= (nb & 0xFu) << (4 * q);
        }
        m &= 0xFFFFu << drop;
        if (m) { pos = a + (uint32_t)__builtin_ctz(m); break; }
        a += 16;
        drop = 0;
    }
    len[i] = (uint32_t)(pos - st) + 1;
    dest[i] = route_dest(codes[i], cls[i], nranks);
}

// The projected records (a keep mask: project_record), each written over its own
// source position in `proj` (a projected record is never longer than the record, so
// route_copy_kernel then moves them like whole records), their lengths and
// destination ranks (route_len_kernel's job for whole records).  One wave per 64 consecutive records: their byte span (up to the
// next record's start; `end` = the byte count, the padding '\n' ends the last) is
// staged in LDS with 16-byte loads, each lane projects its record in place there
// (forward: every byte is written at or before the byte it came from) and the wave
// stores the span back with 16-byte stores (the edge chunks, shared with the
// neighbouring waves' spans, byte by byte within the span).  A span over RP_CAP
// bytes (long records) is projected from global memory by each lane directly.
constexpr uint32_t RP_CAP = 4096;
__global__ __launch_bounds__(256) void route_project_kernel(const uint8_t* __restrict__ g,
                                                            const unsigned long long* __restrict__ recs, uint32_t n,
                                                            uint64_t end, uint64_t mask, uint32_t last_keep,
                                                            uint32_t delim, uint32_t quote,
                                                            const unsigned long long* __restrict__ codes,
                                                            const uint32_t* __restrict__ cls, uint32_t nranks,
                                                            uint32_t* __restrict__ len, uint32_t* __restrict__ dest,
                                                            uint8_t* __restrict__ proj) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[4][RP_CAP];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) & ~63ull;
    const uint64_t i = i0 + lane;
    const bool live = i0 < n;
    uint64_t a = 0, b = 0;
    if (live) {
        a = recs[i0] & ~15ull;
        b = ((i0 + 64 < n ? recs[i0 + 64] : end + 1) + 15) & ~15ull;
    }
    const bool fits = live && b - a <= RP_CAP;
    uint8_t* L = buf[w];
    if (fits)
        for (uint64_t q = a + lane * 16; q < b; q += 64 * 16) *(uint4*)(L + (q - a)) = *(const uint4*)(g + q);
    __syncthreads();
    if (i < n) {
        const uint64_t st = recs[i];
        const uint32_t m = fits ? project_record<true>(L + (st - a), mask, last_keep, delim, quote, L + (st - a))
                                : project_record<true>(g + st, mask, last_keep, delim, quote, proj + st);
        len[i] = m;
        dest[i] = route_dest(codes[i], cls[i], nranks);
    }
    __syncthreads();
    if (fits) {                                            // only [S, E): the edge chunks are shared
        const uint64_t S = recs[i0], E = i0 + 64 < n ? recs[i0 + 64] : end + 1;
        for (uint64_t q = a + lane * 16; q < b; q += 64 * 16) {
            if (q >= S && q + 16 <= E) *(uint4*)(proj + q) = *(const uint4*)(L + (q - a));
            else
                for (uint64_t k = q < S ? S : q; k < q + 16 && k < E; k++) proj[k] = L[k - a];
        }
    }
}

// per-destination record and byte starts from the destination-sorted layout
// (thread j in [0, n]: destinations in (dsorted[j-1], dsorted[j]] start at j)
__global__ void route_bounds_kernel(const uint32_t* __restrict__ dsorted, const unsigned long long* __restrict__ off,
                                    const unsigned long long* __restrict__ lens, uint32_t n, uint32_t nranks,
                                    unsigned long long* __restrict__ starts) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n) return;
    const int64_t lo = j == 0 ? -1 : (int64_t)dsorted[j - 1];
    const int64_t hi = j == n ? (int64_t)nranks - 1 : (int64_t)dsorted[j];
    const unsigned long long b = j < n ? off[j] : off[n - 1] + lens[n - 1];
    for (int64_t d = lo + 1; d <= hi; d++) {
        starts[d] = j;
        starts[nranks + 1 + d] = b;
    }
    if (j == n) {
        starts[nranks] = n;
        starts[2 * nranks + 1] = b;
    }
}

__global__ void gather_len_kernel(const uint32_t* __restrict__ len, const uint32_t* __restrict__ order, uint32_t n,
                                  unsigned long long* __restrict__ out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[j] = len[order[j]];
}

// one wave per 64 consecutive output records: each lane loads one record's
// (source, destination, length) coalesced, then the wave copies them four at a
// time, 16 lanes per record (records are ~30-40 B: two or three bytes per lane)
__global__ void route_copy_kernel(const uint8_t* __restrict__ g, const unsigned long long* __restrict__ recs,
                                  const uint32_t* __restrict__ order, const uint32_t* __restrict__ len,
                                  const unsigned long long* __restrict__ off, uint32_t n, uint64_t gid_base,
                                  uint8_t* __restrict__ out, unsigned long long* __restrict__ gids) {
    const uint64_t j0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~(uint64_t)63;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t j = j0 + lane;
    unsigned long long src = 0, dst = 0;
    uint32_t m = 0;
    if (j < n) {
        const uint32_t i = order[j];
        src = recs[i];
        dst = off[j];
        m = len[i];
        gids[j] = gid_base + i;
    }
    // four records at a time, 16 lanes each (lane k of a group moves bytes k, k + 16, ...)
    const uint32_t grp = lane >> 4, sub = lane & 15;
    for (uint32_t r = 0; r < 64; r += 4) {
        const int from = (int)(r + grp);
        const unsigned long long s = __shfl(src, from);
        const unsigned long long d = __shfl(dst, from);
        const uint32_t mm = (uint32_t)__shfl((int)m, from);     // 0 past n
        for (uint32_t k = sub; k < mm; k += 16) out[d + k] = k + 1 == mm ? (uint8_t)'\n' : g[s + k];
    }
}

// ---- the send buffer by destination runs (nranks <= 64, executor.hip route_plan).
// The send buffer is the records grouped by destination, file order within one; the
// 64 consecutive records of a wave contribute one run per destination they hold.  route_runs_kernel
// writes each (destination d, wave w) run's record and byte count at [d * nw + w]
// (destination-major: one exclusive scan of each array gives every run's send-buffer
// record and byte base), route_scatter_kernel puts each record at its run's byte base
// plus the bytes of the run's records before it, and its global id at the run's
// record base plus its rank in the run.  Every read is a file-order stream (no gather
// through a sorted order); the writes are up to nranks contiguous runs per wave.

// inclusive wave scans: 64-bit through the LDS crossbar, 32-bit by DPP row shifts /
// broadcasts (the runs' byte sums when every record of the wave is under 2^25 bytes,
// so 64 of them fit)
__device__ __forceinline__ unsigned long long wave_incl_u64(unsigned long long x, uint32_t lane) {
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_u32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
__device__ __forceinline__ unsigned long long wave_incl_len(uint32_t x, bool wide, uint32_t lane) {
    return wide ? wave_incl_u64(x, lane) : (unsigned long long)wave_incl_u32(x);
}

// dest == nranks (BCAST): the record goes to every rank (a replicated join record,
// cqgpu_route_plan2) -- it is counted in every destination's run of its wave, so each
// destination's region stays in file order
__global__ __launch_bounds__(256) void route_runs_kernel(const uint32_t* __restrict__ dest,
                                                         const uint32_t* __restrict__ len, uint32_t n, uint32_t nw,
                                                         uint32_t nranks, unsigned long long* __restrict__ rcnt,
                                                         unsigned long long* __restrict__ rbytes) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t w = (uint32_t)(i >> 6);
    if (((uint64_t)w << 6) >= n) return;                 // (a whole wave)
    const bool valid = i < n;
    const uint32_t d = valid ? dest[i] : ~0u;
    const uint32_t m = valid ? len[i] : 0u;
    const bool wide = __ballot(m >= (1u << 25)) != 0;
    if (__ballot(d == nranks) != 0) {                    // broadcast records: every destination in turn
        for (uint32_t d0 = 0; d0 < nranks; d0++) {
            const bool mine = valid && (d == d0 || d == nranks);
            const uint64_t mk = __ballot(mine);
            const unsigned long long b = wave_incl_len(mine ? m : 0u, wide, lane);
            if (lane == 63) {
                rcnt[(uint64_t)d0 * nw + w] = (unsigned long long)__popcll(mk);
                rbytes[(uint64_t)d0 * nw + w] = b;
            }
        }
        return;
    }
    bool todo = valid;
    for (;;) {                                           // one trip per destination present
        const uint64_t pend = __ballot(todo);
        if (!pend) break;
        const uint32_t d0 = (uint32_t)__shfl((int)d, (int)__builtin_ctzll(pend), 64);
        const bool mine = todo && d == d0;
        const uint64_t mk = __ballot(mine);
        const unsigned long long b = wave_incl_len(mine ? m : 0u, wide, lane);
        if (lane == 63) {
            rcnt[(uint64_t)d0 * nw + w] = (unsigned long long)__popcll(mk);
            rbytes[(uint64_t)d0 * nw + w] = b;
        }
        todo = todo && !mine;
    }
}

__global__ __launch_bounds__(256) void route_scatter_kernel(const uint8_t* __restrict__ g,
                                                            const unsigned long long* __restrict__ recs,
                                                            const uint32_t* __restrict__ dest,
                                                            const uint32_t* __restrict__ len, uint32_t n, uint32_t nw,
                                                            uint32_t nranks, uint64_t end,
                                                            const unsigned long long* __restrict__ cbase,
                                                            const unsigned long long* __restrict__ bbase,
                                                            uint64_t gid_base, uint8_t* __restrict__ out,
                                                            unsigned long long* __restrict__ gids) {
    // the wave's source span staged in LDS with 16-byte loads (route_project_kernel's
    // span: up to the next record's start; the padding '\n' ends the last record), so
    // the byte copy below reads LDS instead of waiting on HBM per record group
    __shared__ __attribute__((aligned(16))) uint8_t buf[4][RP_CAP];
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t w = (uint32_t)(i >> 6);
    const uint64_t i0 = (uint64_t)w << 6;
    const bool live = i0 < n;
    uint64_t a = 0, b = 0;
    if (live) {
        a = recs[i0] & ~15ull;
        b = ((i0 + 64 < n ? recs[i0 + 64] : end + 1) + 15) & ~15ull;
    }
    const bool fits = live && b - a <= RP_CAP;
    uint8_t* L = buf[threadIdx.x >> 6];
    if (fits)
        for (uint64_t q = a + lane * 16; q < b; q += 64 * 16) *(uint4*)(L + (q - a)) = *(const uint4*)(g + q);
    __syncthreads();
    if (!live) return;
    const bool valid = i < n;
    const uint32_t d = valid ? dest[i] : ~0u;
    const uint32_t m = valid ? len[i] : 0u;
    const unsigned long long src = valid ? recs[i] : 0ull;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const bool wide = __ballot(m >= (1u << 25)) != 0;
    const uint32_t grp = lane >> 4, sub = lane & 15;
    // four records at a time, 16 lanes each (lane k of a group moves bytes k, k + 16, ...)
    auto copy = [&](unsigned long long dst, uint32_t mlen) {
        for (uint32_t r = 0; r < 64; r += 4) {
            const int from = (int)(r + grp);
            const unsigned long long s = __shfl(src, from, 64);
            const unsigned long long t = __shfl(dst, from, 64);
            const uint32_t mm = (uint32_t)__shfl((int)mlen, from, 64);     // 0 past n / not sent
            if (fits)
                for (uint32_t k = sub; k < mm; k += 16) out[t + k] = k + 1 == mm ? (uint8_t)'\n' : L[s - a + k];
            else
                for (uint32_t k = sub; k < mm; k += 16) out[t + k] = k + 1 == mm ? (uint8_t)'\n' : g[s + k];
        }
    };
    if (__ballot(d == nranks) != 0) {                    // broadcast records: one copy per destination
        for (uint32_t d0 = 0; d0 < nranks; d0++) {
            const bool mine = valid && (d == d0 || d == nranks);
            const uint64_t mk = __ballot(mine);
            const uint32_t x = mine ? m : 0u;
            const unsigned long long pre = wave_incl_len(x, wide, lane) - x;
            unsigned long long dst = 0;
            if (mine) {
                const uint64_t at = (uint64_t)d0 * nw + w;
                dst = bbase[at] + pre;
                gids[cbase[at] + (uint64_t)__popcll(mk & below)] = gid_base + i;
            }
            copy(dst, x);
        }
        return;
    }
    unsigned long long dst = 0;
    bool todo = valid;
    for (;;) {
        const uint64_t pend = __ballot(todo);
        if (!pend) break;
        const uint32_t d0 = (uint32_t)__shfl((int)d, (int)__builtin_ctzll(pend), 64);
        const bool mine = todo && d == d0;
        const uint64_t mk = __ballot(mine);
        const uint32_t x = mine ? m : 0u;
        const unsigned long long pre = wave_incl_len(x, wide, lane) - x;
        if (mine) {
            const uint64_t at = (uint64_t)d0 * nw + w;
            dst = bbase[at] + pre;
            gids[cbase[at] + (uint64_t)__popcll(mk & below)] = gid_base + i;
        }
        todo = todo && !mine;
    }
    copy(dst, m);
}

// starts[0..nranks]: each destination's first send-buffer record (starts[nranks] = n);
// starts[nranks+1 .. 2*nranks+1]: the same in bytes (route_bounds_kernel's layout)
__global__ void route_run_starts_kernel(const unsigned long long* __restrict__ cbase,
                                        const unsigned long long* __restrict__ bbase,
                                        const unsigned long long* __restrict__ rcnt,
                                        const unsigned long long* __restrict__ rbytes, uint32_t nw, uint32_t nranks,
                                        unsigned long long* __restrict__ starts) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d > nranks) return;
    const uint64_t last = (uint64_t)nranks * nw - 1;
    starts[d] = d < nranks ? cbase[(uint64_t)d * nw] : cbase[last] + rcnt[last];
    starts[nranks + 1 + d] = d < nranks ? bbase[(uint64_t)d * nw] : bbase[last] + rbytes[last];
}

// (l, r) pair -> its position key in the reference's output order (perform_join,
// evaluator_joins.c:63-171): (global left id << 32 | global right id) for matched
// pairs, (left id << 32) for an unmatched left row (it is its row's only output),
// (2^32 - 1) << 32 | right id for an unmatched right row (appended after every
// left-driven row, in right-row order).  Ids < 2^32 - 1 (checked on the host).
constexpr uint32_t PAIR_NONE = 0xFFFFFFFFu;       // scan.hip JOIN_NONE
__global__ void pair_gid_kernel(const uint2* __restrict__ pairs, const unsigned long long* __restrict__ pidx,
                                uint32_t n, const unsigned long long* __restrict__ lg,
                                const unsigned long long* __restrict__ rg, unsigned long long* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2 pr = pairs[pidx[i]];
    const unsigned long long l = pr.x == PAIR_NONE ? 0xFFFFFFFFull : lg[pr.x];
    const unsigned long long r = pr.y == PAIR_NONE ? 0ull : rg[pr.y];
    out[i] = (l << 32) | r;
}

// the same for the pairs passing a row-returning WHERE (flags), written at their
// output positions (pos: exclusive scan of flags)
__global__ void pair_gid_flagged_kernel(const uint2* __restrict__ pairs, unsigned long long np,
                                        const unsigned int* __restrict__ flags, const unsigned int* __restrict__ pos,
                                        const unsigned long long* __restrict__ lg,
                                        const unsigned long long* __restrict__ rg, unsigned long long* __restrict__ out) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np || !flags[i]) return;
    const uint2 pr = pairs[i];
    const unsigned long long l = pr.x == PAIR_NONE ? 0xFFFFFFFFull : lg[pr.x];
    const unsigned long long r = pr.y == PAIR_NONE ? 0ull : rg[pr.y];
    out[pos[i]] = (l << 32) | r;
}

// A chain of joins across partials (process_joins, evaluator_joins.c:237-274): the
// reference's output order at level j is the order of the working row, then the
// right row (nested loops), with an outer join's unmatched right rows appended in
// right-row order.  As one 64-bit mixed-radix key: K_j = K_{j-1} * (n_j + 1) + r,
// r = n_j for a NULL right side, and K_{j-1} = S_{j-1} (one past every real key of
// the level before) for an unmatched right row; level 0's key is the global left
// record id.  The host checks that the key space S_j = (S_{j-1} + 1) * (n_j + 1)
// stays below 2^64.  prev / rg null: the row index itself.
__global__ void chain_key_kernel(const uint2* __restrict__ pairs, unsigned long long np,
                                 const unsigned long long* __restrict__ prev, unsigned long long prev_none,
                                 unsigned long long radix, const unsigned long long* __restrict__ rg,
                                 unsigned long long r_none, unsigned long long* __restrict__ out) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const uint2 pr = pairs[i];
    const unsigned long long w = pr.x == PAIR_NONE ? prev_none : (prev ? prev[pr.x] : (unsigned long long)pr.x);
    const unsigned long long r = pr.y == PAIR_NONE ? r_none : (rg ? rg[pr.y] : (unsigned long long)pr.y);
    out[i] = w * radix + r;
}

// keys of selected pairs: out[i] = key[pidx[i]], or the flagged pairs' keys at their
// output positions (pos: exclusive scan of flags)
__global__ void key_pick_kernel(const unsigned long long* __restrict__ key, const unsigned long long* __restrict__ pidx,
                                uint32_t n, unsigned long long* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = key[pidx[i]];
}
// the record holding byte offset q[i] (its start: the last record start <= q[i], by
// binary search over the file-order starts) -> its global id (routed tables) or index
__global__ void offset_gid_kernel(const unsigned long long* __restrict__ starts, unsigned long long n,
                                  const unsigned long long* __restrict__ q, uint32_t nq,
                                  const unsigned long long* __restrict__ gids, unsigned long long* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const unsigned long long o = q[i];
    unsigned long long lo = 0, hi = n;                  // first start > o
    while (lo < hi) {
        const unsigned long long mid = (lo + hi) >> 1;
        if (starts[mid] <= o) lo = mid + 1;
        else hi = mid;
    }
    const unsigned long long idx = lo ? lo - 1 : 0;
    out[i] = n == 0 ? ~0ull : (gids ? gids[idx] : idx);
}
__global__ void key_flagged_kernel(const unsigned long long* __restrict__ key, unsigned long long np,
                                   const unsigned int* __restrict__ flags, const unsigned int* __restrict__ pos,
                                   unsigned long long* __restrict__ out) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < np && flags[i]) out[pos[i]] = key[i];
}

// ---- record starts of a whole table (csv_load's line split, reference
// csv_reader.c:403-427: a record is a maximal non-empty run of bytes other than
// '\n' / '\r'; the header record ends at data_begin).  Two bandwidth passes over
// the bytes, no atomics: per-block counts, an exclusive scan, then each block
// writes its starts in file order.  Each thread owns 16 bytes; the byte before
// them comes from the previous lane (or memory: the table is padded with '\n').
constexpr uint32_t RS_T = 256;                  // threads per block
constexpr uint32_t RS_B = RS_T * 16;            // bytes per block

__device__ __forceinline__ uint32_t start_mask(const uint8_t* __restrict__ g, uint64_t p0, uint64_t lo, uint64_t n) {
    const uint4 v = *(const uint4*)(g + p0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t term = 0;                           // bit b: byte p0+b is a terminator
    for (int q = 0; q < 4; q++)
        for (int b = 0; b < 4; b++) {
            const uint32_t ch = (w[q] >> (8 * b)) & 0xff;
            term |= (uint32_t)(ch == '\n' || ch == '\r') << (4 * q + b);
        }
    const uint8_t prev = g[(int64_t)p0 - 1];
    const uint32_t prev_term = (term << 1) | (uint32_t)(prev == '\n' || prev == '\r');
    uint32_t m = ~term & prev_term & 0xffffu;
    // only positions in [lo, n)
    for (int b = 0; b < 16; b++)
        if (p0 + b < lo || p0 + b >= n) m &= ~(1u << b);
    return m;
}

__global__ void rs_count_kernel(const uint8_t* __restrict__ g, uint64_t lo, uint64_t n,
                                unsigned long long* __restrict__ counts) {
    const uint64_t p0 = (uint64_t)blockIdx.x * RS_B + threadIdx.x * 16;
    const uint32_t c = p0 < n ? (uint32_t)__popc(start_mask(g, p0, lo, n)) : 0u;
    __shared__ uint32_t part[RS_T / 64];
    uint32_t s = c;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x / 64] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (uint32_t k = 0; k < RS_T / 64; k++) t += part[k];
        counts[blockIdx.x] = t;
    }
}

__global__ void rs_write_kernel(const uint8_t* __restrict__ g, uint64_t lo, uint64_t n,
                                const unsigned long long* __restrict__ base, unsigned long long* __restrict__ out) {
    const uint64_t p0 = (uint64_t)blockIdx.x * RS_B + threadIdx.x * 16;
    const uint32_t m = p0 < n ? start_mask(g, p0, lo, n) : 0u;
    const uint32_t c = (uint32_t)__popc(m);
    // block exclusive scan of c
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x / 64;
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    __shared__ uint32_t wt[RS_T / 64];
    if (lane == 63) wt[wv] = inc;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t k = 0; k < wv; k++) before += wt[k];
    unsigned long long pos = base[blockIdx.x] + before + inc - c;
    for (uint32_t mm = m; mm; mm &= mm - 1) out[pos++] = p0 + (uint32_t)__builtin_ctz(mm);
}

// a later RIGHT / FULL level across partials (executor.hip OuterSet): unm[i] = 1 for a
// right record this rank's rows did not match -> matched_out[i] (this rank's matched
// flags), and unm[i] = 1 only for the records no rank matched (gset[i] = 0), on the
// emitting rank
__global__ void outer_global_kernel(unsigned int* __restrict__ unm, uint32_t n, const uint8_t* __restrict__ gset,
                                    uint32_t emit, uint8_t* __restrict__ matched_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned int u = unm[i];
    if (matched_out) matched_out[i] = u ? 0 : 1;
    if (gset) unm[i] = emit && !gset[i] ? 1u : 0u;
}

// cqgpu_route_plan2's destinations beyond the key routing: fixed != ~0 sends every
// record there (a JOIN without ON: the FROM side to its own rank, the JOIN side to
// every rank = nranks); rep (1-3) sends each non-NULL key of another value class to
// every rank (value_compare calls keys of different classes "equal",
// csv_reader.c:126-129, so such a record may match on any rank)
__global__ void route_dest_mode_kernel(const uint32_t* __restrict__ cls, uint32_t n, uint32_t nranks, uint32_t rep,
                                       uint32_t fixed, uint32_t* __restrict__ dest) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (fixed != ~0u) dest[i] = fixed;
    else if (rep && cls[i] && cls[i] != rep) dest[i] = nranks;
}

inline uint32_t blocks(uint64_t n, uint32_t b) { return (uint32_t)((n + b - 1) / b); }

}  // namespace

extern "C" {

hipError_t cq_launch_route_len(const uint8_t* g, const unsigned long long* recs, uint32_t n,
                               const unsigned long long* codes, const uint32_t* cls, uint32_t nranks, uint32_t* len,
                               uint32_t* dest, hipStream_t s) {
    if (!n) return hipSuccess;
    route_len_kernel<<<blocks(n, 256), 256, 0, s>>>(g, recs, n, codes, cls, nranks, len, dest);
    return hipGetLastError();
}

// starts[0..nranks]: record index where each destination begins (starts[nranks] = n);
// starts[nranks+1 .. 2*nranks+1]: the same in send-buffer bytes
hipError_t cq_launch_route_bounds(const uint32_t* dsorted, const unsigned long long* off,
                                  const unsigned long long* lens, uint32_t n, uint32_t nranks,
                                  unsigned long long* starts, hipStream_t s) {
    if (!n) return hipSuccess;
    route_bounds_kernel<<<blocks((uint64_t)n + 1, 256), 256, 0, s>>>(dsorted, off, lens, n, nranks, starts);
    return hipGetLastError();
}

// out[i] = i (the record ids of an unrouted join side)
__global__ void iota_u64_kernel(uint32_t n, unsigned long long* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}
hipError_t cq_launch_iota_u64(uint32_t n, unsigned long long* out, hipStream_t s) {
    if (!n) return hipSuccess;
    iota_u64_kernel<<<blocks(n, 256), 256, 0, s>>>(n, out);
    return hipGetLastError();
}

// stable sort of record indices by destination rank
hipError_t cq_launch_gather_len(const uint32_t* len, const uint32_t* order, uint32_t n, unsigned long long* out,
                                hipStream_t s) {
    if (!n) return hipSuccess;
    gather_len_kernel<<<blocks(n, 256), 256, 0, s>>>(len, order, n, out);
    return hipGetLastError();
}

hipError_t cq_launch_route_dest_mode(const uint32_t* cls, uint32_t n, uint32_t nranks, uint32_t rep, uint32_t fixed,
                                    uint32_t* dest, hipStream_t s) {
    if (!n) return hipSuccess;
    route_dest_mode_kernel<<<blocks(n, 256), 256, 0, s>>>(cls, n, nranks, rep, fixed, dest);
    return hipGetLastError();
}
// the typed exchange's count pass, back to the host in one copy: every destination's
// first region position (roffs[d * nw]), the last window's scan and count (the totals),
// the build side's last window base and records, and the 32-byte control block
// (flags, key range)
__global__ void typed_summary_kernel(const unsigned int* __restrict__ roffs, const unsigned int* __restrict__ rcnt,
                                     const unsigned int* __restrict__ wbase, const unsigned int* __restrict__ wcount,
                                     uint64_t nw, uint32_t nranks, const uint32_t* __restrict__ ctl,
                                     uint32_t* __restrict__ out) {
    const uint32_t t = threadIdx.x;
    const uint64_t nn = nw * nranks;
    if (t < 8) out[t] = ctl[t];
    if (t < nranks) out[8 + t] = nw ? roffs[(uint64_t)t * nw] : 0u;
    if (t == 0) {
        out[8 + nranks] = nw ? roffs[nn - 1] : 0u;
        out[9 + nranks] = nw ? rcnt[nn - 1] : 0u;
        out[10 + nranks] = nw && wbase ? wbase[nw - 1] : 0u;
        out[11 + nranks] = nw && wcount ? wcount[nw - 1] : 0u;
    }
}
hipError_t cq_launch_typed_summary(const unsigned int* roffs, const unsigned int* rcnt, const unsigned int* wbase,
                                   const unsigned int* wcount, uint64_t nw, uint32_t nranks, const uint32_t* ctl,
                                   uint32_t* out, hipStream_t s) {
    if (nranks > 64) return hipErrorInvalidValue;
    typed_summary_kernel<<<1, 64, 0, s>>>(roffs, rcnt, wbase, wcount, nw, nranks, ctl, out);
    return hipGetLastError();
}
hipError_t cq_launch_route_runs(const uint32_t* dest, const uint32_t* len, uint32_t n, uint32_t nw, uint32_t nranks,
                                unsigned long long* rcnt, unsigned long long* rbytes, hipStream_t s) {
    if (!n) return hipSuccess;
    route_runs_kernel<<<blocks((uint64_t)nw * 64, 256), 256, 0, s>>>(dest, len, n, nw, nranks, rcnt, rbytes);
    return hipGetLastError();
}
hipError_t cq_launch_route_run_starts(const unsigned long long* cbase, const unsigned long long* bbase,
                                     const unsigned long long* rcnt, const unsigned long long* rbytes, uint32_t nw,
                                     uint32_t nranks, unsigned long long* starts, hipStream_t s) {
    if (!nw || !nranks) return hipSuccess;
    route_run_starts_kernel<<<blocks((uint64_t)nranks + 1, 256), 256, 0, s>>>(cbase, bbase, rcnt, rbytes, nw, nranks,
                                                                              starts);
    return hipGetLastError();
}
hipError_t cq_launch_route_scatter(const uint8_t* g, const unsigned long long* recs, const uint32_t* dest,
                                   const uint32_t* len, uint32_t n, uint32_t nw, uint32_t nranks, uint64_t end,
                                   const unsigned long long* cbase, const unsigned long long* bbase, uint64_t gid_base,
                                   uint8_t* out, unsigned long long* gids, hipStream_t s) {
    if (!n) return hipSuccess;
    route_scatter_kernel<<<blocks((uint64_t)nw * 64, 256), 256, 0, s>>>(g, recs, dest, len, n, nw, nranks, end,
                                                                        cbase, bbase, gid_base, out, gids);
    return hipGetLastError();
}
// A fused-join partial's packed groups (scan.hip pack layout: group i's record at
// i * rec, its first pair's (left byte offset << 32) at byte 32), mapped in place
// before the mailbox copy: each offset to its record's global id (offset_gid_kernel's
// search over the file-order record starts), so the host reads ids, not offsets
__global__ void pack_first_gid_kernel(uint8_t* __restrict__ pk, const unsigned int* __restrict__ count,
                                      uint32_t cap, uint32_t rec, const unsigned long long* __restrict__ starts,
                                      unsigned long long n, const unsigned long long* __restrict__ gids) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ng = min(*count, cap);
    if (i >= ng) return;
    unsigned long long* f = (unsigned long long*)(pk + (size_t)i * rec + 32);
    const unsigned long long v = *f;
    if (v == ~0ull) return;                               // no first pair
    const unsigned long long o = v >> 32;
    unsigned long long lo = 0, hi = n;                    // first start > o
    while (lo < hi) {
        const unsigned long long mid = (lo + hi) >> 1;
        if (starts[mid] <= o) lo = mid + 1;
        else hi = mid;
    }
    const unsigned long long idx = lo ? lo - 1 : 0;
    const unsigned long long gid = n == 0 ? 0xFFFFFFFFull : (gids ? gids[idx] : idx);
    *f = (gid < 0xFFFFFFFFull ? gid : 0xFFFFFFFFull) << 32;   // (0xFFFFFFFF: out of range, the host refuses)
}
hipError_t cq_launch_pack_first_gid(uint8_t* pk, const unsigned int* count, uint32_t cap, uint32_t rec,
                                    const unsigned long long* starts, unsigned long long n,
                                    const unsigned long long* gids, hipStream_t s) {
    if (!cap) return hipSuccess;
    pack_first_gid_kernel<<<blocks(cap, 256), 256, 0, s>>>(pk, count, cap, rec, starts, n, gids);
    return hipGetLastError();
}
// the join exchange's record ids as 32 bits (every id < 2^32, checked by the caller)
__global__ void gid_narrow_kernel(const unsigned long long* __restrict__ in, uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)in[i];
}
__global__ void gid_widen_kernel(const uint32_t* __restrict__ in, uint64_t n, unsigned long long* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}
hipError_t cq_launch_gid_narrow(const unsigned long long* in, uint64_t n, uint32_t* out, hipStream_t s) {
    if (!n) return hipSuccess;
    gid_narrow_kernel<<<blocks(n, 256), 256, 0, s>>>(in, n, out);
    return hipGetLastError();
}
hipError_t cq_launch_gid_widen(const uint32_t* in, uint64_t n, unsigned long long* out, hipStream_t s) {
    if (!n) return hipSuccess;
    gid_widen_kernel<<<blocks(n, 256), 256, 0, s>>>(in, n, out);
    return hipGetLastError();
}
hipError_t cq_launch_outer_global(unsigned int* unm, uint32_t n, const uint8_t* gset, uint32_t emit, uint8_t* matched_out,
                                  hipStream_t s) {
    if (!n) return hipSuccess;
    outer_global_kernel<<<blocks(n, 256), 256, 0, s>>>(unm, n, gset, emit, matched_out);
    return hipGetLastError();
}
hipError_t cq_launch_route_project(const uint8_t* g, const unsigned long long* recs, uint32_t n, uint64_t end,
                                   uint64_t mask, uint32_t last_keep, uint32_t delim, uint32_t quote,
                                   const unsigned long long* codes, const uint32_t* cls, uint32_t nranks, uint32_t* len,
                                   uint32_t* dest, uint8_t* proj, hipStream_t s) {
    if (!n) return hipSuccess;
    route_project_kernel<<<blocks(n, 256), 256, 0, s>>>(g, recs, n, end, mask, last_keep, delim, quote, codes, cls,
                                                        nranks, len, dest, proj);
    return hipGetLastError();
}

hipError_t cq_launch_route_copy(const uint8_t* g, const unsigned long long* recs, const uint32_t* order,
                                const uint32_t* len, const unsigned long long* off, uint32_t n, uint64_t gid_base,
                                uint8_t* out, unsigned long long* gids, hipStream_t s) {
    if (!n) return hipSuccess;
    route_copy_kernel<<<blocks(n, 256), 256, 0, s>>>(g, recs, order, len, off, n, gid_base, out, gids);
    return hipGetLastError();
}

// record starts of g[lo, n) in file order: first call with out == nullptr returns
// the block count (scratch: counts/base of that many u64); see all_records
uint32_t cq_rs_blocks(uint64_t n) { return blocks(n ? n : 1, RS_B); }
hipError_t cq_launch_rs_count(const uint8_t* g, uint64_t lo, uint64_t n, unsigned long long* counts, hipStream_t s) {
    rs_count_kernel<<<cq_rs_blocks(n), RS_T, 0, s>>>(g, lo, n, counts);
    return hipGetLastError();
}
hipError_t cq_launch_rs_write(const uint8_t* g, uint64_t lo, uint64_t n, const unsigned long long* base,
                              unsigned long long* out, hipStream_t s) {
    rs_write_kernel<<<cq_rs_blocks(n), RS_T, 0, s>>>(g, lo, n, base, out);
    return hipGetLastError();
}

hipError_t cq_launch_pair_gid_flagged(const uint2* pairs, unsigned long long np, const unsigned int* flags,
                                      const unsigned int* pos, const unsigned long long* lg,
                                      const unsigned long long* rg, unsigned long long* out, hipStream_t s) {
    if (!np) return hipSuccess;
    pair_gid_flagged_kernel<<<(unsigned)((np + 255) / 256), 256, 0, s>>>(pairs, np, flags, pos, lg, rg, out);
    return hipGetLastError();
}
hipError_t cq_launch_pair_gid(const uint2* pairs, const unsigned long long* pidx, uint32_t n,
                              const unsigned long long* lg, const unsigned long long* rg, unsigned long long* out,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    pair_gid_kernel<<<blocks(n, 256), 256, 0, s>>>(pairs, pidx, n, lg, rg, out);
    return hipGetLastError();
}

hipError_t cq_launch_chain_key(const uint2* pairs, unsigned long long np, const unsigned long long* prev,
                               unsigned long long prev_none, unsigned long long radix, const unsigned long long* rg,
                               unsigned long long r_none, unsigned long long* out, hipStream_t s) {
    if (!np) return hipSuccess;
    chain_key_kernel<<<(unsigned)((np + 255) / 256), 256, 0, s>>>(pairs, np, prev, prev_none, radix, rg, r_none, out);
    return hipGetLastError();
}
hipError_t cq_launch_key_pick(const unsigned long long* key, const unsigned long long* pidx, uint32_t n,
                              unsigned long long* out, hipStream_t s) {
    if (!n) return hipSuccess;
    key_pick_kernel<<<blocks(n, 256), 256, 0, s>>>(key, pidx, n, out);
    return hipGetLastError();
}
hipError_t cq_launch_offset_gid(const unsigned long long* starts, unsigned long long n, const unsigned long long* q,
                               uint32_t nq, const unsigned long long* gids, unsigned long long* out, hipStream_t s) {
    if (!nq) return hipSuccess;
    offset_gid_kernel<<<blocks(nq, 256), 256, 0, s>>>(starts, n, q, nq, gids, out);
    return hipGetLastError();
}
hipError_t cq_launch_key_flagged(const unsigned long long* key, unsigned long long np, const unsigned int* flags,
                                 const unsigned int* pos, unsigned long long* out, hipStream_t s) {
    if (!np) return hipSuccess;
    key_flagged_kernel<<<(unsigned)((np + 255) / 256), 256, 0, s>>>(key, np, flags, pos, out);
    return hipGetLastError();
}

}  // extern "C"
