// merge.hip -- the multi-GPU GROUP BY merge on the devices (SURVEY.md section 8e,
// steps 1-4): every rank's partial groups are key records in HBM; one all_gather
// of those records (RCCL) gives every rank the same concatenation, from which
// each rank builds the same global dictionary on its device -- a key's dense id is
// the rank of its first occurrence in the concatenation -- and scatters its own
// partial state into dense per-group planes that RCCL reduces: SUM for counts,
// sums and the STDDEV moments, MIN for first-row positions, per-class first
// positions and MIN/MAX order keys.  Two mask passes then keep, per group, only the
// cells of the rank that holds the winning row (the first row for representative
// cells, the first occurrence of the extreme for MIN/MAX), so a SUM reduce
// delivers exactly those cells to rank 0, which finishes the few result rows.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "plan.h"

namespace cq {
namespace mg {

// one partial group's key (cell.h GKey without GK_LONG addresses)
struct KeyRec {
    uint32_t clslen, pad;
    uint64_t w0, w1, pad2;
};
static_assert(sizeof(KeyRec) == 32, "32-byte key records");

__device__ __forceinline__ uint64_t key_hash(const KeyRec& k) {
    return mix64(k.w0 ^ mix64(k.w1 + 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)k.clslen << 17));
}
// text keys over 16 bytes (GK_LONG = 5): w0 / w1 two content hashes, pad2 the byte
// offset of the text in the gathered key blobs; equal only when the bytes are
__device__ __forceinline__ bool key_eq(const KeyRec& a, const KeyRec& b, const uint8_t* __restrict__ text) {
    if (a.clslen != b.clslen || a.w0 != b.w0 || a.w1 != b.w1) return false;
    if ((a.clslen >> 16) != 5u) return true;
    const uint32_t n = a.clslen & 0xffffu;
    const uint8_t* x = text + a.pad2;
    const uint8_t* y = text + b.pad2;
    for (uint32_t i = 0; i < n; i++)
        if (x[i] != y[i]) return false;
    return true;
}

// every record of the concatenation into a table of distinct keys; each slot keeps
// the smallest record index holding its key (the wave-uniform loop as in
// hash_build_kernel: a claimed, unpublished slot is retried on the next trip)
__global__ void dict_build_kernel(const KeyRec* __restrict__ all, const uint8_t* __restrict__ text, uint32_t n,
                                  uint32_t* __restrict__ state,
                                  uint32_t* __restrict__ rec_of, uint32_t* __restrict__ first_of, uint32_t cap,
                                  uint32_t* __restrict__ slot_of, unsigned int* __restrict__ err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool pending = i < n;
    KeyRec k{};
    if (pending) k = all[i];
    const uint32_t mask = cap - 1;
    uint32_t s = (uint32_t)key_hash(k) & mask, probes = 0, slot = 0;
    for (uint32_t trip = 0; __any(pending); trip++) {
        if (pending) {
            uint32_t st = __hip_atomic_load(&state[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st == 0) {
                const uint32_t old = atomicCAS(&state[s], 0u, 1u);
                if (old == 0) {
                    __hip_atomic_store(&rec_of[s], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&state[s], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    slot = s;
                    pending = false;
                }
                st = old;
            }
            if (pending && st == 2) {
                const uint32_t r = __hip_atomic_load(&rec_of[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (key_eq(all[r], k, text)) {
                    slot = s;
                    pending = false;
                } else {
                    s = (s + 1) & mask;
                    if (++probes >= cap) { atomicOr(err, 1u); pending = false; }
                }
            }
        }
        if (trip > (1u << 22)) {
            if (pending) atomicOr(err, 2u);
            break;
        }
    }
    if (i < n) {
        atomicMin(&first_of[slot], i);
        slot_of[i] = slot;
    }
}

// a rank's key records as gathered: their long-text offsets are relative to the
// rank's blob, which starts `add` bytes into the concatenation
__global__ void rebase_kernel(KeyRec* __restrict__ recs, uint32_t n, uint64_t add) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && (recs[i].clslen >> 16) == 5u) recs[i].pad2 += add;
}

// 1 where record i is its key's first occurrence
__global__ void dict_flag_kernel(const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ first_of,
                                 uint32_t n, uint32_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = first_of[slot_of[i]] == i ? 1u : 0u;
}

// rows of `w` 64-bit words, every row set to `row` (the planes' identities: 0 for
// SUM words, "absent" positions for MIN words, a group's empty private state)
__global__ void fill_rows_kernel(unsigned long long* __restrict__ dst, uint64_t g, uint32_t w,
                                 const unsigned long long* __restrict__ row) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < g * w) dst[i] = row[i % w];
}

// this rank's groups (records [mine, mine + m) of the concatenation) into the dense
// planes: row d of each plane is group d's words (SUM plane W, MIN plane P, private
// plane Q; layouts in executor.hip, cqgpu_partial)
__global__ void dict_scatter_kernel(const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ first_of,
                                    const uint32_t* __restrict__ dense_of, uint32_t mine, uint32_t m,
                                    const unsigned long long* __restrict__ st_sum,
                                    const unsigned long long* __restrict__ st_min,
                                    const unsigned long long* __restrict__ st_priv, uint32_t W, uint32_t P, uint32_t Q,
                                    unsigned long long* __restrict__ dsum, unsigned long long* __restrict__ dmin,
                                    unsigned long long* __restrict__ dpriv, uint32_t* __restrict__ dense_id) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t d = dense_of[first_of[slot_of[mine + j]]];
    dense_id[j] = (uint32_t)d;
    for (uint32_t w = 0; w < W; w++) dsum[d * W + w] = st_sum[(uint64_t)j * W + w];
    for (uint32_t w = 0; w < P; w++) dmin[d * P + w] = st_min[(uint64_t)j * P + w];
    for (uint32_t w = 0; w < Q; w++) dpriv[d * Q + w] = st_priv[(uint64_t)j * Q + w];
}

constexpr unsigned long long ABSENT = 0x7FFFFFFFFFFFFFFFULL;   // above every position / key (signed MIN)

// the class of a MIN/MAX accumulator's result: the class (number, string, date)
// whose first cell comes first in the whole file (value_compare calls cells of
// different classes equal, evaluator_aggregates.c:311-326); -1 when none
__device__ __forceinline__ int win_class(const unsigned long long* __restrict__ cf) {
    int best = -1;
    for (int k = 0; k < 3; k++)
        if ((long long)cf[k] != (long long)ABSENT && (best < 0 || (long long)cf[k] < (long long)cf[best])) best = k;
    return best;
}

// after the MIN all-reduce of the MIN plane: per MIN/MAX accumulator, this rank's
// position of the winning class's extreme if its own extreme equals the global one
// (else ABSENT) -- the next MIN all-reduce picks the first occurrence
// MIN plane row: [first, per accumulator: class firsts (3), order keys (3)]
// private row:  [first, per accumulator: keys (3), positions (3), cells (3 x 2)],
//               [representative cells (R x 2)], [STDDEV n, sum, M2 (nv x 3)]
__global__ void ext_mask_kernel(const unsigned long long* __restrict__ dmin, const unsigned long long* __restrict__ dpriv,
                                uint64_t g, uint32_t P, uint32_t Q, uint32_t nmm,
                                unsigned long long* __restrict__ dext) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= g) return;
    for (uint32_t a = 0; a < nmm; a++) {
        const unsigned long long* mrow = dmin + d * P + 1 + 6 * a;
        const unsigned long long* prow = dpriv + d * Q + 1 + 12 * a;
        const int k = win_class(mrow);
        unsigned long long v = ABSENT;
        if (k >= 0 && prow[3 + k] != ABSENT && prow[k] == mrow[3 + k]) v = prow[3 + k];
        dext[d * nmm + a] = v;
    }
}

// after the extreme positions are global: the cells this rank owns (the
// representative cells of groups whose first row is here, the extreme cells whose
// first occurrence is here; zero elsewhere, so a SUM reduce delivers the owner's),
// and per STDDEV its term of the pooled squared deviations around the global mean
// (M2_r + n_r (mean_r - mean)^2; `dsum` already all-reduced)
__global__ void cell_mask_kernel(const unsigned long long* __restrict__ dmin, const unsigned long long* __restrict__ dext,
                                 const unsigned long long* __restrict__ dpriv, const double* __restrict__ dsum,
                                 uint64_t g, uint32_t P, uint32_t Q, uint32_t W, uint32_t nmm, uint32_t R, uint32_t nv,
                                 uint32_t vsum0, unsigned long long* __restrict__ dcell, double* __restrict__ dvla) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= g) return;
    const unsigned long long* prow = dpriv + d * Q;
    const uint32_t C = R + nmm;
    const bool first_here = prow[0] != ABSENT && prow[0] == dmin[d * P];
    for (uint32_t r = 0; r < R; r++) {
        const unsigned long long* pc = prow + 1 + 12 * nmm + 2 * r;
        dcell[(d * C + r) * 2] = first_here ? pc[0] : 0ull;
        dcell[(d * C + r) * 2 + 1] = first_here ? pc[1] : 0ull;
    }
    for (uint32_t a = 0; a < nmm; a++) {
        const int k = win_class(dmin + d * P + 1 + 6 * a);
        const unsigned long long* pa = prow + 1 + 12 * a;
        const bool own = k >= 0 && dext[d * nmm + a] != ABSENT && pa[3 + k] == dext[d * nmm + a];
        dcell[(d * C + R + a) * 2] = own ? pa[6 + 2 * k] : 0ull;
        dcell[(d * C + R + a) * 2 + 1] = own ? pa[7 + 2 * k] : 0ull;
    }
    for (uint32_t v = 0; v < nv; v++) {
        const unsigned long long* pv = prow + 1 + 12 * nmm + 2 * R + 3 * v;
        const double n = __longlong_as_double((long long)pv[0]);
        double t = 0.0;
        if (n > 0) {
            const double sum = __longlong_as_double((long long)pv[1]), m2 = __longlong_as_double((long long)pv[2]);
            const double gn = dsum[d * W + vsum0 + 2 * v], gs = dsum[d * W + vsum0 + 2 * v + 1];
            const double dm = sum / n - gs / gn;
            t = m2 + n * dm * dm;
        }
        dvla[d * nv + v] = t;
    }
}

// ---- gather-merge on the root (executor.hip dist_query): every rank's records
// (plan.h GM layout) side by side, rank r's at buf + r * B.  Record i = r * maxg + j
// (rank-major = file order, the ranges being ordered); a key's dense id is the rank
// of its first occurrence, which is also the group's global first-appearance order
// (create_groups, evaluator_aggregates.c:152-164), and that occurrence holds the
// group's first row -- its representative cells are the result's.
struct GmView {
    const uint8_t* buf;
    uint64_t B;          // bytes per rank
    uint32_t N, maxg, rec, nacc, R;
    __device__ __forceinline__ const GmHdr& hdr(uint32_t r) const { return *(const GmHdr*)(buf + (uint64_t)r * B); }
    __device__ __forceinline__ const uint8_t* rec_at(uint32_t r, uint32_t j) const {
        return buf + (uint64_t)r * B + GM_HDR + (uint64_t)j * rec;
    }
    __device__ __forceinline__ const uint8_t* key_text(const uint8_t* rp) const {
        return rp + 40 + 16 * nacc + (uint64_t)R * GM_CELL + 16;
    }
};
__device__ __forceinline__ bool gm_key_eq(const GmView& V, const uint8_t* a, const uint8_t* b) {
    const uint32_t ca = *(const uint32_t*)a, cb = *(const uint32_t*)b;
    if (ca != cb || ((const uint64_t*)a)[1] != ((const uint64_t*)b)[1] || ((const uint64_t*)a)[2] != ((const uint64_t*)b)[2])
        return false;
    if ((ca >> 16) != 5u) return true;                              // GK_LONG: the bytes
    const uint32_t n = ca & 0xffffu;
    const uint8_t* x = V.key_text(a);
    const uint8_t* y = V.key_text(b);
    for (uint32_t k = 0; k < n; k++)
        if (x[k] != y[k]) return false;
    return true;
}

__global__ void gm_dict_kernel(GmView V, uint32_t* __restrict__ state, uint32_t* __restrict__ rec_of,
                               uint32_t* __restrict__ first_of, uint32_t cap, uint32_t* __restrict__ slot_of,
                               unsigned int* __restrict__ err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = V.N * V.maxg;
    const uint32_t r = i / V.maxg, j = i - r * V.maxg;
    bool pending = i < T && j < min(V.hdr(r).ng, V.maxg);
    const bool valid = pending;
    const uint8_t* rp = pending ? V.rec_at(r, j) : nullptr;
    uint64_t h = 0;
    if (pending)
        h = mix64(((const uint64_t*)rp)[1] ^ mix64(((const uint64_t*)rp)[2] + 0x9E3779B97F4A7C15ULL) ^
                  ((uint64_t)*(const uint32_t*)rp << 17));
    const uint32_t mask = cap - 1;
    uint32_t s = (uint32_t)h & mask, probes = 0, slot = 0;
    for (uint32_t trip = 0; __any(pending); trip++) {
        if (pending) {
            uint32_t st = __hip_atomic_load(&state[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st == 0) {
                const uint32_t old = atomicCAS(&state[s], 0u, 1u);
                if (old == 0) {
                    __hip_atomic_store(&rec_of[s], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&state[s], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    slot = s;
                    pending = false;
                }
                st = old;
            }
            if (pending && st == 2) {
                const uint32_t o = __hip_atomic_load(&rec_of[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t orr = o / V.maxg;
                if (gm_key_eq(V, V.rec_at(orr, o - orr * V.maxg), rp)) {
                    slot = s;
                    pending = false;
                } else {
                    s = (s + 1) & mask;
                    if (++probes >= cap) { atomicOr(err, 1u); pending = false; }
                }
            }
        }
        if (trip > (1u << 22)) {
            if (pending) atomicOr(err, 2u);
            break;
        }
    }
    if (valid) {
        atomicMin(&first_of[slot], i);
        slot_of[i] = slot;
    }
}

// 1 where record i is its key's first occurrence (0 for the empty record slots)
__global__ void gm_flag_kernel(GmView V, const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ first_of,
                               uint32_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = V.N * V.maxg;
    if (i >= T) return;
    const uint32_t r = i / V.maxg, j = i - r * V.maxg;
    flag[i] = (j < min(V.hdr(r).ng, V.maxg) && first_of[slot_of[i]] == i) ? 1u : 0u;
}

// idx[r * T + d] = j: rank r's record of dense group d
__global__ void gm_scatter_kernel(GmView V, const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ first_of,
                                  const uint32_t* __restrict__ dense, uint32_t* __restrict__ idx) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = V.N * V.maxg;
    if (i >= T) return;
    const uint32_t r = i / V.maxg, j = i - r * V.maxg;
    if (j >= min(V.hdr(r).ng, V.maxg)) return;
    idx[(uint64_t)r * T + dense[first_of[slot_of[i]]]] = j;
}

// one thread per dense group (its first occurrence h): COUNT / SUM / numeric counts
// added over the ranks in rank order (a fixed order: the same sums every run), the
// representative cells and first row (made whole-file) from the first occurrence;
// written in pack_result_kernel's layout (executor.hip build_direct reads it).  The
// header of `mail` gets the summed statistics, the group count and the status.
__global__ void gm_combine_kernel(GmView V, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ dense,
                                  const uint32_t* __restrict__ idx, int grouped, uint32_t sb, uint8_t* __restrict__ dst,
                                  unsigned int* __restrict__ gcount, uint8_t* __restrict__ mail,
                                  const unsigned int* __restrict__ err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t T = V.N * V.maxg;
    uint32_t status = *err ? GM_FAILED : GM_OK;
    for (uint32_t r = 0; r < V.N; r++) status = max(status, V.hdr(r).status);
    uint32_t G = T ? dense[T - 1] + flag[T - 1] : 0u;
    const bool zero = !grouped && G == 0;                 // no row anywhere: the one empty group
    if (zero) G = 1;
    const uint32_t nacc = V.nacc, R = V.R, ncell = R + nacc + 1;
    const uint32_t orec = 40u + 40u * nacc;
    if (i == 0) {
        ScanStats st;
        memset(&st, 0, sizeof st);
        for (uint32_t r = 0; r < V.N; r++) {
            st.records += V.hdr(r).records;
            st.passed += V.hdr(r).passed;
            st.slow_records += V.hdr(r).slow_records;
            st.lds_spills += V.hdr(r).lds_spills;
        }
        memcpy(mail, &st, sizeof st);
        *(uint32_t*)(mail + sizeof(ScanStats)) = status == GM_OK ? G : 0u;
        *(uint32_t*)(mail + sizeof(ScanStats) + 4) = status;
        gcount[0] = status == GM_OK ? G : 0u;
        gcount[1] = status;
    }
    if (status != GM_OK) return;
    uint32_t d = 0, hr = 0, hj = 0;
    if (zero) {
        if (i != 0) return;
    } else {
        if (i >= T || !flag[i]) return;
        d = dense[i];
        hr = i / V.maxg;
        hj = i - hr * V.maxg;
    }
    uint8_t* op = dst + (uint64_t)d * orec;
    Cell* oc = (Cell*)(dst + (uint64_t)G * orec) + (uint64_t)d * ncell;
    uint8_t* ob = dst + (uint64_t)G * orec + (uint64_t)G * ncell * sizeof(Cell) + (uint64_t)d * ncell * sb;
    uint64_t* oq = (uint64_t*)(op + 40);
    if (zero) {
        ((uint32_t*)op)[0] = (uint32_t)GK_ALL << 16;
        ((uint32_t*)op)[1] = 0;
        ((uint64_t*)op)[1] = 0;
        ((uint64_t*)op)[2] = 0;
        ((unsigned long long*)op)[3] = 0;
        ((unsigned long long*)op)[4] = ~0ull;
        for (uint32_t a = 0; a < nacc; a++) {
            oq[5 * a] = 0; oq[5 * a + 1] = 0; oq[5 * a + 2] = 0; oq[5 * a + 3] = 0; oq[5 * a + 4] = ~0ull;
        }
        for (uint32_t k = 0; k < ncell; k++) oc[k] = cell_null();
        return;
    }
    const uint8_t* hp = V.rec_at(hr, hj);
    unsigned long long cnt = 0;
    for (uint32_t r = 0; r < V.N; r++) {
        const uint32_t j = idx[(uint64_t)r * T + d];
        if (j == 0xFFFFFFFFu) continue;
        const uint8_t* rp = V.rec_at(r, j);
        cnt += ((const unsigned long long*)rp)[3];
    }
    ((uint32_t*)op)[0] = *(const uint32_t*)hp;
    ((uint32_t*)op)[1] = 0;
    ((uint64_t*)op)[1] = ((const uint64_t*)hp)[1];
    ((uint64_t*)op)[2] = ((const uint64_t*)hp)[2];
    ((unsigned long long*)op)[3] = cnt;
    const unsigned long long f = ((const unsigned long long*)hp)[4];
    ((unsigned long long*)op)[4] = f == ~0ull ? ~0ull : f + V.hdr(hr).base;
    for (uint32_t a = 0; a < nacc; a++) {
        double sum = 0.0;
        unsigned long long num = 0;
        for (uint32_t r = 0; r < V.N; r++) {
            const uint32_t j = idx[(uint64_t)r * T + d];
            if (j == 0xFFFFFFFFu) continue;
            const uint64_t* q = (const uint64_t*)(V.rec_at(r, j) + 40);
            if (q[2 * a + 1]) {
                sum += __longlong_as_double((long long)q[2 * a]);
                num += q[2 * a + 1];
            }
        }
        oq[5 * a] = (uint64_t)__double_as_longlong(sum);
        oq[5 * a + 1] = num;
        oq[5 * a + 2] = 0;
        oq[5 * a + 3] = 0;
        oq[5 * a + 4] = ~0ull;
    }
    // cells: [R representative][nacc extremes (none here)][the key text]
    const uint8_t* hc = hp + 40 + 16 * nacc;
    for (uint32_t k = 0; k < ncell; k++) {
        Cell c = cell_null();
        const uint8_t* cc = nullptr;
        if (k < R) cc = hc + (uint64_t)k * GM_CELL;
        else if (k == ncell - 1) cc = hc + (uint64_t)R * GM_CELL;
        if (cc) {
            c.kind = ((const uint32_t*)cc)[0];
            c.len = ((const uint32_t*)cc)[1];
            c.bits = ((const uint64_t*)cc)[1];
            if (c.kind == K_STR) {
                const uint32_t nb = min(c.len, sb);
                for (uint32_t w = 0; w < nb; w++) ob[(uint64_t)k * sb + w] = cc[16 + w];
            }
        }
        oc[k] = c;
    }
}

}  // namespace mg
}  // namespace cq

extern "C" {

hipError_t cq_excl_sum_u32(void* temp, size_t* temp_bytes, const unsigned int* in, unsigned int* out, size_t n,
                           hipStream_t s);

// the root's whole gather-merge: dictionary, dense ids, per-rank index, combine.
// state / first_of (cap slots) and idx (N * N * maxg words) must hold 0 / 0xFF bytes
// on entry (cq_gm_merge_scratch sizes them); err zero
size_t cq_gm_scan_bytes(uint32_t T) {
    size_t tb = 0;
    (void)cq_excl_sum_u32(nullptr, &tb, nullptr, nullptr, T, nullptr);   // (a size query)
    return tb;
}
hipError_t cq_launch_gm_merge(const uint8_t* buf, uint64_t B, uint32_t N, uint32_t maxg, int nacc, uint32_t R,
                              int grouped, uint32_t sb, uint32_t* state, uint32_t* rec_of, uint32_t* first_of, uint32_t cap,
                              uint32_t* slot_of, uint32_t* flag, uint32_t* dense, uint32_t* idx, void* scan_temp,
                              size_t scan_temp_bytes, unsigned int* err, uint8_t* dst, unsigned int* gcount,
                              uint8_t* mail, hipStream_t s) {
    cq::mg::GmView V{buf, B, N, maxg, cq::gm_rec_bytes(nacc, R), (uint32_t)nacc, R};
    const uint32_t T = N * maxg;
    const unsigned g = (T + 255) / 256;
    hipLaunchKernelGGL(cq::mg::gm_dict_kernel, dim3(g), dim3(256), 0, s, V, state, rec_of, first_of, cap, slot_of, err);
    hipLaunchKernelGGL(cq::mg::gm_flag_kernel, dim3(g), dim3(256), 0, s, V, slot_of, first_of, flag);
    size_t tb = scan_temp_bytes;
    hipError_t e = cq_excl_sum_u32(scan_temp, &tb, flag, dense, T, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cq::mg::gm_scatter_kernel, dim3(g), dim3(256), 0, s, V, slot_of, first_of, dense, idx);
    hipLaunchKernelGGL(cq::mg::gm_combine_kernel, dim3(g), dim3(256), 0, s, V, flag, dense, idx, grouped, sb, dst, gcount,
                       mail, err);
    return hipGetLastError();
}

hipError_t cq_launch_dict_build(const void* all, const void* text, uint32_t n, uint32_t* state, uint32_t* rec_of,
                                uint32_t* first_of, uint32_t cap, uint32_t* slot_of, unsigned int* err, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::dict_build_kernel, dim3((n + 255) / 256), dim3(256), 0, s,
                       (const cq::mg::KeyRec*)all, (const uint8_t*)text, n, state, rec_of, first_of, cap, slot_of, err);
    return hipGetLastError();
}
hipError_t cq_launch_rebase(void* recs, uint32_t n, uint64_t add, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::rebase_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (cq::mg::KeyRec*)recs, n, add);
    return hipGetLastError();
}
hipError_t cq_launch_dict_flag(const uint32_t* slot_of, const uint32_t* first_of, uint32_t n, uint32_t* flag,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::dict_flag_kernel, dim3((n + 255) / 256), dim3(256), 0, s, slot_of, first_of, n, flag);
    return hipGetLastError();
}
hipError_t cq_launch_fill_rows(unsigned long long* dst, uint64_t g, uint32_t w, const unsigned long long* row,
                               hipStream_t s) {
    if (!g || !w) return hipSuccess;
    const uint64_t n = g * w;
    hipLaunchKernelGGL(cq::mg::fill_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dst, g, w, row);
    return hipGetLastError();
}
hipError_t cq_launch_dict_scatter(const uint32_t* slot_of, const uint32_t* first_of, const uint32_t* dense_of,
                                  uint32_t mine, uint32_t m, const unsigned long long* st_sum,
                                  const unsigned long long* st_min, const unsigned long long* st_priv, uint32_t W,
                                  uint32_t P, uint32_t Q, unsigned long long* dsum, unsigned long long* dmin,
                                  unsigned long long* dpriv, uint32_t* dense_id, hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::dict_scatter_kernel, dim3((m + 255) / 256), dim3(256), 0, s, slot_of, first_of, dense_of,
                       mine, m, st_sum, st_min, st_priv, W, P, Q, dsum, dmin, dpriv, dense_id);
    return hipGetLastError();
}
hipError_t cq_launch_ext_mask(const unsigned long long* dmin, const unsigned long long* dpriv, uint64_t g, uint32_t P,
                              uint32_t Q, uint32_t nmm, unsigned long long* dext, hipStream_t s) {
    if (!g || !nmm) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::ext_mask_kernel, dim3((unsigned)((g + 255) / 256)), dim3(256), 0, s, dmin, dpriv, g, P, Q,
                       nmm, dext);
    return hipGetLastError();
}
hipError_t cq_launch_cell_mask(const unsigned long long* dmin, const unsigned long long* dext,
                               const unsigned long long* dpriv, const double* dsum, uint64_t g, uint32_t P, uint32_t Q,
                               uint32_t W, uint32_t nmm, uint32_t R, uint32_t nv, uint32_t vsum0,
                               unsigned long long* dcell, double* dvla, hipStream_t s) {
    if (!g) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::cell_mask_kernel, dim3((unsigned)((g + 255) / 256)), dim3(256), 0, s, dmin, dext, dpriv,
                       dsum, g, P, Q, W, nmm, R, nv, vsum0, dcell, dvla);
    return hipGetLastError();
}

}  // extern "C"
