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

}  // namespace mg
}  // namespace cq

extern "C" {

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
