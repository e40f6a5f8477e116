// merge.hip -- the multi-GPU GROUP BY merge on the devices (SURVEY.md section 8e,
// steps 1-4): every rank's partial groups are key records in HBM; one all_gather
// of those records (RCCL) gives every rank the same concatenation, from which
// each rank builds the same global dictionary on its device -- a key's dense id is
// the rank of its first occurrence in the concatenation -- and scatters its own
// partial state into dense arrays that RCCL reduces: SUM for counts and sums, MIN
// for first-row positions.  Rank 0 finishes the few result rows.
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
__device__ __forceinline__ bool key_eq(const KeyRec& a, const KeyRec& b) {
    return a.clslen == b.clslen && a.w0 == b.w0 && a.w1 == b.w1;
}

// every record of the concatenation into a table of distinct keys; each slot keeps
// the smallest record index holding its key (the wave-uniform loop as in
// hash_build_kernel: a claimed, unpublished slot is retried on the next trip)
__global__ void dict_build_kernel(const KeyRec* __restrict__ all, uint32_t n, uint32_t* __restrict__ state,
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
                if (key_eq(all[r], k)) {
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

// 1 where record i is its key's first occurrence
__global__ void dict_flag_kernel(const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ first_of,
                                 uint32_t n, uint32_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = first_of[slot_of[i]] == i ? 1u : 0u;
}

// this rank's groups (records [mine, mine + m) of the concatenation) into the dense
// arrays: dsum[d * W + 0] = COUNT, [1 + 2a] = SUM_a, [2 + 2a] = numeric count_a (as
// doubles: exact below 2^53); dfirst[d]; drep[2d] = representative cell kind,
// [2d + 1] = its payload bits
__global__ void dict_scatter_kernel(const uint32_t* __restrict__ slot_of, const uint32_t* __restrict__ first_of,
                                    const uint32_t* __restrict__ dense_of, uint32_t mine, uint32_t m,
                                    const double* __restrict__ st_sum, const unsigned long long* __restrict__ st_first,
                                    const unsigned long long* __restrict__ st_rep, uint32_t W,
                                    double* __restrict__ dsum, unsigned long long* __restrict__ dfirst,
                                    unsigned long long* __restrict__ drep) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t d = dense_of[first_of[slot_of[mine + j]]];
    for (uint32_t w = 0; w < W; w++) dsum[(uint64_t)d * W + w] = st_sum[(uint64_t)j * W + w];
    dfirst[d] = st_first[j];
    drep[2 * (uint64_t)d] = st_rep[2 * (uint64_t)j];
    drep[2 * (uint64_t)d + 1] = st_rep[2 * (uint64_t)j + 1];
}

// after the MIN all-reduce of the first positions: only the rank holding a group's
// first row keeps its representative cell, so a SUM reduce delivers exactly it
__global__ void rep_mask_kernel(const unsigned long long* __restrict__ mine, const unsigned long long* __restrict__ global,
                                uint32_t g, unsigned long long* __restrict__ drep) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < g && mine[d] != global[d]) {
        drep[2 * (uint64_t)d] = 0;
        drep[2 * (uint64_t)d + 1] = 0;
    }
}

}  // namespace mg
}  // namespace cq

extern "C" {

hipError_t cq_launch_dict_build(const void* all, uint32_t n, uint32_t* state, uint32_t* rec_of, uint32_t* first_of,
                                uint32_t cap, uint32_t* slot_of, unsigned int* err, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::dict_build_kernel, dim3((n + 255) / 256), dim3(256), 0, s,
                       (const cq::mg::KeyRec*)all, n, state, rec_of, first_of, cap, slot_of, err);
    return hipGetLastError();
}
hipError_t cq_launch_dict_flag(const uint32_t* slot_of, const uint32_t* first_of, uint32_t n, uint32_t* flag,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::dict_flag_kernel, dim3((n + 255) / 256), dim3(256), 0, s, slot_of, first_of, n, flag);
    return hipGetLastError();
}
hipError_t cq_launch_dict_scatter(const uint32_t* slot_of, const uint32_t* first_of, const uint32_t* dense_of,
                                  uint32_t mine, uint32_t m, const double* st_sum, const unsigned long long* st_first,
                                  const unsigned long long* st_rep, uint32_t W, double* dsum,
                                  unsigned long long* dfirst, unsigned long long* drep, hipStream_t s) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::dict_scatter_kernel, dim3((m + 255) / 256), dim3(256), 0, s, slot_of, first_of, dense_of,
                       mine, m, st_sum, st_first, st_rep, W, dsum, dfirst, drep);
    return hipGetLastError();
}
hipError_t cq_launch_rep_mask(const unsigned long long* mine, const unsigned long long* global, uint32_t g,
                              unsigned long long* drep, hipStream_t s) {
    if (!g) return hipSuccess;
    hipLaunchKernelGGL(cq::mg::rep_mask_kernel, dim3((g + 255) / 256), dim3(256), 0, s, mine, global, g, drep);
    return hipGetLastError();
}

}  // extern "C"
