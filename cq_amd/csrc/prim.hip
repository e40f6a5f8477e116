// prim.hip -- device primitives owned by the executor: exclusive prefix sums of
// u32 / u64 arrays (match counts -> pair offsets, pass flags -> output positions,
// formatted-row lengths -> byte offsets).
//
// Three launches per level: every 2,048-element tile is reduced by one 256-thread
// block, the tile sums are scanned (recursively when there are more than a tile's
// worth), and every tile is scanned again with its base added.  Inside a block a
// thread owns 8 consecutive elements; the 256 per-thread totals are scanned with
// wave64 shuffles and one LDS round for the four wave totals.  HBM traffic: the
// input read twice, the output written once.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace cq {
namespace prim {

constexpr int ST = 256;            // threads per block
constexpr int SE = 8;              // elements per thread
constexpr int TILE = ST * SE;      // elements per block

template <class T>
__device__ __forceinline__ T wave_incl(T x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// exclusive scan of one value per thread over the block; *total = block sum
template <class T>
__device__ __forceinline__ T block_excl(T x, T* total) {
    __shared__ T wsum[ST / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const T inc = wave_incl(x);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    T base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < ST / 64; w++) {
        const T s = wsum[w];
        base += w < wv ? s : (T)0;
        all += s;
    }
    __syncthreads();                     // wsum is reused by the next call
    *total = all;
    return base + inc - x;
}

template <class T>
__global__ __launch_bounds__(ST) void tile_sum_kernel(const T* __restrict__ in, uint64_t n, T* __restrict__ sums) {
    const uint64_t b0 = (uint64_t)blockIdx.x * TILE + (uint64_t)threadIdx.x * SE;
    T s = 0;
#pragma unroll
    for (int k = 0; k < SE; k++)
        if (b0 + k < n) s += in[b0 + k];
    T total;
    (void)block_excl(s, &total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// base: exclusive prefix of the tile sums (nullptr: one tile, base 0)
template <class T>
__global__ __launch_bounds__(ST) void tile_scan_kernel(const T* __restrict__ in, uint64_t n,
                                                       const T* __restrict__ base, T* __restrict__ out,
                                                       T* __restrict__ total_out) {
    const uint64_t b0 = (uint64_t)blockIdx.x * TILE + (uint64_t)threadIdx.x * SE;
    T v[SE];
    T s = 0;
#pragma unroll
    for (int k = 0; k < SE; k++) {
        v[k] = b0 + k < n ? in[b0 + k] : (T)0;
        s += v[k];
    }
    T total;
    T run = block_excl(s, &total) + (base ? base[blockIdx.x] : (T)0);
#pragma unroll
    for (int k = 0; k < SE; k++) {
        if (b0 + k < n) out[b0 + k] = run;
        run += v[k];
    }
    if (total_out && blockIdx.x == gridDim.x - 1 && threadIdx.x == ST - 1) *total_out = run;
}

inline uint64_t tiles_of(uint64_t n) { return (n + TILE - 1) / TILE; }

// scratch elements the scan of n elements needs (the tile sums of every level)
inline uint64_t scan_scratch(uint64_t n) {
    uint64_t s = 0;
    for (uint64_t t = tiles_of(n); t > 1; t = tiles_of(t)) s += 2 * t;
    return s + 2;
}

template <class T>
hipError_t excl_scan(const T* in, T* out, uint64_t n, T* scratch, T* total, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t t = tiles_of(n);
    if (t > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (t == 1) {
        hipLaunchKernelGGL(tile_scan_kernel<T>, dim3(1), dim3(ST), 0, st, in, n, (const T*)nullptr, out, total);
        return hipGetLastError();
    }
    T* sums = scratch;
    T* bases = scratch + t;
    hipLaunchKernelGGL(tile_sum_kernel<T>, dim3((uint32_t)t), dim3(ST), 0, st, in, n, sums);
    hipError_t e = excl_scan<T>(sums, bases, t, scratch + 2 * t, (T*)nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tile_scan_kernel<T>, dim3((uint32_t)t), dim3(ST), 0, st, in, n, (const T*)bases, out, total);
    return hipGetLastError();
}

}  // namespace prim
}  // namespace cq

extern "C" {

// scratch bytes for cq_scan_u64 / cq_scan_u32 of n elements
size_t cq_scan_scratch_bytes(uint64_t n, int elem_bytes) { return cq::prim::scan_scratch(n) * (size_t)elem_bytes; }

// out[i] = in[0] + ... + in[i - 1]; *total (device, optional) = the sum of all
hipError_t cq_scan_u64(const unsigned long long* in, unsigned long long* out, uint64_t n, void* scratch,
                       unsigned long long* total, hipStream_t s) {
    return cq::prim::excl_scan<unsigned long long>(in, out, n, (unsigned long long*)scratch, total, s);
}
hipError_t cq_scan_u32(const unsigned int* in, unsigned int* out, uint64_t n, void* scratch, unsigned int* total,
                       hipStream_t s) {
    return cq::prim::excl_scan<unsigned int>(in, out, n, (unsigned int*)scratch, total, s);
}

}  // extern "C"
