// prim.hip -- device primitives owned by the executor (no library sorts or scans
// on any query path): exclusive prefix sums of u32 / u64 arrays (match counts ->
// pair offsets, pass flags -> output positions, row lengths -> byte offsets) and a
// stable LSD radix sort of u32 / u64 keys with optional u32 values (record
// offsets to file order, join rows by key slot / value class, routed records by
// destination rank, MEDIAN values per group).
//
// Scan:
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

// ------------------------------------------------------------------ radix sort
// One pass per 8-bit digit, least significant first; each pass is stable, so the
// whole sort is.  A pass: every 4,096-element tile counts its digits in LDS
// (digit-major counts[d * tiles + t]), one exclusive scan of the counts gives each
// (digit, tile) its output base, and every tile scatters its elements in order.
// Inside a tile the elements go in chunks of 256 (one per thread, in index
// order); a thread's rank among the chunk's earlier elements with its digit is
// the popcount of its wave peers below it (peers by eight ballots over the digit
// bits) plus the counts of the same digit in the lower waves of the chunk.
// HBM traffic per pass: keys (+ values) read twice, written once.
constexpr int RT = 256;
constexpr int RPT = 16;
constexpr int RTILE = RT * RPT;

template <class K>
__global__ __launch_bounds__(RT) void radix_hist_kernel(const K* __restrict__ keys, uint64_t n, int shift,
                                                        uint32_t dmask, uint32_t* __restrict__ counts,
                                                        uint32_t tiles) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b = (uint64_t)blockIdx.x * RTILE + threadIdx.x;
#pragma unroll 4
    for (int k = 0; k < RPT; k++) {
        const uint64_t i = b + (uint64_t)k * RT;
        if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & dmask], 1u);
    }
    __syncthreads();
    counts[(uint64_t)threadIdx.x * tiles + blockIdx.x] = h[threadIdx.x];
}

template <class K, bool PAIRS>
__global__ __launch_bounds__(RT) void radix_scatter_kernel(const K* __restrict__ kin, K* __restrict__ kout,
                                                           const uint32_t* __restrict__ vin, uint32_t* __restrict__ vout,
                                                           uint64_t n, int shift, uint32_t dmask,
                                                           const uint32_t* __restrict__ offs, uint32_t tiles) {
    __shared__ uint32_t run[256];
    __shared__ uint32_t wc[RT / 64][256];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    run[tid] = offs[(uint64_t)tid * tiles + blockIdx.x];
    const uint64_t below = (1ull << lane) - 1;
    for (int k = 0; k < RPT; k++) {
#pragma unroll
        for (int w = 0; w < RT / 64; w++) wc[w][tid] = 0;
        __syncthreads();
        const uint64_t i = (uint64_t)blockIdx.x * RTILE + (uint64_t)k * RT + tid;
        const bool valid = i < n;
        K key = 0;
        uint32_t val = 0, d = 0;
        if (valid) {
            key = kin[i];
            if (PAIRS) val = vin[i];
            d = (uint32_t)(key >> shift) & dmask;
        }
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const uint64_t bb = __ballot((d >> bit) & 1u);
            peers &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & below);
        if (valid && rank == 0) wc[wv][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pre = 0;
#pragma unroll
            for (int w = 0; w < RT / 64; w++) pre += w < wv ? wc[w][d] : 0u;
            const uint32_t pos = run[d] + pre + rank;
            kout[pos] = key;
            if (PAIRS) vout[pos] = val;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < RT / 64; w++) add += wc[w][tid];
        run[tid] += add;
    }
}

template <class K, bool PAIRS>
hipError_t radix_sort(void* temp, size_t* temp_bytes, const K* kin, K* kout, const uint32_t* vin, uint32_t* vout,
                      uint64_t n, int bit_lo, int bit_hi, hipStream_t st) {
    if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;            // 32-bit output positions
    const uint64_t tiles = (n + RTILE - 1) / RTILE;
    const uint64_t ncnt = tiles * 256;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t kb = al(n * sizeof(K)), vb = PAIRS ? al(n * 4) : 0, cb = al(ncnt * 4);
    const size_t sb = al(scan_scratch(ncnt) * 4);
    const size_t need = kb + vb + 2 * cb + sb + 256;
    if (!temp) { *temp_bytes = need; return hipSuccess; }
    if (*temp_bytes < need) return hipErrorInvalidValue;
    uint8_t* t = (uint8_t*)temp;
    K* kbuf = (K*)t;
    uint32_t* vbuf = (uint32_t*)(t + kb);
    uint32_t* counts = (uint32_t*)(t + kb + vb);
    uint32_t* offs = (uint32_t*)(t + kb + vb + cb);
    uint32_t* scr = (uint32_t*)(t + kb + vb + 2 * cb);
    if (n == 0) return hipSuccess;
    const int passes = bit_hi > bit_lo ? (bit_hi - bit_lo + 7) / 8 : 0;
    if (passes == 0) {
        hipError_t e = hipMemcpyAsync(kout, kin, n * sizeof(K), hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess && PAIRS) e = hipMemcpyAsync(vout, vin, n * 4, hipMemcpyDeviceToDevice, st);
        return e;
    }
    const K* ks = kin;
    const uint32_t* vs = vin;
    for (int p = 0; p < passes; p++) {
        const int shift = bit_lo + 8 * p;
        const int width = bit_hi - shift < 8 ? bit_hi - shift : 8;
        const uint32_t dmask = (1u << width) - 1;
        const bool last_to_out = ((passes - 1 - p) & 1) == 0;
        K* kd = last_to_out ? kout : kbuf;
        uint32_t* vd = last_to_out ? vout : vbuf;
        hipLaunchKernelGGL(radix_hist_kernel<K>, dim3((uint32_t)tiles), dim3(RT), 0, st, ks, n, shift, dmask, counts,
                           (uint32_t)tiles);
        hipError_t e = excl_scan<uint32_t>(counts, offs, ncnt, scr, (uint32_t*)nullptr, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((radix_scatter_kernel<K, PAIRS>), dim3((uint32_t)tiles), dim3(RT), 0, st, ks, kd, vs, vd, n,
                           shift, dmask, offs, (uint32_t)tiles);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        ks = kd;
        vs = vd;
    }
    return hipSuccess;
}

template <class T>
hipError_t excl_sum_tmp(void* temp, size_t* temp_bytes, const T* in, T* out, uint64_t n, hipStream_t st) {
    const size_t need = scan_scratch(n) * sizeof(T) + 256;
    if (!temp) { *temp_bytes = need; return hipSuccess; }
    return excl_scan<T>(in, out, n, (T*)temp, (T*)nullptr, st);
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


// ---- the executor's sorts and scans (temp == nullptr: *temp_bytes = scratch needed)
// record byte offsets to file order (row-returning SELECT, evaluator_utils.c:249-549)
hipError_t cq_sort_offsets(void* temp, size_t* temp_bytes, const unsigned long long* in, unsigned long long* out,
                           size_t n, int bits, hipStream_t s) {
    return cq::prim::radix_sort<unsigned long long, false>(temp, temp_bytes, in, out, nullptr, nullptr, n, 0, bits, s);
}
// (u64 key, u32 value) pairs by the whole key, stable
hipError_t cq_sort_codes(void* temp, size_t* temp_bytes, const unsigned long long* kin, unsigned long long* kout,
                         const unsigned int* vin, unsigned int* vout, size_t n, hipStream_t s) {
    return cq::prim::radix_sort<unsigned long long, true>(temp, temp_bytes, kin, kout, vin, vout, n, 0, 64, s);
}
// (u32 key, u32 value) pairs by the low `bits` key bits, stable (value classes, destination ranks, key slots)
hipError_t cq_sort_u32(void* temp, size_t* temp_bytes, const unsigned int* kin, unsigned int* kout,
                       const unsigned int* vin, unsigned int* vout, size_t n, int bits, hipStream_t s) {
    return cq::prim::radix_sort<unsigned int, true>(temp, temp_bytes, kin, kout, vin, vout, n, 0, bits, s);
}
hipError_t cq_sort_classes(void* temp, size_t* temp_bytes, const unsigned int* kin, unsigned int* kout,
                           const unsigned int* vin, unsigned int* vout, size_t n, hipStream_t s) {
    return cq_sort_u32(temp, temp_bytes, kin, kout, vin, vout, n, 2, s);
}
hipError_t cq_sort_dest(void* temp, size_t* temp_bytes, const unsigned int* kin, unsigned int* kout,
                        const unsigned int* vin, unsigned int* vout, size_t n, int bits, hipStream_t s) {
    return cq_sort_u32(temp, temp_bytes, kin, kout, vin, vout, n, bits, s);
}
hipError_t cq_excl_sum_u64(void* temp, size_t* temp_bytes, const unsigned long long* in, unsigned long long* out,
                           size_t n, hipStream_t s) {
    return cq::prim::excl_sum_tmp<unsigned long long>(temp, temp_bytes, in, out, n, s);
}
hipError_t cq_excl_sum_u32(void* temp, size_t* temp_bytes, const unsigned int* in, unsigned int* out, size_t n,
                           hipStream_t s) {
    return cq::prim::excl_sum_tmp<unsigned int>(temp, temp_bytes, in, out, n, s);
}

}  // extern "C"
