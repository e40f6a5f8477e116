// Per-step launch overhead: constant kernel inputs (the __constant__ plan and table
// descriptors, small descriptor buffers) are uploaded only when their bytes differ
// from the last upload to the same destination on the same device, and a kernel's
// dynamic-LDS attribute is set once.  Every upload and launch of the library is
// ordered on its device's one stream (executor.hip DevCtx), so a skipped upload's
// destination still holds exactly those bytes when the next launch reads it.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace cq {

struct UploadShadow {
    std::mutex mu;
    std::unordered_map<uint64_t, std::vector<uint8_t>> last;   // (device, destination) -> bytes
    std::unordered_map<uint64_t, int> lds;                      // (device, kernel) -> LDS bytes set
};
inline UploadShadow& upload_shadow() {
    static UploadShadow* S = new UploadShadow;   // never destroyed (used from static teardown)
    return *S;
}
inline uint64_t upload_key(const void* dst) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return (uint64_t)(uintptr_t)dst ^ ((uint64_t)(uint32_t)dev << 56);
}

// hipMemcpyToSymbolAsync / hipMemcpyAsync(H2D) of n bytes, skipped when unchanged
inline hipError_t upload_symbol(const void* symbol, const void* src, size_t n, hipStream_t s) {
    UploadShadow& S = upload_shadow();
    const uint64_t k = upload_key(symbol);
    std::lock_guard<std::mutex> g(S.mu);
    std::vector<uint8_t>& v = S.last[k];
    if (v.size() == n && memcmp(v.data(), src, n) == 0) return hipSuccess;
    const hipError_t e = hipMemcpyToSymbolAsync(symbol, src, n, 0, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) v.assign((const uint8_t*)src, (const uint8_t*)src + n);
    else v.clear();
    return e;
}
inline hipError_t upload_buffer(void* dst, const void* src, size_t n, hipStream_t s) {
    UploadShadow& S = upload_shadow();
    const uint64_t k = upload_key(dst);
    std::lock_guard<std::mutex> g(S.mu);
    std::vector<uint8_t>& v = S.last[k];
    if (v.size() == n && memcmp(v.data(), src, n) == 0) return hipSuccess;
    const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) v.assign((const uint8_t*)src, (const uint8_t*)src + n);
    else v.clear();
    return e;
}
// a device buffer written by other means than upload_buffer: its shadow is stale
inline void upload_forget(const void* dst) {
    UploadShadow& S = upload_shadow();
    const uint64_t k = upload_key(dst);
    std::lock_guard<std::mutex> g(S.mu);
    S.last.erase(k);
}
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per kernel and device
inline void set_max_lds(const void* fn, int bytes) {
    UploadShadow& S = upload_shadow();
    const uint64_t k = upload_key(fn);
    {
        std::lock_guard<std::mutex> g(S.mu);
        auto it = S.lds.find(k);
        if (it != S.lds.end() && it->second >= bytes) return;
    }
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess) {
        std::lock_guard<std::mutex> g(S.mu);
        S.lds[k] = bytes;
    }
}

}  // namespace cq
