// Issue cost (SIMD cycles per wave64 instruction, 8 and 16 waves per CU) of more of
// the integer instructions the scan kernels use; each loop step is exactly one
// instruction (inline asm), 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define K(NAME, ASM, CON)                                                                             \
    __global__ void __launch_bounds__(1024) NAME(uint32_t* out, uint32_t seed, int iters) {           \
        uint32_t a[8];                                                                                \
        for (int i = 0; i < 8; i++) a[i] = seed ^ (threadIdx.x * (i + 3));                            \
        const uint32_t c = seed | 1;                                                                  \
        for (int i = 0; i < iters; i++) {                                                             \
            _Pragma("unroll") for (int j = 0; j < 16; j++) {                                          \
                _Pragma("unroll") for (int q = 0; q < 8; q++) asm volatile(ASM : "+v"(a[q]) : CON(c)); \
            }                                                                                         \
        }                                                                                             \
        uint32_t x = 0;                                                                               \
        for (int i = 0; i < 8; i++) x ^= a[i];                                                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                               \
    }
#define VC(c) "v"(c)
#define SC(c) "s"(c)
K(k_cndmask, "v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc", VC)    // 2 insts
K(k_bfe, "v_bfe_u32 %0, %0, 3, %1", VC)
K(k_bcnt, "v_bcnt_u32_b32 %0, %0, %1", VC)
K(k_umul24, "v_mul_u32_u24 %0, %0, %1", VC)
K(k_mullo, "v_mul_lo_u32 %0, %0, %1", VC)
K(k_min3, "v_min3_u32 %0, %0, %1, %0", VC)
K(k_lshlor, "v_lshl_or_b32 %0, %0, 3, %1", VC)
K(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 1", VC)
K(k_ffbh, "v_ffbh_u32 %0, %0", VC)
K(k_add3, "v_add3_u32 %0, %0, %1, %0", VC)
K(k_xor_sgpr, "v_xor_b32 %0, %1, %0", SC)
K(k_xor_v, "v_xor_b32 %0, %0, %1", VC)
K(k_add_v, "v_add_u32 %0, %0, %1", VC)
K(k_perm_v, "v_perm_b32 %0, %1, %0, %0", VC)
K(k_bitop3_v, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96", VC)
K(k_and_v, "v_and_b32 %0, %0, %1", VC)
K(k_xor_lit, "v_xor_b32 %0, 0x30303030, %0", VC)
K(k_add_inl, "v_add_u32 %0, 5, %0", VC)
K(k_shr_inl, "v_lshrrev_b32 %0, 3, %0", VC)
K(k_shr_v, "v_lshrrev_b32 %0, %1, %0", VC)
K(k_or_v, "v_or_b32 %0, %0, %1", VC)
K(k_sub_v, "v_sub_u32 %0, %0, %1", VC)
K(k_cndmask_v, "v_cndmask_b32 %0, %0, %1, vcc", VC)
K(k_cmp_v, "v_cmp_gt_u32 vcc, %0, %1\n\tv_xor_b32 %0, %0, %1", VC)
K(k_mov_v, "v_mov_b32 %0, %1", VC)
K(k_lshladd_inl, "v_lshl_add_u32 %0, %0, 3, %1", VC)
K(k_bitop3_s, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96", SC)
K(k_cndmask_s, "v_cndmask_b32 %0, %0, %1, s[4:5]", VC)
K(k_perm_sgpr, "v_perm_b32 %0, %1, %0, %0", SC)

// 64-bit: one chain per pair
#define K64(NAME, ASM)                                                                               \
    __global__ void __launch_bounds__(1024) NAME(uint32_t* out, uint32_t seed, int iters) {          \
        uint64_t a[4];                                                                               \
        for (int i = 0; i < 4; i++) a[i] = ((uint64_t)seed << 32) ^ (threadIdx.x * (i + 3));          \
        const uint64_t c = seed | 1;                                                                 \
        for (int i = 0; i < iters; i++) {                                                            \
            _Pragma("unroll") for (int j = 0; j < 32; j++) {                                         \
                _Pragma("unroll") for (int q = 0; q < 4; q++) asm volatile(ASM : "+v"(a[q]) : "v"(c)); \
            }                                                                                        \
        }                                                                                            \
        uint64_t x = 0;                                                                              \
        for (int i = 0; i < 4; i++) x ^= a[i];                                                       \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)x ^ (uint32_t)(x >> 32);              \
    }
K64(k_add64, "v_lshl_add_u64 %0, %0, 0, %1")
K64(k_shl64, "v_lshlrev_b64 %0, 3, %0")
K64(k_cmp64, "v_cmp_eq_u64 vcc, %0, %1\n\tv_mov_b64 %0, %1")   // 2 insts: subtract mov_b64
K64(k_mov64, "v_mov_b64 %0, %1")

__global__ void __launch_bounds__(1024) k_clock(unsigned long long* out, int iters) {
    uint32_t a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * (i + 3);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        _Pragma("unroll") for (int j = 0; j < 16; j++) {
            _Pragma("unroll") for (int q = 0; q < 8; q++) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[q]) : "v"(a[(q + 1) & 7]));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = 0;
    for (int i = 0; i < 8; i++) x ^= a[i];
    if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = x; }
}
typedef void (*fn_t)(uint32_t*, uint32_t, int);
int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 512 * 1024 * 4);
    struct { const char* n; fn_t f; double per_step; } ks[] = {
        {"cmp_gt+cndmask (2)", k_cndmask, 2}, {"bfe", k_bfe, 1}, {"bcnt", k_bcnt, 1}, {"mul_u32_u24", k_umul24, 1},
        {"mul_lo_u32", k_mullo, 1}, {"min3", k_min3, 1}, {"lshl_or", k_lshlor, 1}, {"alignbyte", k_alignbyte, 1},
        {"ffbh", k_ffbh, 1}, {"add3", k_add3, 1}, {"xor (vgpr)", k_xor_v, 1}, {"add_u32 (vgpr)", k_add_v, 1}, {"perm (vgpr)", k_perm_v, 1}, {"bitop3 (vgpr)", k_bitop3_v, 1}, {"and (vgpr)", k_and_v, 1}, {"xor (literal)", k_xor_lit, 1}, {"add (inline const)", k_add_inl, 1},
        {"lshrrev (inline)", k_shr_inl, 1}, {"lshrrev (vgpr)", k_shr_v, 1}, {"or (vgpr)", k_or_v, 1}, {"sub (vgpr)", k_sub_v, 1},
        {"cndmask vcc", k_cndmask_v, 1}, {"cmp_gt vcc + xor (2)", k_cmp_v, 2}, {"mov_b32 (vgpr)", k_mov_v, 1},
        {"cndmask s[4:5]", k_cndmask_s, 1}, {"xor (sgpr)", k_xor_sgpr, 1}, {"perm (sgpr)", k_perm_sgpr, 1},
        {"lshl_add_u64", k_add64, 1}, {"lshlrev_b64", k_shl64, 1}, {"cmp_eq_u64+mov_b64 (2)", k_cmp64, 2},
        {"mov_b64", k_mov64, 1}};
    const int iters = 1000;
    {
        unsigned long long* d;
        (void)hipMalloc(&d, 32);
        hipLaunchKernelGGL(k_clock, dim3(256), dim3(1024), 0, 0, d, 20000);
        unsigned long long h[3];
        (void)hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
        printf("shader clock under a VALU loop: %.0f MHz (memtime %llu ticks over memrealtime %llu x 10 ns)\n",
               h[0] * 100.0 / (double)h[1], h[0], h[1]);
    }
    for (auto& k : ks) {
        for (int waves : {8, 16}) {
            const int threads = waves * 64, blocks = 256;
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 7u, 10);
            (void)hipDeviceSynchronize();
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 7u, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double steps = (k.f == k_add64 || k.f == k_shl64 || k.f == k_cmp64 || k.f == k_mov64) ? 32.0 * 4 : 16.0 * 8;
            const double insts_per_simd = (double)blocks * waves / 1024.0 * iters * steps * k.per_step;
            printf("%-24s waves/CU %2d: %.3f ms, %.2f ns per wave-inst per SIMD\n", k.n, waves, ms, ms * 1e6 / insts_per_simd);
        }
    }
    return 0;
}
