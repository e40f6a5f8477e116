// VALU issue rate on gfx950: cycles per wave64 instruction per SIMD for the integer
// ops the scan kernels use (v_xor / v_perm / v_add / v_bitop3 / v_dot4 / v_alignbit /
// 64-bit add), at 4 and 8 waves per SIMD.  Prints SIMD-cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int OP>
__global__ void __launch_bounds__(1024) k(uint32_t* out, uint32_t seed, int iters, unsigned long long* clk) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
    const uint32_t c = seed | 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
#define STEP(x)                                                                          \
            if (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(c));                                               \
            if (OP == 1) x = __builtin_amdgcn_perm(c, x, x);                             \
            if (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(c));                                                      \
            if (OP == 3) x = __builtin_amdgcn_bitop3_b32(x, c, x >> 1, 0x96);            \
            if (OP == 4) x = __builtin_amdgcn_udot4(x, c, x, false);                     \
            if (OP == 5) x = __builtin_amdgcn_alignbit(x, c, x);                         \
            if (OP == 6) { uint64_t y = ((uint64_t)c << 32) | x; asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(y)); x = (uint32_t)y ^ (uint32_t)(y >> 32); }  \
            if (OP == 7) asm volatile("v_ffbl_b32 %0, %0" : "+v"(x));
            STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) atomicAdd(clk, t1 - t0);
}

int main() {
    uint32_t* out;
    unsigned long long* clk;
    hipMalloc(&out, 256 * 1024 * 8 * 4);
    hipMalloc(&clk, 8);
    const char* names[] = {"xor (asm)", "perm", "add_u32 (asm)", "bitop3+shr(2)", "dot4", "alignbit", "lshl_add_u64+xor", "ffbl (asm)"};
    void (*fns[])(uint32_t*, uint32_t, int, unsigned long long*) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>};
    for (int op = 0; op < 8; op++) {
        for (int waves : {4, 8, 16, 32}) {   // waves per CU (1024-thread blocks: 16; two blocks: 32)
            const int threads = waves <= 16 ? waves * 64 : 1024, blocks = waves <= 16 ? 256 : 512;
            const int iters = 2000;
            hipLaunchKernelGGL(fns[op], dim3(blocks), dim3(threads), 0, 0, out, 7u, 10, clk);
            hipDeviceSynchronize();
            hipMemset(clk, 0, 8);
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(fns[op], dim3(blocks), dim3(threads), 0, 0, out, 7u, iters, clk);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long c = 0;
            hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
            // wave-instructions per SIMD: blocks * waves_per_block / (256 CU * 4 SIMD) * iters * 16 * 8
            const double wpb = threads / 64.0;
            const double insts_per_simd = blocks * wpb / 1024.0 * iters * 16.0 * 8.0 * (op == 3 ? 2 : (op == 6 ? 3 : 1));
            const double avg_clk = (double)c / blocks;   // per-block loop cycles (s_memtime ticks)
            // every SIMD runs the same number of waves: ticks of one block's loop / wave-insts one SIMD issues meanwhile
            const double simd_insts_per_block = insts_per_simd * 1024.0 / blocks / 4.0 * (blocks > 256 ? 2.0 : 1.0) / 1.0;
            printf("%-16s waves/CU %2d: %.3f ms, %.2f ns per wave-inst per SIMD, %.2f ticks per wave-inst per SIMD\n",
                   names[op], waves, ms, ms * 1e6 / insts_per_simd, avg_clk / (insts_per_simd / (blocks > 256 ? 2.0 : 1.0)));
        }
    }
    return 0;
}
