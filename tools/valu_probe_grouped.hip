// Issue probe (grouped ChaCha): ChaCha20 rounds emitted grouped by instruction kind (tools/gen_chacha_grp.py),
// 1 or 2 blocks per lane, with s_barrier after every BAR-th rotate group, at
// 1/2/4 waves of one workgroup per SIMD.  Run under rocprofv3 --pmc.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "chacha_grp.inc"  // python tools/gen_chacha_grp.py tools/chacha_grp.inc

#define OPS16(x, o) "+v"(x[o + 0]), "+v"(x[o + 1]), "+v"(x[o + 2]), "+v"(x[o + 3]), "+v"(x[o + 4]), "+v"(x[o + 5]), \
    "+v"(x[o + 6]), "+v"(x[o + 7]), "+v"(x[o + 8]), "+v"(x[o + 9]), "+v"(x[o + 10]), "+v"(x[o + 11]),           \
    "+v"(x[o + 12]), "+v"(x[o + 13]), "+v"(x[o + 14]), "+v"(x[o + 15])

template <int NB, int BAR>
__device__ __forceinline__ void dr(uint32_t* x) {
    if constexpr (NB == 1) {
        if constexpr (BAR == 0) asm volatile(SG_CHACHA_DR_NB1_BAR0 : OPS16(x, 0));
        if constexpr (BAR == 1) asm volatile(SG_CHACHA_DR_NB1_BAR1 : OPS16(x, 0));
        if constexpr (BAR == 2) asm volatile(SG_CHACHA_DR_NB1_BAR2 : OPS16(x, 0));
        if constexpr (BAR == 4) asm volatile(SG_CHACHA_DR_NB1_BAR4 : OPS16(x, 0));
    } else {
        if constexpr (BAR == 0) asm volatile(SG_CHACHA_DR_NB2_BAR0 : OPS16(x, 0), OPS16(x, 16));
        if constexpr (BAR == 1) asm volatile(SG_CHACHA_DR_NB2_BAR1 : OPS16(x, 0), OPS16(x, 16));
        if constexpr (BAR == 2) asm volatile(SG_CHACHA_DR_NB2_BAR2 : OPS16(x, 0), OPS16(x, 16));
        if constexpr (BAR == 4) asm volatile(SG_CHACHA_DR_NB2_BAR4 : OPS16(x, 0), OPS16(x, 16));
    }
}

template <int NB, int BAR, int WG>
__global__ __launch_bounds__(WG) void chacha(uint32_t* out, uint32_t seed, int nblk) {
    const uint32_t t = threadIdx.x + blockIdx.x * WG;
    uint32_t acc = 0;
    for (int blk = 0; blk < nblk; blk += NB) {
        uint32_t x[16 * NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            x[16 * b + 0] = 0x61707865u; x[16 * b + 1] = 0x3320646eu; x[16 * b + 2] = 0x79622d32u; x[16 * b + 3] = 0x6b206574u;
#pragma unroll
            for (int i = 4; i < 12; ++i) x[16 * b + i] = seed + i;
            x[16 * b + 12] = t * 64u + blk + b; x[16 * b + 13] = 0; x[16 * b + 14] = seed ^ 9; x[16 * b + 15] = seed ^ 10;
        }
#pragma unroll 1
        for (int r = 0; r < 10; ++r) dr<NB, BAR>(x);
#pragma unroll
        for (int i = 0; i < 16 * NB; ++i) acc ^= x[i] + i;
    }
    if (acc == 0x12345678u) out[t] = acc;
}

template <typename F>
static void timeit(const char* name, F launch) {
    launch();
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-36s %8.3f ms\n", name, ms);
    fflush(stdout);
}

int main() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&chacha<1, 1, 1024>), hipFuncAttributeMaxDynamicSharedMemorySize, 100000);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&chacha<2, 1, 1024>), hipFuncAttributeMaxDynamicSharedMemorySize, 100000);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&chacha<1, 0, 1024>), hipFuncAttributeMaxDynamicSharedMemorySize, 100000);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&chacha<2, 2, 1024>), hipFuncAttributeMaxDynamicSharedMemorySize, 100000);
    uint32_t* out;
    (void)hipMalloc(&out, 1 << 28);
    const int waves = 256 * 32;
    const int nblk = 32;
#define CH(NB, BAR, WG) \
    timeit("grp NB=" #NB " BAR=" #BAR " WG=" #WG, [&] { hipLaunchKernelGGL((chacha<NB, BAR, WG>), dim3(waves * 64 / WG), dim3(WG), 0, 0, out, 1u, nblk); })
    CH(1, 0, 256); CH(2, 0, 256); CH(1, 0, 1024); CH(2, 0, 1024);
    CH(1, 1, 512); CH(1, 1, 1024); CH(2, 1, 512); CH(2, 1, 1024); CH(2, 2, 1024); CH(2, 4, 1024);
    CH(1, 2, 1024); CH(2, 1, 256);
    // exclusive residency: one 1024-thread workgroup per CU (LDS request forces it), long loop
    const int nb2 = 256;
    timeit("EXCL grp NB=1 BAR=1 WG=1024", [&] { hipLaunchKernelGGL((chacha<1, 1, 1024>), dim3(256), dim3(1024), 100000, 0, out, 1u, nb2); });
    timeit("EXCL grp NB=2 BAR=1 WG=1024", [&] { hipLaunchKernelGGL((chacha<2, 1, 1024>), dim3(256), dim3(1024), 100000, 0, out, 1u, nb2); });
    timeit("EXCL grp NB=1 BAR=0 WG=1024", [&] { hipLaunchKernelGGL((chacha<1, 0, 1024>), dim3(256), dim3(1024), 100000, 0, out, 1u, nb2); });
    timeit("EXCL grp NB=2 BAR=2 WG=1024", [&] { hipLaunchKernelGGL((chacha<2, 2, 1024>), dim3(256), dim3(1024), 100000, 0, out, 1u, nb2); });
    return 0;
}
