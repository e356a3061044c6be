// Issue probe for the two-blocks-per-lane question (round-4 verdict, item 1a):
// the grouped lock-step ChaCha20 rounds (tools/gen_chacha_grp.py, s_barrier
// after every rotate group) with 1 or 2 blocks per lane, in 512-thread
// workgroups, at the residencies the 16 KiB kernel could run at:
//   * 2 workgroups per CU = 4 waves per SIMD (the product's residency, ~80 KB LDS each)
//   * 1 workgroup per CU  = 2 waves per SIMD (what 8 KiB per wave iteration needs:
//     2 x 8 KiB chunk buffers + 2 KiB lines per wave = ~147 KB per workgroup)
// The LDS request only forces the residency; nothing is read or written there.
// Same total work for every configuration (blocks per launch); prints ms and
// ns per block.  Build: hipcc --offload-arch=gfx950 -O3 -I suruga_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "sg_chacha_grp.inc"

#define OPS16(x, o)                                                                                                  \
    "+v"(x[o + 0]), "+v"(x[o + 1]), "+v"(x[o + 2]), "+v"(x[o + 3]), "+v"(x[o + 4]), "+v"(x[o + 5]), "+v"(x[o + 6]), \
        "+v"(x[o + 7]), "+v"(x[o + 8]), "+v"(x[o + 9]), "+v"(x[o + 10]), "+v"(x[o + 11]), "+v"(x[o + 12]),          \
        "+v"(x[o + 13]), "+v"(x[o + 14]), "+v"(x[o + 15])

template <int NB>
__global__ __launch_bounds__(512) void chacha(uint32_t* out, uint32_t seed, int iters) {
    extern __shared__ uint32_t lds[];
    const uint32_t t = threadIdx.x + blockIdx.x * 512u;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t x[16 * NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            x[16 * b + 0] = 0x61707865u; x[16 * b + 1] = 0x3320646eu; x[16 * b + 2] = 0x79622d32u; x[16 * b + 3] = 0x6b206574u;
#pragma unroll
            for (int i = 4; i < 12; ++i) x[16 * b + i] = seed + i;
            x[16 * b + 12] = t * 64u + it * NB + b; x[16 * b + 13] = 0; x[16 * b + 14] = seed ^ 9; x[16 * b + 15] = seed ^ 10;
        }
#pragma unroll 1
        for (int r = 0; r < 10; ++r) {
            if constexpr (NB == 1) asm volatile(SG_CHACHA_DR_NB1_BAR1 : OPS16(x, 0));
            else asm volatile(SG_CHACHA_DR_NB2_BAR1 : OPS16(x, 0), OPS16(x, 16));
        }
#pragma unroll
        for (int i = 0; i < 16 * NB; ++i) acc ^= x[i] + i;
    }
    if (acc == 0x12345678u) { out[t] = acc; lds[threadIdx.x] = acc; }
}

template <int NB>
static void run(const char* name, int wgs, int blocks_per_lane, size_t lds_bytes) {
    uint32_t* out;
    (void)hipMalloc(&out, (size_t)wgs * 512 * 4);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&chacha<NB>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_bytes);
    const int iters = blocks_per_lane / NB;
    auto launch = [&] { hipLaunchKernelGGL((chacha<NB>), dim3(wgs), dim3(512), lds_bytes, 0, out, 1u, iters); };
    for (int w = 0; w < 3; ++w) launch();
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double blocks = (double)wgs * 512 * blocks_per_lane;
    printf("%-44s %8.3f ms  %.4f ns/block\n", name, best, 1e6 * best / blocks);
    fflush(stdout);
    (void)hipFree(out);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int wgs = cus * 8;  // several waves of workgroups at either residency
    const int bpl = 256;      // 256 blocks per lane = one 16 KiB record per wave
    const size_t two_per_cu = 80 * 1024, one_per_cu = 147 * 1024;
    run<1>("NB=1, 2 WG/CU (4 waves/SIMD) [product]", wgs, bpl, two_per_cu);
    run<2>("NB=2, 2 WG/CU (4 waves/SIMD)", wgs, bpl, two_per_cu);
    run<1>("NB=1, 1 WG/CU (2 waves/SIMD)", wgs, bpl, one_per_cu);
    run<2>("NB=2, 1 WG/CU (2 waves/SIMD) [8 KiB iters]", wgs, bpl, one_per_cu);
    run<1>("NB=1, 2 WG/CU (4 waves/SIMD) [product]", wgs, bpl, two_per_cu);
    run<2>("NB=2, 1 WG/CU (2 waves/SIMD) [8 KiB iters]", wgs, bpl, one_per_cu);
    return 0;
}
