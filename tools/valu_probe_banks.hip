// VGPR-bank probe for the lock-step ARX stream (round 5): the grouped ChaCha20
// double round of the product (s_barrier after every rotate group) on explicit
// VGPRs v64..v79, with the state words either contiguous (word i in v64 + i:
// every column-round operand pair in one bank mod 4) or spread (word 4k + j in
// bank (j + k) mod 4: no instruction reads two operands of one bank);
// tools/gen_bank_probe.py writes both asm bodies.  512-thread workgroups, two
// per CU (the 16 KiB kernel's residency, forced by the LDS request), the same
// blocks per launch for both; prints ms and ns per block.
// Build: hipcc --offload-arch=gfx950 -O3 -I tools/probe_banks tools/valu_probe_banks.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "banks.inc"

template <int SPREAD>
__global__ __launch_bounds__(512) void chacha(uint32_t* out, uint32_t seed, int iters) {
    extern __shared__ uint32_t lds[];
    uint32_t acc = seed + threadIdx.x + blockIdx.x * 512u;
    if constexpr (SPREAD) {
        asm volatile(BANK_INIT_SPREAD : : "v"(acc) : BANK_CLOBBER_SPREAD);
    } else {
        asm volatile(BANK_INIT_CONTIG : : "v"(acc) : BANK_CLOBBER_CONTIG);
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll 1
        for (int r = 0; r < 10; ++r) {
            if constexpr (SPREAD) asm volatile(BANK_DR_SPREAD ::: BANK_CLOBBER_SPREAD);
            else asm volatile(BANK_DR_CONTIG ::: BANK_CLOBBER_CONTIG);
        }
    }
    if constexpr (SPREAD) {
        asm volatile(BANK_FOLD_SPREAD : "+v"(acc) : : BANK_CLOBBER_SPREAD);
    } else {
        asm volatile(BANK_FOLD_CONTIG : "+v"(acc) : : BANK_CLOBBER_CONTIG);
    }
    if (acc == 0x12345678u) { out[threadIdx.x] = acc; lds[threadIdx.x] = acc; }
}

template <int SPREAD>
static void run(const char* name, int wgs, int iters, size_t lds_bytes) {
    uint32_t* out;
    (void)hipMalloc(&out, 512 * 4);
    auto launch = [&] { hipLaunchKernelGGL((chacha<SPREAD>), dim3(wgs), dim3(512), lds_bytes, 0, out, 1u, iters); };
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
    const double blocks = (double)wgs * 512 * iters;
    printf("%-40s %8.3f ms  %.4f ns/block\n", name, best, 1e6 * best / blocks);
    fflush(stdout);
    (void)hipFree(out);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int wgs = cus * 8, iters = 256;
    const size_t two_per_cu = 80 * 1024;
    for (int rep = 0; rep < 2; ++rep) {
        run<0>("contiguous (same-bank operand pairs)", wgs, iters, two_per_cu);
        run<1>("spread (operands in different banks)", wgs, iters, two_per_cu);
    }
    return 0;
}
