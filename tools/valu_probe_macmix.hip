// Issue probe (MAC beside lock-step ChaCha): can one wave per SIMD run slow-op MAC work (Poly1305 Horner steps)
// beside three lock-step waves running grouped ChaCha20 rounds, without
// breaking their add/xor pairing?  1024-thread workgroups, waves 0-3 (one per
// SIMD) = MAC waves, waves 4-15 = ChaCha waves; barrier counts matched.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "chacha_grp.inc"  // python tools/gen_chacha_grp.py tools/chacha_grp.inc

#define X16 "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
    "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])

struct H32 { uint32_t h0, h1, h2, h3, h4; };
__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
    return __builtin_addc(a, b, cin, cout);
}
__device__ __forceinline__ void horner_step(H32& h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t r0,
                                            uint32_t r1, uint32_t r2, uint32_t r3, uint32_t s1, uint32_t s2, uint32_t s3) {
    uint32_t c;
    const uint32_t a0 = addc(h.h0, m0, 0u, &c), a1 = addc(h.h1, m1, c, &c), a2 = addc(h.h2, m2, c, &c),
                   a3 = addc(h.h3, m3, c, &c);
    const uint32_t a4 = h.h4 + 1u + c;
    const uint64_t d0 = (uint64_t)a0 * r0 + (uint64_t)a1 * s3 + (uint64_t)a2 * s2 + (uint64_t)a3 * s1;
    const uint64_t d1 = (uint64_t)a0 * r1 + (uint64_t)a1 * r0 + (uint64_t)a2 * s3 + (uint64_t)a3 * s2 + (uint64_t)a4 * s1;
    const uint64_t d2 = (uint64_t)a0 * r2 + (uint64_t)a1 * r1 + (uint64_t)a2 * r0 + (uint64_t)a3 * s3 + (uint64_t)a4 * s2;
    const uint64_t d3 = (uint64_t)a0 * r3 + (uint64_t)a1 * r2 + (uint64_t)a2 * r1 + (uint64_t)a3 * r0 + (uint64_t)a4 * s3;
    const uint32_t e1 = addc((uint32_t)d1, (uint32_t)(d0 >> 32), 0u, &c);
    const uint32_t e2 = addc((uint32_t)d2, (uint32_t)(d1 >> 32), c, &c);
    const uint32_t e3 = addc((uint32_t)d3, (uint32_t)(d2 >> 32), c, &c);
    uint32_t e4 = a4 * r0 + (uint32_t)(d3 >> 32) + c;
    const uint32_t f = (e4 >> 2) * 5u;
    e4 &= 3u;
    h.h0 = addc((uint32_t)d0, f, 0u, &c); h.h1 = addc(e1, 0u, c, &c); h.h2 = addc(e2, 0u, c, &c);
    h.h3 = addc(e3, 0u, c, &c); h.h4 = e4 + c;
}

// MODE bit 0: ChaCha waves compute (else barriers only); bit 1: MAC waves compute (else barriers only)
// MAC waves: one Horner step per SPB barriers.
template <int MODE, int SPB>
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t seed, int nblk) {
    const uint32_t t = threadIdx.x + blockIdx.x * 1024u;
    const uint32_t wave = threadIdx.x >> 6;
    const int nbar = nblk * 80;
    if (wave < 4u) {
        const uint32_t r0 = __builtin_amdgcn_readfirstlane(seed & 0x0fffffffu), r1 = __builtin_amdgcn_readfirstlane((seed * 3u) & 0x0ffffffcu);
        const uint32_t r2 = __builtin_amdgcn_readfirstlane((seed * 5u) & 0x0ffffffcu), r3 = __builtin_amdgcn_readfirstlane((seed * 7u) & 0x0ffffffcu);
        const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
        H32 h = {t, t * 3u, t ^ 5u, t + 9u, 1u};
        uint32_t m0 = t;
        for (int i = 0; i < nbar; ++i) {
            if ((MODE & 2) && (i % SPB) == 0) { horner_step(h, m0, m0 ^ 7u, m0 + 3u, m0 * 5u, r0, r1, r2, r3, s1, s2, s3); m0 += 0x9e3779b9u; }
            __builtin_amdgcn_s_barrier();
        }
        if ((h.h0 ^ h.h1 ^ h.h2 ^ h.h3 ^ h.h4) == 0x12345678u) out[t] = 1;
    } else {
        uint32_t acc = 0;
        for (int blk = 0; blk < nblk; ++blk) {
            if (MODE & 1) {
                uint32_t x[16];
                for (int i = 0; i < 16; ++i) x[i] = seed + i * 0x01010101u + (i == 12 ? t * 64u + blk : 0u);
#pragma unroll 1
                for (int r = 0; r < 10; ++r) asm volatile(SG_CHACHA_DR_NB1_BAR1 : X16);
                for (int i = 0; i < 16; ++i) acc ^= x[i];
            } else {
#pragma unroll 1
                for (int i = 0; i < 80; ++i) __builtin_amdgcn_s_barrier();
            }
        }
        if (acc == 0x12345678u) out[t] = acc;
    }
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
    printf("%-40s %8.3f ms\n", name, ms);
    fflush(stdout);
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 1 << 28);
    const int grid = 256 * 2;  // two 1024-thread workgroups per CU over time
    const int nblk = 32;
#define K(MODE, SPB) timeit("mode=" #MODE " steps/barrier=1/" #SPB, [&] { hipLaunchKernelGGL((k<MODE, SPB>), dim3(grid), dim3(1024), 0, 0, out, 0x12345u, nblk); })
    K(0, 4); K(1, 4); K(2, 4); K(3, 4); K(2, 8); K(3, 8); K(2, 2); K(3, 2);
    return 0;
}
