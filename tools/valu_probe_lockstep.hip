// Issue probe (lock-step): does lock-step between the waves of a SIMD let the fast VALU ops
// (add/xor) pair up inside a mixed stream?  Same instruction streams as probe 4
// with and without an s_barrier per iteration, at 1, 2 and 4 waves of the same
// workgroup per SIMD; plus a compiled ChaCha20 block loop with a barrier per
// double round.  Run under rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 256
#define R8(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define I_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define I_XOR(r) "v_xor_b32 " r ", " r ", %8\n"
#define I_ALN(r) "v_alignbit_b32 " r ", " r ", " r ", 7\n"
#define I_QRA(r) I_ADD(r) I_XOR(r) I_ALN(r)

// V: 0 = grp8 add|xor|aln, 1 = per-reg add,xor,aln.  BAR: barrier every BAR iterations (0 = none)
template <int V, int BAR, int WG>
__global__ __launch_bounds__(WG) void mix(uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * WG;
    uint32_t x0 = t ^ seed, x1 = t * 3u, x2 = t + 7u, x3 = t * 5u ^ seed, x4 = t + 11u, x5 = t * 13u, x6 = t ^ 0x55u,
             x7 = t + seed;
    const uint32_t y = seed | 1u;
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (V == 0)
            asm volatile(R8(I_ADD) R8(I_XOR) R8(I_ALN) : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5),
                         "+v"(x6), "+v"(x7) : "v"(y));
        else
            asm volatile(R8(I_QRA) : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                         : "v"(y));
        if constexpr (BAR > 0)
            if ((i % BAR) == BAR - 1) __builtin_amdgcn_s_barrier();
    }
    const uint32_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (r == 0x12345678u) out[t] = r;
}

__device__ __forceinline__ uint32_t rot_sh(uint32_t a, int e) { return (a << e) | (a >> (32 - e)); }
#define QRX(a, b, c, d) \
    a += b; d ^= a; d = rot_sh(d, 16); c += d; b ^= c; b = rot_sh(b, 12); \
    a += b; d ^= a; d = rot_sh(d, 8); c += d; b ^= c; b = rot_sh(b, 7);
template <int BAR, int WG>
__global__ __launch_bounds__(WG) void chacha(uint32_t* out, uint32_t seed, int nblk) {
    const uint32_t t = threadIdx.x + blockIdx.x * WG;
    uint32_t acc = 0;
    for (int blk = 0; blk < nblk; ++blk) {
        uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u, x4 = seed, x5 = seed + 1,
                 x6 = seed + 2, x7 = seed + 3, x8 = seed + 4, x9 = seed + 5, x10 = seed + 6, x11 = seed + 7,
                 x12 = t * 64u + blk, x13 = 0, x14 = seed ^ 9, x15 = seed ^ 10;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            QRX(x0, x4, x8, x12) QRX(x1, x5, x9, x13) QRX(x2, x6, x10, x14) QRX(x3, x7, x11, x15)
            QRX(x0, x5, x10, x15) QRX(x1, x6, x11, x12) QRX(x2, x7, x8, x13) QRX(x3, x4, x9, x14)
            if constexpr (BAR > 0)
                if ((r % BAR) == BAR - 1) __builtin_amdgcn_s_barrier();
        }
        acc ^= x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ x15;
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
    printf("%-40s %8.3f ms\n", name, ms);
    fflush(stdout);
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 1 << 28);
    // same total waves (256 CUs x 32 waves) in every case
    const int waves = 256 * 32;
#define MIX(V, BAR, WG) \
    timeit("mix V=" #V " BAR=" #BAR " WG=" #WG, [&] { hipLaunchKernelGGL((mix<V, BAR, WG>), dim3(waves * 64 / WG), dim3(WG), 0, 0, out, 1u); })
    MIX(0, 0, 256); MIX(0, 1, 256); MIX(0, 0, 512); MIX(0, 1, 512); MIX(0, 4, 512);
    MIX(0, 0, 1024); MIX(0, 1, 1024);
    MIX(1, 0, 256); MIX(1, 1, 512); MIX(1, 1, 1024);
#define CH(BAR, WG) \
    timeit("chacha BAR=" #BAR " WG=" #WG, [&] { hipLaunchKernelGGL((chacha<BAR, WG>), dim3(waves * 64 / WG), dim3(WG), 0, 0, out, 1u, 8); })
    CH(0, 256); CH(0, 512); CH(1, 512); CH(2, 512); CH(0, 1024); CH(1, 1024);
    return 0;
}
