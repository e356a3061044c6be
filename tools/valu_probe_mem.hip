// Issue probe (streaming ChaCha20): does the lock-step pairing of grouped
// ChaCha rounds (valu_probe_grouped.hip: ~2.6 cycles per VALU instruction
// with no memory traffic) survive the loads, XOR and stores of a real
// keystream pass?  Every lane XORs 64-byte blocks of a 2 GiB buffer with
// ChaCha20 keystream and writes them out, one or two blocks per lane per
// step, as
//   cc   : compiled C++ rounds (the product kernel's form), 256-thread WGs
//   grpN : grouped asm rounds, s_barrier after every N-th rotate group
//          (0 = none), 1024-thread WGs
// with and without the next step's loads issued before the rounds (pf).
// Build: hipcc --offload-arch=gfx950 -O3 -I tools tools/valu_probe_mem.hip -o tools/valu_probe_mem
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "chacha_grp.inc"  // python tools/gen_chacha_grp.py tools/chacha_grp.inc

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define OPS16(x, o) "+v"(x[o + 0]), "+v"(x[o + 1]), "+v"(x[o + 2]), "+v"(x[o + 3]), "+v"(x[o + 4]), "+v"(x[o + 5]), \
    "+v"(x[o + 6]), "+v"(x[o + 7]), "+v"(x[o + 8]), "+v"(x[o + 9]), "+v"(x[o + 10]), "+v"(x[o + 11]),           \
    "+v"(x[o + 12]), "+v"(x[o + 13]), "+v"(x[o + 14]), "+v"(x[o + 15])

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(a, b, c, d)                   \
    a += b; d ^= a; d = rotl32(d, 16);   \
    c += d; b ^= c; b = rotl32(b, 12);   \
    a += b; d ^= a; d = rotl32(d, 8);    \
    c += d; b ^= c; b = rotl32(b, 7);

template <int NB, int BAR>
__device__ __forceinline__ void dr(uint32_t* x) {
    if constexpr (BAR < 0) {  // compiled
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            uint32_t* y = x + 16 * b;
            QR(y[0], y[4], y[8], y[12]); QR(y[1], y[5], y[9], y[13]); QR(y[2], y[6], y[10], y[14]); QR(y[3], y[7], y[11], y[15]);
            QR(y[0], y[5], y[10], y[15]); QR(y[1], y[6], y[11], y[12]); QR(y[2], y[7], y[8], y[13]); QR(y[3], y[4], y[9], y[14]);
        }
    } else if constexpr (NB == 1) {
        if constexpr (BAR == 0) asm volatile(SG_CHACHA_DR_NB1_BAR0 : OPS16(x, 0));
        if constexpr (BAR == 1) asm volatile(SG_CHACHA_DR_NB1_BAR1 : OPS16(x, 0));
        if constexpr (BAR == 2) asm volatile(SG_CHACHA_DR_NB1_BAR2 : OPS16(x, 0));
    } else {
        if constexpr (BAR == 0) asm volatile(SG_CHACHA_DR_NB2_BAR0 : OPS16(x, 0), OPS16(x, 16));
        if constexpr (BAR == 1) asm volatile(SG_CHACHA_DR_NB2_BAR1 : OPS16(x, 0), OPS16(x, 16));
        if constexpr (BAR == 2) asm volatile(SG_CHACHA_DR_NB2_BAR2 : OPS16(x, 0), OPS16(x, 16));
    }
}

// block id (blk, b) of thread g: data at in + 4 * ((blk + b) * T + g)
template <int NB, int BAR, int WG, bool PF, int MODE = 0>  // MODE 1: no rounds (copy), 2: no memory
__global__ __launch_bounds__(WG) void stream(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint32_t seed,
                                             int nblk) {
    const uint32_t g = threadIdx.x + blockIdx.x * WG;
    const uint32_t T = gridDim.x * WG;
    u32x4 d[NB][4], dn[NB][4];
    auto load = [&](u32x4 (&dst)[NB][4], int blk) {
        if constexpr (MODE == 2) {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int q = 0; q < 4; ++q) dst[b][q] = u32x4{g, (uint32_t)blk, 3u, 4u};
            return;
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const u32x4* p = in + 4ull * ((uint64_t)(blk + b) * T + g);
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[b][q] = __builtin_nontemporal_load(p + q);
        }
    };
    if constexpr (PF) load(dn, 0);
    for (int blk = 0; blk < nblk; blk += NB) {
        if constexpr (PF) {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int q = 0; q < 4; ++q) d[b][q] = dn[b][q];
            if (blk + NB < nblk) load(dn, blk + NB);
        } else {
            load(d, blk);
        }
        uint32_t x[16 * NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            x[16 * b + 0] = 0x61707865u; x[16 * b + 1] = 0x3320646eu; x[16 * b + 2] = 0x79622d32u; x[16 * b + 3] = 0x6b206574u;
#pragma unroll
            for (int i = 4; i < 12; ++i) x[16 * b + i] = seed + i;
            x[16 * b + 12] = g * 64u + blk + b; x[16 * b + 13] = 0; x[16 * b + 14] = seed ^ 9; x[16 * b + 15] = seed ^ 10;
        }
        if constexpr (MODE != 1) {
#pragma unroll 1
            for (int r = 0; r < 10; ++r) dr<NB, BAR>(x);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            uint32_t ks[16];
            ks[0] = x[16 * b + 0] + 0x61707865u; ks[1] = x[16 * b + 1] + 0x3320646eu;
            ks[2] = x[16 * b + 2] + 0x79622d32u; ks[3] = x[16 * b + 3] + 0x6b206574u;
#pragma unroll
            for (int i = 4; i < 12; ++i) ks[i] = x[16 * b + i] + seed + i;
            ks[12] = x[16 * b + 12] + g * 64u + blk + b; ks[13] = x[16 * b + 13];
            ks[14] = x[16 * b + 14] + (seed ^ 9); ks[15] = x[16 * b + 15] + (seed ^ 10);
            u32x4* p = out + 4ull * ((uint64_t)(blk + b) * T + g);
            u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32x4 v = d[b][q] ^ u32x4{ks[4 * q], ks[4 * q + 1], ks[4 * q + 2], ks[4 * q + 3]};
                if constexpr (MODE == 2) acc ^= v;
                else p[q] = v;
            }
            if constexpr (MODE == 2)
                if (acc.x == 0x12345678u && acc.y == 7u) p[0] = acc;
        }
    }
}


// Coalesced form: wave w's step covers one contiguous 4 KiB chunk; global
// loads/stores are lane-contiguous (16 B per lane, 1 KiB per instruction) and
// the chunk is transposed through a wave-private LDS slot so that lane t still
// owns 64-byte block t of the chunk (MODE 3: copy only, no rounds, no LDS).
template <int BAR, int WG, int MODE, bool SWZ>
__global__ __launch_bounds__(WG) void stream_co(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint32_t seed,
                                                int nblk) {
    __shared__ u32x4 lds[WG * 4];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t nw = gridDim.x * (WG / 64);
    const uint32_t gw = blockIdx.x * (WG / 64) + w;
    u32x4* slot = lds + w * 256;
    // 16-byte unit u of the chunk lives at slot[u ^ swz(u)]: spreads lane t's
    // block-reads (units 4t + q) over banks
    auto phys = [](uint32_t u) { return SWZ ? (u ^ ((u >> 4) & 3u)) : u; };
    u32x4 v[4], vn[4];
    auto gload = [&](u32x4 (&dst)[4], int blk) {
        const u32x4* p = in + 256ull * ((uint64_t)blk * nw + gw);
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = __builtin_nontemporal_load(p + lane + 64 * q);
    };
    gload(vn, 0);
    for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = vn[q];
        if (blk + 1 < nblk) gload(vn, blk + 1);
        u32x4* po = out + 256ull * ((uint64_t)blk * nw + gw);
        if constexpr (MODE == 3) {
#pragma unroll
            for (int q = 0; q < 4; ++q) po[lane + 64 * q] = v[q] ^ u32x4{seed, 1u, 2u, 3u};
            continue;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) slot[phys(lane + 64 * q)] = v[q];
        __builtin_amdgcn_wave_barrier();
        u32x4 d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = slot[phys(4 * lane + q)];
        uint32_t x[16];
        x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
#pragma unroll
        for (int i = 4; i < 12; ++i) x[i] = seed + i;
        x[12] = gw * 64u + lane + blk; x[13] = 0; x[14] = seed ^ 9; x[15] = seed ^ 10;
#pragma unroll 1
        for (int r = 0; r < 10; ++r) dr<1, BAR>(x);
        uint32_t ks[16];
        ks[0] = x[0] + 0x61707865u; ks[1] = x[1] + 0x3320646eu; ks[2] = x[2] + 0x79622d32u; ks[3] = x[3] + 0x6b206574u;
#pragma unroll
        for (int i = 4; i < 12; ++i) ks[i] = x[i] + seed + i;
        ks[12] = x[12] + gw * 64u + lane + blk; ks[13] = x[13]; ks[14] = x[14] + (seed ^ 9); ks[15] = x[15] + (seed ^ 10);
        if constexpr (MODE == 5) {  // strided store straight from registers (lane t: its own 64 B)
#pragma unroll
            for (int q = 0; q < 4; ++q) po[4 * lane + q] = d[q] ^ u32x4{ks[4 * q], ks[4 * q + 1], ks[4 * q + 2], ks[4 * q + 3]};
            continue;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) slot[phys(4 * lane + q)] = d[q] ^ u32x4{ks[4 * q], ks[4 * q + 1], ks[4 * q + 2], ks[4 * q + 3]};
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) po[lane + 64 * q] = slot[phys(lane + 64 * q)];
        __builtin_amdgcn_wave_barrier();
    }
}

// Wave-specialised form: 8 lock-step ChaCha waves (two records' worth of
// 4 KiB chunks, as stream_co with BAR = 1) plus NMAC waves that stand in for
// the MAC: between every two barriers of the rounds they issue MACW
// dependent-pair v_mad_u64_u32 (half-rate, like the Horner step), so every
// wave of the workgroup hits the same 80 barriers per block.
template <int NMAC, int MACW>
__global__ __launch_bounds__(512 + 64 * NMAC) void stream_ws(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                            uint32_t seed, int nblk) {
    __shared__ u32x4 lds[512 * 4];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    if (w >= 8) {  // MAC stand-in waves
        uint64_t a0 = seed + lane, a1 = lane * 3u, a2 = lane ^ 5u, a3 = lane + 7u;
        uint32_t m = lane | 1u;
        for (int blk = 0; blk < nblk; ++blk) {
            for (int g = 0; g < 80; ++g) {
#pragma unroll
                for (int i = 0; i < MACW / 4; ++i) {
                    a0 = (uint64_t)(uint32_t)a0 * m + (a1 >> 32);
                    a1 = (uint64_t)(uint32_t)a1 * m + (a2 >> 32);
                    a2 = (uint64_t)(uint32_t)a2 * m + (a3 >> 32);
                    a3 = (uint64_t)(uint32_t)a3 * m + (a0 >> 32);
                }
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if ((a0 ^ a1 ^ a2 ^ a3) == 0x123456789ull) out[threadIdx.x] = u32x4{1u, 2u, 3u, 4u};
        return;
    }
    const uint32_t nw = gridDim.x * 8u;
    const uint32_t gw = blockIdx.x * 8u + w;
    u32x4* slot = lds + w * 256;
    auto phys = [](uint32_t u) { return u ^ ((u >> 4) & 3u); };
    u32x4 v[4], vn[4];
    auto gload = [&](u32x4 (&dst)[4], int blk) {
        const u32x4* p = in + 256ull * ((uint64_t)blk * nw + gw);
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = __builtin_nontemporal_load(p + lane + 64 * q);
    };
    gload(vn, 0);
    for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = vn[q];
        if (blk + 1 < nblk) gload(vn, blk + 1);
        u32x4* po = out + 256ull * ((uint64_t)blk * nw + gw);
#pragma unroll
        for (int q = 0; q < 4; ++q) slot[phys(lane + 64 * q)] = v[q];
        __builtin_amdgcn_wave_barrier();
        u32x4 d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = slot[phys(4 * lane + q)];
        uint32_t x[16];
        x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
#pragma unroll
        for (int i = 4; i < 12; ++i) x[i] = seed + i;
        x[12] = gw * 64u + lane + blk; x[13] = 0; x[14] = seed ^ 9; x[15] = seed ^ 10;
#pragma unroll 1
        for (int r = 0; r < 10; ++r) dr<1, 1>(x);
        uint32_t ks[16];
        ks[0] = x[0] + 0x61707865u; ks[1] = x[1] + 0x3320646eu; ks[2] = x[2] + 0x79622d32u; ks[3] = x[3] + 0x6b206574u;
#pragma unroll
        for (int i = 4; i < 12; ++i) ks[i] = x[i] + seed + i;
        ks[12] = x[12] + gw * 64u + lane + blk; ks[13] = x[13]; ks[14] = x[14] + (seed ^ 9); ks[15] = x[15] + (seed ^ 10);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) slot[phys(4 * lane + q)] = d[q] ^ u32x4{ks[4 * q], ks[4 * q + 1], ks[4 * q + 2], ks[4 * q + 3]};
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) po[lane + 64 * q] = slot[phys(lane + 64 * q)];
        __builtin_amdgcn_wave_barrier();
    }
}

template <typename F>
static void timeit(const char* name, double gib, F launch) {
    launch();
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("%-28s %8.3f ms  %7.1f GiB/s keystream\n", name, best, gib / (best * 1e-3));
    fflush(stdout);
}

int main() {
    const int threads = 256 * 2048;  // 2048 threads per CU over 256 CUs
    const int nblk = 64;             // 64-byte blocks per thread: 2 GiB in, 2 GiB out
    const size_t bytes = (size_t)threads * nblk * 64;
    const double gib = (double)bytes / (1 << 30);
    u32x4 *in, *out;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, bytes) != hipSuccess) return 1;
    (void)hipMemset(in, 0x5a, bytes);
#define RUNM(NB, BAR, WG, PF, M, name) \
    timeit(name, gib, [&] { hipLaunchKernelGGL((stream<NB, BAR, WG, PF, M>), dim3(threads / WG), dim3(WG), 0, 0, in, out, 1u, nblk); })
#define RUN(NB, BAR, WG, PF, name) RUNM(NB, BAR, WG, PF, 0, name)
#define RUNC(BAR, WG, M, SWZ, name) \
    timeit(name, gib, [&] { hipLaunchKernelGGL((stream_co<BAR, WG, M, SWZ>), dim3(threads / WG), dim3(WG), 0, 0, in, out, 1u, nblk); })
    {  // wave-specialised: 3 workgroups of 8 ChaCha + NMAC waves per CU
        const int wgs = 256 * 3, nb = 85;
        const double g2 = (double)wgs * 512 * nb * 64 / (1 << 30);
#define RUNW(NMAC, MACW, name) \
    timeit(name, g2, [&] { hipLaunchKernelGGL((stream_ws<NMAC, MACW>), dim3(wgs), dim3(512 + 64 * NMAC), 0, 0, in, out, 1u, nb); })
        RUNW(0, 4, "ws 8 chacha + 0 mac");
        RUNW(2, 4, "ws 8 chacha + 2 mac x4");
        RUNW(2, 8, "ws 8 chacha + 2 mac x8");
        RUNW(2, 12, "ws 8 chacha + 2 mac x12");
        RUNW(2, 16, "ws 8 chacha + 2 mac x16");
        RUNW(4, 12, "ws 8 chacha + 4 mac x12");
    }
    RUNC(1, 512, 0, true, "co grp1 WG=512 swz (ref)");
    RUNC(-1, 256, 3, false, "co copy only WG=256");
    RUNC(-1, 1024, 3, false, "co copy only WG=1024");
    RUNC(-1, 256, 0, false, "co cc WG=256");
    RUNC(-1, 256, 0, true, "co cc WG=256 swz");
    RUNC(0, 1024, 0, true, "co grp0 WG=1024 swz");
    RUNC(1, 1024, 0, false, "co grp1 WG=1024");
    RUNC(1, 1024, 0, true, "co grp1 WG=1024 swz");
    RUNC(1, 512, 0, true, "co grp1 WG=512 swz");
    RUNC(1, 512, 5, true, "co-in strided-out grp1 WG=512");
    RUNC(-1, 256, 5, true, "co-in strided-out cc WG=256");
    RUNM(1, -1, 256, false, 1, "copy only WG=256");
    RUNM(1, -1, 256, true, 1, "copy only WG=256 pf");
    RUNM(1, -1, 256, false, 2, "cc compute only WG=256");
    RUNM(2, -1, 256, false, 2, "cc compute only NB=2 WG=256");
    RUNM(1, 1, 1024, false, 2, "grp1 compute only WG=1024");
    RUNM(1, 0, 1024, false, 2, "grp0 compute only WG=1024");
    RUN(1, -1, 256, false, "cc NB=1 WG=256");
    RUN(1, -1, 256, true, "cc NB=1 WG=256 pf");
    RUN(2, -1, 256, true, "cc NB=2 WG=256 pf");
    RUN(1, 0, 1024, true, "grp0 NB=1 WG=1024 pf");
    RUN(1, 1, 1024, false, "grp1 NB=1 WG=1024");
    RUN(1, 1, 1024, true, "grp1 NB=1 WG=1024 pf");
    RUN(2, 1, 1024, true, "grp1 NB=2 WG=1024 pf");
    RUN(1, 1, 512, true, "grp1 NB=1 WG=512 pf");
    RUN(2, 2, 1024, true, "grp2 NB=2 WG=1024 pf");
    (void)hipFree(in);
    (void)hipFree(out);
    return 0;
}
