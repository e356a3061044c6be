// Issue probe (MAC): issue rates of the Poly1305 arithmetic (64-bit multiply-add, carry
// chains), a compiled radix-2^32 Horner step loop, and ChaCha20 with one vs
// two interleaved blocks per lane.  Wall-clock rates per SIMD are the primary
// output (s_memtime per wave as a cross-check).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <utility>

#define ITERS 512
#define R8(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define R32(OP) R8(OP) R8(OP) R8(OP) R8(OP)
#define I_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define I_MULLO(r) "v_mul_lo_u32 " r ", " r ", %8\n"
#define I_MULHI(r) "v_mul_hi_u32 " r ", " r ", %8\n"
#define I_MUL24(r) "v_mul_u32_u24 " r ", " r ", %8\n"
#define I_MULHI24(r) "v_mul_hi_u32_u24 " r ", " r ", %8\n"
#define I_ADDC(r) "v_addc_co_u32 " r ", vcc, " r ", %8, vcc\n"
#define I_CND(r) "v_cndmask_b32 " r ", " r ", %8, vcc\n"
#define I_DPP(r) "v_add_u32_dpp " r ", " r ", " r " row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define I_FMA64(r) ""

struct Var { const char* name; int per_iter; };
static const Var kVars[] = {
    {"v_add_u32", 32}, {"v_mul_lo_u32", 32}, {"v_mul_hi_u32", 32}, {"v_mul_u32_u24", 32},
    {"v_mul_hi_u32_u24", 32}, {"v_addc_co_u32", 32}, {"v_cndmask_b32", 32}, {"v_add_u32_dpp", 32},
};
constexpr int kNumVars = sizeof(kVars) / sizeof(kVars[0]);

template <int V>
__device__ __forceinline__ void body(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                     uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y) {
#define SG_ASM(S) asm volatile(S : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y) : "vcc")
    if constexpr (V == 0) SG_ASM(R32(I_ADD));
    if constexpr (V == 1) SG_ASM(R32(I_MULLO));
    if constexpr (V == 2) SG_ASM(R32(I_MULHI));
    if constexpr (V == 3) SG_ASM(R32(I_MUL24));
    if constexpr (V == 4) SG_ASM(R32(I_MULHI24));
    if constexpr (V == 5) SG_ASM(R32(I_ADDC));
    if constexpr (V == 6) SG_ASM(R32(I_CND));
    if constexpr (V == 7) SG_ASM(R32(I_DPP));
#undef SG_ASM
}

template <int V>
__global__ __launch_bounds__(256) void probe(unsigned long long* cyc, uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint32_t x0 = t ^ seed, x1 = t * 3u, x2 = t + 7u, x3 = t * 5u ^ seed, x4 = t + 11u, x5 = t * 13u, x6 = t ^ 0x55u,
             x7 = t + seed;
    const uint32_t y = seed | 0x01234567u;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) body<V>(x0, x1, x2, x3, x4, x5, x6, x7, y);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const uint32_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (r == 0x12345678u) out[t] = r;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

// v_mad_u64_u32 chains: 8 independent 64-bit accumulators
__global__ __launch_bounds__(256) void mad64(unsigned long long* cyc, uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint64_t a0 = t, a1 = t * 3u, a2 = t + 7u, a3 = t ^ seed, a4 = t + 11u, a5 = t * 13u, a6 = t ^ 0x55u, a7 = t + seed;
    const uint32_t y = seed | 0x01234567u;
    const uint32_t x0 = t * 7u, x1 = t * 9u, x2 = t + 5u, x3 = t ^ 77u;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a0 = (uint64_t)x0 * y + a0; a1 = (uint64_t)x1 * y + a1; a2 = (uint64_t)x2 * y + a2; a3 = (uint64_t)x3 * y + a3;
            a4 = (uint64_t)x0 * (y + 1u) + a4; a5 = (uint64_t)x1 * (y + 1u) + a5; a6 = (uint64_t)x2 * (y + 1u) + a6;
            a7 = (uint64_t)x3 * (y + 1u) + a7;
            asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((uint32_t)(r ^ (r >> 32)) == 0x12345678u) out[t] = (uint32_t)r;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

// fp64 fma chains
__global__ __launch_bounds__(256) void fma64(unsigned long long* cyc, uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    double a0 = t, a1 = t * 3.0, a2 = t + 7.0, a3 = t * 0.5, a4 = t + 11.0, a5 = t * 13.0, a6 = t * 0.25, a7 = t + 1.0;
    const double m = 1.0 + seed * 1e-12, c = 1e-3;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
            a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const double r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (r == 0.123) out[t] = 1;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

// ---- the product's radix-2^32 Horner step (sg_kernels.hip horner_step) ----
struct H32 { uint32_t h0, h1, h2, h3, h4; };
__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
    return __builtin_addc(a, b, cin, cout);
}
__device__ __forceinline__ void horner_step(H32& h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t pad,
                                            uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t s1,
                                            uint32_t s2, uint32_t s3) {
    uint32_t c;
    const uint32_t a0 = addc(h.h0, m0, 0u, &c);
    const uint32_t a1 = addc(h.h1, m1, c, &c);
    const uint32_t a2 = addc(h.h2, m2, c, &c);
    const uint32_t a3 = addc(h.h3, m3, c, &c);
    const uint32_t a4 = h.h4 + pad + c;
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
    h.h0 = addc((uint32_t)d0, f, 0u, &c);
    h.h1 = addc(e1, 0u, c, &c);
    h.h2 = addc(e2, 0u, c, &c);
    h.h3 = addc(e3, 0u, c, &c);
    h.h4 = e4 + c;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void horner(unsigned long long* cyc, uint32_t* out, uint32_t seed, int steps) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    const uint32_t r0 = __builtin_amdgcn_readfirstlane(seed & 0x0fffffffu);
    const uint32_t r1 = __builtin_amdgcn_readfirstlane((seed * 3u) & 0x0ffffffcu);
    const uint32_t r2 = __builtin_amdgcn_readfirstlane((seed * 5u) & 0x0ffffffcu);
    const uint32_t r3 = __builtin_amdgcn_readfirstlane((seed * 7u) & 0x0ffffffcu);
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
    H32 h[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) h[c] = H32{t + c, t * 3u, t ^ 5u, t + 9u, 1u};
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    uint32_t m0 = t, m1 = t * 7u, m2 = t ^ 0xabcdu, m3 = t + 3u;
    for (int i = 0; i < steps; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) horner_step(h[c], m0 + c, m1, m2, m3, 1u, r0, r1, r2, r3, s1, s2, s3);
        m0 += 0x9e3779b9u; m1 ^= m0;
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc ^= h[c].h0 ^ h[c].h1 ^ h[c].h2 ^ h[c].h3 ^ h[c].h4;
    if (acc == 0x12345678u) out[t] = acc;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

// ---- ChaCha20 with NB blocks per lane interleaved ----
__device__ __forceinline__ uint32_t rot_sh(uint32_t a, int e) { return (a << e) | (a >> (32 - e)); }
#define QRX(a, b, c, d) \
    a += b; d ^= a; d = rot_sh(d, 16); c += d; b ^= c; b = rot_sh(b, 12); \
    a += b; d ^= a; d = rot_sh(d, 8); c += d; b ^= c; b = rot_sh(b, 7);
template <int NB>
__global__ __launch_bounds__(256) void chacha(unsigned long long* cyc, uint32_t* out, uint32_t seed, int nblk) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint32_t acc = 0;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int blk = 0; blk < nblk; blk += NB) {
        uint32_t x[NB][16];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, seed, seed + 1, seed + 2,
                                    seed + 3, seed + 4, seed + 5, seed + 6, seed + 7, t * 64u + blk + b, 0, seed ^ 9,
                                    seed ^ 10};
#pragma unroll
            for (int i = 0; i < 16; ++i) x[b][i] = s[i];
        }
#pragma unroll
        for (int r = 0; r < 10; ++r) {
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                QRX(x[b][0], x[b][4], x[b][8], x[b][12]) QRX(x[b][1], x[b][5], x[b][9], x[b][13])
                QRX(x[b][2], x[b][6], x[b][10], x[b][14]) QRX(x[b][3], x[b][7], x[b][11], x[b][15])
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                QRX(x[b][0], x[b][5], x[b][10], x[b][15]) QRX(x[b][1], x[b][6], x[b][11], x[b][12])
                QRX(x[b][2], x[b][7], x[b][8], x[b][13]) QRX(x[b][3], x[b][4], x[b][9], x[b][14])
            }
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc ^= x[b][i] + (i == 12 ? t * 64u + blk + b : seed + i);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    if (acc == 0x12345678u) out[t] = acc;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

static unsigned long long* g_cyc;
static uint32_t* g_out;

template <typename F>
static void measure(const char* name, double units_per_wave, int wps, F launch) {
    const int blocks = 256 * wps;
    launch(blocks);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    launch(blocks);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(blocks * 4);
    (void)hipMemcpy(c.data(), g_cyc, c.size() * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double med = (double)c[c.size() / 2];
    const double rate = (double)blocks * 4 * units_per_wave / (ms * 1e-3) / 1024.0;
    printf("%-26s wps=%2d wall=%8.3fms  %.3e units/s/SIMD  (med wave cyc %9.0f, cyc/unit/wave %.2f)\n", name, wps, ms,
           rate, med, med / units_per_wave);
    fflush(stdout);
}

template <int V>
static void run_var() {
    for (int wps : {4, 8, 16})
        measure(kVars[V].name, (double)ITERS * kVars[V].per_iter, wps,
                [](int blocks) { hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), 0, 0, g_cyc, g_out, 1u); });
}
template <int... Vs>
static void run_all(std::integer_sequence<int, Vs...>) {
    (run_var<Vs>(), ...);
}

int main() {
    (void)hipMalloc(&g_cyc, 256 * 64 * 4 * 8);
    (void)hipMalloc(&g_out, 1 << 26);
    run_all(std::make_integer_sequence<int, kNumVars>{});
    for (int wps : {4, 8, 16}) {
        measure("v_mad_u64_u32 (C)", ITERS * 32.0, wps,
                [](int b) { hipLaunchKernelGGL(mad64, dim3(b), dim3(256), 0, 0, g_cyc, g_out, 1u); });
        measure("v_fma_f64", ITERS * 32.0, wps,
                [](int b) { hipLaunchKernelGGL(fma64, dim3(b), dim3(256), 0, 0, g_cyc, g_out, 1u); });
    }
    const int steps = 64;
    for (int wps : {4, 8, 16}) {
        measure("horner step x1 chain", steps * 1.0, wps,
                [](int b) { hipLaunchKernelGGL(horner<1>, dim3(b), dim3(256), 0, 0, g_cyc, g_out, 0x12345u, 64); });
        measure("horner step x2 chains", steps * 2.0, wps,
                [](int b) { hipLaunchKernelGGL(horner<2>, dim3(b), dim3(256), 0, 0, g_cyc, g_out, 0x12345u, 64); });
    }
    const int nblk = 16;
    for (int wps : {4, 8, 16}) {
        measure("chacha 1 blk/lane", nblk, wps,
                [](int b) { hipLaunchKernelGGL(chacha<1>, dim3(b), dim3(256), 0, 0, g_cyc, g_out, 1u, 16); });
        measure("chacha 2 blk/lane", nblk, wps,
                [](int b) { hipLaunchKernelGGL(chacha<2>, dim3(b), dim3(256), 0, 0, g_cyc, g_out, 1u, 16); });
    }
    return 0;
}
