// Timing probe for the wave-per-record C1 kernel (suruga_amd/csrc/sg_wpr.hip).
// NOT product code: a copy of the record kernel with knobs that remove parts of
// the work (the MAC, the rounds, the LDS output staging, the lock-step
// barriers, the epilogue) so that each part's cost can be measured on the GPU.
// Variants with a part removed produce wrong output; only the full variant is
// checked, against the library's own sg_seal_batch result.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I suruga_amd/csrc -I tools tools/wpr_probe.hip \
//          -L suruga_amd -lsuruga_gpu -Wl,-rpath,$PWD/suruga_amd -o tools/wpr_probe
// Run:   tools/wpr_probe [records]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/suruga_gpu.h"
#include "chacha_grp.inc"  // tools/gen_chacha_grp.py: every barrier variant
#include "sg_device.h"
#include "sg_internal.h"

using namespace sg;
using namespace sg::dev;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr uint32_t kWaves = 8, kChunk = 4096, kLines = 40, kLineBytes = 48, kLinesOff = 2 * kChunk;
constexpr uint32_t kWaveLds = 2 * kChunk + kLines * kLineBytes + 64;

enum : int { NOMAC = 1, NOROUNDS = 2, OUTDIRECT = 4, NOBAR = 8, NOEPI = 16, NOMEM = 32, BAR2 = 64, NOTREAD = 128 };

__device__ __forceinline__ uint32_t bytes_from(uint32_t w, uint32_t lo) {
    if (lo <= 4u * w) return 0xffffffffu;
    if (lo >= 4u * w + 4u) return 0u;
    return 0xffffffffu << (8u * (lo - 4u * w));
}
typedef const __attribute__((address_space(4))) uint32_t* cu32p;
__device__ __forceinline__ uint32_t cload(const void* base, uint64_t word) { return ((cu32p)(uintptr_t)base)[word]; }
__device__ __forceinline__ void dma_chunk(uint32_t l0, const uint8_t* g0) {
    const uint8_t* g1 = g0 + 1024;
    const uint8_t* g2 = g0 + 2048;
    const uint8_t* g3 = g0 + 3072;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
        "s_mov_b32 m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, off\n\t"
        "s_mov_b32 m0, %8\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g0), "v"(g1), "v"(g2), "v"(g3), "s"(l0), "s"(uniform(l0 + 1024u)), "s"(uniform(l0 + 2048u)),
          "s"(uniform(l0 + 3072u))
        : "memory");
}
__device__ __forceinline__ void dma_one(uint32_t l0, const void* g) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(l0)
                 : "memory");
}
__device__ __forceinline__ F26 reduce_words8(const uint32_t w[8]) {
    uint64_t t = (uint64_t)__builtin_amdgcn_alignbit(w[5], w[4], 2) * 5u + w[0];
    const uint32_t y0 = (uint32_t)t;
    t = (uint64_t)__builtin_amdgcn_alignbit(w[6], w[5], 2) * 5u + w[1] + (t >> 32);
    const uint32_t y1 = (uint32_t)t;
    t = (uint64_t)__builtin_amdgcn_alignbit(w[7], w[6], 2) * 5u + w[2] + (t >> 32);
    const uint32_t y2 = (uint32_t)t;
    t = (uint64_t)(w[7] >> 2) * 5u + w[3] + (t >> 32);
    const uint32_t y3 = (uint32_t)t;
    t = (uint64_t)(w[4] & 3u) + (t >> 32);
    const uint64_t u = (uint64_t)(uint32_t)(t >> 2) * 5u + y0;
    uint32_t c;
    const uint32_t z1 = addc(y1, (uint32_t)(u >> 32), 0u, &c);
    const uint32_t z2 = addc(y2, 0u, c, &c);
    const uint32_t z3 = addc(y3, 0u, c, &c);
    const uint32_t z4 = ((uint32_t)t & 3u) + c;
    F26 f = words_to_f26((uint32_t)u, z1, z2, z3, 0u);
    f.v4 += z4 << 24;
    return f;
}

template <int V>
__device__ __forceinline__ void rounds(uint32_t* x) {
#pragma unroll 1
    for (int r = 0; r < 10; ++r) {
        if constexpr (V & NOBAR)
            asm volatile(SG_CHACHA_DR_NB1_BAR0
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                           "+v"(x[14]), "+v"(x[15]));
        else if constexpr (V & BAR2)
            asm volatile(SG_CHACHA_DR_NB1_BAR2
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                           "+v"(x[14]), "+v"(x[15]));
        else
            asm volatile(SG_CHACHA_DR_NB1_BAR1
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                           "+v"(x[14]), "+v"(x[15]));
    }
}

// seal, TLS mode only (the C1 shape)
template <int V>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void probe_kernel(const KParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    uint8_t* buf = lds + wave * kWaveLds;
    uint8_t* lines = buf + kLinesOff;
    const uint32_t lds_wave = uniform((uint32_t)(uintptr_t)buf);
    const uint32_t lds_lines = uniform(lds_wave + kLinesOff);
    const uint32_t hh = lane >> 5, q = lane & 31u;
    const uint32_t sigma = 5u;
    const uint32_t nv = 16u - sigma;
    const u32x4 vmask = {~bytes_from(0u, nv), ~bytes_from(1u, nv), ~bytes_from(2u, nv), ~bytes_from(3u, nv)};
    const uint32_t wunit = (lane & ~3u) | ((lane ^ (lane >> 4)) & 3u);
    const uint32_t xq = (lane >> 2) & 3u;
    const uint32_t ngroups = (p.count + kWaves - 1u) / kWaves;
    auto dma_chunk_of = [&](uint32_t rec, uint32_t c) {
        if constexpr (!(V & NOMEM))
            dma_chunk(lds_wave + kChunk * (c & 1u), p.in + p.in_stride * rec + kChunk * c + 16u * wunit);
    };
    auto dma_table_of = [&](uint32_t rec) {
        if (lane < kWprRecWords / 4u) dma_one(lds_lines, p.ws + (uint64_t)rec * kWprRecWords + 4u * lane);
    };
    uint32_t g = blockIdx.x;
    if (g < ngroups && g * kWaves + wave < p.count) {
        dma_chunk_of(g * kWaves + wave, 0u);
        dma_table_of(g * kWaves + wave);
    }
    bool first = true;
    for (; g < ngroups; g += gridDim.x) {
        const uint32_t rec = g * kWaves + wave;
        const bool active = rec < p.count;
        const uint32_t recl = rec < p.count ? rec : p.count - 1u;
        const uint32_t gn = g + gridDim.x, nrec = gn * kWaves + wave;
        const bool next = gn < ngroups && nrec < p.count;
        uint8_t* out = p.out + p.out_stride * recl;
        uint32_t kw[8];
#pragma unroll
        for (uint32_t i = 0; i < 8u; ++i) kw[i] = cload(p.keys, i);
        const uint64_t seq = p.seq0 + recl;
        const uint32_t n14 = bswap32((uint32_t)(seq >> 32)), n15 = bswap32((uint32_t)seq);
        if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        first = false;
        wave_lds_sync();
        const uint32_t* tab = reinterpret_cast<const uint32_t*>(lines);
        const uint32_t e = 31u - q;
        const F26 W = fmul(load_f26(tab + kWHi + 20u * hh + 5u * (e >> 3)), load_f26(tab + kWLo + 5u * (e & 7u)));
        const F26 ctot = {uniform(tab[kWCtot + 0]), uniform(tab[kWCtot + 1]), uniform(tab[kWCtot + 2]),
                          uniform(tab[kWCtot + 3]), uniform(tab[kWCtot + 4])};
        const uint32_t sk[4] = {uniform(tab[kWS + 0]), uniform(tab[kWS + 1]), uniform(tab[kWS + 2]),
                                uniform(tab[kWS + 3])};
        F26 lv = f26_zero();
        if (lane < kLines) {
            const uint32_t k = lane / 5u, u = lane - 5u * k;
            lv = fmul(load_f26(tab + kWRd + 5u * u), load_f26(tab + kWTk + 5u * k));
        }
        wave_lds_sync();
        if (lane < kLines) {
            const F26 v = canonical(lv);
            uint32_t c;
            uint32_t d[5];
            d[0] = addc(v.v0 | (v.v1 << 26), 0x80808080u, 0u, &c) ^ 0x80808080u;
            d[1] = addc((v.v1 >> 6) | (v.v2 << 20), 0x80808080u, c, &c) ^ 0x80808080u;
            d[2] = addc((v.v2 >> 12) | (v.v3 << 14), 0x80808080u, c, &c) ^ 0x80808080u;
            d[3] = addc((v.v3 >> 18) | (v.v4 << 8), 0x80808080u, c, &c) ^ 0x80808080u;
            d[4] = ((v.v4 >> 24) + 0x80u + c) ^ 0x80u;
            uint8_t* ln = lines + kLineBytes * lane;
            st16(ln, u32x4{0u, 0u, 0u, 0u});
            st16(ln + 16, u32x4{0u, 0u, 0u, 0u});
            st16(ln + 32, u32x4{0u, 0u, 0u, 0u});
#pragma unroll
            for (uint32_t i = 0; i < 17u; ++i) ln[47u - sigma - i] = (uint8_t)(d[i >> 2] >> (8u * (i & 3u)));
        } else if (lane == kLines) {
            st16(lines + kLines * kLineBytes, u32x4{0u, 0u, 0u, 0u});
        }
        wave_lds_sync();
        i32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 1 << 24;
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
            if (j > 0u) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            wave_lds_sync();
            uint8_t* cb = buf + kChunk * (j & 1u);
            u32x4 D[4];
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) D[i] = ld16(cb + 16u * (4u * lane + (i ^ xq)));
            if (j < 3u) {
                if (active) dma_chunk_of(rec, j + 1u);
            } else if (next) {
                dma_chunk_of(nrec, 0u);
            }
            const uint32_t ctr = 64u * j + lane + 1u;
            uint32_t x[16] = {kSigma0, kSigma1, kSigma2, kSigma3, kw[0], kw[1], kw[2], kw[3],
                              kw[4],   kw[5],   kw[6],   kw[7],   ctr,   0u,    n14,   n15};
            if constexpr (!(V & NOROUNDS)) rounds<V>(x);
            const u32x4 ks[4] = {u32x4{x[0] + kSigma0, x[1] + kSigma1, x[2] + kSigma2, x[3] + kSigma3},
                                 u32x4{x[4] + kw[0], x[5] + kw[1], x[6] + kw[2], x[7] + kw[3]},
                                 u32x4{x[8] + kw[4], x[9] + kw[5], x[10] + kw[6], x[11] + kw[7]},
                                 u32x4{x[12] + ctr, x[13], x[14] + n14, x[15] + n15}};
            const uint32_t kk = (1u - hh) + 2u * (3u - j);
            u32x4 O[4];
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
                O[i] = D[i] ^ ks[i];
                if constexpr (!(V & NOMAC)) {
                    const uint32_t iv = 5u * kk + 4u - i;
                    u32x4 f;
                    if constexpr (V & NOTREAD) {
                        f = u32x4{iv, iv + 1u, iv + 2u, iv + 3u};
                    } else {
                        const u32x4 Vw = ldu16(lines + kLineBytes * iv + 47u - q);
                        const u32x4 Pw = ldu16(lines + kLineBytes * iv - 17u - q);
                        f = (Vw & vmask) | (Pw & ~vmask);
                    }
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, f),
                                                                 __builtin_bit_cast(i32x4, O[i] ^ 0x80808080u), acc, 0,
                                                                 0, 0);
                }
            }
            if (j == 3u && next) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                wave_lds_sync();
                dma_table_of(nrec);
            }
            if constexpr (V & OUTDIRECT) {
                if (active) {
                    uint8_t* dst = out + kChunk * j + 64u * lane;
#pragma unroll
                    for (uint32_t i = 0; i < 4u; ++i) st16(dst + 16u * i, O[i]);
                }
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 4u; ++i) st16(cb + 16u * (4u * lane + (i ^ xq)), O[i]);
                wave_lds_sync();
                const u32x4 o0 = ld16(cb + 16u * wunit), o1 = ld16(cb + 1024u + 16u * wunit);
                const u32x4 o2 = ld16(cb + 2048u + 16u * wunit), o3 = ld16(cb + 3072u + 16u * wunit);
                if (active && !(V & NOMEM)) {
                    uint8_t* dst = out + kChunk * j + 16u * lane;
                    st16(dst, o0);
                    st16(dst + 1024, o1);
                    st16(dst + 2048, o2);
                    st16(dst + 3072, o3);
                } else if (active) {  // keep the data live
                    if ((o0.x ^ o1.y ^ o2.z ^ o3.w) == 0x12345679u) st16(out, o0);
                }
            }
            wave_lds_sync();
        }
        uint32_t tw[4] = {0u, 0u, 0u, 0u};
        if constexpr (!(V & NOEPI)) {
            uint32_t xw[8];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                uint64_t yv = (uint64_t)(uint32_t)acc[4 * m + 1] * 256u + (uint32_t)acc[4 * m];
                yv += (uint64_t)(uint32_t)acc[4 * m + 2] * 65536u;
                yv += (uint64_t)(uint32_t)acc[4 * m + 3] * 16777216u;
                xw[2 * m] = (uint32_t)yv;
                xw[2 * m + 1] = (uint32_t)(yv >> 32);
            }
            F26 f = fmul(reduce_words8(xw), W);
            auto level = [&](auto dpp) {
                f.v0 += dpp(f.v0); f.v1 += dpp(f.v1); f.v2 += dpp(f.v2); f.v3 += dpp(f.v3); f.v4 += dpp(f.v4);
            };
            level([](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true); });
            level([](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true); });
            level([](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true); });
            level([](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true); });
            level([](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xf, 0xf, true); });
            f = carry1(f);
            level([](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xf, 0xf, true); });
            auto lane63 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); };
            const F26 fs = {lane63(f.v0) + ctot.v0, lane63(f.v1) + ctot.v1, lane63(f.v2) + ctot.v2,
                            lane63(f.v3) + ctot.v3, lane63(f.v4) + ctot.v4};
            tag_words(fs, sk, tw);
        } else {
            tw[0] = (uint32_t)acc[0] ^ W.v0 ^ ctot.v0 ^ sk[0];
        }
        if (active && lane == 0u) st16(out + kWprN, u32x4{tw[0], tw[1], tw[2], tw[3]});
    }
}

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

template <int V>
float run_variant(const KParams& p, int grid, int reps) {
    const size_t lds = kWaves * kWaveLds;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((probe_kernel<V>), dim3(grid), dim3(512), lds, 0, p);  // warm-up
    CK(hipGetLastError());
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe_kernel<V>), dim3(grid), dim3(512), lds, 0, p);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const uint32_t count = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const uint32_t n = 16384;
    uint8_t *pt, *ct, *ct2, *keys, *ws;
    const size_t wsz = sg_workspace_size(count);
    CK(hipMalloc(&pt, (size_t)count * n));
    CK(hipMalloc(&ct, (size_t)count * (n + 16)));
    CK(hipMalloc(&ct2, (size_t)count * (n + 16)));
    CK(hipMalloc(&keys, 32));
    CK(hipMalloc(&ws, wsz));
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)i;
    CK(hipMemcpy(keys, key, 32, hipMemcpyHostToDevice));
    if (sg_fill_records(pt, n, n, count, 0x53555255ull, 0, nullptr) != SG_OK) return 1;
    sg_batch b;
    memset(&b, 0, sizeof b);
    b.count = count;
    b.flags = SG_BATCH_TLS;
    b.keys = keys;
    b.num_keys = 1;
    b.content_type = 23;
    b.ver_major = 3;
    b.ver_minor = 3;
    b.in = pt;
    b.in_stride = n;
    b.out = ct;
    b.out_stride = n + 16;
    b.uniform_len = n;
    b.workspace = ws;
    b.workspace_size = wsz;
    if (sg_seal_batch(&b) != SG_OK) {
        fprintf(stderr, "seal: %s\n", sg_last_error());
        return 1;
    }
    CK(hipDeviceSynchronize());
    KParams p;
    memset(&p, 0, sizeof p);
    p.keys = keys;
    p.in = pt;
    p.in_stride = n;
    p.out = ct2;
    p.out_stride = n + 16;
    p.ws = (uint32_t*)ws;
    p.uniform_len = n;
    p.count = count;
    p.tls = 1;
    p.ad_len = 13;
    p.tls_hdr = 23u | (3u << 8) | (3u << 16);
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid2 = 2 * cus, grid1 = cus;
    const int reps = 5;
    // full variant: correctness against the library
    run_variant<0>(p, grid2, 1);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> h1((size_t)count * (n + 16)), h2((size_t)count * (n + 16));
    CK(hipMemcpy(h1.data(), ct, h1.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), ct2, h2.size(), hipMemcpyDeviceToHost));
    printf("full variant matches the library: %s\n", memcmp(h1.data(), h2.data(), h1.size()) == 0 ? "yes" : "NO");
    // library timing
    hipEvent_t a, bb;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&bb));
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) sg_seal_batch(&b);
    CK(hipEventRecord(bb, 0));
    CK(hipEventSynchronize(bb));
    float lib_ms = 0;
    CK(hipEventElapsedTime(&lib_ms, a, bb));
    printf("library sg_seal_batch (keying + record kernel): %.3f ms\n", lib_ms / reps);
#define RUN(V, G, NAME) printf("%-44s grid %4d: %.3f ms\n", NAME, G, run_variant<V>(p, G, reps))
    RUN(0, grid2, "full");
    RUN(0, grid1, "full, 1 WG/CU");
    RUN(NOMAC, grid2, "no MAC");
    RUN(NOTREAD, grid2, "MAC without T-window LDS reads");
    RUN(NOEPI, grid2, "no epilogue");
    RUN(NOROUNDS, grid2, "no rounds");
    RUN(NOROUNDS | NOMAC, grid2, "no rounds, no MAC (memory path)");
    RUN(OUTDIRECT, grid2, "direct 64-B-stride stores");
    RUN(NOBAR, grid2, "rounds without s_barrier");
    RUN(BAR2, grid2, "s_barrier every 2nd rotate group");
    RUN(NOMEM, grid2, "no global loads/stores");
    RUN(NOMEM | NOMAC, grid2, "no memory, no MAC (rounds only)");
    return 0;
}
