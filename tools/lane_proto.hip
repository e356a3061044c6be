// Prototype: one record per LANE (sequential ChaCha20 + Poly1305 Horner per lane)
// vs the library's one-record-per-workgroup seal kernel, C1 shape (TLS mode,
// n multiple of 64, 16-aligned records).  Checks bit-exactness against the
// library output and times both in one process.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/suruga_gpu.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(a, b, c, d) a += b; d ^= a; d = rotl32(d, 16); c += d; b ^= c; b = rotl32(b, 12); \
                       a += b; d ^= a; d = rotl32(d, 8); c += d; b ^= c; b = rotl32(b, 7);

__device__ __forceinline__ void chacha_block(uint32_t ks[16], const uint32_t k[8], uint32_t ctr, uint32_t n14, uint32_t n15) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x12 = ctr, x13 = 0u, x14 = n14, x15 = n15;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        QR(x0, x4, x8, x12) QR(x1, x5, x9, x13) QR(x2, x6, x10, x14) QR(x3, x7, x11, x15)
        QR(x0, x5, x10, x15) QR(x1, x6, x11, x12) QR(x2, x7, x8, x13) QR(x3, x4, x9, x14)
    }
    ks[0] = x0 + 0x61707865u; ks[1] = x1 + 0x3320646eu; ks[2] = x2 + 0x79622d32u; ks[3] = x3 + 0x6b206574u;
    ks[4] = x4 + k[0]; ks[5] = x5 + k[1]; ks[6] = x6 + k[2]; ks[7] = x7 + k[3];
    ks[8] = x8 + k[4]; ks[9] = x9 + k[5]; ks[10] = x10 + k[6]; ks[11] = x11 + k[7];
    ks[12] = x12 + ctr; ks[13] = x13; ks[14] = x14 + n14; ks[15] = x15 + n15;
}

__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) { return __builtin_addc(a, b, cin, cout); }

struct H32 { uint32_t h0, h1, h2, h3, h4; };
struct RK { uint32_t r0, r1, r2, r3, s1, s2, s3; };

__device__ __forceinline__ void horner(H32& h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t pad, const RK& k) {
    uint32_t c;
    const uint32_t a0 = addc(h.h0, m0, 0u, &c), a1 = addc(h.h1, m1, c, &c), a2 = addc(h.h2, m2, c, &c), a3 = addc(h.h3, m3, c, &c);
    const uint32_t a4 = h.h4 + pad + c;
    const uint64_t d0 = (uint64_t)a0 * k.r0 + (uint64_t)a1 * k.s3 + (uint64_t)a2 * k.s2 + (uint64_t)a3 * k.s1;
    const uint64_t d1 = (uint64_t)a0 * k.r1 + (uint64_t)a1 * k.r0 + (uint64_t)a2 * k.s3 + (uint64_t)a3 * k.s2 + (uint64_t)a4 * k.s1;
    const uint64_t d2 = (uint64_t)a0 * k.r2 + (uint64_t)a1 * k.r1 + (uint64_t)a2 * k.r0 + (uint64_t)a3 * k.s3 + (uint64_t)a4 * k.s2;
    const uint64_t d3 = (uint64_t)a0 * k.r3 + (uint64_t)a1 * k.r2 + (uint64_t)a2 * k.r1 + (uint64_t)a3 * k.r0 + (uint64_t)a4 * k.s3;
    const uint32_t e1 = addc((uint32_t)d1, (uint32_t)(d0 >> 32), 0u, &c);
    const uint32_t e2 = addc((uint32_t)d2, (uint32_t)(d1 >> 32), c, &c);
    const uint32_t e3 = addc((uint32_t)d3, (uint32_t)(d2 >> 32), c, &c);
    uint32_t e4 = a4 * k.r0 + (uint32_t)(d3 >> 32) + c;
    const uint32_t f = (e4 >> 2) * 5u;
    e4 &= 3u;
    h.h0 = addc((uint32_t)d0, f, 0u, &c); h.h1 = addc(e1, 0u, c, &c); h.h2 = addc(e2, 0u, c, &c); h.h3 = addc(e3, 0u, c, &c);
    h.h4 = e4 + c;
}

// final: h mod p, + s mod 2^128 (h < 2^131 partially reduced)
__device__ __forceinline__ void finish(H32 h, const uint32_t s[4], uint32_t t[4]) {
    // fully reduce: fold h4 >> 2 again, then conditional subtract p
    uint32_t c;
    uint32_t f = (h.h4 >> 2) * 5u; h.h4 &= 3u;
    h.h0 = addc(h.h0, f, 0u, &c); h.h1 = addc(h.h1, 0u, c, &c); h.h2 = addc(h.h2, 0u, c, &c); h.h3 = addc(h.h3, 0u, c, &c); h.h4 += c;
    // g = h + 5; if g >= 2^130 then h = g - 2^130
    uint32_t g0 = addc(h.h0, 5u, 0u, &c), g1 = addc(h.h1, 0u, c, &c), g2 = addc(h.h2, 0u, c, &c), g3 = addc(h.h3, 0u, c, &c);
    uint32_t g4 = h.h4 + c;
    const uint32_t m = 0u - (g4 >> 2);  // all ones if g >= 2^130
    h.h0 = (g0 & m) | (h.h0 & ~m); h.h1 = (g1 & m) | (h.h1 & ~m); h.h2 = (g2 & m) | (h.h2 & ~m); h.h3 = (g3 & m) | (h.h3 & ~m);
    t[0] = addc(h.h0, s[0], 0u, &c); t[1] = addc(h.h1, s[1], c, &c); t[2] = addc(h.h2, s[2], c, &c); t[3] = addc(h.h3, s[3], c, &c);
}

__device__ __forceinline__ uint32_t ab24(uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbit(hi, lo, 24); }

// seal, TLS mode, n = 64 m, record i at in + i*n, out + i*(n+16)
__global__ __launch_bounds__(256) void lane_seal(const uint8_t* in, uint8_t* out, const uint32_t* key, uint64_t seq0,
                                                 uint32_t n, uint32_t count, uint64_t istride, uint64_t ostride) {
    const uint32_t rec = blockIdx.x * 256u + threadIdx.x;
    if (rec >= count) return;
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = key[i];
    const uint64_t seq = seq0 + rec;
    const uint32_t n14 = __builtin_bswap32((uint32_t)(seq >> 32)), n15 = __builtin_bswap32((uint32_t)seq);
    uint32_t ks[16];
    chacha_block(ks, k, 0u, n14, n15);
    RK rk;
    rk.r0 = ks[0] & 0x0fffffffu; rk.r1 = ks[1] & 0x0ffffffcu; rk.r2 = ks[2] & 0x0ffffffcu; rk.r3 = ks[3] & 0x0ffffffcu;
    rk.s1 = rk.r1 + (rk.r1 >> 2); rk.s2 = rk.r2 + (rk.r2 >> 2); rk.s3 = rk.r3 + (rk.r3 >> 2);
    const uint32_t s[4] = {ks[4], ks[5], ks[6], ks[7]};
    // MAC block 0: ad[0..13) || 13 || 0 0  ; ad = be64(seq) || 23 3 3 || be16(n)
    H32 h = {0, 0, 0, 0, 0};
    const uint32_t ad0 = __builtin_bswap32((uint32_t)(seq >> 32)), ad1 = __builtin_bswap32((uint32_t)seq);
    const uint32_t ad2 = 23u | (3u << 8) | (3u << 16) | ((n >> 8) & 0xffu) << 24;
    const uint32_t ad3 = (n & 0xffu) | (13u << 8);
    horner(h, ad0, ad1, ad2, ad3, 1u, rk);
    const u32x4* src = reinterpret_cast<const u32x4*>(in + (uint64_t)rec * istride);
    u32x4* dst = reinterpret_cast<u32x4*>(out + (uint64_t)rec * ostride);
    uint32_t p14 = 0, p15 = 0;  // ct dwords 14, 15 of the previous chunk (stream "len" bytes for chunk 0)
    const uint32_t m = n >> 6;
    for (uint32_t c = 0; c < m; ++c) {
        const u32x4 d0 = src[4 * c], d1 = src[4 * c + 1], d2 = src[4 * c + 2], d3 = src[4 * c + 3];
        chacha_block(ks, k, c + 1u, n14, n15);
        const u32x4 c0 = d0 ^ u32x4{ks[0], ks[1], ks[2], ks[3]};
        const u32x4 c1 = d1 ^ u32x4{ks[4], ks[5], ks[6], ks[7]};
        const u32x4 c2 = d2 ^ u32x4{ks[8], ks[9], ks[10], ks[11]};
        const u32x4 c3 = d3 ^ u32x4{ks[12], ks[13], ks[14], ks[15]};
        dst[4 * c] = c0; dst[4 * c + 1] = c1; dst[4 * c + 2] = c2; dst[4 * c + 3] = c3;
        // MAC blocks 4c+1..4c+4: stream dword s = ab24(ct[s-5], ct[s-6]); for c = 0 the two
        // "previous" dwords are stream dwords 4 (len bytes 3..6 = 0) -> handled by p = 0 and
        // block 1 dword 0 = stream dword 4 = 0.
        const uint32_t b1w0 = c == 0 ? 0u : ab24(p15, p14);
        horner(h, b1w0, ab24(c0.x, p15), ab24(c0.y, c0.x), ab24(c0.z, c0.y), 1u, rk);
        horner(h, ab24(c0.w, c0.z), ab24(c1.x, c0.w), ab24(c1.y, c1.x), ab24(c1.z, c1.y), 1u, rk);
        horner(h, ab24(c1.w, c1.z), ab24(c2.x, c1.w), ab24(c2.y, c2.x), ab24(c2.z, c2.y), 1u, rk);
        horner(h, ab24(c2.w, c2.z), ab24(c3.x, c2.w), ab24(c3.y, c3.x), ab24(c3.z, c3.y), 1u, rk);
        p14 = c3.z; p15 = c3.w;
    }
    // last block: ct bytes 64m-5..64m (5 bytes) || le64(n) : 13 bytes, pad bit at byte 13
    {
        const uint32_t w0 = ab24(p15, p14);
        const uint32_t w1 = ab24(n, p15);
        const uint32_t w2 = ab24(0u, n);
        const uint32_t w3 = 0x100u;  // byte 12 = len byte 7 = 0, pad at byte 13
        horner(h, w0, w1, w2, w3, 0u, rk);
    }
    uint32_t t[4];
    finish(h, s, t);
    uint32_t* tp = reinterpret_cast<uint32_t*>(out + (uint64_t)rec * ostride + n);
    tp[0] = t[0]; tp[1] = t[1]; tp[2] = t[2]; tp[3] = t[3];
}

__global__ void fill(uint8_t* p, size_t bytes) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < bytes / 8; i += (size_t)gridDim.x * 256) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
        reinterpret_cast<uint64_t*>(p)[i] = x;
    }
}

int main(int argc, char** argv) {
    const uint32_t n = 16384, count = argc > 1 ? atoi(argv[1]) : (1u << 20);
    uint8_t *pt, *ct_lib, *ct_lane, *keys, *st;
    void* ws;
    CHECK(hipMalloc(&pt, (size_t)(n + 4096) * count));
    CHECK(hipMalloc(&ct_lib, (size_t)(n + 16) * count));
    CHECK(hipMalloc(&ct_lane, (size_t)(n + 4096) * count));
    CHECK(hipMalloc(&keys, 64));
    CHECK(hipMalloc(&st, count));
    CHECK(hipMalloc(&ws, sg_workspace_size(count)));
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)i;
    CHECK(hipMemcpy(keys, key, 32, hipMemcpyHostToDevice));
    fill<<<4096, 256>>>(pt, (size_t)(n + 4096) * count);
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    sg_batch b;
    memset(&b, 0, sizeof b);
    b.count = count; b.flags = SG_BATCH_TLS; b.keys = keys; b.num_keys = 1; b.content_type = 23; b.ver_major = 3; b.ver_minor = 3;
    b.in = pt; b.in_stride = n; b.out = ct_lib; b.out_stride = n + 16; b.uniform_len = n; b.stream = s; b.workspace = ws;
    b.workspace_size = sg_workspace_size(count);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int round = 0; round < 4; ++round) {
        CHECK(hipEventRecord(e0, s));
        if (sg_seal_batch(&b) != 0) { printf("lib err %s\n", sg_last_error()); return 1; }
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms_lib; CHECK(hipEventElapsedTime(&ms_lib, e0, e1));
        CHECK(hipEventRecord(e0, s));
        lane_seal<<<(count + 255) / 256, 256, 0, s>>>(pt, ct_lane, (const uint32_t*)keys, 0, n, count, n, n + 16);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms_lane; CHECK(hipEventElapsedTime(&ms_lane, e0, e1));
        printf("round %d: library seal (keying+wg kernel) %.3f ms, lane-per-record seal %.3f ms\n", round, ms_lib, ms_lane);
    }
    const uint64_t strides[][2] = {{16384, 16400}, {16448, 16464}, {16384 + 1088, 16400 + 1088}, {16384 + 4096, 16400 + 4000}};
    for (auto& st2 : strides) {
        float best = 1e9;
        for (int r = 0; r < 3; ++r) {
            CHECK(hipEventRecord(e0, s));
            lane_seal<<<(count + 255) / 256, 256, 0, s>>>(pt, ct_lane, (const uint32_t*)keys, 0, n, count, st2[0], st2[1]);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("lane seal, in stride %lu out stride %lu: %.3f ms\n", (unsigned long)st2[0], (unsigned long)st2[1], best);
    }
    lane_seal<<<(count + 255) / 256, 256, 0, s>>>(pt, ct_lane, (const uint32_t*)keys, 0, n, count, n, n + 16);
    CHECK(hipStreamSynchronize(s));
    std::vector<uint8_t> a((size_t)(n + 16) * 4096), c((size_t)(n + 16) * 4096);
    CHECK(hipMemcpy(a.data(), ct_lib, a.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(c.data(), ct_lane, c.size(), hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < a.size(); ++i) bad += a[i] != c[i];
    printf("first 4096 records: %zu differing bytes (tags: %s)\n", bad, memcmp(a.data() + n, c.data() + n, 16) == 0 ? "rec0 tag equal" : "rec0 tag DIFFERS");
    return bad != 0;
}
