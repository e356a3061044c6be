// sg_wpr.hip -- gfx950 wave-per-record ChaCha20-Poly1305 for full 16 KiB TLS
// records (klutzy/suruga src/cipher/chacha20_poly1305.rs:48-94 on records of
// RECORD_MAX_LEN = 2^14 bytes, tls.rs:32,137-147).
//
// One wave owns one record; a 512-thread workgroup holds eight records, two
// workgroups share a CU (four waves per SIMD), and the persistent grid takes
// record groups from a device counter.  Per record the wave runs four
// iterations over 4 KiB chunks:
//
//   * the chunk arrives by LDS-DMA, lane-contiguously (16 B per lane, 1 KiB
//     per instruction, prefetched one chunk ahead, one piece per double round)
//     into the wave's LDS slice through an XOR swizzle, so that lane t then
//     reads its own 64-byte block 64 j + t conflict-free;
//   * lane t computes keystream block 64 j + t + 1 (chacha20.rs:111-135, block
//     0 being the Poly1305 key, chacha20_poly1305.rs:50-52) with grouped ARX
//     rounds and an s_barrier after every rotate group (sg_chacha_grp.inc),
//     which keeps the waves of each SIMD in lock-step so that their full-rate
//     add/xor instructions pair up;
//   * the XOR result is staged in the same swizzled slice and leaves
//     lane-contiguously during the next chunk's first double rounds;
//   * Poly1305 is fed from the ciphertext registers themselves: the wave's 64
//     lanes hold 256 consecutive 16-byte ciphertext chunks, which are the B
//     operands of four v_mfma_i32_32x32x32_i8 per iteration, issued during the
//     next iteration's rounds (see "MAC" below).
//
// MAC.  The reference evaluates h = sum_b v_b r^(B - b) over the 16-byte
// blocks of ad || le64(|ad|) || ct || le64(|ct|) (chacha20_poly1305.rs:19-42,
// poly1305.rs:207-228).  Ciphertext chunk m (bytes 16 m .. 16 m + 15) starts
// at stream offset o + 16 m, o = |ad| + 8 = 16 beta + sigma, so its byte a' has
// weight 2^(8 (sigma + a')) r^(E(m) + 1) when sigma + a' < 16 and
// 2^(8 (sigma + a' - 16)) r^E(m) otherwise, with E(m) = B - beta - 1 - m.
// Chunk m = 256 j + 128 h + 4 q + i (iteration j, lane 32 h + q, chunk i of
// the lane's block) factors as E(m) = 4 (31 - q) + e(j, h, i),
// e = 128 (1 - h) + 256 (3 - j) + (4 - i) + delta.  Each MFMA step (j, i) then
// computes D[c][q] += sum_{h, a'} T[c][(h, a')] (byte - 128), where column q
// is the lane's chunk and row c a base-256 digit position: T holds the signed
// digits of r^(e + 1) and r^e, shifted by sigma + a' (a Toeplitz band).  The
// eight powers per step, r^(128 k + 1 + delta + u) (k = 0..7, u = 0..4), are
// built once per record as 48-byte digit lines in LDS; a lane reads its
// 16-byte T fragment as two windows of two adjacent lines (aligned dwords
// shifted with v_alignbyte).  |D| <
// 2^23, so with the accumulator seeded at 2^24 every entry is a positive
// 25-bit integer.  At the end each lane assembles its 16 entries exactly,
// X = sum_r D[c_r][q] 2^(8 c_r), reduces it mod 2^130 - 5, multiplies by
// W = r^(4 (31 - q)) (times 2^32 for the upper half-wave) and a DPP sum adds
// the 64 terms.  The keying kernel supplies the per-record constant ctot:
// the AD / length blocks, the pad bits, the i8 bias and the seed.  Every step
// is exact arithmetic mod p, so tags equal the reference's bit for bit
// (tests/test_wpr_mac_model.py pins this decomposition against the CPU
// restatement of poly1305.rs).
#include "sg_internal.h"
#include "sg_device.h"
#include "sg_chacha_grp.inc"  // grouped ChaCha20 double round (tools/gen_chacha_grp.py --product)

#include <stdint.h>
#include <stdlib.h>

namespace sg {
namespace {

using namespace dev;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr uint32_t kWprWaves = 8;           // records per 512-thread workgroup
constexpr uint32_t kWprChunk = 4096;        // bytes per wave iteration
constexpr uint32_t kWprLines = 40;          // T digit lines per record
constexpr uint32_t kWprLineBytes = 48;
constexpr uint32_t kWprLinesOff = 2 * kWprChunk;  // two chunk buffers, then the T lines
constexpr uint32_t kWprWaveLds = 2 * kWprChunk + kWprLines * kWprLineBytes + 64;  // 10176: two workgroups per CU
constexpr uint32_t kWprKeyThreads = 64;
constexpr uint32_t kWprKeyStride = 81;      // LDS words per record and half

// Geometry of the MAC stream ad || le64(|ad|) || ct || le64(n) for n = 2^14.
struct WprGeom {
    uint32_t o, sigma, beta, B, rem, delta;
};
__device__ __forceinline__ WprGeom wpr_geom(uint32_t adlen) {
    WprGeom g;
    g.o = adlen + 8u;
    g.sigma = g.o & 15u;
    g.beta = g.o >> 4;
    const uint32_t L = adlen + 16u + kWprN;
    g.B = (L + 15u) >> 4;
    g.rem = L - 16u * (g.B - 1u);
    g.delta = g.B - g.beta - 1u - 1024u;  // 0 or 1
    return g;
}

// bytes >= lo of a little-endian word set: mask of the bytes whose index
// (4 w + byte) is >= lo
__device__ __forceinline__ uint32_t bytes_from(uint32_t w, uint32_t lo) {
    if (lo <= 4u * w) return 0xffffffffu;
    if (lo >= 4u * w + 4u) return 0u;
    return 0xffffffffu << (8u * (lo - 4u * w));
}

// p - (2^24 * sum_{c<32} 2^(8c) mod p) in radix 2^26: the seed of the 32 x 32
// accumulator, negated (tests/test_wpr_mac_model.py: CJ)
constexpr uint32_t kCJ0 = 0x1bd2d2bu, kCJ1 = 0x36f6f6fu, kCJ2 = 0x3dbdbdbu, kCJ3 = 0x2f6f6f6u, kCJ4 = 0x1bdbdbdu;

// ---------------------------------------------------------------------------
// Keying pre-pass: one lane per record, 64 records per wave, the 160-word
// record (sg_internal.h, kW*) staged in LDS by halves and stored coalesced.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wpr_flush_half(const KParams& p, uint32_t rec0, uint32_t half, const uint32_t* stage,
                                               uint32_t lane) {
    const uint32_t nrec = p.count - rec0 < kWprKeyThreads ? p.count - rec0 : kWprKeyThreads;
    const uint32_t nvec = nrec * 20u;  // 80 words = 20 x 16 B per record and half
    for (uint32_t v = lane; v < nvec; v += kWprKeyThreads) {
        const uint32_t rr = v / 20u, c = v - rr * 20u;
        const uint32_t* src = stage + rr * kWprKeyStride + 4u * c;
        st16(p.ws + (uint64_t)(rec0 + rr) * kWprRecWords + 80u * half + 4u * c, u32x4{src[0], src[1], src[2], src[3]});
    }
}

template <bool OPEN>
__global__ __launch_bounds__(64) void sg_wpr_keying_kernel(const KParams p) {
    __shared__ uint32_t stage[kWprKeyThreads * kWprKeyStride];
    const uint32_t lane = threadIdx.x;
    const uint32_t rec0 = blockIdx.x * kWprKeyThreads;
    const uint32_t rec = rec0 + lane;
    uint32_t* st = stage + lane * kWprKeyStride;
    const uint32_t adlen = p.tls ? 13u : p.ad_len;
    const WprGeom G = wpr_geom(adlen);
    if (blockIdx.x == 0u && lane == 0u) p.ws[(uint64_t)p.count * kWprRecWords] = 0u;  // the AEAD kernel's group counter

    F26 r = f26_zero();
    uint32_t s[4] = {0u, 0u, 0u, 0u};
    RecKey rk = {};
    const bool act = rec < p.count;
    if (act) {
        rk = record_key(p, rec);
        uint32_t ks[16];
        chacha_block(ks, rk.k, 0u, rk.n14, rk.n15);  // block 0 -> poly key (chacha20_poly1305.rs:50,75)
        // r = clamp(pk[0..16]) (poly1305.rs:197-203), s = pk[16..32] (chacha20_poly1305.rs:32-39)
        r = words_to_f26(ks[0] & 0x0fffffffu, ks[1] & 0x0ffffffcu, ks[2] & 0x0ffffffcu, ks[3] & 0x0ffffffcu, 0u);
        s[0] = ks[4]; s[1] = ks[5]; s[2] = ks[6]; s[3] = ks[7];
    }

    // ---- second half: lo[b] = R^b, hi[h][a] = 2^(32 h) R^(8 a) (R = r^4) ----
    const F26 r2 = fmul(r, r), R = fmul(r2, r2);
    F26 x = f26_one(), sum_lo = f26_zero();
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        store_f26(st + (kWLo - 80u) + 5u * b, x);
        sum_lo = f26_add(sum_lo, x);
        x = fmul(x, R);
    }
    const F26 R8 = x;
    F26 y = f26_one(), sum_hi = f26_zero();
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        store_f26(st + (kWHi - 80u) + 5u * a, y);
        store_f26(st + (kWHi - 80u) + 20u + 5u * a, mul_add(y, 0u, 64u, 0u, 0u, 0u, f26_zero()));  // * 2^32
        sum_hi = f26_add(sum_hi, y);
        y = fmul(y, R8);
    }
    const F26 T = y;  // R^32 = r^128
    __syncthreads();
    wpr_flush_half(p, rec0, 1u, stage, lane);
    __syncthreads();

    // ---- first half: s, ctot, rd[u] = r^(1 + delta + u), tk[k] = T^k ----
    st[kWS + 0] = s[0]; st[kWS + 1] = s[1]; st[kWS + 2] = s[2]; st[kWS + 3] = s[3];
    const F26 r3 = fmul(r2, r), r5 = fmul(R, r), r6 = fmul(R, r2);
    const bool d1 = G.delta != 0u;
    const F26 pw[6] = {r, r2, r3, R, r5, r6};
#pragma unroll
    for (int u = 0; u < 5; ++u) store_f26(st + kWRd + 5u * u, d1 ? pw[u + 1] : pw[u]);
    const F26 rd0 = d1 ? r2 : r;        // r^(1 + delta)
    const F26 rdel = d1 ? r : f26_one();  // r^delta
    F26 t = f26_one(), sum_t = f26_zero();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        store_f26(st + kWTk + 5u * k, t);
        sum_t = f26_add(sum_t, t);
        t = fmul(t, T);
    }
    const F26 T8 = t;  // r^1024

    // geometric sums: SW = sum_{u<32} R^u, g = G(1024) = (r + r^2 + r^3 + r^4) SW sum_k T^k
    const F26 SW = fmul(carry1(sum_hi), carry1(sum_lo));
    const F26 G4 = carry1(f26_add(f26_add(r, r2), f26_add(r3, R)));
    const F26 g = fmul(fmul(G4, SW), carry1(sum_t));
    // pads (poly1305.rs:224-225): 2^128 sum_{b < B-1} r^(B-b) + 2^(8 rem) r
    //   = 2^128 G(B) + (2^(8 rem) + p - 2^128) r,  G(B) = G(1024) + r^1024 G(B - 1024)
    const F26 GB = fmul_add(T8, geo_sum(r, G.B - 1024u), g);
    F26 pads = mul_add(GB, 0u, 0u, 0u, 0u, 1u << 24, f26_zero());
    {
        F26 cf = F26{0x3fffffbu, 0x3ffffffu, 0x3ffffffu, 0x3ffffffu, 0x2ffffffu};  // p - 2^128
        const uint32_t bit = 8u * G.rem, li = bit / 26u, v = 1u << (bit - 26u * li);
        cf.v0 += li == 0u ? v : 0u;
        cf.v1 += li == 1u ? v : 0u;
        cf.v2 += li == 2u ? v : 0u;
        cf.v3 += li == 3u ? v : 0u;
        cf.v4 += li == 4u ? v : 0u;
        pads = fmul_add(cf, r, pads);
    }
    // i8 bias: 128 sum over the ciphertext bytes of their weights
    //   = r^delta G(1024) (A1 r + A2),  A1 = sum_{k=sigma}^{15} 128 2^(8k),  A2 = sum_{k<sigma} 128 2^(8k)
    F26 bias;
    {
        uint32_t a1[4], a2[4];
#pragma unroll
        for (uint32_t w = 0; w < 4; ++w) {
            const uint32_t m = bytes_from(w, G.sigma);
            a1[w] = 0x80808080u & m;
            a2[w] = 0x80808080u & ~m;
        }
        const F26 A1 = words_to_f26(a1[0], a1[1], a1[2], a1[3], 0u);
        const F26 A2 = words_to_f26(a2[0], a2[1], a2[2], a2[3], 0u);
        bias = fmul(fmul(g, fmul_add(A1, r, A2)), rdel);
    }
    // accumulator seed: -(2^24 sum_c 2^(8c)) SW
    const F26 seed = mul_add(SW, kCJ0, kCJ1, kCJ2, kCJ3, kCJ4, f26_zero());
    // prefix ad || le64(|ad|) (stream bytes < o) as blocks 0..beta: Horner, then r^(B - beta) = r^1024 r^(1 + delta)
    F26 hp = f26_zero();
    if (act) {
        for (uint32_t b = 0; b <= G.beta; ++b) {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (uint32_t i = 0; i < 16u; ++i) {
                const uint32_t pos = 16u * b + i;
                if (pos < G.o) w[i >> 2] |= (uint32_t)prefix_byte(p, rec, rk.seq, kWprN, adlen, pos) << (8u * (i & 3u));
            }
            hp = fmul_add(hp, r, words_to_f26(w[0], w[1], w[2], w[3], 0u));
        }
    }
    const F26 prefix = fmul(fmul(hp, T8), rd0);
    // suffix le64(n) at stream offset o + n = 16 (beta + 1024) + sigma: n 2^(8 sigma) split at 2^128
    F26 suffix;
    {
        const uint32_t wi = G.sigma >> 2, bs = 8u * (G.sigma & 3u);
        const uint64_t v = (uint64_t)kWprN << bs;
        uint32_t w[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            if (i == wi) {
                w[i] = (uint32_t)v;
                w[i + 1] = (uint32_t)(v >> 32);
            }
        }
        suffix = fmul_add(words_to_f26(w[0], w[1], w[2], w[3], 0u), rd0, fmul(F26{w[4], 0u, 0u, 0u, 0u}, rdel));
    }
    const F26 ctot = carry1(f26_add(f26_add(f26_add(pads, bias), f26_add(seed, prefix)), suffix));
    store_f26(st + kWCtot, ctot);
    __syncthreads();
    wpr_flush_half(p, rec0, 0u, stage, lane);
}

// ---------------------------------------------------------------------------
// The record kernel.
// ---------------------------------------------------------------------------
// Four LDS-DMA loads (global_load_lds_dwordx4, 1 KiB each) of one 4 KiB chunk:
// instruction k writes LDS bytes [l0 + 1024 k, +1024) from each lane's
// g0 + 1024 k.  hipcc does not count these loads: the kernel waits for them
// with its own s_waitcnt vmcnt.
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
        : "v"(g0), "v"(g1), "v"(g2), "v"(g3), "s"(l0), "s"(uniform(l0 + 1024u)), "s"(uniform(l0 + 2048u)), "s"(uniform(l0 + 3072u))
        : "memory");
}

// X = sum_m Y_m 2^(64 m) < 2^242 (eight words) -> F26 with limb 4 < 2^27.
__device__ __forceinline__ F26 reduce_words8(const uint32_t w[8]) {
    // y = (X mod 2^130) + 5 (X >> 130) < 2^131, then once more
    uint64_t t = (uint64_t)__builtin_amdgcn_alignbit(w[5], w[4], 2) * 5u + w[0];
    const uint32_t y0 = (uint32_t)t;
    t = (uint64_t)__builtin_amdgcn_alignbit(w[6], w[5], 2) * 5u + w[1] + (t >> 32);
    const uint32_t y1 = (uint32_t)t;
    t = (uint64_t)__builtin_amdgcn_alignbit(w[7], w[6], 2) * 5u + w[2] + (t >> 32);
    const uint32_t y2 = (uint32_t)t;
    t = (uint64_t)(w[7] >> 2) * 5u + w[3] + (t >> 32);
    const uint32_t y3 = (uint32_t)t;
    t = (uint64_t)(w[4] & 3u) + (t >> 32);                     // y = y0..y3 + t 2^128
    const uint64_t u = (uint64_t)(uint32_t)(t >> 2) * 5u + y0;  // (y mod 2^130) + 5 (y >> 130)
    uint32_t c;
    const uint32_t z1 = addc(y1, (uint32_t)(u >> 32), 0u, &c);
    const uint32_t z2 = addc(y2, 0u, c, &c);
    const uint32_t z3 = addc(y3, 0u, c, &c);
    const uint32_t z4 = ((uint32_t)t & 3u) + c;  // <= 4
    F26 f = words_to_f26((uint32_t)u, z1, z2, z3, 0u);
    f.v4 += z4 << 24;
    return f;
}

// Phase timing (experiment builds only, -DSG_WPR_PROFILE=1; the output is
// unchanged): each wave accumulates s_memtime deltas per phase in SGPRs and
// writes them once at its end; tools/wpr_phase.py reads them back through
// sg_wpr_profile_read.
#ifndef SG_WPR_PROFILE
#define SG_WPR_PROFILE 0
#endif
constexpr uint32_t kProfPhases = 10, kProfWaves = 4096;
#if SG_WPR_PROFILE
__device__ unsigned long long g_wpr_prof[kProfWaves][kProfPhases];
#define SG_TICK(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define SG_ACC(k, a, b) prof[k] += (b) - (a)
#else
#define SG_TICK(v)
#define SG_ACC(k, a, b)
#endif

// The double-round body (experiment builds may pick another barrier spacing
// from tools/chacha_grp.inc; every form computes the same rounds)
#ifndef SG_WPR_DR_ASM
#define SG_WPR_DR_ASM SG_CHACHA_DR_NB1_BAR1
#endif

// A zero vector materialised where it is used (a hoisted constant would hold
// four VGPRs across the whole record loop).
__device__ __forceinline__ u32x4 zero4() {
    u32x4 z;
    asm volatile("v_mov_b32 %0, 0\nv_mov_b32 %1, 0\nv_mov_b32 %2, 0\nv_mov_b32 %3, 0"
                 : "=v"(z[0]), "=v"(z[1]), "=v"(z[2]), "=v"(z[3]));
    return z;
}

// Scalar loads of wave-uniform inputs (key table, key index, sequence numbers,
// explicit nonces, the received tag): the constant address space makes hipcc
// emit s_load (counted on lgkmcnt), so no compiler-counted vector load ever
// waits behind the kernel's own LDS-DMA queue.
typedef const __attribute__((address_space(4))) uint32_t* cu32p;
__device__ __forceinline__ uint32_t cload(const void* base, uint64_t word) {
    return ((cu32p)(uintptr_t)base)[word];
}

// One 16-byte LDS-DMA per lane: LDS [l0 + 16 lane, +16) <- g (lanes with exec set).
// The same with a wave-uniform base address in SGPRs and the lane's 32-bit
// offset in a VGPR (global_load_lds_dwordx4 saddr form): one VGPR per lane for
// every DMA of the kernel instead of a 64-bit address per instruction.
__device__ __forceinline__ void dma_sv(uint32_t l0, const void* sbase, uint32_t voff) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(l0)
                 : "memory");
}

__device__ __forceinline__ void dma_one(uint32_t l0, const void* g) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(l0)
                 : "memory");
}

template <bool OPEN, bool TLS>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void sg_wpr_kernel(const KParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    uint8_t* buf = lds + wave * kWprWaveLds;
    uint8_t* lines = buf + kWprLinesOff;  // also the landing area of the record's keying table
    const uint32_t lds_wave = uniform((uint32_t)(uintptr_t)buf);
    const uint32_t lds_lines = uniform(lds_wave + kWprLinesOff);
    const uint32_t hh = lane >> 5, q = lane & 31u;
    const uint32_t adlen = TLS ? 13u : p.ad_len;
    const uint32_t sigma = (adlen + 8u) & 15u;
    // T fragment byte a' comes from the V window for a' < 16 - sigma, else from P
    const uint32_t nv = 16u - sigma;
    const u32x4 vmask = {~bytes_from(0u, nv), ~bytes_from(1u, nv), ~bytes_from(2u, nv), ~bytes_from(3u, nv)};
    // LDS swizzle: 16-byte unit 4 t + c of a chunk lives at 4 t + (c ^ ((t >> 2) & 3))
    const uint32_t wunit = (lane & ~3u) | ((lane ^ (lane >> 4)) & 3u);  // unit of global position 64 k + lane
    const uint32_t xq = (lane >> 2) & 3u;
    // the lane's MAC window base (line 5 (1 - hh), dword of byte 47 - q) and shift
    const uint8_t* mac_base = lines + 240u * (1u - hh) + 4u * ((47u - q) >> 2);
    const uint32_t mac_shift = (47u - q) & 3u;
    const uint32_t ngroups = (p.count + kWprWaves - 1u) / kWprWaves;

    // Chunk c of a record is fetched by LDS-DMA into buffer c & 1, one chunk
    // ahead: lane l of DMA instruction k lands at LDS unit 64 k + l and reads
    // global unit 64 k + wunit(l), so LDS unit phi(g) holds global unit g
    // (phi = wunit within each 64-unit piece, an involution).  The record's
    // keying table (640 B) is fetched into the line area the same way.  The
    // only vector-memory operations of the kernel are these DMAs and the
    // output stores, so the waits below count exactly.
    auto dma_chunk_of = [&](uint32_t rec, uint32_t c) {
        dma_chunk(lds_wave + kWprChunk * (c & 1u), p.in + p.in_stride * rec + kWprChunk * c + 16u * wunit);
    };
    auto dma_table_of = [&](uint32_t rec) {  // into the line area
        if (lane < kWprRecWords / 4u) dma_one(lds_lines, p.ws + (uint64_t)rec * kWprRecWords + 4u * lane);
    };
    // Record groups are handed out dynamically: the first one is the
    // workgroup's index, every later one comes from a device counter (zeroed by
    // the keying kernel), fetched by wave 0 at the start of the previous group
    // and passed to the other waves through LDS.  The two workgroups sharing a
    // CU do not progress at the same rate (a static g += gridDim.x split left
    // the fastest waves idle for the last 40 % of the launch).
    uint32_t* const ctr = p.ws + (uint64_t)p.count * kWprRecWords;
    uint32_t* const gslot = reinterpret_cast<uint32_t*>(lds + kWprLinesOff + kWprLines * kWprLineBytes + 32u);
    uint32_t g = blockIdx.x;
    if (g < ngroups && g * kWprWaves + wave < p.count) {
        dma_chunk_of(g * kWprWaves + wave, 0u);
        dma_table_of(g * kWprWaves + wave);
    }
    bool first = true;
    // the previous chunk's output waits in its LDS buffer and leaves during
    // the next chunk's first double rounds (pend: it belongs to an active record)
    bool pend = false;
    uint8_t* pend_dst = p.out;

#if SG_WPR_PROFILE
    uint64_t prof[kProfPhases] = {};
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    uint64_t t_prev = t_start;
#endif
    while (g < ngroups) {
        SG_TICK(t_rs);
        SG_ACC(7, t_prev, t_rs);  // epilogue + loop overhead of the previous record
#if SG_WPR_PROFILE
        prof[6] += 1;  // records (groups) this wave ran
#endif
        const uint32_t rec = g * kWprWaves + wave;
        const bool active = rec < p.count;  // an inactive wave still runs every round and barrier
        const uint32_t recl = rec < p.count ? rec : p.count - 1u;
        uint32_t gn = ngroups, nrec = 0u;  // the next group: known from iteration 3 on
        bool next = false;
        uint8_t* out = p.out + p.out_stride * recl;
        // key, nonce (chacha20.rs:25-51; TLS: be64(seq), tls.rs:103), received tag
        uint32_t kw[8];
        {
            const uint32_t ki = p.key_index ? cload(p.key_index, recl) : 0u;
#pragma unroll
            for (uint32_t i = 0; i < 8u; ++i) kw[i] = cload(p.keys, 8ull * ki + i);
        }
        uint32_t n14, n15;
        if constexpr (TLS) {
            uint64_t seq = p.seq0 + recl;
            if (p.seq) seq = (uint64_t)cload(p.seq, 2ull * recl) | ((uint64_t)cload(p.seq, 2ull * recl + 1u) << 32);
            n14 = bswap32((uint32_t)(seq >> 32));
            n15 = bswap32((uint32_t)seq);
        } else {
            n14 = cload(p.nonces, 2ull * recl);
            n15 = cload(p.nonces, 2ull * recl + 1u);
        }
        // The column quarter rounds 1-3 of the first double round see no block
        // counter (word 13 is 0, chacha20.rs:114-121): the same for every lane
        // and chunk of the record, so they run once per record on the SALU.
        uint32_t u[16] = {kSigma0, kSigma1, kSigma2, kSigma3, kw[0], kw[1], kw[2], kw[3],
                          kw[4],   kw[5],   kw[6],   kw[7],   0u,    0u,    n14,   n15};
        SG_QR(u[1], u[5], u[9], u[13]) SG_QR(u[2], u[6], u[10], u[14]) SG_QR(u[3], u[7], u[11], u[15])
        // and the steps of the double round whose operands are all uniform
        // (tools/gen_chacha_grp.py, SG_CHACHA_DR1S_*; tests/test_chacha_asm_model.py)
        const uint32_t S0 = u[0] + u[4], T1 = u[1] + u[6], T2 = u[2] + u[7];
        const uint32_t T13 = rotl32(u[13] ^ T2, 16);
        uint32_t rx[4] = {0u, 0u, 0u, 0u};
        if constexpr (OPEN) {  // the received tag (chacha20_poly1305.rs:72-73)
            const uint8_t* tg = p.in + p.in_stride * recl + kWprN;
            rx[0] = cload(tg, 0); rx[1] = cload(tg, 1); rx[2] = cload(tg, 2); rx[3] = cload(tg, 3);
        }

        // ---- the keying table has landed (it was followed only by the previous
        // record's tag / status store; the chunk-0 DMA is older)
        if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        first = false;
        wave_lds_sync();
        uint32_t fetched = 0u;
        if (wave == 0u && lane == 0u)
            fetched = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        SG_TICK(t_tw);
        SG_ACC(0, t_rs, t_tw);  // wait for the keying table
        const uint32_t* tab = reinterpret_cast<const uint32_t*>(lines);
        // row weight W = 2^(32 hh) r^(4 (31 - q)) = hi[hh][a] lo[b], 31 - q = 8 a + b
        const uint32_t e = 31u - q;
        const F26 W = fmul(load_f26(tab + kWHi + 20u * hh + 5u * (e >> 3)), load_f26(tab + kWLo + 5u * (e & 7u)));
        const F26 ctot = {uniform(tab[kWCtot + 0]), uniform(tab[kWCtot + 1]), uniform(tab[kWCtot + 2]),
                          uniform(tab[kWCtot + 3]), uniform(tab[kWCtot + 4])};
        const uint32_t sk[4] = {uniform(tab[kWS + 0]), uniform(tab[kWS + 1]), uniform(tab[kWS + 2]),
                                uniform(tab[kWS + 3])};
        // ---- T digit lines: line l = 5 k + u holds r^(128 k + 1 + delta + u) as
        // 17 signed base-256 digits, digit i at byte 47 - sigma - i, zeros elsewhere
        F26 lv = f26_zero();
        if (lane < kWprLines) {
            const uint32_t k = lane / 5u, u = lane - 5u * k;
            lv = fmul(load_f26(tab + kWRd + 5u * u), load_f26(tab + kWTk + 5u * k));
        }
        wave_lds_sync();  // every table read is done before the lines overwrite it
        if (lane < kWprLines) {
            const F26 v = canonical(lv);
            uint32_t c;  // digits = the bytes of v + 0x80..80, each ^ 0x80
            uint32_t d[5];
            d[0] = addc(v.v0 | (v.v1 << 26), 0x80808080u, 0u, &c) ^ 0x80808080u;
            d[1] = addc((v.v1 >> 6) | (v.v2 << 20), 0x80808080u, c, &c) ^ 0x80808080u;
            d[2] = addc((v.v2 >> 12) | (v.v3 << 14), 0x80808080u, c, &c) ^ 0x80808080u;
            d[3] = addc((v.v3 >> 18) | (v.v4 << 8), 0x80808080u, c, &c) ^ 0x80808080u;
            d[4] = ((v.v4 >> 24) + 0x80u + c) ^ 0x80u;
            uint8_t* ln = lines + kWprLineBytes * lane;
            const u32x4 z = zero4();
            st16(ln, z);
            st16(ln + 16, z);
            st16(ln + 32, z);
#pragma unroll
            for (uint32_t i = 0; i < 17u; ++i) ln[47u - sigma - i] = (uint8_t)(d[i >> 2] >> (8u * (i & 3u)));
        } else if (lane == kWprLines) {
            st16(lines + kWprLines * kWprLineBytes, zero4());
        }
        wave_lds_sync();
        SG_TICK(t_pl);
        SG_ACC(1, t_tw, t_pl);  // W and the digit lines

        i32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 1 << 24;

        // MAC step (jj, i): T fragment = the V window of line iv = 5 k + 4 - i for
        // bytes a' < 16 - sigma, else the P window of line iv - 1 (k = (1 - hh) +
        // 2 (3 - jj)); B operand = chunk i of the lane's block, byte - 128.
        // The windows start at byte 47 - q of line iv and 31 - q of line iv - 1:
        // both are read as aligned dwords (an unaligned 16-byte LDS read stalls
        // the LDS pipe for the whole CU) and shifted into place with
        // v_alignbyte by the lane's (47 - q) & 3.  TLS (sigma = 5) needs V words
        // 0-2 and P words 2-3 only.
        struct MacRaw {
            uint32_t v[5], p[5];
        };
        auto mac_load = [&](uint32_t jj, uint32_t i, MacRaw& R) {
            const uint8_t* b = mac_base + 480u * (3u - jj) + 48u * (4u - i);
            const uint32_t* vb = reinterpret_cast<const uint32_t*>(b);
            const uint32_t* pb = reinterpret_cast<const uint32_t*>(b - 64);
            if constexpr (TLS) {
#pragma unroll
                for (int t = 0; t < 4; ++t) R.v[t] = vb[t];
#pragma unroll
                for (int t = 2; t < 5; ++t) R.p[t] = pb[t];
            } else {
#pragma unroll
                for (int t = 0; t < 5; ++t) {
                    R.v[t] = vb[t];
                    R.p[t] = pb[t];
                }
            }
        };
        auto mac_frag = [&](const MacRaw& R) -> u32x4 {
            u32x4 f;
            if constexpr (TLS) {  // bytes 0-10 from V, 11-15 from P
                f[0] = __builtin_amdgcn_alignbyte(R.v[1], R.v[0], mac_shift);
                f[1] = __builtin_amdgcn_alignbyte(R.v[2], R.v[1], mac_shift);
                const uint32_t v2 = __builtin_amdgcn_alignbyte(R.v[3], R.v[2], mac_shift);
                const uint32_t p2 = __builtin_amdgcn_alignbyte(R.p[3], R.p[2], mac_shift);
                f[2] = (v2 & 0x00ffffffu) | (p2 & 0xff000000u);
                f[3] = __builtin_amdgcn_alignbyte(R.p[4], R.p[3], mac_shift);
            } else {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t vt = __builtin_amdgcn_alignbyte(R.v[t + 1], R.v[t], mac_shift);
                    const uint32_t pt = __builtin_amdgcn_alignbyte(R.p[t + 1], R.p[t], mac_shift);
                    f[t] = (vt & vmask[t]) | (pt & ~vmask[t]);
                }
            }
            return f;
        };
        auto mac_mfma_f = [&](const u32x4& f, const u32x4& a) {
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, f),
                                                         __builtin_bit_cast(i32x4, a ^ 0x80808080u), acc, 0, 0, 0);
        };
        auto mac_mfma = [&](const MacRaw& R, const u32x4& a) { mac_mfma_f(mac_frag(R), a); };
        // The MAC of iteration j - 1 runs inside iteration j's rounds: its T
        // windows are read one double round ahead of each MFMA and the MFMAs are
        // two double rounds apart, so neither an LDS latency nor the MFMA chain
        // ever stalls a wave at a lock-step barrier (sched_barrier pins the
        // placement).  A holds the previous iteration's ciphertext chunks.  The
        // last iteration reads its own T fragments (F3) during its rounds, so the
        // line area is free for the next record's keying table before this
        // record's last stores are issued.
        u32x4 A[4] = {};
        MacRaw R0 = {}, R1 = {};
        u32x4 F3[4] = {};
#define SG_DR()                                                                                                   \
    asm volatile(SG_WPR_DR_ASM                                                                                    \
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
                   "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]),         \
                   "+v"(x[15]))
#define SG_PIN() __builtin_amdgcn_sched_barrier(0)

#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
            SG_TICK(t_js);
            // chunk j has landed in buffer j & 1 (j >= 1: its DMA was the last
            // memory operation of iteration j - 1; j = 0: waited for with the table)
            if (j > 0u) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (j == 1u && wave == 0u && lane == 0u) *gslot = gridDim.x + fetched;  // the atomic has returned
            wave_lds_sync();
            if (j == 3u) {  // wave 0 published it before the barriers of iterations 1 and 2
                gn = uniform(*gslot);
                nrec = gn * kWprWaves + wave;
                next = gn < ngroups && nrec < p.count;
            }
            SG_TICK(t_jw);
            SG_ACC(2, t_js, t_jw);  // wait for the chunk
            uint8_t* cb = buf + kWprChunk * (j & 1u);
            uint8_t* pb = buf + kWprChunk * ((j + 1u) & 1u);  // the pending output

            // keystream block 64 j + lane + 1 (chacha20_poly1305.rs:52), lock-step rounds
            const uint32_t ctr = 64u * j + lane + 1u;
            uint32_t x[16];
            x[12] = ctr;
            u32x4 D[4];
            SG_PIN();
            // first double round: every word but the counter enters from SGPRs
            asm volatile(SG_CHACHA_DR1S_COL : "=v"(x[0]), "=v"(x[4]), "=v"(x[8]), "+v"(x[12])
                         : "s"(S0), "s"(kw[0]), "s"(kw[4]));
            asm volatile(SG_CHACHA_DR1S_DIAG
                         : "+v"(x[0]), "+v"(x[4]), "+v"(x[8]), "+v"(x[12]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]),
                           "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[13]),
                           "=v"(x[14]), "=v"(x[15])
                         : "s"(u[5]), "s"(u[15]), "s"(T1), "s"(u[3]), "s"(u[14]), "s"(u[10]), "s"(u[11]), "s"(T13),
                           "s"(u[9]), "s"(u[6]), "s"(u[7]), "s"(T2));
            SG_PIN();
            // The previous chunk's output leaves lane-contiguously one 1 KiB piece
            // per double round (read from LDS one gap ahead of its store), and
            // piece k of the next chunk's DMA follows the store of output piece k
            // (the same LDS range): the stores and DMAs of the 16 waves of a CU
            // spread over five gaps instead of queueing behind each other.
            auto out_piece = [&](uint32_t k) { return ld16(pb + 1024u * k + 16u * wunit); };
            auto store_piece = [&](uint32_t k, const u32x4& v) { st16(pend_dst + 1024u * k + 16u * lane, v); };
            auto dma_piece = [&](uint32_t k) {
                if (j < 3u) {
                    if (active)
                        dma_sv(uniform(lds_wave + kWprChunk * ((j + 1u) & 1u) + 1024u * k),
                               p.in + p.in_stride * rec + kWprChunk * (j + 1u) + 1024u * k, 16u * wunit);
                } else if (next) {
                    dma_sv(uniform(lds_wave + 1024u * k), p.in + p.in_stride * nrec + 1024u * k, 16u * wunit);
                }
            };
            u32x4 oa = {}, ob = {};
            if (j > 0u) mac_load(j - 1u, 0u, R0);
            if (pend) oa = out_piece(0u);
            SG_PIN();
            SG_DR();
            SG_PIN();
            if (j > 0u) {
                mac_mfma(R0, A[0]);
                mac_load(j - 1u, 1u, R1);
            }
            if (pend) {
                store_piece(0u, oa);
                ob = out_piece(1u);
            }
            SG_PIN();
            SG_DR();
            SG_PIN();
            if (j > 0u) {
                mac_mfma(R1, A[1]);
                mac_load(j - 1u, 2u, R0);
            }
            if (pend) {
                store_piece(1u, ob);
                oa = out_piece(2u);
            }
            dma_piece(0u);
            SG_PIN();
            SG_DR();
            SG_PIN();
            if (j > 0u) {
                mac_mfma(R0, A[2]);
                mac_load(j - 1u, 3u, R1);
            }
            if (pend) {
                store_piece(2u, oa);
                ob = out_piece(3u);
            }
            dma_piece(1u);
            SG_PIN();
            SG_DR();
            SG_PIN();
            if (j > 0u) mac_mfma(R1, A[3]);
            if (pend) store_piece(3u, ob);
            dma_piece(2u);
            SG_PIN();
            SG_DR();
            SG_PIN();
            dma_piece(3u);
            if (j == 3u) {
                mac_load(3u, 0u, R0);
                mac_load(3u, 1u, R1);
            }
            SG_PIN();
            SG_DR();
            SG_PIN();
            if (j == 3u) {
                F3[0] = mac_frag(R0);
                F3[1] = mac_frag(R1);
                mac_load(3u, 2u, R0);
                mac_load(3u, 3u, R1);
            }
            SG_PIN();
            SG_DR();
            SG_PIN();
            if (j == 3u) {
                F3[2] = mac_frag(R0);
                F3[3] = mac_frag(R1);
            }
            SG_PIN();
            SG_DR();
            SG_PIN();
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) D[i] = ld16(cb + 16u * (4u * lane + (i ^ xq)));
            SG_PIN();
            SG_DR();
            SG_PIN();
            SG_TICK(t_jr);
            SG_ACC(3, t_jw, t_jr);  // rounds (+ MAC of the previous chunk)
            if (j == 3u && next) {  // the line area is read out: the next record's table lands there
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                dma_table_of(nrec);
            }
            // feed-forward (chacha20.rs:104-106) and XOR (chacha20.rs:143-153)
            u32x4 O[4];
            O[0] = D[0] ^ u32x4{x[0] + kSigma0, x[1] + kSigma1, x[2] + kSigma2, x[3] + kSigma3};
            O[1] = D[1] ^ u32x4{x[4] + kw[0], x[5] + kw[1], x[6] + kw[2], x[7] + kw[3]};
            O[2] = D[2] ^ u32x4{x[8] + kw[4], x[9] + kw[5], x[10] + kw[6], x[11] + kw[7]};
            O[3] = D[3] ^ u32x4{x[12] + ctr, x[13], x[14] + n14, x[15] + n15};
            // the MAC reads the ciphertext: received (open) or just produced (seal)
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) A[i] = OPEN ? D[i] : O[i];
            if (j == 3u) {
                SG_PIN();
#pragma unroll
                for (uint32_t i = 0; i < 4u; ++i) mac_mfma_f(F3[i], A[i]);
                SG_PIN();
            }

            // the output waits in the same slice; it leaves during the next
            // chunk's first double rounds
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) st16(cb + 16u * (4u * lane + (i ^ xq)), O[i]);
            pend = active;
            pend_dst = out + kWprChunk * j;
            SG_TICK(t_je);
            SG_ACC(4, t_jr, t_je);  // feed-forward, XOR, staging, stores
#if SG_WPR_PROFILE
            t_prev = t_je;
#endif
        }
#undef SG_DR
#undef SG_PIN

        // ---- assemble X = sum_r D[c_r][q] 2^(8 c_r - 32 hh), c_r = (r & 3) + 8 (r >> 2) + 4 hh
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
        {  // sum the 64 lane terms into lane 63: row_shr 1, 2, 4, 8, row_bcast:15, carry, row_bcast:31
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
        }
        auto lane63 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); };
        const F26 fs = {lane63(f.v0) + ctot.v0, lane63(f.v1) + ctot.v1, lane63(f.v2) + ctot.v2,
                        lane63(f.v3) + ctot.v3, lane63(f.v4) + ctot.v4};
        uint32_t tw[4];
        tag_words(fs, sk, tw);
        if (active && lane == 0u) {
            if constexpr (!OPEN) {
                st16(out + kWprN, u32x4{tw[0], tw[1], tw[2], tw[3]});  // ct || tag (chacha20_poly1305.rs:55)
            } else {
                // constant-time compare: diff |= a ^ b over all 16 bytes (chacha20_poly1305.rs:84-87)
                const uint32_t diff = (rx[0] ^ tw[0]) | (rx[1] ^ tw[1]) | (rx[2] ^ tw[2]) | (rx[3] ^ tw[3]);
                p.status[rec] = diff != 0u ? 1u : 0u;
            }
        }
        g = gn;
    }
    if (pend) {  // the last record's last chunk
        wave_lds_sync();
        const uint8_t* pb = buf + kWprChunk;
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) st16(pend_dst + 1024u * k + 16u * lane, ld16(pb + 1024u * k + 16u * wunit));
    }
#if SG_WPR_PROFILE
    SG_TICK(t_end);
    SG_ACC(7, t_prev, t_end);
    prof[5] = t_end - t_start;  // the wave's whole life
    prof[8] = __builtin_amdgcn_s_memrealtime() - rt_start;  // the same in 100 MHz ticks
    prof[9] = rt_start;
    const uint32_t wid = blockIdx.x * kWprWaves + wave;
    if (lane == 0u && wid < kProfWaves) {
#pragma unroll
        for (uint32_t k = 0; k < kProfPhases; ++k) g_wpr_prof[wid][k] = prof[k];
    }
#endif
}

int g_cus[64];  // CUs per device ordinal (0: not read yet)

}  // namespace

#if SG_WPR_PROFILE
}  // namespace sg
extern "C" int sg_wpr_profile_read(unsigned long long* host, size_t n) {
    const size_t bytes = sizeof(sg::g_wpr_prof);
    if (n * sizeof(unsigned long long) < bytes) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(sg::g_wpr_prof), bytes) != hipSuccess) return -2;
    static unsigned long long zero[sg::kProfWaves][sg::kProfPhases];
    if (hipMemcpyToSymbol(HIP_SYMBOL(sg::g_wpr_prof), zero, bytes) != hipSuccess) return -3;
    return (int)(bytes / sizeof(unsigned long long));
}
namespace sg {
#endif

hipError_t launch_wpr(const KParams& p, bool open, hipStream_t s, hipEvent_t ev_keyed, hipEvent_t ev_start) {
    const uint32_t kgrid = (p.count + kWprKeyThreads - 1u) / kWprKeyThreads;
    if (open)
        hipLaunchKernelGGL((sg_wpr_keying_kernel<true>), dim3(kgrid), dim3(kWprKeyThreads), 0, s, p);
    else
        hipLaunchKernelGGL((sg_wpr_keying_kernel<false>), dim3(kgrid), dim3(kWprKeyThreads), 0, s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ev_keyed && (e = hipEventRecord(ev_keyed, s)) != hipSuccess) return e;
    if (ev_start && (e = hipEventRecord(ev_start, s)) != hipSuccess) return e;
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    int cus = dev >= 0 && dev < 64 ? __atomic_load_n(&g_cus[dev], __ATOMIC_RELAXED) : 0;
    if (cus <= 0) {
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        if (dev >= 0 && dev < 64) __atomic_store_n(&g_cus[dev], cus, __ATOMIC_RELAXED);
    }
    const uint32_t ngroups = (p.count + kWprWaves - 1u) / kWprWaves;
    uint32_t grid = 2u * (uint32_t)cus;  // two workgroups (16 waves) per CU
    if (grid > ngroups) grid = ngroups;
    const size_t lds = kWprWaves * kWprWaveLds;
#define SG_WPR_LAUNCH(O, T) hipLaunchKernelGGL((sg_wpr_kernel<O, T>), dim3(grid), dim3(512), lds, s, p)
    if (open) {
        if (p.tls) SG_WPR_LAUNCH(true, true); else SG_WPR_LAUNCH(true, false);
    } else {
        if (p.tls) SG_WPR_LAUNCH(false, true); else SG_WPR_LAUNCH(false, false);
    }
#undef SG_WPR_LAUNCH
    return hipGetLastError();
}

#ifndef SG_WPR_DEFAULT
#define SG_WPR_DEFAULT 1
#endif
static int g_wpr = -1;  // -1: not read from the environment yet
bool wpr_enabled() {
    if (__atomic_load_n(&g_wpr, __ATOMIC_ACQUIRE) < 0) {
        const char* e = getenv("SG_LOCKSTEP");
        int expect = -1;
        __atomic_compare_exchange_n(&g_wpr, &expect, e ? (e[0] == '1' ? 1 : 0) : (SG_WPR_DEFAULT ? 1 : 0), false,
                                    __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
    }
    return __atomic_load_n(&g_wpr, __ATOMIC_ACQUIRE) == 1;
}
int set_wpr(int enable) {
    const int prev = wpr_enabled() ? 1 : 0;
    if (enable >= 0) __atomic_store_n(&g_wpr, enable ? 1 : 0, __ATOMIC_RELEASE);
    return prev;
}

const char* wpr_kernel_config() {
    return "sg_wpr_kernel v14: full 16 KiB records, one wave per record (8 per 512-thread workgroup, persistent "
           "2 per CU, record groups handed out by a device counter), 4 KiB chunks LDS-DMA prefetched lane-contiguously into an XOR-swizzled LDS slice, output "
           "read out during the next chunk's first double rounds, lock-step grouped ChaCha20 rounds (s_barrier per "
           "rotate group; the first double round takes its uniform words from SGPRs, the counter-free steps once "
           "per record on the SALU), Poly1305 as 16 "
           "v_mfma_i32_32x32x32_i8 per record fed from the ciphertext registers one chunk behind (Toeplitz digit "
           "lines of r^(128k+d) in LDS, read as aligned dwords + v_alignbyte), exact per-lane assembly, "
           "W = r^(4(31-q)) scaling, DPP sum; keying pre-pass with the constant term";
}

}  // namespace sg
