// sg_device.h -- device-side building blocks shared by the gfx950 kernels
// (sg_kernels.hip: size-class kernels, keying, bucketing; sg_wpr.hip: the
// wave-per-record kernel for full 16 KiB records).  Not part of the public ABI.
//
//   ChaCha20 block function        klutzy/suruga src/crypto/chacha20.rs:25-135
//   Poly1305 field arithmetic      src/crypto/poly1305.rs:25-192 (exact mod 2^130-5)
//   tag = (h mod 2^128) + s        poly1305.rs:230-312
//   TLS nonce / additional data    src/tls.rs:103-112, 250-265
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sg_internal.h"

namespace sg {
namespace dev {

constexpr uint32_t M26 = (1u << 26) - 1;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
    return __builtin_addc(a, b, cin, cout);  // v_add_co / v_addc_co chain
}

// 16-byte accesses: aligned (global / LDS) and unaligned (LDS: one ds_read_b128)
__device__ __forceinline__ u32x4 ld16(const void* p) {
    return *reinterpret_cast<const u32x4*>(__builtin_assume_aligned(p, 16));
}
__device__ __forceinline__ void st16(void* p, u32x4 v) {
    *reinterpret_cast<u32x4*>(__builtin_assume_aligned(p, 16)) = v;
}
// Record bytes are read once and written once: the wave-per-record kernel
// moves them with the non-temporal policy (SG_STREAM_NT, default on): its
// LDS-DMA loads carry `nt` (SG_DMA_POL) and its lane-contiguous stores are
// nontemporal.  Same-box A/B on C1 (round 3): +1.5-1.7 % (seal 7.52 -> 7.42 ms,
// open 7.57 -> 7.44 ms).  The kernels whose lanes each move a 64-byte block
// (packed, size classes) keep the default policy (nt measured -1.3 % on C2).
#ifndef SG_STREAM_NT
#define SG_STREAM_NT 1
#endif
#if SG_STREAM_NT
#define SG_DMA_POL " nt"
#else
#define SG_DMA_POL ""
#endif
__device__ __forceinline__ u32x4 gld16(const void* p) {
    const u32x4* q = reinterpret_cast<const u32x4*>(__builtin_assume_aligned(p, 16));
    if constexpr (SG_STREAM_NT) return __builtin_nontemporal_load(q);
    return *q;
}
__device__ __forceinline__ void gst16(void* p, u32x4 v) {
    u32x4* q = reinterpret_cast<u32x4*>(__builtin_assume_aligned(p, 16));
    if constexpr (SG_STREAM_NT) {
        __builtin_nontemporal_store(v, q);
    } else {
        *q = v;
    }
}

typedef u32x4 u32x4_u __attribute__((aligned(1)));
__device__ __forceinline__ u32x4 ldu16(const void* p) { return *reinterpret_cast<const u32x4_u*>(p); }

// LDS writes of one lane visible to the other lanes of its wave, and no
// compiler reordering of LDS accesses across this point
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---- ChaCha20 (chacha20.rs) ------------------------------------------------
// quarter round, chacha20.rs:63-81
#define SG_QR(a, b, c, d)                   \
    a += b; d ^= a; d = rotl32(d, 16);      \
    c += d; b ^= c; b = rotl32(b, 12);      \
    a += b; d ^= a; d = rotl32(d, 8);       \
    c += d; b ^= c; b = rotl32(b, 7);

// Wave-uniform variants for the scalar unit.  The SALU has no rotate and no
// byte swap: the opaque asm keeps the shift-or from being matched to
// v_alignbit / v_perm (which would move the whole uniform chain to the VALU).
__device__ __forceinline__ uint32_t srotl32(uint32_t x, int n) {
    uint32_t hi = x << n, lo = x >> (32 - n);
    asm volatile("" : "+s"(hi));
    return hi | lo;
}
__device__ __forceinline__ uint32_t sbswap32(uint32_t x) {
    uint32_t a = x << 24, b = (x << 8) & 0x00ff0000u;
    asm volatile("" : "+s"(a), "+s"(b));
    return a | b | ((x >> 8) & 0x0000ff00u) | (x >> 24);
}
#define SG_QR_S(a, b, c, d)                  \
    a += b; d ^= a; d = srotl32(d, 16);      \
    c += d; b ^= c; b = srotl32(b, 12);      \
    a += b; d ^= a; d = srotl32(d, 8);       \
    c += d; b ^= c; b = srotl32(b, 7);

constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646eu, kSigma2 = 0x79622d32u, kSigma3 = 0x6b206574u;

// One keystream block (chacha20.rs:25-51 state, :53-109 round20).  k[8] key
// words, ctr = state word 12 (word 13 is always 0: chacha20.rs:114-121),
// n14/n15 = nonce words.  ks[i] = round20(state)[i] (little-endian words).
__device__ __forceinline__ void chacha_block(uint32_t ks[16], const uint32_t k[8], uint32_t ctr, uint32_t n14,
                                             uint32_t n15) {
    uint32_t x0 = kSigma0, x1 = kSigma1, x2 = kSigma2, x3 = kSigma3;
    uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3];
    uint32_t x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x12 = ctr, x13 = 0u, x14 = n14, x15 = n15;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        SG_QR(x0, x4, x8, x12) SG_QR(x1, x5, x9, x13) SG_QR(x2, x6, x10, x14) SG_QR(x3, x7, x11, x15)
        SG_QR(x0, x5, x10, x15) SG_QR(x1, x6, x11, x12) SG_QR(x2, x7, x8, x13) SG_QR(x3, x4, x9, x14)
    }
    ks[0] = x0 + kSigma0; ks[1] = x1 + kSigma1; ks[2] = x2 + kSigma2; ks[3] = x3 + kSigma3;
    ks[4] = x4 + k[0]; ks[5] = x5 + k[1]; ks[6] = x6 + k[2]; ks[7] = x7 + k[3];
    ks[8] = x8 + k[4]; ks[9] = x9 + k[5]; ks[10] = x10 + k[6]; ks[11] = x11 + k[7];
    ks[12] = x12 + ctr; ks[13] = x13; ks[14] = x14 + n14; ks[15] = x15 + n15;
}

// ---- Poly1305 field arithmetic, radix 2^26 ---------------------------------
// Invariant of a "reduced" element: limbs 0,2,3,4 < 2^26, limb 1 < 2^26 + 2^8.
struct F26 {
    uint32_t v0, v1, v2, v3, v4;
};

__device__ __forceinline__ F26 f26_zero() { return F26{0u, 0u, 0u, 0u, 0u}; }
__device__ __forceinline__ F26 f26_one() { return F26{1u, 0u, 0u, 0u, 0u}; }
__device__ __forceinline__ F26 f26_add(const F26& a, const F26& b) {
    return F26{a.v0 + b.v0, a.v1 + b.v1, a.v2 + b.v2, a.v3 + b.v3, a.v4 + b.v4};
}
__device__ __forceinline__ void store_f26(uint32_t* p, const F26& x) {
    p[0] = x.v0; p[1] = x.v1; p[2] = x.v2; p[3] = x.v3; p[4] = x.v4;
}
__device__ __forceinline__ F26 load_f26(const uint32_t* p) { return F26{p[0], p[1], p[2], p[3], p[4]}; }

// a * b + c (mod p, reduced) -- the Int1305::mult of poly1305.rs:51-128 in
// one carry pass.  b reduced; a and c limbs < 2^27.
__device__ __forceinline__ F26 mul_add(const F26 a, const uint32_t b0, const uint32_t b1, const uint32_t b2,
                                       const uint32_t b3, const uint32_t b4, const F26 c) {
    const uint32_t s1 = b1 * 5u, s2 = b2 * 5u, s3 = b3 * 5u, s4 = b4 * 5u;
    F26 h;
    uint64_t d = (uint64_t)c.v0 + (uint64_t)a.v0 * b0 + (uint64_t)a.v1 * s4 + (uint64_t)a.v2 * s3 +
                 (uint64_t)a.v3 * s2 + (uint64_t)a.v4 * s1;
    h.v0 = (uint32_t)d & M26;
    uint32_t cy = (uint32_t)(d >> 26);
    d = (uint64_t)(c.v1 + cy) + (uint64_t)a.v0 * b1 + (uint64_t)a.v1 * b0 + (uint64_t)a.v2 * s4 +
        (uint64_t)a.v3 * s3 + (uint64_t)a.v4 * s2;
    h.v1 = (uint32_t)d & M26;
    cy = (uint32_t)(d >> 26);
    d = (uint64_t)(c.v2 + cy) + (uint64_t)a.v0 * b2 + (uint64_t)a.v1 * b1 + (uint64_t)a.v2 * b0 +
        (uint64_t)a.v3 * s4 + (uint64_t)a.v4 * s3;
    h.v2 = (uint32_t)d & M26;
    cy = (uint32_t)(d >> 26);
    d = (uint64_t)(c.v3 + cy) + (uint64_t)a.v0 * b3 + (uint64_t)a.v1 * b2 + (uint64_t)a.v2 * b1 +
        (uint64_t)a.v3 * b0 + (uint64_t)a.v4 * s4;
    h.v3 = (uint32_t)d & M26;
    cy = (uint32_t)(d >> 26);
    d = (uint64_t)(c.v4 + cy) + (uint64_t)a.v0 * b4 + (uint64_t)a.v1 * b3 + (uint64_t)a.v2 * b2 +
        (uint64_t)a.v3 * b1 + (uint64_t)a.v4 * b0;
    h.v4 = (uint32_t)d & M26;
    cy = (uint32_t)(d >> 26);
    const uint64_t e = (uint64_t)h.v0 + (uint64_t)cy * 5u;  // 2^130 == 5 (mod p)
    h.v0 = (uint32_t)e & M26;
    h.v1 += (uint32_t)(e >> 26);
    return h;
}
__device__ __forceinline__ F26 fmul(const F26 a, const F26 b) { return mul_add(a, b.v0, b.v1, b.v2, b.v3, b.v4, f26_zero()); }
__device__ __forceinline__ F26 fmul_add(const F26 a, const F26 b, const F26 c) {
    return mul_add(a, b.v0, b.v1, b.v2, b.v3, b.v4, c);
}

// One carry pass over limbs < 2^32 (value unchanged mod p): limbs < 2^26 + 2^8.
__device__ __forceinline__ F26 carry1(F26 f) {
    uint32_t c;
    c = f.v0 >> 26; f.v0 &= M26; f.v1 += c;
    c = f.v1 >> 26; f.v1 &= M26; f.v2 += c;
    c = f.v2 >> 26; f.v2 &= M26; f.v3 += c;
    c = f.v3 >> 26; f.v3 &= M26; f.v4 += c;
    c = f.v4 >> 26; f.v4 &= M26; f.v0 += c * 5u;
    c = f.v0 >> 26; f.v0 &= M26; f.v1 += c;
    return f;
}

// Strict normal form: every limb < 2^26 (value < 2^130), for limbs < 2^32.
__device__ __forceinline__ F26 ripple_full(F26 h) {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        uint32_t c;
        c = h.v0 >> 26; h.v0 &= M26; h.v1 += c;
        c = h.v1 >> 26; h.v1 &= M26; h.v2 += c;
        c = h.v2 >> 26; h.v2 &= M26; h.v3 += c;
        c = h.v3 >> 26; h.v3 &= M26; h.v4 += c;
        c = h.v4 >> 26; h.v4 &= M26; h.v0 += c * 5u;
    }
    // a second-pass fold implies v1..v4 wrapped to 0, so this cannot overflow v1
    const uint32_t c = h.v0 >> 26;
    h.v0 &= M26;
    h.v1 += c;
    return h;
}

// Canonical representative in [0, p): subtract p when h >= p, branch-free
// (the role of Int1305::normalize, poly1305.rs:165-192).
__device__ __forceinline__ F26 canonical(F26 h) {
    h = ripple_full(h);
    uint32_t g0 = h.v0 + 5u, c = g0 >> 26; g0 &= M26;
    uint32_t g1 = h.v1 + c; c = g1 >> 26; g1 &= M26;
    uint32_t g2 = h.v2 + c; c = g2 >> 26; g2 &= M26;
    uint32_t g3 = h.v3 + c; c = g3 >> 26; g3 &= M26;
    uint32_t g4 = h.v4 + c;
    const uint32_t ge = 0u - (g4 >> 26);  // all ones when h + 5 >= 2^130, i.e. h >= p
    g4 &= M26;
    h.v0 = (g0 & ge) | (h.v0 & ~ge);
    h.v1 = (g1 & ge) | (h.v1 & ~ge);
    h.v2 = (g2 & ge) | (h.v2 & ~ge);
    h.v3 = (g3 & ge) | (h.v3 & ~ge);
    h.v4 = (g4 & ge) | (h.v4 & ~ge);
    return h;
}

// tag = (h mod 2^128) + s mod 2^128, little-endian words (poly1305.rs:231-312)
__device__ __forceinline__ void tag_words(F26 h, const uint32_t s[4], uint32_t t[4]) {
    h = canonical(h);
    const uint32_t w0 = h.v0 | (h.v1 << 26);
    const uint32_t w1 = (h.v1 >> 6) | (h.v2 << 20);
    const uint32_t w2 = (h.v2 >> 12) | (h.v3 << 14);
    const uint32_t w3 = (h.v3 >> 18) | (h.v4 << 8);
    uint64_t acc = (uint64_t)w0 + s[0];
    t[0] = (uint32_t)acc;
    acc = (acc >> 32) + w1 + s[1];
    t[1] = (uint32_t)acc;
    acc = (acc >> 32) + w2 + s[2];
    t[2] = (uint32_t)acc;
    acc = (acc >> 32) + w3 + s[3];
    t[3] = (uint32_t)acc;
}

// 128-bit little-endian value (4 words) + extra high bits -> radix 2^26
__device__ __forceinline__ F26 words_to_f26(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t hi) {
    F26 c;
    c.v0 = w0 & M26;
    c.v1 = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
    c.v2 = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    c.v3 = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
    c.v4 = (w3 >> 8) | (hi << 24);
    return c;
}

// sum_{e=1..m} x^e by binary doubling (G(2a) = G(a) + x^a G(a), G(a+1) = G(a) + x^(a+1))
__device__ __forceinline__ F26 geo_sum(const F26 x, const uint32_t m) {
    F26 g = f26_zero(), pw = f26_one();
    if (m == 0u) return g;
    for (int bit = 31 - __builtin_clz(m); bit >= 0; --bit) {
        g = mul_add(g, pw.v0, pw.v1, pw.v2, pw.v3, pw.v4, g);
        pw = fmul(pw, pw);
        if ((m >> bit) & 1u) {
            pw = fmul(pw, x);
            g = f26_add(g, pw);
        }
    }
    return g;
}

// ---- Poly1305 Horner step with the clamped r, radix 2^32 ------------------
// h = h0 + h1 2^32 + h2 2^64 + h3 2^96 + h4 2^128 (h4 small).  r0..r3 are the
// clamped key words: r0 < 2^28, r1..r3 < 2^28 and divisible by 4, so
// r_j 2^128 == (r_j / 4) * 5 (mod p) and s_j = r_j + (r_j >> 2) stays exact.
struct H32 {
    uint32_t h0, h1, h2, h3, h4;
};

// h = (h + m + pad * 2^128) * r  (partially reduced: h4 <= 4)
__device__ __forceinline__ void horner_step(H32& h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                            uint32_t pad, uint32_t r0, uint32_t r1, uint32_t r2,
                                            uint32_t r3, uint32_t s1, uint32_t s2, uint32_t s3) {
    // h += m (poly1305.rs:227 c.add(&h))
    uint32_t c;
    const uint32_t a0 = addc(h.h0, m0, 0u, &c);
    const uint32_t a1 = addc(h.h1, m1, c, &c);
    const uint32_t a2 = addc(h.h2, m2, c, &c);
    const uint32_t a3 = addc(h.h3, m3, c, &c);
    const uint32_t a4 = h.h4 + pad + c;
    // * r (poly1305.rs:227 .mult(&r)): column sums < 2^63, then one carry ripple
    const uint64_t d0 = (uint64_t)a0 * r0 + (uint64_t)a1 * s3 + (uint64_t)a2 * s2 + (uint64_t)a3 * s1;
    const uint64_t d1 = (uint64_t)a0 * r1 + (uint64_t)a1 * r0 + (uint64_t)a2 * s3 + (uint64_t)a3 * s2 +
                        (uint64_t)a4 * s1;
    const uint64_t d2 = (uint64_t)a0 * r2 + (uint64_t)a1 * r1 + (uint64_t)a2 * r0 + (uint64_t)a3 * s3 +
                        (uint64_t)a4 * s2;
    const uint64_t d3 = (uint64_t)a0 * r3 + (uint64_t)a1 * r2 + (uint64_t)a2 * r1 + (uint64_t)a3 * r0 +
                        (uint64_t)a4 * s3;
    const uint32_t e1 = addc((uint32_t)d1, (uint32_t)(d0 >> 32), 0u, &c);
    const uint32_t e2 = addc((uint32_t)d2, (uint32_t)(d1 >> 32), c, &c);
    const uint32_t e3 = addc((uint32_t)d3, (uint32_t)(d2 >> 32), c, &c);
    uint32_t e4 = a4 * r0 + (uint32_t)(d3 >> 32) + c;
    // fold bits >= 2^130: (e4 >> 2) * 2^130 == (e4 >> 2) * 5
    const uint32_t f = (e4 >> 2) * 5u;
    e4 &= 3u;
    h.h0 = addc((uint32_t)d0, f, 0u, &c);
    h.h1 = addc(e1, 0u, c, &c);
    h.h2 = addc(e2, 0u, c, &c);
    h.h3 = addc(e3, 0u, c, &c);
    h.h4 = e4 + c;
}

// ---- per-record parameters ---------------------------------------------------
struct RecKey {
    uint32_t k[8];
    uint32_t n14, n15;
    uint64_t seq;
};

__device__ __forceinline__ RecKey record_key(const KParams& p, uint32_t rec) {
    RecKey rk;
    uint32_t ki = p.key_index ? p.key_index[rec] : 0u;
    ki = ki < p.num_keys ? ki : p.num_keys - 1u;  // out-of-range indices stay inside the key table
    const uint32_t* kw = reinterpret_cast<const uint32_t*>(p.keys + 32u * ki);
#pragma unroll
    for (int i = 0; i < 8; ++i) rk.k[i] = kw[i];  // keys are little-endian words (chacha20.rs:37-39)
    if (p.tls) {
        // nonce = u64_be_array(seq) (tls.rs:103, util.rs:43-45) loaded as two
        // little-endian words (chacha20.rs:45-46)
        rk.seq = p.seq ? p.seq[rec] : p.seq0 + rec;
        rk.n14 = bswap32((uint32_t)(rk.seq >> 32));
        rk.n15 = bswap32((uint32_t)rk.seq);
    } else {
        const uint8_t* nb = p.nonces + 8ull * rec;
        rk.seq = 0;
        rk.n14 = (uint32_t)nb[0] | ((uint32_t)nb[1] << 8) | ((uint32_t)nb[2] << 16) | ((uint32_t)nb[3] << 24);
        rk.n15 = (uint32_t)nb[4] | ((uint32_t)nb[5] << 8) | ((uint32_t)nb[6] << 16) | ((uint32_t)nb[7] << 24);
    }
    return rk;
}

__device__ __forceinline__ uint32_t record_len(const KParams& p, uint32_t rec) {
    return p.len ? p.len[rec] : p.uniform_len;
}

// AD byte i of the TLS record-layer additional data (tls.rs:103-112, 250-265):
// be64(seq) || type || major || minor || be16(n)
__device__ __forceinline__ uint8_t tls_ad_byte(uint64_t seq, uint32_t hdr, uint32_t n, uint32_t i) {
    if (i < 8) return (uint8_t)(seq >> (56 - 8 * i));
    if (i < 11) return (uint8_t)(hdr >> (8 * (i - 8)));
    if (i == 11) return (uint8_t)(n >> 8);
    return (uint8_t)n;
}

// Byte i (< adlen + 8) of the MAC stream prefix ad || le64(|ad|)
// (chacha20_poly1305.rs:24-26).
__device__ __forceinline__ uint8_t prefix_byte(const KParams& p, uint32_t rec, uint64_t seq, uint32_t n, uint32_t adlen,
                                               uint32_t i) {
    if (i < adlen) return p.tls ? tls_ad_byte(seq, p.tls_hdr, n, i) : p.ads[(uint64_t)p.ad_stride * rec + i];
    return (uint8_t)((uint64_t)adlen >> (8u * (i - adlen)));
}

}  // namespace dev
}  // namespace sg
