// sg_kernels.hip -- gfx950 (CDNA4) kernels for suruga's ChaCha20-Poly1305
// record AEAD (draft-agl-tls-chacha20poly1305-04 as in klutzy/suruga).
//
// Work decomposition (one TLS record per 256-thread workgroup):
//
//   sg_keying_kernel   one lane per record: ChaCha20 block 0 -> Poly1305 key
//                      (r clamped, s; chacha20_poly1305.rs:50,75,32-39,
//                      poly1305.rs:197-203) and the 16 powers of r^k
//                      that combine the MAC lanes.
//   sg_aead_kernel<OPEN>
//     phase 1, all 4 waves: lane t owns 64-byte data blocks t, t+256, ...;
//       computes keystream block b+1 in registers (chacha20.rs:53-135),
//       XORs the record bytes (chacha20.rs:143-153), writes the result to HBM
//       and the ciphertext into LDS.
//     phase 2, wave 0: Poly1305 over ad || le64(|ad|) || ct || le64(|ct|)
//       (chacha20_poly1305.rs:19-42), read from LDS.  The B MAC blocks are
//       preceded by z zero "virtual" blocks (leading zeros do not change a
//       Horner polynomial) so that B + z = 64k; lane t runs the reference's
//       Horner step h = (h + c) * r (poly1305.rs:213-228) over its k
//       contiguous blocks in radix 2^32 with the clamped r; each lane then
//       scales its sum by r^(k*(63-t)) (radix 2^26, powers from the keying
//       record) and a shuffle reduction adds the 64 terms.  Lane 0 reduces mod 2^130-5, adds s
//       (poly1305.rs:230-312) and seals (chacha20_poly1305.rs:55) or
//       compares in constant time (:84-93) after decrypting
//       unconditionally (:80-82).
//
// All Poly1305 arithmetic is exact mod p = 2^130 - 5, so the tag equals the
// reference's sequential Horner result bit for bit.
#include "sg_internal.h"
#include "sg_chacha_grp.inc"  // grouped ChaCha20 double round (tools/gen_chacha_grp.py --product)

#include <stdint.h>
#include <stdlib.h>

#ifndef SG_SALU_PRE
#define SG_SALU_PRE 1  // hoist the counter-free part of ChaCha round 1 to the SALU
#endif
#ifndef SG_LS_NOMAC
#define SG_LS_NOMAC 0  // timing experiments only: the lock-step kernel skips the MAC (tags are wrong)
#endif
#ifndef SG_LS_NOROUNDS
#define SG_LS_NOROUNDS 0
#endif
#ifndef SG_LS_COMPILED
#define SG_LS_COMPILED 0  // experiments: the lock-step kernel with compiled (unsynchronised) rounds
#endif

namespace sg {
namespace {

constexpr uint32_t M26 = (1u << 26) - 1;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ u32x4 ld16(const void* p) {
    return *reinterpret_cast<const u32x4*>(__builtin_assume_aligned(p, 16));
}
__device__ __forceinline__ void st16(void* p, u32x4 v) {
    *reinterpret_cast<u32x4*>(__builtin_assume_aligned(p, 16)) = v;
}
// streamed record bytes: read once, written once.  SG_NT sets non-temporal
// hints (1 loads, 2 stores); measured on C1 they cost 5-9 % (loads),
// 7-12 % (stores) and 40 % (both), so the product leaves them off.
#ifndef SG_NT
#define SG_NT 0
#endif
__device__ __forceinline__ u32x4 ldg16(const void* p) {
    const u32x4* q = reinterpret_cast<const u32x4*>(__builtin_assume_aligned(p, 16));
    if constexpr (SG_NT & 1) return __builtin_nontemporal_load(q);
    else return *q;
}
__device__ __forceinline__ void stg16(void* p, u32x4 v) {
    u32x4* q = reinterpret_cast<u32x4*>(__builtin_assume_aligned(p, 16));
    if constexpr (SG_NT & 2) __builtin_nontemporal_store(v, q);
    else *q = v;
}
// 16 bytes at any byte address (LDS: one ds_read_b128 on gfx950)
typedef u32x4 u32x4_u __attribute__((aligned(1)));
__device__ __forceinline__ u32x4 ldu16(const void* p) { return *reinterpret_cast<const u32x4_u*>(p); }

// chacha20.rs:63-81
#define SG_QR(a, b, c, d)                   \
    a += b; d ^= a; d = rotl32(d, 16);      \
    c += d; b ^= c; b = rotl32(b, 12);      \
    a += b; d ^= a; d = rotl32(d, 8);       \
    c += d; b ^= c; b = rotl32(b, 7);

// One ChaCha20 keystream block (chacha20.rs:25-51 state, :53-109 round20).
// k[8] key words, ctr = state word 12 (word 13 is always 0: chacha20.rs:114-121),
// n14/n15 = nonce words.  ks[i] = round20(state)[i] (little-endian words).
__device__ __forceinline__ void chacha_block(uint32_t ks[16], const uint32_t k[8], uint32_t ctr,
                                             uint32_t n14, uint32_t n15) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3];
    uint32_t x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x12 = ctr, x13 = 0u, x14 = n14, x15 = n15;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        SG_QR(x0, x4, x8, x12) SG_QR(x1, x5, x9, x13) SG_QR(x2, x6, x10, x14) SG_QR(x3, x7, x11, x15)
        SG_QR(x0, x5, x10, x15) SG_QR(x1, x6, x11, x12) SG_QR(x2, x7, x8, x13) SG_QR(x3, x4, x9, x14)
    }
    ks[0] = x0 + 0x61707865u; ks[1] = x1 + 0x3320646eu; ks[2] = x2 + 0x79622d32u; ks[3] = x3 + 0x6b206574u;
    ks[4] = x4 + k[0]; ks[5] = x5 + k[1]; ks[6] = x6 + k[2]; ks[7] = x7 + k[3];
    ks[8] = x8 + k[4]; ks[9] = x9 + k[5]; ks[10] = x10 + k[6]; ks[11] = x11 + k[7];
    ks[12] = x12 + ctr; ks[13] = x13; ks[14] = x14 + n14; ks[15] = x15 + n15;
}

// ---- uniform-record variant: the counter-free part of round 1 on the SALU ----
// Within one record only state word 12 (the block counter) differs between
// blocks.  The column quarter-rounds on words (1,5,9,13), (2,6,10,14),
// (3,7,11,15) and the first add of (0,4,8,12) are therefore the same for
// every block; when the record is wave-uniform (key and nonce in SGPRs) they
// are computed once on the scalar unit, which otherwise idles, instead of
// costing ~37 VALU per block.  The SALU has no rotate: the opaque asm keeps the
// shift-or from being matched to v_alignbit.
__device__ __forceinline__ uint32_t srotl32(uint32_t x, int n) {
    uint32_t hi = x << n, lo = x >> (32 - n);
    asm volatile("" : "+s"(hi));
    return hi | lo;
}
#define SG_QR_S(a, b, c, d)                  \
    a += b; d ^= a; d = srotl32(d, 16);      \
    c += d; b ^= c; b = srotl32(b, 12);      \
    a += b; d ^= a; d = srotl32(d, 8);       \
    c += d; b ^= c; b = srotl32(b, 7);

struct ChaChaPre {
    uint32_t x[16];  // state after the counter-free part of round 1 (x12 unused)
};

// k, n14, n15 must be wave-uniform.
__device__ __forceinline__ ChaChaPre chacha_pre(const uint32_t k[8], uint32_t n14, uint32_t n15) {
    uint32_t x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x5 = k[1], x6 = k[2], x7 = k[3], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x13 = 0u, x14 = n14, x15 = n15;
    SG_QR_S(x1, x5, x9, x13) SG_QR_S(x2, x6, x10, x14) SG_QR_S(x3, x7, x11, x15)
    return ChaChaPre{{0x61707865u + k[0], x1, x2, x3, k[0], x5, x6, x7, k[4], x9, x10, x11, 0u, x13, x14, x15}};
}

// Same result as chacha_block(ks, k, ctr, n14, n15), starting from chacha_pre.
__device__ __forceinline__ void chacha_block_pre(uint32_t ks[16], const ChaChaPre& P, const uint32_t k[8],
                                                 uint32_t ctr, uint32_t n14, uint32_t n15) {
    uint32_t x0 = P.x[0], x1 = P.x[1], x2 = P.x[2], x3 = P.x[3];
    uint32_t x4 = P.x[4], x5 = P.x[5], x6 = P.x[6], x7 = P.x[7];
    uint32_t x8 = P.x[8], x9 = P.x[9], x10 = P.x[10], x11 = P.x[11];
    uint32_t x12 = ctr, x13 = P.x[13], x14 = P.x[14], x15 = P.x[15];
    // rest of round 1, column (0,4,8,12): its first add is in x0 already
    x12 ^= x0; x12 = rotl32(x12, 16);
    x8 += x12; x4 ^= x8; x4 = rotl32(x4, 12);
    x0 += x4; x12 ^= x0; x12 = rotl32(x12, 8);
    x8 += x12; x4 ^= x8; x4 = rotl32(x4, 7);
    SG_QR(x0, x5, x10, x15) SG_QR(x1, x6, x11, x12) SG_QR(x2, x7, x8, x13) SG_QR(x3, x4, x9, x14)
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        SG_QR(x0, x4, x8, x12) SG_QR(x1, x5, x9, x13) SG_QR(x2, x6, x10, x14) SG_QR(x3, x7, x11, x15)
        SG_QR(x0, x5, x10, x15) SG_QR(x1, x6, x11, x12) SG_QR(x2, x7, x8, x13) SG_QR(x3, x4, x9, x14)
    }
    ks[0] = x0 + 0x61707865u; ks[1] = x1 + 0x3320646eu; ks[2] = x2 + 0x79622d32u; ks[3] = x3 + 0x6b206574u;
    ks[4] = x4 + k[0]; ks[5] = x5 + k[1]; ks[6] = x6 + k[2]; ks[7] = x7 + k[3];
    ks[8] = x8 + k[4]; ks[9] = x9 + k[5]; ks[10] = x10 + k[6]; ks[11] = x11 + k[7];
    ks[12] = x12 + ctr; ks[13] = x13; ks[14] = x14 + n14; ks[15] = x15 + n15;
}

// ---- Poly1305 field arithmetic, radix 2^26 (general multiplier) ----------
// Invariant of a "reduced" element: limbs 0,2,3,4 < 2^26, limb 1 < 2^26 + 2^8.
struct F26 {
    uint32_t v0, v1, v2, v3, v4;
};

// returns a * b + c (mod p, reduced); b fully reduced (< 2^26 per limb),
// a limbs < 2^27, c limbs < 2^27.
__device__ __forceinline__ F26 mul_add(const F26 a, const uint32_t b0, const uint32_t b1,
                                       const uint32_t b2, const uint32_t b3, const uint32_t b4,
                                       const F26 c) {
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

__device__ __forceinline__ F26 f26_zero() { return F26{0u, 0u, 0u, 0u, 0u}; }

__device__ __forceinline__ void store_f26(uint32_t* p, const F26& x) {
    p[0] = x.v0; p[1] = x.v1; p[2] = x.v2; p[3] = x.v3; p[4] = x.v4;
}
__device__ __forceinline__ F26 load_f26(const uint32_t* p) { return F26{p[0], p[1], p[2], p[3], p[4]}; }

// Full carry: every limb < 2^26 (value < 2^130, not yet < p).
__device__ __forceinline__ F26 carry_full(F26 h) {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        uint32_t c;
        c = h.v1 >> 26; h.v1 &= M26; h.v2 += c;
        c = h.v2 >> 26; h.v2 &= M26; h.v3 += c;
        c = h.v3 >> 26; h.v3 &= M26; h.v4 += c;
        c = h.v4 >> 26; h.v4 &= M26; h.v0 += c * 5u;
        c = h.v0 >> 26; h.v0 &= M26; h.v1 += c;
    }
    return h;
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
__device__ __forceinline__ F26 words_to_f26(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                            uint32_t hi) {
    F26 c;
    c.v0 = w0 & M26;
    c.v1 = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
    c.v2 = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    c.v3 = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
    c.v4 = (w3 >> 8) | (hi << 24);
    return c;
}

// ---- Poly1305 Horner step with the clamped r, radix 2^32 ------------------
// h = h0 + h1 2^32 + h2 2^64 + h3 2^96 + h4 2^128 (h4 small).  r0..r3 are the
// clamped key words: r0 < 2^28, r1..r3 < 2^28 and divisible by 4, so
// r_j 2^128 == (r_j / 4) * 5 (mod p) and s_j = r_j + (r_j >> 2) stays exact.
struct H32 {
    uint32_t h0, h1, h2, h3, h4;
};

__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
    return __builtin_addc(a, b, cin, cout);  // v_add_co / v_addc_co chain
}

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

// MAC geometry: stream length L, blocks B, lane chunk k (odd: spreads the
// lanes' LDS reads over banks), leading virtual zero blocks z = PL*k - B, for
// PL MAC lanes per record.
struct MacGeom {
    uint32_t L, B, k, z;
};
__device__ __forceinline__ MacGeom mac_geom(uint32_t adlen, uint32_t n, uint32_t PL) {
    MacGeom g;
    g.L = adlen + 16u + n;
    g.B = (g.L + 15u) >> 4;
    g.k = (g.B + PL - 1u) / PL;
    g.k |= 1u;
    g.z = PL * g.k - g.B;
    return g;
}

// MAC lanes per record, a function of the payload length only so that the
// keying kernel and every AEAD size class agree on k (see size_class).
__device__ __forceinline__ uint32_t mac_lanes(uint32_t n) { return class_mac_lanes(size_class(n)); }

// Per-record parameters shared by the keying and AEAD kernels.
struct RecKey {
    uint32_t k[8];
    uint32_t n14, n15;
    uint64_t seq;
};

__device__ __forceinline__ RecKey record_key(const KParams& p, uint32_t rec) {
    RecKey rk;
    const uint32_t ki = p.key_index ? p.key_index[rec] : 0u;
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

// ---------------------------------------------------------------------------
// Keying pre-pass: one lane per record.
// ---------------------------------------------------------------------------
// The 64 records of a wave are staged in LDS (row stride 97 words: no bank
// conflicts) and leave as one contiguous 24 KiB run of 16-byte stores; one
// lane writing its own 384-byte record would touch 64 cache lines per store.
constexpr uint32_t kKeyingThreads = 64;

// sum_{e=1..m} x^e by binary doubling (G(2a) = G(a) + x^a G(a), G(a+1) = G(a) + x^(a+1))
__device__ __forceinline__ F26 geo_sum(const F26 x, const uint32_t m) {
    F26 g = f26_zero(), pw = F26{1u, 0u, 0u, 0u, 0u};
    if (m == 0u) return g;
    for (int bit = 31 - __builtin_clz(m); bit >= 0; --bit) {
        g = mul_add(g, pw.v0, pw.v1, pw.v2, pw.v3, pw.v4, g);
        pw = mul_add(pw, pw.v0, pw.v1, pw.v2, pw.v3, pw.v4, f26_zero());
        if ((m >> bit) & 1u) {
            pw = mul_add(pw, x.v0, x.v1, x.v2, x.v3, x.v4, f26_zero());
            g = F26{g.v0 + pw.v0, g.v1 + pw.v1, g.v2 + pw.v2, g.v3 + pw.v3, g.v4 + pw.v4};
        }
    }
    return g;
}

template <bool OPEN, bool LS>
__global__ __launch_bounds__(64) void sg_keying_kernel(const KParams p) {
    // words [0, kRSmallOff) go through LDS; the lock-step extras (LS) are
    // written straight from the lane, so the stage stays small (occupancy)
    constexpr uint32_t RW = LS ? kKeyRecWordsLs : kKeyRecWords;
    constexpr uint32_t SW = LS ? kRSmallOff : kKeyRecWords;  // staged words per record
    constexpr uint32_t kKeyLdsStride = SW + 1;
    __shared__ uint32_t stage[kKeyingThreads * kKeyLdsStride];
    const uint32_t lane = threadIdx.x;
    const uint32_t rec0 = blockIdx.x * kKeyingThreads;
    const uint32_t rec = rec0 + lane;
    uint32_t* out = stage + lane * kKeyLdsStride;
    uint32_t* gout = p.ws + (uint64_t)rec * RW;
    if (rec < p.count) {
        const uint32_t len = record_len(p, rec);
        const uint32_t n = OPEN ? (len >= 16u ? len - 16u : 0u) : len;
        const RecKey rk = record_key(p, rec);
        uint32_t ks[16];
        chacha_block(ks, rk.k, 0u, rk.n14, rk.n15);  // block 0 -> poly key (chacha20_poly1305.rs:50)
        // r = clamp(pk[0..16]) (poly1305.rs:197-203), s = pk[16..32]
        const uint32_t r0 = ks[0] & 0x0fffffffu, r1 = ks[1] & 0x0ffffffcu;
        const uint32_t r2 = ks[2] & 0x0ffffffcu, r3 = ks[3] & 0x0ffffffcu;
        out[kR32Off + 0] = r0;
        out[kR32Off + 1] = r1;
        out[kR32Off + 2] = r2;
        out[kR32Off + 3] = r3;
        out[kSOff + 0] = ks[4];
        out[kSOff + 1] = ks[5];
        out[kSOff + 2] = ks[6];
        out[kSOff + 3] = ks[7];
        const uint32_t adlen = p.tls ? 13u : p.ad_len;
        const MacGeom g = mac_geom(adlen, n, LS ? 64u : mac_lanes(n));
        const F26 r = words_to_f26(r0, r1, r2, r3, 0u);
        if constexpr (!LS) {
            // R = r^k by square-and-multiply; then R^0..R^7 and R^0, R^8, .., R^56.
            // mul_add outputs are valid multipliers as they stand (limb 1 may exceed
            // 2^26 by < 2^8), so no extra carry passes are needed here.
            F26 R = r;
            for (int bit = 30 - __builtin_clz(g.k); bit >= 0; --bit) {
                R = mul_add(R, R.v0, R.v1, R.v2, R.v3, R.v4, f26_zero());
                if ((g.k >> bit) & 1u) R = mul_add(R, r.v0, r.v1, r.v2, r.v3, r.v4, f26_zero());
            }
            F26 x = F26{1u, 0u, 0u, 0u, 0u};
            for (int j = 0; j < 8; ++j) {  // lo[j] = R^j
                store_f26(out + kPowLoOff + 5 * j, x);
                x = mul_add(x, R.v0, R.v1, R.v2, R.v3, R.v4, f26_zero());
            }
            const F26 R8 = x;
            x = F26{1u, 0u, 0u, 0u, 0u};
            for (int i = 0; i < 8; ++i) {  // hi[i] = R^(8 i)
                store_f26(out + kPowHiOff + 5 * i, x);
                if (i < 7) x = mul_add(x, R8.v0, R8.v1, R8.v2, R8.v3, R8.v4, f26_zero());
            }
        } else {
            // power tables of the MFMA evaluation (mfma_mac)
            F26 x = F26{1u, 0u, 0u, 0u, 0u};
            for (int j = 0; j < 8; ++j) {  // rs[j] = r^j
                store_f26(gout + kRSmallOff + 5 * j, x);
                x = mul_add(x, r.v0, r.v1, r.v2, r.v3, r.v4, f26_zero());
            }
            const F26 r8 = x;
            x = F26{1u, 0u, 0u, 0u, 0u};
            for (int i = 0; i < 4; ++i) {  // rm[i] = r^(8 i); x ends at r^32
                store_f26(gout + kRMidOff + 5 * i, x);
                x = mul_add(x, r8.v0, r8.v1, r8.v2, r8.v3, r8.v4, f26_zero());
            }
            const F26 r32 = x;
            x = r;
            for (int j = 0; j < 8; ++j) {  // pl[j] = r^(32 j + 1)
                store_f26(out + kPowLoOff + 5 * j, x);
                x = mul_add(x, r32.v0, r32.v1, r32.v2, r32.v3, r32.v4, f26_zero());
            }
            F26 r256 = mul_add(r32, r32.v0, r32.v1, r32.v2, r32.v3, r32.v4, f26_zero());
            r256 = mul_add(r256, r256.v0, r256.v1, r256.v2, r256.v3, r256.v4, f26_zero());
            r256 = mul_add(r256, r256.v0, r256.v1, r256.v2, r256.v3, r256.v4, f26_zero());
            x = F26{1u, 0u, 0u, 0u, 0u};
            for (int i = 0; i < 6; ++i) {  // ph[i] = r^(256 i)
                store_f26(out + kPowHiOff + 5 * i, x);
                if (i < 5) x = mul_add(x, r256.v0, r256.v1, r256.v2, r256.v3, r256.v4, f26_zero());
            }
            // Constant term (mfma_mac): with N = 64 k slots, K = 0x80 x 16 bytes
            // (the i8 bias of the block bytes), J = sum_c 2^(24 + 8 c) (the seed of
            // the 32 product columns), G(m) = sum_{e=1..m} r^e and the row weights
            // W_q = r^(31 - q), sum_q W_q = 1 + G(31):
            //   ctot = K G(N) + 2^128 G(B) + [rem < 16] (2^(8 rem) - 2^128) r - J (1 + G(31))
            // with G(N) = G(32) sum_{t < 2k} r^(32 t).
            const uint32_t rem = g.L - 16u * (g.B - 1u);
            const F26 G31 = geo_sum(r, 31u);
            const F26 G32 = F26{G31.v0 + r32.v0, G31.v1 + r32.v1, G31.v2 + r32.v2, G31.v3 + r32.v3, G31.v4 + r32.v4};
            const F26 T = geo_sum(r32, 2u * g.k - 1u);
            const F26 GN = mul_add(G32, T.v0 + 1u, T.v1, T.v2, T.v3, T.v4, f26_zero());
            const F26 GB = geo_sum(r, g.B);
            F26 c = mul_add(GN, 0x808080u, 0x202020u, 0x80808u, 0x2020202u, 0x808080u, f26_zero());  // K G(N)
            c = mul_add(GB, 0u, 0u, 0u, 0u, 0x1000000u, c);                                      // 2^128 G(B)
            c = mul_add(F26{G31.v0 + 1u, G31.v1, G31.v2, G31.v3, G31.v4}, 0x1bd2d2bu, 0x36f6f6fu, 0x3dbdbdbu,
                        0x2f6f6f6u, 0x1bdbdbdu, c);                                                // (p - J)(1 + G(31))
            if (rem < 16u) {  // (2^(8 rem) + p - 2^128) r
                F26 cf = F26{0x3fffffbu, 0x3ffffffu, 0x3ffffffu, 0x3ffffffu, 0x2ffffffu};
                const uint32_t bit = 8u * rem, li = bit / 26u, v = 1u << (bit - 26u * li);
                cf.v0 += li == 0u ? v : 0u;
                cf.v1 += li == 1u ? v : 0u;
                cf.v2 += li == 2u ? v : 0u;
                cf.v3 += li == 3u ? v : 0u;
                cf.v4 += li == 4u ? v : 0u;
                c = mul_add(cf, r.v0, r.v1, r.v2, r.v3, r.v4, c);
            }
            store_f26(gout + kCtotOff, c);
        }
    }
    __syncthreads();
    // coalesced flush: the wave's records are contiguous in the workspace
    const uint32_t nrec = p.count - rec0 < kKeyingThreads ? p.count - rec0 : kKeyingThreads;
    u32x4* dst = reinterpret_cast<u32x4*>(p.ws + (uint64_t)rec0 * RW);
    const uint32_t nvec = nrec * (SW / 4u);
    for (uint32_t v = lane; v < nvec; v += kKeyingThreads) {
        const uint32_t w = 4u * v;
        const uint32_t rr = w / SW, c = w - rr * SW;
        const uint32_t* src = stage + rr * kKeyLdsStride + c;
        dst[(rr * RW + c) / 4u] = u32x4{src[0], src[1], src[2], src[3]};
    }
}

// AD byte i of the TLS record-layer additional data (tls.rs:103-112, 250-265):
// be64(seq) || type || major || minor || be16(n)
__device__ __forceinline__ uint8_t tls_ad_byte(uint64_t seq, uint32_t hdr, uint32_t n, uint32_t i) {
    if (i < 8) return (uint8_t)(seq >> (56 - 8 * i));
    if (i < 11) return (uint8_t)(hdr >> (8 * (i - 8)));
    if (i == 11) return (uint8_t)(n >> 8);
    return (uint8_t)n;
}

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// ---------------------------------------------------------------------------
// Fused seal / open.  A 256-thread workgroup serves RPW = 256 / L records with
// L lanes each (size classes: L = 16 for n <= 1 KiB, 64 for n <= 4 KiB, 256
// otherwise); PL = min(L, 64) of them run the MAC.  Per record, in LDS:
//   [0, S) virtual-block space | S: ad | le64(adlen) | A: ct (n) | le64(n) | zeros
// ---------------------------------------------------------------------------
template <bool OPEN, uint32_t L>
__device__ __forceinline__ void aead_record(const KParams& p, const uint32_t rec, const bool active,
                                            uint8_t* lds, const uint32_t t) {
    constexpr uint32_t PL = L < 64u ? L : 64u;
    constexpr uint32_t Z = 32u * PL;  // space for the virtual blocks in front: 16 * max z
    uint32_t n = 0;
    bool work = active;
    const uint32_t len = active ? record_len(p, rec) : 0u;
    if (active) {
        n = len;
        if constexpr (OPEN) {
            if (len < 16u) {  // chacha20_poly1305.rs:68-70 "message too short"
                if (t == 0) p.status[rec] = 2u;
                work = false;
            }
            n = len - 16u;
        }
    }
    const uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    RecKey rk = {};
    const uint32_t adlen = p.tls ? 13u : p.ad_len;
    const uint32_t A = Z + ((adlen + 8u + 15u) & ~15u);
    const uint32_t S = A - adlen - 8u;  // stream start, >= Z
    uint8_t* ct_lds = lds + A;
    if (work) {
        in = p.in + (p.in_off ? p.in_off[rec] : p.in_stride * rec);
        out = p.out + (p.out_off ? p.out_off[rec] : p.out_stride * rec);
        rk = record_key(p, rec);

        // ---- phase 1: keystream XOR, 64 bytes per lane-block ----------------
        const bool vec_ok = (((uintptr_t)in | (uintptr_t)out) & 15u) == 0u;
        const uint32_t nblocks = (n + 63u) >> 6;
        ChaChaPre pre;
        if constexpr (SG_SALU_PRE && L >= 64u) pre = chacha_pre(rk.k, rk.n14, rk.n15);
        for (uint32_t b = t; b < nblocks; b += L) {
            const uint32_t off = b << 6;
            if (vec_ok && off + 64u <= n) {
                const u32x4 d0 = ldg16(in + off), d1 = ldg16(in + off + 16);
                const u32x4 d2 = ldg16(in + off + 32), d3 = ldg16(in + off + 48);
                uint32_t ks[16];
                // data uses blocks 1.. (chacha20_poly1305.rs:52)
                if constexpr (SG_SALU_PRE && L >= 64u) chacha_block_pre(ks, pre, rk.k, b + 1u, rk.n14, rk.n15);
                else chacha_block(ks, rk.k, b + 1u, rk.n14, rk.n15);
                const u32x4 r0 = d0 ^ u32x4{ks[0], ks[1], ks[2], ks[3]};
                const u32x4 r1 = d1 ^ u32x4{ks[4], ks[5], ks[6], ks[7]};
                const u32x4 r2 = d2 ^ u32x4{ks[8], ks[9], ks[10], ks[11]};
                const u32x4 r3 = d3 ^ u32x4{ks[12], ks[13], ks[14], ks[15]};
                stg16(out + off, r0);
                stg16(out + off + 16, r1);
                stg16(out + off + 32, r2);
                stg16(out + off + 48, r3);
                if constexpr (OPEN) {
                    st16(ct_lds + off, d0);
                    st16(ct_lds + off + 16, d1);
                    st16(ct_lds + off + 32, d2);
                    st16(ct_lds + off + 48, d3);
                } else {
                    st16(ct_lds + off, r0);
                    st16(ct_lds + off + 16, r1);
                    st16(ct_lds + off + 32, r2);
                    st16(ct_lds + off + 48, r3);
                }
            } else {
                // partial last block or misaligned record: byte granular
                uint32_t ks[16];
                if constexpr (SG_SALU_PRE && L >= 64u) chacha_block_pre(ks, pre, rk.k, b + 1u, rk.n14, rk.n15);
                else chacha_block(ks, rk.k, b + 1u, rk.n14, rk.n15);
#pragma unroll
                for (uint32_t w = 0; w < 16; ++w) {
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) {
                        const uint32_t idx = off + 4u * w + k;
                        if (idx < n) {
                            const uint8_t x = in[idx];
                            const uint8_t y = x ^ (uint8_t)(ks[w] >> (8u * k));
                            out[idx] = y;
                            ct_lds[idx] = OPEN ? x : y;
                        }
                    }
                }
            }
        }

        // ---- MAC stream framing: ad || le64(|ad|) || ct || le64(|ct|) --------
        if (t < PL) {
            for (uint32_t i = t; i < adlen + 8u; i += PL) {
                uint8_t v;
                if (i < adlen)
                    v = p.tls ? tls_ad_byte(rk.seq, p.tls_hdr, n, i) : p.ads[(uint64_t)p.ad_stride * rec + i];
                else
                    v = (uint8_t)((uint64_t)adlen >> (8u * (i - adlen)));
                lds[S + i] = v;
            }
            // suffix le64(n), then zeros to the end of the last block
            for (uint32_t i = t; i < 28u; i += PL) ct_lds[n + i] = i < 8u ? (uint8_t)((uint64_t)n >> (8u * i)) : 0;
        }
    }
    __syncthreads();
#ifdef SG_EXP_NOMAC  // timing experiments only: skip the MAC (tags are wrong)
    return;
#endif
    if (!work || t >= PL) return;

    // ---- phase 2: Poly1305 on PL lanes -----------------------------------------
    // open: the finishing lane fetches the received tag now so that its memory latency
    // hides behind the Horner loop instead of stalling the final compare
    uint32_t rx[4] = {0u, 0u, 0u, 0u};
    if constexpr (OPEN) {
        if (t == PL - 1u) {  // the lane that finishes the tag
            const uint8_t* ep = in + n;
            if ((((uintptr_t)ep) & 3u) == 0u) {
                const uint32_t* e32 = reinterpret_cast<const uint32_t*>(ep);
                rx[0] = e32[0]; rx[1] = e32[1]; rx[2] = e32[2]; rx[3] = e32[3];
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) rx[i >> 2] |= (uint32_t)ep[i] << (8 * (i & 3));
            }
        }
    }
    const MacGeom g = mac_geom(adlen, n, PL);
    const uint32_t* kr = p.ws + (uint64_t)rec * kKeyRecWords;
    uint32_t r0 = kr[kR32Off + 0], r1 = kr[kR32Off + 1], r2 = kr[kR32Off + 2], r3 = kr[kR32Off + 3];
    if constexpr (PL == 64u) {  // one record per wave: keep the key in SGPRs
        r0 = uniform(r0); r1 = uniform(r1); r2 = uniform(r2); r3 = uniform(r3);
    }
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);

    // lane t: virtual blocks [t*k, t*k + k); virtual block v is real iff v >= z
    const uint32_t v0 = t * g.k;
    const uint32_t rem = g.L - 16u * (g.B - 1u);  // bytes in the final block, 1..16
    H32 h = {0u, 0u, 0u, 0u, 0u};
    // Every block is stepped with the 2^128 pad bit; the virtual blocks (the
    // first z of the record, all in lanes t <= tp = z / k) are then discarded
    // instead of being masked block by block: lanes t < tp hold only virtual
    // blocks and drop their sum at the end, lane tp restarts from h = 0 after
    // its first nv = z mod k blocks.  Dropping a prefix of a Horner chain is
    // exact (h = 0 is the state after leading zero blocks), so the tag is the
    // reference's (poly1305.rs:213-228).  Blocks are read as one unaligned
    // 16-byte LDS load each, one block ahead of the multiply.
    {
        const uint8_t* blk = lds + (S - 16u * g.z + 16u * v0);
        const uint32_t tp = g.z / g.k, nv = g.z - tp * g.k;
        // m holds block j; run(e) steps blocks j .. e-1 (e <= k - 1), each
        // load issued one block ahead; unrolled by two so that the
        // prefetched block needs no register copy
        u32x4 m = ldu16(blk);
        uint32_t j = 0;
        auto run = [&](const uint32_t e) {
            for (; j + 2u <= e; j += 2u) {
                const u32x4 ma = ldu16(blk + 16u * (j + 1u));
                __builtin_amdgcn_sched_barrier(0);
                horner_step(h, m.x, m.y, m.z, m.w, 1u, r0, r1, r2, r3, s1, s2, s3);
                m = ldu16(blk + 16u * (j + 2u));
                __builtin_amdgcn_sched_barrier(0);
                horner_step(h, ma.x, ma.y, ma.z, ma.w, 1u, r0, r1, r2, r3, s1, s2, s3);
            }
            if (j < e) {
                const u32x4 mn = ldu16(blk + 16u * (j + 1u));
                __builtin_amdgcn_sched_barrier(0);
                horner_step(h, m.x, m.y, m.z, m.w, 1u, r0, r1, r2, r3, s1, s2, s3);
                m = mn;
                ++j;
            }
        };
        run(nv);
        if (t == tp) h = H32{0u, 0u, 0u, 0u, 0u};
        run(g.k - 1u);
        // final block: a partial one carries its pad bit at 8 * rem
        // (poly1305.rs:216-225; the bytes after the stream are zero)
        uint32_t pad = 1u;
        if (rem < 16u && t == PL - 1u) {
            const uint32_t fb = 1u << (8u * (rem & 3u));
            const uint32_t fw = rem >> 2;
            m.x |= fw == 0u ? fb : 0u;
            m.y |= fw == 1u ? fb : 0u;
            m.z |= fw == 2u ? fb : 0u;
            m.w |= fw == 3u ? fb : 0u;
            pad = 0u;
        }
        horner_step(h, m.x, m.y, m.z, m.w, pad, r0, r1, r2, r3, s1, s2, s3);
        if (t < tp) h = H32{0u, 0u, 0u, 0u, 0u};
    }
    // radix 2^32 -> 2^26 (h < 2^131)
    F26 f = words_to_f26(h.h0, h.h1, h.h2, h.h3, 0u);
    f.v4 += h.h4 << 24;
    {
        const uint32_t c = f.v4 >> 26;
        f.v4 &= M26;
        f.v0 += c * 5u;
    }
    // combine lanes: total = sum_t h_t R^(PL-1-t), R = r^k; R^e = hi[e >> 3] * lo[e & 7]
    {
        const uint32_t e = PL - 1u - t;
        const F26 plo = load_f26(kr + kPowLoOff + 5u * (e & 7u));
        const F26 phi = load_f26(kr + kPowHiOff + 5u * (e >> 3));
        const F26 P = mul_add(phi, plo.v0, plo.v1, plo.v2, plo.v3, plo.v4, f26_zero());
        f = mul_add(f, P.v0, P.v1, P.v2, P.v3, P.v4, f26_zero());
    }
    // Sum the PL lane terms into the group's last lane with DPP row shifts
    // (groups of PL <= 16 lanes lie inside one 16-lane row) and the row
    // broadcasts for 32 and 64.  mul_add leaves limbs < 2^27, so 32 terms sum
    // below 2^32; one carry pass precedes the last doubling.
    {
        auto level = [&](auto dpp) {
            f.v0 += dpp(f.v0); f.v1 += dpp(f.v1); f.v2 += dpp(f.v2); f.v3 += dpp(f.v3); f.v4 += dpp(f.v4);
        };
        auto carry = [&]() {
            uint32_t c;
            c = f.v0 >> 26; f.v0 &= M26; f.v1 += c;
            c = f.v1 >> 26; f.v1 &= M26; f.v2 += c;
            c = f.v2 >> 26; f.v2 &= M26; f.v3 += c;
            c = f.v3 >> 26; f.v3 &= M26; f.v4 += c;
            c = f.v4 >> 26; f.v4 &= M26; f.v0 += c * 5u;
        };
        // row_shr:n = 0x110 + n, row_bcast:15 = 0x142, row_bcast:31 = 0x143; only the
        // group's last lane (31 or 63 for the broadcasts) is read afterwards
        if constexpr (PL == 2u) carry();
        level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true); });
        if constexpr (PL == 4u) carry();
        if constexpr (PL >= 4u)
            level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true); });
        if constexpr (PL == 8u) carry();
        if constexpr (PL >= 8u)
            level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true); });
        if constexpr (PL == 16u) carry();
        if constexpr (PL >= 16u)
            level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true); });
        if constexpr (PL == 32u) carry();
        if constexpr (PL >= 32u)
            level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xf, 0xf, true); });
        if constexpr (PL == 64u) {
            carry();
            level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xf, 0xf, true); });
        }
    }
    uint32_t tw[4];
    if constexpr (PL == 64u) {
        // one record per wave: lift the sum out of lane 63 into SGPRs so the
        // final reduction and s addition run on the scalar unit instead of
        // occupying the whole wave's VALU for one lane's arithmetic
        auto lane63 = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); };
        const F26 fs = {lane63(f.v0), lane63(f.v1), lane63(f.v2), lane63(f.v3), lane63(f.v4)};
        uint32_t s[4] = {uniform(kr[kSOff + 0]), uniform(kr[kSOff + 1]), uniform(kr[kSOff + 2]),
                         uniform(kr[kSOff + 3])};
        tag_words(fs, s, tw);
        if (t != PL - 1u) return;
    } else {
        if (t != PL - 1u) return;
        uint32_t s[4] = {kr[kSOff + 0], kr[kSOff + 1], kr[kSOff + 2], kr[kSOff + 3]};
        tag_words(f, s, tw);
    }

    if constexpr (!OPEN) {
        uint8_t* tp = out + n;  // ct || tag (chacha20_poly1305.rs:55)
        if ((((uintptr_t)tp) & 3u) == 0u) {
            uint32_t* t32 = reinterpret_cast<uint32_t*>(tp);
            t32[0] = tw[0]; t32[1] = tw[1]; t32[2] = tw[2]; t32[3] = tw[3];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) tp[i] = (uint8_t)(tw[i >> 2] >> (8 * (i & 3)));
        }
    } else {
        // constant-time compare: diff |= a ^ b over all 16 bytes (:84-87)
        const uint32_t diff = (rx[0] ^ tw[0]) | (rx[1] ^ tw[1]) | (rx[2] ^ tw[2]) | (rx[3] ^ tw[3]);
        p.status[rec] = diff != 0u ? 1u : 0u;
    }
}

// Record slot of this lane's group.  For L >= 64 a group is a whole wave (or
// the workgroup), so the slot is made provably uniform: the record's key,
// nonce and lengths then live in SGPRs and the uniform first-round
// quarter-rounds are hoisted to scalar code.
template <uint32_t L>
__device__ __forceinline__ uint32_t group_of_thread() {
    if constexpr (L == 256u) return 0u;
    else if constexpr (L >= 64u) return __builtin_amdgcn_readfirstlane(threadIdx.x / L);
    else return threadIdx.x / L;
}

// Direct launch: workgroup w serves records w*RPW .. w*RPW + RPW - 1.
template <bool OPEN, uint32_t L>
__global__ __launch_bounds__(256) void sg_aead_kernel(const KParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr uint32_t RPW = 256u / L;
    const uint32_t g = group_of_thread<L>(), t = threadIdx.x % L;
    const uint32_t rec = blockIdx.x * RPW + g;
    aead_record<OPEN, L>(p, rec, rec < p.count, lds + g * p.lds_rec_bytes, t);
}

// Bucketed launch: records listed by sg_classify_kernel for this size class.
// PERSIST = false: the host read the class population back and sized the grid
// exactly (one record group per workgroup, like the direct kernel: waves that
// finish their ChaCha20 share exit and free their slots while wave 0 runs the
// MAC).  PERSIST = true (stream capture, where the host cannot wait): a fixed
// grid walks the list; the barrier closing each iteration makes waves 1-3
// wait for wave 0's MAC, ~30 % slower per byte (tools/exp_list.py).
template <bool OPEN, uint32_t L, bool PERSIST>
__global__ __launch_bounds__(256) void sg_aead_list_kernel(const KParams p, const uint32_t* __restrict__ list,
                                                           const uint32_t* __restrict__ list_count) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr uint32_t RPW = 256u / L;
    const uint32_t g = group_of_thread<L>(), t = threadIdx.x % L;
    const uint32_t cnt = *list_count;
    const uint32_t stride = PERSIST ? gridDim.x * RPW : 0xffffffffu;
    for (uint32_t base = blockIdx.x * RPW; base < cnt; base += stride) {
        const uint32_t slot = base + g;
        const bool active = slot < cnt;
        uint32_t rec = active ? list[slot] : 0u;
        if constexpr (L >= 64u) rec = __builtin_amdgcn_readfirstlane(rec);
        aead_record<OPEN, L>(p, rec, active, lds + g * p.lds_rec_bytes, t);
        if constexpr (!PERSIST) break;
        __syncthreads();  // LDS is reused by the next iteration
    }
}

// ---------------------------------------------------------------------------
// Lock-step form of a uniform 16 KiB-class batch (KParams::ls; every record
// has the same length n, 8192 < n <= 16384).  Two records per 512-thread
// workgroup, so each SIMD holds two waves of one workgroup:
// * the record enters LDS with lane-contiguous 16-byte loads (1 KiB per
//   wave instruction; a lane that loads its own 64-byte block directly -- the
//   sg_aead_kernel pattern -- caps read+write at ~3.6 TB/s on MI355X, lane-
//   contiguous access streams ~5 TB/s, profiles/r01_valu_issue_probes.md);
// * lane t computes keystream block t + 1 (chacha20_poly1305.rs:52) with the
//   grouped rounds of sg_chacha_grp.inc -- four adds, four xors, four rotates,
//   s_barrier -- which keep the two waves of a SIMD in lock-step so that
//   their full-rate add/xor pair (2 cycles instead of 4);
// * Poly1305 runs on one wave per record as an i8 MFMA product (mfma_mac:
//   17 v_mfma_i32_32x32x32_i8 for a 16 KiB record, ~300 VALU instead of the
//   ~870 of v9's Horner MAC or ~1100 of the earlier 256-lane form).
// Measured (profiles/r01_mfma_mac_ab.md): seal 10.1 ms / open 9.6 ms against
// v9's 9.75 / 9.70; the MAC's LDS operand loads queue behind the lock-step
// data path and its one-wave tail holds the workgroup's LDS, so the kernel is
// off by default (sg_set_lockstep).
// Seal: load -> rounds -> ct into LDS -> store + MAC.  Open: load -> MAC over
// the received ciphertext -> rounds -> plaintext -> store (the reference
// decrypts unconditionally, chacha20_poly1305.rs:80-82).  Every wave runs the
// same rounds and barriers whatever its record holds: an inactive slot runs
// on dummy state.
// ---------------------------------------------------------------------------
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// LDS writes of one lane visible to the other lanes of its wave (and no
// compiler reordering across it)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Poly1305 of one record on one wave as an i8 MFMA product.
//
// The reference evaluates h = sum_j v_j r^(B - j) by Horner's rule
// (poly1305.rs:213-228), v_j = block j + pad bit.  Take the slot grid of the
// PL = 64 geometry (mac_geom: N = 64 k slots, the first z virtual and zero)
// as 32 rows of 2k blocks, slot i = 32 s + q in row q (so the 32 lanes of a
// half-wave read 32 consecutive blocks): its weight r^(N - i) = W_q P_s with
// W_q = r^(31 - q) and P_s = r^(32 (2k - 1 - s) + 1) (keying tables).
// Writing P_s in signed base-256 digits P_s[0..16], the byte convolution of a row
//   S[q][c] = sum_s sum_a (b_{q,s,a} - 128) P_s[c - a],   c = 0..31
// is one 32 x 32 x (32 k) i8 matrix product: A = the stream bytes with the
// top bit flipped (row q, K = (s, a)), B = the Toeplitz matrix of the
// digits (K = (s, a), column c), k MFMA 32x32x32 steps.  |S| < 2^24, so
// with the accumulator seeded at 2^24 every entry is a positive 25-bit
// integer and X_q = sum_c S[q][c] 2^(8c) is assembled exactly in radix 2^32.
// Then h = sum_q W_q X_q + ctot (mod p), where ctot (keying kernel) restores
// the i8 bias, the 2^24 seed and the pad bits.  Every step is exact integer
// arithmetic mod 2^130 - 5, so the tag equals the reference's.
template <bool OPEN>
__device__ __forceinline__ void mfma_mac(const KParams& p, const uint32_t rec, const uint32_t n, const uint32_t adlen,
                                         uint8_t* slot, const uint32_t S, const uint8_t* in, uint8_t* out,
                                         const uint32_t lane) {
    const MacGeom g = mac_geom(adlen, n, 64u);
    const uint32_t rows = 2u * g.k;
    const uint32_t* kr = p.ws + (uint64_t)rec * kKeyRecWordsLs;
    // every global operand of the combine is fetched now, so its latency hides
    // behind the power table and the matrix product: W_q = r^(31 - q) = rm[e >> 3] rs[e & 7]
    const uint32_t we = 31u - (lane & 31u);
    const F26 plo = load_f26(kr + kRSmallOff + 5u * (we & 7u));
    const F26 phi = load_f26(kr + kRMidOff + 5u * (we >> 3));
    const F26 ctot = {uniform(kr[kCtotOff + 0]), uniform(kr[kCtotOff + 1]), uniform(kr[kCtotOff + 2]),
                      uniform(kr[kCtotOff + 3]), uniform(kr[kCtotOff + 4])};
    uint32_t sk[4] = {uniform(kr[kSOff + 0]), uniform(kr[kSOff + 1]), uniform(kr[kSOff + 2]), uniform(kr[kSOff + 3])};
    uint32_t rx[4] = {0u, 0u, 0u, 0u};
    if constexpr (OPEN) {  // the received tag, fetched early (lane 0 compares)
        if (lane == 0u) {
            const uint8_t* ep = in + n;
            if ((((uintptr_t)ep) & 3u) == 0u) {
                const uint32_t* e32 = reinterpret_cast<const uint32_t*>(ep);
                rx[0] = e32[0]; rx[1] = e32[1]; rx[2] = e32[2]; rx[3] = e32[3];
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) rx[i >> 2] |= (uint32_t)ep[i] << (8 * (i & 3));
            }
        }
    }
    // ---- power table: row s = P_s's digits, reversed, at slot + 48 s: the 16
    // bytes at + 31 - c are P_s[c], P_s[c - 1], .., P_s[c - 15] (0 outside 0..16);
    // P_s = r^(32 t + 1), t = 2k - 1 - s
    if (lane < rows) {
        const uint32_t e = rows - 1u - lane;
        const F26 pm = load_f26(kr + kPowHiOff + 5u * (e >> 3));
        const F26 ps = load_f26(kr + kPowLoOff + 5u * (e & 7u));
        const F26 v = canonical(mul_add(pm, ps.v0, ps.v1, ps.v2, ps.v3, ps.v4, f26_zero()));
        // signed digits of V = the bytes of V + 0x80..80 (17 bytes), each minus 0x80
        uint32_t c;
        const uint32_t w0 = addc(v.v0 | (v.v1 << 26), 0x80808080u, 0u, &c);
        const uint32_t w1 = addc((v.v1 >> 6) | (v.v2 << 20), 0x80808080u, c, &c);
        const uint32_t w2 = addc((v.v2 >> 12) | (v.v3 << 14), 0x80808080u, c, &c);
        const uint32_t w3 = addc((v.v3 >> 18) | (v.v4 << 8), 0x80808080u, c, &c);
        const uint32_t w4 = (v.v4 >> 24) + 0x80u + c;
        uint8_t* F = slot + 48u * lane;
        st16(F, u32x4{0u, 0u, 0u, ((w4 ^ 0x80u) & 0xffu) << 24});
        st16(F + 16, u32x4{bswap32(w3 ^ 0x80808080u), bswap32(w2 ^ 0x80808080u), bswap32(w1 ^ 0x80808080u),
                           bswap32(w0 ^ 0x80808080u)});
        st16(F + 32, u32x4{0u, 0u, 0u, 0u});
    }
    wave_lds_sync();
    // ---- S = A B on the matrix cores: lane = (half h, row/column q) ----------
    const uint32_t q = lane & 31u, hh = lane >> 5;
    const uint32_t zoff = S + adlen + 8u + n + 8u;  // 16 zero bytes behind le64(n): the virtual blocks
    i32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 1 << 24;
    auto a_at = [&](const uint32_t i) {
        const uint32_t si = 32u * (2u * i + hh) + q;  // lanes q read consecutive blocks
        return slot + (si < g.z ? zoff : S + 16u * (si - g.z));
    };
    auto b_at = [&](const uint32_t i) { return slot + 48u * (2u * i + hh) + 31u - q; };
#ifndef SG_MAC_GLOBAL_A
#define SG_MAC_GLOBAL_A 0
#endif
    // Experiment switch (off): A blocks that lie wholly inside the ciphertext
    // read from the record in global memory (L2-resident: this workgroup just
    // stored it (seal) or loaded it (open)) instead of LDS; the AD / length
    // blocks and the virtual blocks still come from LDS.  Measured on C1:
    // seal 12.8 / open 12.6 ms against 10.2 / 9.9 from LDS (the 11-byte
    // misaligned 16-byte global loads are slower than the LDS queue)
    const uint8_t* ctg = OPEN ? in : out;
    const uint32_t pre = adlen + 8u;
    auto a_load = [&](const uint32_t i) -> u32x4 {
        if (SG_MAC_GLOBAL_A) {
            const uint32_t si = 32u * (2u * i + hh) + q;
            const uint32_t jb = si - g.z;
            if (si >= g.z && 16u * jb >= pre && 16u * jb + 16u <= pre + n) return ldu16(ctg + (16u * jb - pre));
        }
        return ldu16(a_at(i));
    };
    // operands of step i + 1 are loaded while step i runs
    u32x4 a = a_load(0), b = ldu16(b_at(0));
    for (uint32_t i = 0; i < g.k; ++i) {
        const uint32_t nx = i + 1u < g.k ? i + 1u : i;
        const u32x4 an = a_load(nx), bn = ldu16(b_at(nx));
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, a ^ 0x80808080u),
                                                     __builtin_bit_cast(i32x4, b), acc, 0, 0, 0);
        a = an;
        b = bn;
    }
    // ---- transpose through LDS (over the power table), 16 rows at a time:
    // accumulator i of lane (h, q) is S[(i & 3) + 8 (i >> 2) + 4 h][q]; lane q' < 32 takes row q'
    uint32_t X[32];
    wave_lds_sync();
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = 8 * pass + j;
            const uint32_t row = (uint32_t)((i & 3) + 8 * (i >> 2) - 16 * pass) + 4u * hh;
            *reinterpret_cast<int*>(slot + kLsTileStride * row + 4u * q) = acc[i];
        }
        wave_lds_sync();
        if ((lane >> 4) == (uint32_t)pass) {
            const uint8_t* rp = slot + kLsTileStride * (lane & 15u);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const u32x4 v = ldu16(rp + 16 * j);
                X[4 * j] = v.x; X[4 * j + 1] = v.y; X[4 * j + 2] = v.z; X[4 * j + 3] = v.w;
            }
        }
        wave_lds_sync();
    }
    // ---- X_q = sum_c S'[q][c] 2^(8c) (radix 2^32, 9 words): the four byte
    // phases c = 4m + j are each a run of non-overlapping 25-bit words
    uint32_t wv[9];
    {
        uint32_t c1 = 0u, c2 = 0u, c3 = 0u;
#pragma unroll
        for (int m = 0; m < 9; ++m) {
            const uint32_t t0 = m < 8 ? X[4 * m] : 0u;
            const uint32_t t1 = __builtin_amdgcn_alignbit(m < 8 ? X[4 * m + 1] : 0u, m > 0 ? X[4 * m - 3] : 0u, 24);
            const uint32_t t2 = __builtin_amdgcn_alignbit(m < 8 ? X[4 * m + 2] : 0u, m > 0 ? X[4 * m - 2] : 0u, 16);
            const uint32_t t3 = __builtin_amdgcn_alignbit(m < 8 ? X[4 * m + 3] : 0u, m > 0 ? X[4 * m - 1] : 0u, 8);
            uint32_t x = addc(t0, t1, c1, &c1);
            x = addc(x, t2, c2, &c2);
            wv[m] = addc(x, t3, c3, &c3);
        }
    }
    // ---- mod p: fold everything from 2^130 up twice (2^130 == 5 mod p)
    F26 f;
    {
        uint64_t t = (uint64_t)__builtin_amdgcn_alignbit(wv[5], wv[4], 2) * 5u + wv[0];
        const uint32_t y0 = (uint32_t)t;
        t = (uint64_t)__builtin_amdgcn_alignbit(wv[6], wv[5], 2) * 5u + wv[1] + (t >> 32);
        const uint32_t y1 = (uint32_t)t;
        t = (uint64_t)__builtin_amdgcn_alignbit(wv[7], wv[6], 2) * 5u + wv[2] + (t >> 32);
        const uint32_t y2 = (uint32_t)t;
        t = (uint64_t)__builtin_amdgcn_alignbit(wv[8], wv[7], 2) * 5u + wv[3] + (t >> 32);
        const uint32_t y3 = (uint32_t)t;
        t = (uint64_t)(wv[8] >> 2) * 5u + (wv[4] & 3u) + (t >> 32);  // y = y0..y3 + t 2^128 < 2^162
        const uint64_t u = (uint64_t)(uint32_t)(t >> 2) * 5u + y0;   // (y mod 2^130) + 5 (y >> 130)
        uint32_t c;
        const uint32_t z1 = addc(y1, (uint32_t)(u >> 32), 0u, &c);
        const uint32_t z2 = addc(y2, 0u, c, &c);
        const uint32_t z3 = addc(y3, 0u, c, &c);
        const uint32_t z4 = ((uint32_t)t & 3u) + c;  // <= 4
        f = words_to_f26((uint32_t)u, z1, z2, z3, 0u);
        f.v4 += z4 << 24;
    }
    {  // * W_q
        f = mul_add(f, plo.v0, plo.v1, plo.v2, plo.v3, plo.v4, f26_zero());
        f = mul_add(f, phi.v0, phi.v1, phi.v2, phi.v3, phi.v4, f26_zero());
    }
    if (lane >= 32u) f = f26_zero();
    {  // sum lanes 0..31 into lane 31: row_shr 1, 2, 4, 8, then row_bcast:15
        auto level = [&](auto dpp) {
            f.v0 += dpp(f.v0); f.v1 += dpp(f.v1); f.v2 += dpp(f.v2); f.v3 += dpp(f.v3); f.v4 += dpp(f.v4);
        };
        level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true); });
        level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true); });
        level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true); });
        level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true); });
        uint32_t c;
        c = f.v0 >> 26; f.v0 &= M26; f.v1 += c;
        c = f.v1 >> 26; f.v1 &= M26; f.v2 += c;
        c = f.v2 >> 26; f.v2 &= M26; f.v3 += c;
        c = f.v3 >> 26; f.v3 &= M26; f.v4 += c;
        c = f.v4 >> 26; f.v4 &= M26; f.v0 += c * 5u;
        level([](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xf, 0xf, true); });
    }
    // the sum leaves lane 31 for SGPRs: + ctot, canonical residue, + s (poly1305.rs:231-312)
    auto lane31 = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 31); };
    const F26 fs = {lane31(f.v0) + ctot.v0, lane31(f.v1) + ctot.v1, lane31(f.v2) + ctot.v2, lane31(f.v3) + ctot.v3,
                    lane31(f.v4) + ctot.v4};
    uint32_t tw[4];
    tag_words(fs, sk, tw);
    if (lane != 0u) return;
    if constexpr (!OPEN) {
        uint8_t* tp = out + n;  // ct || tag (chacha20_poly1305.rs:55)
        if ((((uintptr_t)tp) & 3u) == 0u) {
            uint32_t* t32 = reinterpret_cast<uint32_t*>(tp);
            t32[0] = tw[0]; t32[1] = tw[1]; t32[2] = tw[2]; t32[3] = tw[3];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) tp[i] = (uint8_t)(tw[i >> 2] >> (8 * (i & 3)));
        }
    } else {
        // constant-time compare: diff |= a ^ b over all 16 bytes (chacha20_poly1305.rs:84-87)
        const uint32_t diff = (rx[0] ^ tw[0]) | (rx[1] ^ tw[1]) | (rx[2] ^ tw[2]) | (rx[3] ^ tw[3]);
        p.status[rec] = diff != 0u ? 1u : 0u;
    }
}

// le64(n) and zeros to the end of the last MAC block, after the ciphertext
__device__ __forceinline__ void ls_suffix(uint8_t* ct, const uint32_t n) {
    if ((n & 3u) == 0u) {
        uint32_t* q = reinterpret_cast<uint32_t*>(ct + n);
        q[0] = n; q[1] = 0u; q[2] = 0u; q[3] = 0u; q[4] = 0u; q[5] = 0u; q[6] = 0u;
    } else {
        for (uint32_t i = 0; i < 28u; ++i) ct[n + i] = i < 8u ? (uint8_t)((uint64_t)n >> (8u * i)) : 0;
    }
}

template <bool OPEN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) void sg_aead_ls_kernel(const KParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
    const uint32_t t = threadIdx.x & 255u;
    const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63u;
    const uint32_t rec = blockIdx.x * 2u + g;
    const bool active = rec < p.count;
    uint8_t* slot = lds + g * p.lds_rec_bytes;
    const uint32_t n = OPEN ? p.uniform_len - 16u : p.uniform_len;
    const uint32_t adlen = p.tls ? 13u : p.ad_len;
    const uint32_t A = kLsHead + ((adlen + 8u + 15u) & ~15u);
    const uint32_t S = A - adlen - 8u;  // stream start
    uint8_t* ct = slot + A;
    const uint8_t* in = p.in;
    uint8_t* out = p.out;
    RecKey rk = {};
    if (active) {
        in = p.in + (p.in_off ? p.in_off[rec] : p.in_stride * rec);
        out = p.out + (p.out_off ? p.out_off[rec] : p.out_stride * rec);
        rk = record_key(p, rec);
        // ---- the record into LDS, lane-contiguous ----
        const uint32_t tail = n & ~15u;
        if ((((uintptr_t)in) & 15u) == 0u) {
#pragma unroll
            for (uint32_t q = 0; q < 4u; ++q) {
                const uint32_t off = 4096u * w + 16u * (lane + 64u * q);
                if (off + 16u <= n) st16(ct + off, ldg16(in + off));
            }
            if (t < (n & 15u)) ct[tail + t] = in[tail + t];
        } else {
#pragma unroll 1
            for (uint32_t i = t; i < n; i += 256u) ct[i] = in[i];
        }
        // ---- MAC stream framing: ad || le64(|ad|) || ct || le64(|ct|) ----
        for (uint32_t i = t; i < adlen + 8u; i += 256u) {
            uint8_t v;
            if (i < adlen)
                v = p.tls ? tls_ad_byte(rk.seq, p.tls_hdr, n, i) : p.ads[(uint64_t)p.ad_stride * rec + i];
            else
                v = (uint8_t)((uint64_t)adlen >> (8u * (i - adlen)));
            slot[S + i] = v;
        }
        if constexpr (OPEN) {
            if (t == 0u) ls_suffix(ct, n);
        }
    }
    __syncthreads();
    if constexpr (OPEN) {
        // one wave per record (spread over the SIMDs) runs the MAC over the received ciphertext
        if (active && w == (rec & 3u) && !SG_LS_NOMAC) mfma_mac<true>(p, rec, n, adlen, slot, S, in, out, lane);
        __syncthreads();  // every MAC read is done before the plaintext replaces the ciphertext
    }
    // ---- keystream block t + 1 in lock-step; XOR in LDS ----
    const uint32_t off = 64u * t;
    const bool mine = active && off < n;
    u32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    if (mine) {
        d0 = ld16(ct + off); d1 = ld16(ct + off + 16u); d2 = ld16(ct + off + 32u); d3 = ld16(ct + off + 48u);
    }
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, rk.k[0], rk.k[1], rk.k[2], rk.k[3],
                      rk.k[4],     rk.k[5],     rk.k[6],     rk.k[7],     t + 1u,  0u,      rk.n14,  rk.n15};
#if SG_LS_NOROUNDS  // experiment: no rounds (the memory path alone; output is wrong)
#elif SG_LS_COMPILED  // experiment: compiled rounds, no lock-step barriers
    {
        uint32_t ks[16];
        chacha_block(ks, rk.k, t + 1u, rk.n14, rk.n15);
        for (int i = 0; i < 16; ++i) x[i] = ks[i] - (i < 4 ? (i == 0 ? 0x61707865u : i == 1 ? 0x3320646eu : i == 2 ? 0x79622d32u : 0x6b206574u)
                                                         : i < 12 ? rk.k[i - 4] : i == 12 ? t + 1u : i == 13 ? 0u : i == 14 ? rk.n14 : rk.n15);
    }
#else
#pragma unroll 1
    for (int r = 0; r < 10; ++r)
        asm volatile(SG_CHACHA_DR_NB1_BAR1
                     : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                       "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                       "+v"(x[14]), "+v"(x[15]));
#endif
    if (mine) {
        d0 ^= u32x4{x[0] + 0x61707865u, x[1] + 0x3320646eu, x[2] + 0x79622d32u, x[3] + 0x6b206574u};
        d1 ^= u32x4{x[4] + rk.k[0], x[5] + rk.k[1], x[6] + rk.k[2], x[7] + rk.k[3]};
        d2 ^= u32x4{x[8] + rk.k[4], x[9] + rk.k[5], x[10] + rk.k[6], x[11] + rk.k[7]};
        d3 ^= u32x4{x[12] + t + 1u, x[13], x[14] + rk.n14, x[15] + rk.n15};
        st16(ct + off, d0); st16(ct + off + 16u, d1); st16(ct + off + 32u, d2); st16(ct + off + 48u, d3);
    }
    if constexpr (!OPEN) {
        // the suffix lies behind the last (possibly partial) block: written by that block's lane
        if (active && t == ((n >> 6) < 255u ? (n >> 6) : 255u)) ls_suffix(ct, n);
    }
    __syncthreads();
    // ---- the output leaves lane-contiguous ----
    if (active) {
        const uint32_t tail = n & ~15u;
        if ((((uintptr_t)out) & 15u) == 0u) {
#pragma unroll
            for (uint32_t q = 0; q < 4u; ++q) {
                const uint32_t o = 4096u * w + 16u * (lane + 64u * q);
                if (o + 16u <= n) stg16(out + o, ld16(ct + o));
            }
            if (t < (n & 15u)) out[tail + t] = ct[tail + t];
        } else {
#pragma unroll 1
            for (uint32_t i = t; i < n; i += 256u) out[i] = ct[i];
        }
    }
    if constexpr (!OPEN) {
        // the MAC reads the stored ciphertext back (SG_MAC_GLOBAL_A): every wave's stores first
        if (SG_MAC_GLOBAL_A) __syncthreads();
        if (active && w == (rec & 3u) && !SG_LS_NOMAC) mfma_mac<false>(p, rec, n, adlen, slot, S, in, out, lane);
    }
}

// Size-class bucketing.  A 1024-thread workgroup classifies 4096 records:
// per-wave ballots, then one device atomic per class per workgroup (a single
// counter word takes only ~88 atomics/us, so per-wave atomics cost ~0.5 ms
// for 1M records).
constexpr uint32_t kClassifyThreads = 1024;
constexpr uint32_t kClassifyPerThread = 4;

template <bool OPEN>
__global__ __launch_bounds__(1024) void sg_classify_kernel(const KParams p, uint32_t* __restrict__ lists,
                                                           uint32_t* __restrict__ counts) {
    __shared__ uint32_t wave_cnt[kNumClasses][kClassifyThreads / 64];
    __shared__ uint32_t wg_base[kNumClasses];
    const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
    const uint32_t rec0 = blockIdx.x * (kClassifyThreads * kClassifyPerThread);
    uint32_t cls[kClassifyPerThread];
    uint32_t mine[kNumClasses] = {};  // this wave's records per class
#pragma unroll
    for (uint32_t i = 0; i < kClassifyPerThread; ++i) {
        const uint32_t rec = rec0 + i * kClassifyThreads + threadIdx.x;
        cls[i] = kNumClasses;
        if (rec < p.count) {
            const uint32_t len = record_len(p, rec);
            const uint32_t n = OPEN ? (len >= 16u ? len - 16u : 0u) : len;
            cls[i] = size_class(n);
        }
#pragma unroll
        for (uint32_t c = 0; c < kNumClasses; ++c) mine[c] += (uint32_t)__popcll(__ballot(cls[i] == c));
    }
    if (lane == 0)
        for (uint32_t c = 0; c < kNumClasses; ++c) wave_cnt[c][wave] = mine[c];
    __syncthreads();
    if (threadIdx.x < kNumClasses) {
        uint32_t tot = 0;
        for (uint32_t w = 0; w < kClassifyThreads / 64; ++w) {
            const uint32_t x = wave_cnt[threadIdx.x][w];
            wave_cnt[threadIdx.x][w] = tot;  // exclusive prefix over waves
            tot += x;
        }
        wg_base[threadIdx.x] = tot ? atomicAdd(&counts[threadIdx.x], tot) : 0u;
    }
    __syncthreads();
    uint32_t off[kNumClasses];
#pragma unroll
    for (uint32_t c = 0; c < kNumClasses; ++c) off[c] = wg_base[c] + wave_cnt[c][wave];
#pragma unroll
    for (uint32_t i = 0; i < kClassifyPerThread; ++i) {
        const uint32_t rec = rec0 + i * kClassifyThreads + threadIdx.x;
#pragma unroll
        for (uint32_t c = 0; c < kNumClasses; ++c) {
            const uint64_t mask = __ballot(cls[i] == c);
            if (cls[i] == c) lists[(uint64_t)c * p.count + off[c] + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull))] = rec;
            off[c] += (uint32_t)__popcll(mask);
        }
    }
}

// ---------------------------------------------------------------------------
// synthetic records + compare (bench/test plumbing)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void sg_fill_kernel(uint8_t* buf, uint64_t stride, uint32_t len,
                                                      uint32_t count, uint64_t seed, uint64_t j0) {
    const uint32_t wpr = (len + 7u) >> 3;  // 8-byte words per record
    const uint64_t total = (uint64_t)wpr * count;
    const bool aligned = ((stride | (uintptr_t)buf) & 7u) == 0u && (len & 7u) == 0u;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t j = g / wpr;
        const uint32_t w = (uint32_t)(g - j * wpr);
        const uint64_t v = splitmix64(seed ^ ((j0 + j) << 32) ^ (uint64_t)w);
        uint8_t* dst = buf + stride * j + 8ull * w;
        if (aligned) {
            *reinterpret_cast<uint64_t*>(dst) = v;
        } else {
            for (uint32_t b = 0; b < 8u && 8u * w + b < len; ++b) dst[b] = (uint8_t)(v >> (8 * b));
        }
    }
}

__global__ __launch_bounds__(256) void sg_compare_kernel(const uint8_t* a, uint64_t sa, const uint8_t* b,
                                                         uint64_t sb, uint32_t len, uint32_t count,
                                                         unsigned long long* mism) {
    __shared__ uint32_t bad;
    for (uint32_t rec = blockIdx.x; rec < count; rec += gridDim.x) {
        if (threadIdx.x == 0) bad = 0;
        __syncthreads();
        const uint8_t* pa = a + sa * rec;
        const uint8_t* pb = b + sb * rec;
        uint32_t diff = 0;
        const bool vec = (((uintptr_t)pa | (uintptr_t)pb) & 15u) == 0u;
        const uint32_t nvec = vec ? (len >> 4) : 0u;
        for (uint32_t i = threadIdx.x; i < nvec; i += blockDim.x) {
            const uint4 x = reinterpret_cast<const uint4*>(pa)[i];
            const uint4 y = reinterpret_cast<const uint4*>(pb)[i];
            diff |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
        }
        for (uint32_t i = nvec * 16u + threadIdx.x; i < len; i += blockDim.x) diff |= pa[i] ^ pb[i];
        if (diff) atomicOr(&bad, 1u);
        __syncthreads();
        if (threadIdx.x == 0 && bad) atomicAdd(mism, 1ull);
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_keying(const KParams& p, bool open, hipStream_t s) {
    const uint32_t grid = (p.count + kKeyingThreads - 1u) / kKeyingThreads;
    if (p.ls) {
        if (open)
            hipLaunchKernelGGL((sg_keying_kernel<true, true>), dim3(grid), dim3(kKeyingThreads), 0, s, p);
        else
            hipLaunchKernelGGL((sg_keying_kernel<false, true>), dim3(grid), dim3(kKeyingThreads), 0, s, p);
    } else if (open) {
        hipLaunchKernelGGL((sg_keying_kernel<true, false>), dim3(grid), dim3(kKeyingThreads), 0, s, p);
    } else {
        hipLaunchKernelGGL((sg_keying_kernel<false, false>), dim3(grid), dim3(kKeyingThreads), 0, s, p);
    }
    return hipGetLastError();
}

template <bool OPEN, uint32_t L>
hipError_t launch_direct(const KParams& p, hipStream_t s) {
    constexpr uint32_t RPW = 256u / L;
    const uint32_t grid = (p.count + RPW - 1u) / RPW;
    hipLaunchKernelGGL((sg_aead_kernel<OPEN, L>), dim3(grid), dim3(kThreads), RPW * p.lds_rec_bytes, s, p);
    return hipGetLastError();
}

// n_exact: the class population when the host knows it (exact grid), or
// UINT32_MAX for a persistent grid capped at kListGridPerCU workgroups per CU.
template <bool OPEN, uint32_t L>
hipError_t launch_list(const KParams& p, const uint32_t* list, const uint32_t* cnt, uint32_t n_exact,
                       hipStream_t s) {
    constexpr uint32_t RPW = 256u / L;
    const size_t lds = RPW * p.lds_rec_bytes;
    if (n_exact != 0xffffffffu) {
        if (n_exact == 0) return hipSuccess;
        hipLaunchKernelGGL((sg_aead_list_kernel<OPEN, L, false>), dim3((n_exact + RPW - 1u) / RPW), dim3(kThreads),
                           lds, s, p, list, cnt);
        return hipGetLastError();
    }
    uint32_t grid = (p.count + RPW - 1u) / RPW;
    const uint32_t cap = kListGridPerCU * 256u;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL((sg_aead_list_kernel<OPEN, L, true>), dim3(grid), dim3(kThreads), lds, s, p, list, cnt);
    return hipGetLastError();
}

template <bool OPEN>
hipError_t launch_class(uint32_t c, const KParams& q, const uint32_t* list, const uint32_t* cnt, uint32_t n_exact,
                        hipStream_t s) {
#define SG_CLASS_CASE(C)                                                                  \
    case C:                                                                               \
        return list ? launch_list<OPEN, class_lanes(C)>(q, list, cnt, n_exact, s)         \
                    : launch_direct<OPEN, class_lanes(C)>(q, s);
    switch (c) {
        SG_CLASS_CASE(0) SG_CLASS_CASE(1) SG_CLASS_CASE(2) SG_CLASS_CASE(3)
        SG_CLASS_CASE(4) SG_CLASS_CASE(5) SG_CLASS_CASE(6)
        default: return list ? launch_list<OPEN, class_lanes(7)>(q, list, cnt, n_exact, s)
                             : launch_direct<OPEN, class_lanes(7)>(q, s);
    }
#undef SG_CLASS_CASE
}

template <bool OPEN>
hipError_t launch_aead_t(const KParams& p, uint32_t max_n, bool uniform, uint32_t* lists, uint32_t* counts,
                         hipStream_t s) {
    if (uniform && p.ls) {  // uniform 16 KiB-class batch: lock-step kernel, two records per workgroup
        KParams q = p;
        q.lds_rec_bytes = lds_ls_rec_bytes(q.ad_len, max_n);
        hipLaunchKernelGGL(sg_aead_ls_kernel<OPEN>, dim3((p.count + 1u) / 2u), dim3(512), 2u * q.lds_rec_bytes, s, q);
        return hipGetLastError();
    }
    if (uniform) {  // every record in one class: direct launch
        KParams q = p;
        const uint32_t c = size_class(max_n);
        q.lds_rec_bytes = lds_rec_bytes(c, q.ad_len, max_n);
        return launch_class<OPEN>(c, q, nullptr, nullptr, 0, s);
    }
    hipError_t e = hipMemsetAsync(counts, 0, kNumClasses * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint32_t per_wg = kClassifyThreads * kClassifyPerThread;
    hipLaunchKernelGGL(sg_classify_kernel<OPEN>, dim3((p.count + per_wg - 1u) / per_wg), dim3(kClassifyThreads), 0, s,
                       p, lists, counts);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // Read the class populations back (one stream sync per mixed batch) so every
    // class runs on an exact grid; under stream capture the host cannot wait,
    // so the classes run on persistent grids instead.
    uint32_t pop[kNumClasses];
    hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
    if ((e = hipStreamIsCapturing(s, &cap_status)) != hipSuccess) return e;
    const bool exact = cap_status == hipStreamCaptureStatusNone;
    if (exact) {
        if ((e = hipMemcpyAsync(pop, counts, sizeof pop, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    }
    // one launch per populated class, largest records first
    KParams q = p;
    for (int c = (int)size_class(max_n); c >= 0; --c) {
        const uint32_t cap = max_n < class_max((uint32_t)c) ? max_n : class_max((uint32_t)c);
        q.lds_rec_bytes = lds_rec_bytes((uint32_t)c, q.ad_len, cap);
        if ((e = launch_class<OPEN>((uint32_t)c, q, lists + (uint64_t)c * p.count, counts + c,
                                    exact ? pop[c] : 0xffffffffu, s)) != hipSuccess)
            return e;
    }
    return hipSuccess;
}

hipError_t launch_aead(const KParams& p, bool open, uint32_t max_n, bool uniform, uint32_t* lists,
                       uint32_t* counts, hipStream_t s) {
    return open ? launch_aead_t<true>(p, max_n, uniform, lists, counts, s)
                : launch_aead_t<false>(p, max_n, uniform, lists, counts, s);
}

hipError_t launch_fill(uint8_t* buf, uint64_t stride, uint32_t len, uint32_t count, uint64_t seed,
                       uint64_t j0, hipStream_t s) {
    const uint64_t words = (uint64_t)((len + 7u) >> 3) * count;
    uint64_t grid = (words + 255u) / 256u;
    if (grid > 65536u) grid = 65536u;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(sg_fill_kernel, dim3((uint32_t)grid), dim3(256), 0, s, buf, stride, len, count, seed, j0);
    return hipGetLastError();
}

hipError_t launch_compare(const uint8_t* a, uint64_t sa, const uint8_t* b, uint64_t sb, uint32_t len,
                          uint32_t count, unsigned long long* mism, hipStream_t s) {
    uint32_t grid = count < 16384u ? count : 16384u;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(sg_compare_kernel, dim3(grid), dim3(256), 0, s, a, sa, b, sb, len, count, mism);
    return hipGetLastError();
}

#ifndef SG_LOCKSTEP_DEFAULT
#define SG_LOCKSTEP_DEFAULT 0
#endif
static int g_lockstep = -1;  // -1: not read from the environment yet
bool lockstep_enabled() {
    if (__atomic_load_n(&g_lockstep, __ATOMIC_ACQUIRE) < 0) {
        const char* e = getenv("SG_LOCKSTEP");
        int expect = -1;
        __atomic_compare_exchange_n(&g_lockstep, &expect, e ? (e[0] == '1' ? 1 : 0) : (SG_LOCKSTEP_DEFAULT ? 1 : 0),
                                    false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
    }
    return __atomic_load_n(&g_lockstep, __ATOMIC_ACQUIRE) == 1;
}
int set_lockstep(int enable) {
    const int prev = lockstep_enabled() ? 1 : 0;
    if (enable >= 0) __atomic_store_n(&g_lockstep, enable ? 1 : 0, __ATOMIC_RELEASE);
    return prev;
}

const char* kernel_config() {
#define SG_STR2(x) #x
#define SG_STR(x) SG_STR2(x)
    if (lockstep_enabled())
        return "gfx950 sg_aead_kernel v11" "/salu_pre=" SG_STR(SG_SALU_PRE) "/mac_v2=1/lockstep=1"
               ": uniform 8-16 KiB batches on sg_aead_ls_kernel (two records per 512-thread workgroup, lane-contiguous "
               "loads/stores through LDS, grouped lock-step ChaCha20 rounds with s_barrier per rotate group, Poly1305 as an "
               "i8 MFMA product on one wave per record: 32 rows x 2k blocks, Toeplitz digit matrix of r^1..r^2k, "
               "v_mfma_i32_32x32x32_i8, exact row assembly, W_q scaling + DPP sum, keying constant term); other batches: "
               "8 size classes as v9, keying pre-pass";
    return "gfx950 sg_aead_kernel v9" "/salu_pre=" SG_STR(SG_SALU_PRE) "/mac_v2=1"
           ": 8 size classes (2..256 lanes per record, one 64-B block per lane, device bucketing, exact class grids), "
           "lane=64B ChaCha block (counter-free round-1 QRs on SALU for wave-uniform records), Poly1305 contiguous-chunk "
           "Horner radix-2^32 (clamped r, unaligned 16-B LDS block loads, folded pad bit) on min(L,64) lanes + per-lane "
           "r^(k(PL-1-t)) scale + DPP sum, tag finalised on the SALU for one-record waves, keying pre-pass";
}

}  // namespace sg
