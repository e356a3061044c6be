// sg_kernels.hip -- gfx950 (CDNA4) kernels for suruga's ChaCha20-Poly1305
// record AEAD (draft-agl-tls-chacha20poly1305-04 as in klutzy/suruga).
//
// Work decomposition (one TLS record per 256-thread workgroup):
//
//   sg_keying_kernel   one lane per record: ChaCha20 block 0 -> Poly1305 key
//                      (r clamped, s) and the powers r, r^2, r^4 .. r^64 the
//                      MAC kernels multiply by.  (chacha20_poly1305.rs:50,75;
//                      poly1305.rs:197-205)
//   sg_aead_kernel<OPEN>
//     phase 1, all 4 waves: lane t owns 64-byte data blocks t, t+256, ...;
//       computes keystream block b+1 in registers (chacha20.rs:53-135),
//       XORs the record bytes (chacha20.rs:143-153), writes the result to HBM
//       and the ciphertext into LDS.
//     phase 2, wave 0: Poly1305 over ad || le64(|ad|) || ct || le64(|ct|)
//       (chacha20_poly1305.rs:19-42) read from LDS.  Lane t runs Horner over
//       MAC blocks t, t+64, t+128, ... with multiplier r^64, then a 6-level
//       shuffle tree with r^1..r^32 combines the 64 partial sums; lane 0
//       multiplies by r, reduces mod 2^130-5 and adds s (poly1305.rs:230-312).
//       Seal appends the tag (chacha20_poly1305.rs:55); open compares it in
//       constant time (:84-93) after having decrypted unconditionally (:80-82).
//
// All Poly1305 arithmetic is exact mod p = 2^130 - 5 in radix 2^26 with
// 64-bit v_mad_u64_u32 accumulation; the result equals the reference's
// sequential Horner (poly1305.rs:207-228) because both compute the same
// polynomial in the field and reduce it to the canonical representative.
#include "sg_internal.h"

#include <stdint.h>

namespace sg {
namespace {

constexpr uint32_t M26 = (1u << 26) - 1;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

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

// ---- Poly1305 field arithmetic, radix 2^26 ------------------------------
// Invariant of a "reduced" element: limbs 0,2,3,4 < 2^26, limb 1 < 2^26 + 2^8.
struct F26 {
    uint32_t v0, v1, v2, v3, v4;
};

// returns a * b + c (mod p, reduced), b fully reduced (< 2^26 per limb),
// a reduced, c limbs < 2^27.
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

__device__ __forceinline__ F26 mul_add(const F26 a, const uint32_t* b, const F26 c) {
    return mul_add(a, b[0], b[1], b[2], b[3], b[4], c);
}

__device__ __forceinline__ F26 f26_zero() { return F26{0u, 0u, 0u, 0u, 0u}; }

// Full carry: every limb < 2^26, value < 2^130 (not yet < p).
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

// Canonical representative in [0, p): subtract p when h >= p, branch-free
// (the role of Int1305::normalize, poly1305.rs:165-192).
__device__ __forceinline__ F26 canonical(F26 h) {
    h = carry_full(h);
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

// 16 little-endian bytes (4 words) + the 2^(8*valid) pad bit -> radix-2^26
// (poly1305.rs:130-162, :216-225).  valid in [1, 16].
__device__ __forceinline__ F26 block_to_f26(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                            uint32_t hibit) {
    F26 c;
    c.v0 = w0 & M26;
    c.v1 = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
    c.v2 = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    c.v3 = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
    c.v4 = (w3 >> 8) | hibit;
    return c;
}

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
__global__ __launch_bounds__(256) void sg_keying_kernel(const KParams p) {
    const uint32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
    if (rec >= p.count) return;
    const RecKey rk = record_key(p, rec);
    uint32_t ks[16];
    chacha_block(ks, rk.k, 0u, rk.n14, rk.n15);  // block 0 -> poly key (chacha20_poly1305.rs:50)
    // r = clamp(pk[0..16]) (poly1305.rs:197-203), s = pk[16..32]
    const uint32_t r0 = ks[0] & 0x0fffffffu, r1 = ks[1] & 0x0ffffffcu;
    const uint32_t r2 = ks[2] & 0x0ffffffcu, r3 = ks[3] & 0x0ffffffcu;
    F26 pw = block_to_f26(r0, r1, r2, r3, 0u);
    uint32_t* out = p.ws + (uint64_t)rec * kKeyRecWords;
    for (int k = 0; k < 7; ++k) {
        out[kPowOff + 5 * k + 0] = pw.v0;
        out[kPowOff + 5 * k + 1] = pw.v1;
        out[kPowOff + 5 * k + 2] = pw.v2;
        out[kPowOff + 5 * k + 3] = pw.v3;
        out[kPowOff + 5 * k + 4] = pw.v4;
        if (k < 6) pw = carry_full(mul_add(pw, pw.v0, pw.v1, pw.v2, pw.v3, pw.v4, f26_zero()));
    }
    out[kSOff + 0] = ks[4];
    out[kSOff + 1] = ks[5];
    out[kSOff + 2] = ks[6];
    out[kSOff + 3] = ks[7];
    out[kSOff + 4] = 0u;
}

// AD byte i of the TLS record-layer additional data (tls.rs:103-112, 250-265):
// be64(seq) || type || major || minor || be16(n)
__device__ __forceinline__ uint8_t tls_ad_byte(uint64_t seq, uint32_t hdr, uint32_t n, uint32_t i) {
    if (i < 8) return (uint8_t)(seq >> (56 - 8 * i));
    if (i < 11) return (uint8_t)(hdr >> (8 * (i - 8)));
    if (i == 11) return (uint8_t)(n >> 8);
    return (uint8_t)n;
}

// ---------------------------------------------------------------------------
// Fused seal / open: one record per workgroup.
// ---------------------------------------------------------------------------
template <bool OPEN>
__global__ __launch_bounds__(256) void sg_aead_kernel(const KParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t rec = blockIdx.x;
    const uint32_t tid = threadIdx.x;

    const uint32_t len = record_len(p, rec);
    uint32_t n = len;
    if constexpr (OPEN) {
        if (len < 16u) {  // chacha20_poly1305.rs:68-70 "message too short"
            if (tid == 0) p.status[rec] = 2u;
            return;
        }
        n = len - 16u;
    }
    const uint8_t* in = p.in + (p.in_off ? p.in_off[rec] : p.in_stride * rec);
    uint8_t* out = p.out + (p.out_off ? p.out_off[rec] : p.out_stride * rec);
    const RecKey rk = record_key(p, rec);
    const uint32_t A = p.lds_ct_off;
    uint8_t* ct_lds = lds + A;

    // ---- phase 1: keystream XOR, 64 bytes per lane-block ------------------
    const bool vec_ok = (((uintptr_t)in | (uintptr_t)out) & 15u) == 0u;
    const uint32_t nblocks = (n + 63u) >> 6;
    for (uint32_t b = tid; b < nblocks; b += kThreads) {
        const uint32_t off = b << 6;
        if (vec_ok && off + 64u <= n) {
            const uint4* src = reinterpret_cast<const uint4*>(in + off);
            const uint4 d0 = src[0], d1 = src[1], d2 = src[2], d3 = src[3];
            uint32_t ks[16];
            chacha_block(ks, rk.k, b + 1u, rk.n14, rk.n15);  // data uses blocks 1.. (chacha20_poly1305.rs:52)
            const uint4 r0 = make_uint4(d0.x ^ ks[0], d0.y ^ ks[1], d0.z ^ ks[2], d0.w ^ ks[3]);
            const uint4 r1 = make_uint4(d1.x ^ ks[4], d1.y ^ ks[5], d1.z ^ ks[6], d1.w ^ ks[7]);
            const uint4 r2 = make_uint4(d2.x ^ ks[8], d2.y ^ ks[9], d2.z ^ ks[10], d2.w ^ ks[11]);
            const uint4 r3 = make_uint4(d3.x ^ ks[12], d3.y ^ ks[13], d3.z ^ ks[14], d3.w ^ ks[15]);
            uint4* dst = reinterpret_cast<uint4*>(out + off);
            dst[0] = r0; dst[1] = r1; dst[2] = r2; dst[3] = r3;
            uint4* cl = reinterpret_cast<uint4*>(ct_lds + off);
            if constexpr (OPEN) {
                cl[0] = d0; cl[1] = d1; cl[2] = d2; cl[3] = d3;
            } else {
                cl[0] = r0; cl[1] = r1; cl[2] = r2; cl[3] = r3;
            }
        } else {
            // partial last block or misaligned record: byte granular
            uint32_t ks[16];
            chacha_block(ks, rk.k, b + 1u, rk.n14, rk.n15);
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

    // ---- MAC stream framing in LDS: ad || le64(|ad|) || ct || le64(|ct|) ----
    const uint32_t adlen = p.tls ? 13u : p.ad_len;
    const uint32_t S = A - adlen - 8u;  // stream start
    if (tid < 64u) {
        for (uint32_t i = tid; i < adlen + 8u; i += 64u) {
            uint8_t v;
            if (i < adlen)
                v = p.tls ? tls_ad_byte(rk.seq, p.tls_hdr, n, i) : p.ads[(uint64_t)p.ad_stride * rec + i];
            else
                v = (uint8_t)((uint64_t)adlen >> (8u * (i - adlen)));
            lds[S + i] = v;
        }
        if (tid < 8u) ct_lds[n + tid] = (uint8_t)((uint64_t)n >> (8u * tid));
    }
    __syncthreads();
    if (tid >= 64u) return;

    // ---- phase 2 (wave 0): Poly1305 ----------------------------------------
    const uint32_t* kr = p.ws + (uint64_t)rec * kKeyRecWords;
    uint32_t pw[7][5];
#pragma unroll
    for (int k = 0; k < 7; ++k)
#pragma unroll
        for (int i = 0; i < 5; ++i) pw[k][i] = kr[kPowOff + 5 * k + i];

    const uint32_t L = adlen + 16u + n;         // MAC stream length
    const uint32_t B = (L + 15u) >> 4;          // MAC blocks
    const uint32_t z = (64u - (B & 63u)) & 63u; // leading virtual zero blocks
    const uint32_t J = (B + z) >> 6;
    const uint32_t sh = (S & 3u) * 8u;
    const uint32_t* l32 = reinterpret_cast<const uint32_t*>(lds);

    F26 h = f26_zero();
    for (uint32_t j = 0; j < J; ++j) {
        const int32_t i = (int32_t)(tid + 64u * j) - (int32_t)z;
        F26 c = f26_zero();
        if (i >= 0) {
            const uint32_t pos = S + 16u * (uint32_t)i;
            const uint32_t q = pos >> 2;
            const uint32_t a0 = l32[q], a1 = l32[q + 1], a2 = l32[q + 2], a3 = l32[q + 3], a4 = l32[q + 4];
            uint32_t w0 = __builtin_amdgcn_alignbit(a1, a0, sh);
            uint32_t w1 = __builtin_amdgcn_alignbit(a2, a1, sh);
            uint32_t w2 = __builtin_amdgcn_alignbit(a3, a2, sh);
            uint32_t w3 = __builtin_amdgcn_alignbit(a4, a3, sh);
            uint32_t hibit = 1u << 24;  // 2^128 pad bit of a full block
            const uint32_t rem = L - 16u * (uint32_t)i;
            if (rem < 16u) {  // final partial block: zero-pad, pad bit at 8*rem (poly1305.rs:216-225)
                hibit = 0u;
                const uint32_t bit = 8u * rem;
                uint32_t m0 = bit >= 32u ? ~0u : ((1u << bit) - 1u);
                uint32_t m1 = bit >= 64u ? ~0u : (bit <= 32u ? 0u : ((1u << (bit - 32u)) - 1u));
                uint32_t m2 = bit >= 96u ? ~0u : (bit <= 64u ? 0u : ((1u << (bit - 64u)) - 1u));
                uint32_t m3 = bit <= 96u ? 0u : ((1u << (bit - 96u)) - 1u);
                w0 &= m0; w1 &= m1; w2 &= m2; w3 &= m3;
                const uint32_t fb = 1u << (bit & 31u);
                const uint32_t fw = bit >> 5;
                w0 |= fw == 0u ? fb : 0u;
                w1 |= fw == 1u ? fb : 0u;
                w2 |= fw == 2u ? fb : 0u;
                w3 |= fw == 3u ? fb : 0u;
            }
            c = block_to_f26(w0, w1, w2, w3, hibit);
        }
        h = (j == 0) ? c : mul_add(h, pw[6], c);  // h = h * r^64 + c
    }
    // combine lanes: after level l, lane t (t % 2^(l+1) == 0) holds
    // sum_{u=t}^{t+2^(l+1)-1} h_u r^(t+2^(l+1)-1-u)
#pragma unroll
    for (int l = 0; l < 6; ++l) {
        const int d = 1 << l;
        F26 o;
        o.v0 = __shfl_down(h.v0, d, 64);
        o.v1 = __shfl_down(h.v1, d, 64);
        o.v2 = __shfl_down(h.v2, d, 64);
        o.v3 = __shfl_down(h.v3, d, 64);
        o.v4 = __shfl_down(h.v4, d, 64);
        h = mul_add(h, pw[l], o);
    }
    if (tid != 0) return;
    h = mul_add(h, pw[0], f26_zero());  // * r
    uint32_t s[4] = {kr[kSOff + 0], kr[kSOff + 1], kr[kSOff + 2], kr[kSOff + 3]};
    uint32_t t[4];
    tag_words(h, s, t);

    if constexpr (!OPEN) {
        uint8_t* tp = out + n;  // ct || tag (chacha20_poly1305.rs:55)
        if ((((uintptr_t)tp) & 3u) == 0u) {
            uint32_t* t32 = reinterpret_cast<uint32_t*>(tp);
            t32[0] = t[0]; t32[1] = t[1]; t32[2] = t[2]; t32[3] = t[3];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) tp[i] = (uint8_t)(t[i >> 2] >> (8 * (i & 3)));
        }
    } else {
        // constant-time compare: diff |= a ^ b over all 16 bytes (:84-87)
        const uint8_t* ep = in + n;
        uint32_t diff = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) diff |= (uint32_t)(ep[i] ^ (uint8_t)(t[i >> 2] >> (8 * (i & 3))));
        p.status[rec] = diff != 0u ? 1u : 0u;
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

hipError_t launch_keying(const KParams& p, hipStream_t s) {
    const uint32_t grid = (p.count + 255u) / 256u;
    hipLaunchKernelGGL(sg_keying_kernel, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_seal(const KParams& p, uint32_t lds, hipStream_t s) {
    hipLaunchKernelGGL(sg_aead_kernel<false>, dim3(p.count), dim3(kThreads), lds, s, p);
    return hipGetLastError();
}

hipError_t launch_open(const KParams& p, uint32_t lds, hipStream_t s) {
    hipLaunchKernelGGL(sg_aead_kernel<true>, dim3(p.count), dim3(kThreads), lds, s, p);
    return hipGetLastError();
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

const char* kernel_config() {
    return "gfx950 sg_aead_kernel v1: 256 threads/record, lane=64B ChaCha block, "
           "wave0 Poly1305 radix-2^26 strided-Horner(r^64)+6-level tree, keying pre-pass";
}

}  // namespace sg
