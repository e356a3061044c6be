// sg_kernels.hip -- gfx950 (CDNA4) size-class kernels for suruga's
// ChaCha20-Poly1305 record AEAD (draft-agl-tls-chacha20poly1305-04 as in
// klutzy/suruga), used for every batch the wave-per-record kernel of
// sg_wpr.hip does not take (mixed sizes, records other than 16 KiB,
// unaligned or offset-table layouts).
//
// Work decomposition (records of one size class per 256-thread workgroup):
//
//   sg_keying_kernel   one lane per record: ChaCha20 block 0 -> Poly1305 key
//                      (r clamped, s; chacha20_poly1305.rs:50,75,32-39,
//                      poly1305.rs:197-203) and the 16 powers of r^k
//                      that combine the MAC lanes.
//   sg_aead_kernel<OPEN, L>   L lanes per record:
//     phase 1, all lanes: lane t owns 64-byte data blocks t, t+L, ...;
//       computes keystream block b+1 in registers (chacha20.rs:53-135),
//       XORs the record bytes (chacha20.rs:143-153), writes the result to HBM
//       and the ciphertext into LDS.
//     phase 2, PL = min(L, 64) lanes: Poly1305 over ad || le64(|ad|) || ct ||
//       le64(|ct|) (chacha20_poly1305.rs:19-42), read from LDS.  The B MAC
//       blocks are preceded by z zero "virtual" blocks (leading zeros do not
//       change a Horner polynomial) so that B + z = PL k; lane t runs the
//       reference's Horner step h = (h + c) * r (poly1305.rs:213-228) over its
//       k contiguous blocks in radix 2^32 with the clamped r; each lane then
//       scales its sum by r^(k (PL-1-t)) (radix 2^26, powers from the keying
//       record) and a DPP reduction adds the PL terms.  The last lane reduces
//       mod 2^130-5, adds s (poly1305.rs:230-312) and seals
//       (chacha20_poly1305.rs:55) or compares in constant time (:84-93) after
//       decrypting unconditionally (:80-82).
//   sg_classify_kernel   buckets a mixed-size batch into per-class lists.
//
// All Poly1305 arithmetic is exact mod p = 2^130 - 5, so the tag equals the
// reference's sequential Horner result bit for bit.
#include "sg_internal.h"
#include "../../include/suruga_gpu.h"  // SG_HEADER_LEN (record-layer framing kernels)

#include <mutex>
#include <vector>
#include "sg_device.h"

#include <stdint.h>
#include <stdlib.h>

#define SG_STR2(x) #x
#define SG_STR(x) SG_STR2(x)


namespace sg {
namespace {

using namespace dev;

// ---- uniform-record variant: the counter-free part of round 1 on the SALU ----
// Within one record only state word 12 (the block counter) differs between
// blocks.  The column quarter-rounds on words (1,5,9,13), (2,6,10,14),
// (3,7,11,15) and the first add of (0,4,8,12) are therefore the same for
// every block; when the record is wave-uniform (key and nonce in SGPRs) they
// are computed once on the scalar unit, which otherwise idles, instead of
// costing ~37 VALU per block (srotl32 / SG_QR_S, sg_device.h).

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

// ---------------------------------------------------------------------------
// Keying pre-pass: one lane per record.
// ---------------------------------------------------------------------------
// The 64 records of a wave are staged in LDS (row stride kKeyRecWords + 1
// words: no bank conflicts) and leave as one contiguous run of 16-byte stores
// (skipping the powers a record's class never reads); one lane writing its own
// record would touch a cache line per store.
constexpr uint32_t kKeyingThreads = 64;

// The wave-per-record bucket of record rec of a mixed batch (0: a size class);
// n is the plaintext length.  The classify and keying kernels agree on it.
__device__ __forceinline__ uint32_t rec_wpr_bucket(const KParams& p, uint32_t rec, uint32_t n) {
    if (!p.wpr_mix) return 0u;
    const uint64_t ia = (uint64_t)(uintptr_t)p.in + (p.in_off ? p.in_off[rec] : p.in_stride * rec);
    const uint64_t oa = (uint64_t)(uintptr_t)p.out + (p.out_off ? p.out_off[rec] : p.out_stride * rec);
    return wpr_bucket_of(n, ia, oa);
}
// ... and for the packed small-record kernel (sg_pack.hip)
__device__ __forceinline__ bool rec_pack(const KParams& p, uint32_t rec, uint32_t n) {
    if (!p.pack_mix) return false;
    const uint64_t ia = (uint64_t)(uintptr_t)p.in + (p.in_off ? p.in_off[rec] : p.in_stride * rec);
    const uint64_t oa = (uint64_t)(uintptr_t)p.out + (p.out_off ? p.out_off[rec] : p.out_stride * rec);
    return pack_ok(n, ia, oa);
}


// Keying pre-pass of the size-class kernels: ChaCha20 block 0 -> Poly1305 key
// (chacha20_poly1305.rs:50,75,32-39; r clamped as poly1305.rs:197-203), and
// with R = r^k (k = MAC blocks per lane, mac_geom) the tables R^0..R^7 and
// R^0, R^8, .., R^56 that scale the MAC lanes' partial sums.
// KeyJobs (sg_internal.h): njobs == 0 keys every record of the batch by
// index; otherwise the records of up to kNumClasses lists (mixed batches key
// only their size-class records here), job i on blocks [blk0[i], blk0[i+1]).
template <bool OPEN>
__global__ __launch_bounds__(64) void sg_keying_kernel(const KParams p, const KeyJobs jobs) {
    constexpr uint32_t kKeyLdsStride = kKeyRecWords + 1;
    __shared__ uint32_t stage[kKeyingThreads * kKeyLdsStride];
    __shared__ uint32_t recs[kKeyingThreads];
    const uint32_t lane = threadIdx.x;
    const uint32_t* list = nullptr;
    uint32_t cnt = p.count, b0 = 0;
#pragma unroll
    for (uint32_t i = 0; i < kNumClasses; ++i)  // (constant indices: the kernarg table stays in SGPRs)
        if (i < jobs.njobs && blockIdx.x >= jobs.blk0[i]) {
            list = jobs.list[i];
            cnt = jobs.count[i];
            b0 = jobs.blk0[i];
        }
    const uint32_t slot0 = (blockIdx.x - b0) * kKeyingThreads;
    const uint32_t slot = slot0 + lane;
    const bool act = slot < cnt;
    const uint32_t rec = act ? (list ? list[slot] : slot) : 0u;
    recs[lane] = rec;
    uint32_t* out = stage + lane * kKeyLdsStride;
    const uint32_t len = act ? record_len(p, rec) : 0u;
    const uint32_t n = OPEN ? (len >= 16u ? len - 16u : 0u) : len;
    out[kKeyRecWords] = 0u;  // nothing to write unless keyed below
    if (act) {
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
        const MacGeom g = mac_geom(adlen, n, mac_lanes(n));
        const F26 r = words_to_f26(r0, r1, r2, r3, 0u);
        // R = r^k by square-and-multiply; then R^0..R^7 and R^0, R^8, .., R^56.
        // mul_add outputs are valid multipliers as they stand (limb 1 may exceed
        // 2^26 by < 2^8), so no extra carry passes are needed here.
        F26 R = r;
        for (int bit = 30 - __builtin_clz(g.k); bit >= 0; --bit) {
            R = fmul(R, R);
            if ((g.k >> bit) & 1u) R = fmul(R, r);
        }
        // only the powers the record's PL MAC lanes read (a prefix of the layout)
        const uint32_t PL = mac_lanes(n);
        store_f26(out + key_hi_off(0u), f26_one());
        F26 x = f26_one();
        const uint32_t nlo = PL < 8u ? PL : 8u;
        for (uint32_t j = 0; j < nlo; ++j) {  // lo[j] = R^j
            store_f26(out + key_lo_off(j), x);
            x = fmul(x, R);
        }
        if (PL > 8u) {
            const F26 R8 = x;
            for (uint32_t i = 1; i < PL / 8u; ++i) {  // hi[i] = R^(8 i)
                store_f26(out + key_hi_off(i), x);
                if (i + 1u < PL / 8u) x = fmul(x, R8);
            }
        }
        out[kKeyRecWords] = key_used_words(PL);  // the stage row's pad word
    }
    __syncthreads();
    // coalesced flush: 16-byte stores of consecutive words of a record
    // (records by index are contiguous in the workspace; listed ones are not)
    const uint32_t nrec = cnt - slot0 < kKeyingThreads ? cnt - slot0 : kKeyingThreads;
    const uint32_t nvec = nrec * (kKeyRecWords / 4u);
    for (uint32_t v = lane; v < nvec; v += kKeyingThreads) {
        const uint32_t w = 4u * v;
        const uint32_t rr = w / kKeyRecWords, c = w - rr * kKeyRecWords;
        const uint32_t* src = stage + rr * kKeyLdsStride + c;
        if (c < stage[rr * kKeyLdsStride + kKeyRecWords])  // unread powers are not written
            *reinterpret_cast<u32x4*>(p.ws + (uint64_t)recs[rr] * kKeyRecWords + c) = u32x4{src[0], src[1], src[2], src[3]};
    }
}

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
        if constexpr (L >= 64u) pre = chacha_pre(rk.k, rk.n14, rk.n15);
        for (uint32_t b = t; b < nblocks; b += L) {
            const uint32_t off = b << 6;
            if (vec_ok && off + 64u <= n) {
                const u32x4 d0 = ld16(in + off), d1 = ld16(in + off + 16);
                const u32x4 d2 = ld16(in + off + 32), d3 = ld16(in + off + 48);
                uint32_t ks[16];
                // data uses blocks 1.. (chacha20_poly1305.rs:52)
                if constexpr (L >= 64u) chacha_block_pre(ks, pre, rk.k, b + 1u, rk.n14, rk.n15);
                else chacha_block(ks, rk.k, b + 1u, rk.n14, rk.n15);
                const u32x4 r0 = d0 ^ u32x4{ks[0], ks[1], ks[2], ks[3]};
                const u32x4 r1 = d1 ^ u32x4{ks[4], ks[5], ks[6], ks[7]};
                const u32x4 r2 = d2 ^ u32x4{ks[8], ks[9], ks[10], ks[11]};
                const u32x4 r3 = d3 ^ u32x4{ks[12], ks[13], ks[14], ks[15]};
                st16(out + off, r0);
                st16(out + off + 16, r1);
                st16(out + off + 32, r2);
                st16(out + off + 48, r3);
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
                if constexpr (L >= 64u) chacha_block_pre(ks, pre, rk.k, b + 1u, rk.n14, rk.n15);
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
    if (!work || t >= PL) return;

    // ---- phase 2: Poly1305 on PL lanes -----------------------------------------
    const MacGeom g = mac_geom(adlen, n, PL);
    const uint32_t* kr = p.ws + (uint64_t)rec * kKeyRecWords;
    uint32_t r0 = kr[kR32Off + 0], r1 = kr[kR32Off + 1], r2 = kr[kR32Off + 2], r3 = kr[kR32Off + 3];
    if constexpr (PL == 64u) {  // one record per wave: keep the key in SGPRs
        r0 = uniform(r0); r1 = uniform(r1); r2 = uniform(r2); r3 = uniform(r3);
    }
    const uint32_t s1 = r1 + (r1 >> 2), s2 = r2 + (r2 >> 2), s3 = r3 + (r3 >> 2);
    // open: the finishing lane fetches the received tag after the keying record's r
    // words (loads retire in order: waiting for r must not wait for the tag), so
    // that its latency hides behind the Horner loop
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
        const F26 plo = load_f26(kr + key_lo_off(e & 7u));
        const F26 phi = load_f26(kr + key_hi_off(e >> 3));
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
    // XCD-aware order: workgroup b runs on XCD b % 8, and each XCD takes one
    // contiguous run of the list, so neighbouring records (which share cache
    // lines: records are packed byte-tight) are fetched by the same L2.
    const uint32_t nb = gridDim.x, x = blockIdx.x & 7u, q = nb >> 3, r = nb & 7u;
    const uint32_t wg = x * q + (x < r ? x : r) + (blockIdx.x >> 3);
    for (uint32_t base = wg * RPW; base < cnt; base += stride) {
        const uint32_t slot = base + g;
        const bool active = slot < cnt;
        uint32_t rec = active ? list[slot] : 0u;
        if constexpr (L >= 64u) rec = __builtin_amdgcn_readfirstlane(rec);
        aead_record<OPEN, L>(p, rec, active, lds + g * p.lds_rec_bytes, t);
        if constexpr (!PERSIST) break;
        __syncthreads();  // LDS is reused by the next iteration
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
                                                           uint32_t* __restrict__ counts, const uint32_t max_n) {
    // counts: the kNumLists populations, then the over-long count
    __shared__ uint32_t wave_cnt[kNumLists][kClassifyThreads / 64];
    __shared__ uint32_t wg_base[kNumLists];
    const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
    const uint32_t rec0 = blockIdx.x * (kClassifyThreads * kClassifyPerThread);
    uint32_t cls[kClassifyPerThread];
    uint32_t mine[kNumLists] = {};  // this wave's records per list
#pragma unroll
    for (uint32_t i = 0; i < kClassifyPerThread; ++i) {
        const uint32_t rec = rec0 + i * kClassifyThreads + threadIdx.x;
        cls[i] = kNumLists;
        if (rec < p.count) {
            const uint32_t len = record_len(p, rec);
            const uint32_t n = OPEN ? (len >= 16u ? len - 16u : 0u) : len;
            if (n <= max_n) {
                const uint32_t J = rec_wpr_bucket(p, rec, n);
                cls[i] = J ? kNumClasses + J - kWprMinJ : rec_pack(p, rec, n) ? kPackList : size_class(n);
            } else {  // longer than the batch's max_len: no class (its LDS slot would overflow), flagged
                atomicAdd(&counts[kNumLists], 1u);
                if constexpr (OPEN) p.status[rec] = 3u;
            }
        }
#pragma unroll
        for (uint32_t c = 0; c < kNumLists; ++c) mine[c] += (uint32_t)__popcll(__ballot(cls[i] == c));
    }
    if (lane == 0)
        for (uint32_t c = 0; c < kNumLists; ++c) wave_cnt[c][wave] = mine[c];
    __syncthreads();
    if (threadIdx.x < kNumLists) {
        uint32_t tot = 0;
        for (uint32_t w = 0; w < kClassifyThreads / 64; ++w) {
            const uint32_t x = wave_cnt[threadIdx.x][w];
            wave_cnt[threadIdx.x][w] = tot;  // exclusive prefix over waves
            tot += x;
        }
        wg_base[threadIdx.x] = tot ? atomicAdd(&counts[threadIdx.x], tot) : 0u;
    }
    __syncthreads();
    uint32_t off[kNumLists];
#pragma unroll
    for (uint32_t c = 0; c < kNumLists; ++c) off[c] = wg_base[c] + wave_cnt[c][wave];
#pragma unroll
    for (uint32_t i = 0; i < kClassifyPerThread; ++i) {
        const uint32_t rec = rec0 + i * kClassifyThreads + threadIdx.x;
#pragma unroll
        for (uint32_t c = 0; c < kNumLists; ++c) {
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

// ---------------------------------------------------------------------------
// Record-layer framing on the device (sg_record.cpp, registered caller
// buffers): the wire image of a chunk is built / taken apart in HBM so that
// the host link moves one contiguous run each way (a strided host-side copy
// at the wire's 16,405-byte pitch measured ~1.3 s per GiB).  Wire record r
// sits at r * pitch: the 5-byte header (tls.rs:126-130) and its fragment.
// One thread per 4-byte word of the destination; source words are read
// aligned and funnel-shifted (v_alignbyte) into place.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3u));
}

// dst[0, image) <- headers and fragments; fragment r = src + r * src_stride,
// frag bytes (last: last_frag); hdr = type | major << 8 | minor << 16.
// rdiv: ceil(2^40 / pitch) (r = b * rdiv >> 40 is exact for b < 2^40 / pitch;
// launch_frame caps the image at 2^24 bytes, a chunk is ~4.2 MB).
__global__ __launch_bounds__(256) void sg_frame_kernel(const uint8_t* __restrict__ src, uint32_t src_stride,
                                                       uint8_t* __restrict__ dst, uint32_t pitch, uint64_t rdiv,
                                                       uint32_t count, uint32_t frag, uint32_t last_frag,
                                                       uint32_t hdr) {
    const uint32_t image = (count - 1u) * pitch + SG_HEADER_LEN + last_frag;
    const uint32_t nw = (image + 3u) >> 2;
    for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < nw; w += gridDim.x * 256u) {
        const uint32_t b0 = 4u * w;
        const uint32_t r = (uint32_t)(((uint64_t)b0 * rdiv) >> 40);
        const uint32_t o = b0 - r * pitch;  // offset in record r's wire slot
        const uint32_t fl = r + 1u == count ? last_frag : frag;
        if (o >= SG_HEADER_LEN && o + 4u <= SG_HEADER_LEN + fl) {  // inside one fragment
            reinterpret_cast<uint32_t*>(dst)[w] = ld_u32_unaligned(src + (uint64_t)r * src_stride + (o - SG_HEADER_LEN));
            continue;
        }
        uint32_t v = 0u;
        for (uint32_t k = 0; k < 4u; ++k) {  // header bytes and record boundaries
            const uint32_t b = b0 + k;
            if (b >= image) break;
            uint32_t rr = r, oo = o + k;
            if (oo >= pitch) {
                rr += 1u;
                oo -= pitch;
            }
            const uint32_t f = rr + 1u == count ? last_frag : frag;
            uint32_t byte;
            if (oo < SG_HEADER_LEN) {
                const uint32_t n = f;  // be16 fragment length
                byte = oo < 3u ? (hdr >> (8u * oo)) & 0xffu : (oo == 3u ? (n >> 8) & 0xffu : n & 0xffu);
            } else {
                byte = src[(uint64_t)rr * src_stride + (oo - SG_HEADER_LEN)];
            }
            v |= byte << (8u * k);
        }
        if (b0 + 4u <= image) {
            reinterpret_cast<uint32_t*>(dst)[w] = v;
        } else {
            for (uint32_t k = 0; b0 + k < image; ++k) dst[b0 + k] = (uint8_t)(v >> (8u * k));
        }
    }
}

// dst + r * dst_stride <- the frag bytes of wire record r (src + r * pitch + 5),
// count records of one fragment length.  The image is count * pitch bytes; a
// word whose aligned loads would reach past it is read byte by byte, so that
// no load leaves the image (src may be the caller's registered host buffer,
// read over the host link, whose next page need not be mapped).
__global__ __launch_bounds__(256) void sg_unframe_kernel(const uint8_t* __restrict__ src, uint32_t pitch,
                                                         uint8_t* __restrict__ dst, uint32_t dst_stride,
                                                         uint32_t count, uint32_t frag) {
    const uint32_t wpr = (frag + 3u) >> 2;  // destination words per record
    const uint32_t total = wpr * count;
    const uint64_t image = (uint64_t)count * pitch;
    for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < total; g += gridDim.x * 256u) {
        const uint32_t r = g / wpr, w = g - r * wpr;
        const uint64_t off = (uint64_t)r * pitch + SG_HEADER_LEN + 4u * w;
        const uint64_t a0 = ((uintptr_t)src + off) & 3u;  // the aligned loads cover [off - a0, off - a0 + 8)
        uint32_t v;
        if (off - a0 + 8u <= image && off >= a0) {
            v = ld_u32_unaligned(src + off);
        } else {
            v = 0u;
            for (uint32_t k = 0; k < 4u && off + k < image; ++k) v |= (uint32_t)src[off + k] << (8u * k);
        }
        uint8_t* d = dst + (uint64_t)r * dst_stride + 4u * w;
        if (4u * w + 4u <= frag) {
            *reinterpret_cast<uint32_t*>(d) = v;
        } else {
            for (uint32_t k = 0; 4u * w + k < frag; ++k) d[k] = (uint8_t)(v >> (8u * k));
        }
    }
}

// dst[0, n) <- src[0, n): the zero-copy read's plaintext from HBM into the
// caller's registered `out` over the host link (sg_record.cpp).  src is 4-byte
// aligned; dst may not be.  Every thread writes one 4-byte aligned word of dst
// (a funnel shift of two source words: the lanes' stores cover whole 256-byte
// segments) and the partial words at either end byte by byte, so that no store
// leaves [dst, dst + n), and no load leaves [src, src + n + 3] rounded to words.
__global__ __launch_bounds__(256) void sg_copy_out_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         uint64_t n) {
    const uint32_t a = (uint32_t)((4u - ((uintptr_t)dst & 3u)) & 3u);  // bytes before dst's first aligned word
    const uint64_t nw = n > a ? (n - a) >> 2 : 0;                       // whole aligned words of dst
    const uint64_t tid = blockIdx.x * 256ull + threadIdx.x, nth = (uint64_t)gridDim.x * 256ull;
    if (tid < a && tid < n) dst[tid] = src[tid];
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + a);
    for (uint64_t w = tid; w < nw; w += nth) {
        const uint64_t b = a + 4u * w;  // source byte of the word's first byte
        const uint64_t q = b >> 2;
        const uint32_t lo = s32[q];
        const uint32_t hi = (b & 3u) ? s32[q + 1] : 0u;
        d32[w] = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(b & 3u));
    }
    const uint64_t t0 = a + 4u * nw;  // the byte tail
    if (tid < 4u && t0 + tid < n) dst[t0 + tid] = src[t0 + tid];
}

// Failed opens release no plaintext (chacha20_poly1305.rs:80-93 decrypts
// unconditionally but returns only Err on a tag mismatch): every record whose
// status is 1 (wrong mac) gets its output range zeroed after the open
// kernels, by the wave that finds it.  Records that failed are rare, so the
// launch costs one status byte per record when none did.  Status 2 (too
// short) has no output and status 3 (longer than max_len) was never written.
// Each wave scans 64 statuses and zeroes the output of every failed record in
// its ballot with the whole wave: byte stores up to the first 16-byte boundary,
// then 16-byte stores (1 KiB per wave instruction), then the byte tail
// (one byte per lane made a batch of failed 16 KiB records cost more
// than the AEAD launch itself).
__global__ __launch_bounds__(256) void sg_scrub_kernel(const KParams p) {
    const uint32_t base = blockIdx.x * 256u + (threadIdx.x & ~63u), lane = threadIdx.x & 63u;
    const uint32_t i = base + lane;
    uint64_t m = __ballot(i < p.count && p.status[i] == 1u);
    while (m) {
        const uint32_t rec = base + (uint32_t)__builtin_ctzll(m);
        m &= m - 1ull;
        const uint32_t len = record_len(p, rec);
        const uint32_t n = len >= 16u ? len - 16u : 0u;
        uint8_t* o = p.out + (p.out_off ? p.out_off[rec] : p.out_stride * rec);
        const uint32_t head = (uint32_t)((16u - ((uintptr_t)o & 15u)) & 15u);
        const uint32_t h = head < n ? head : n;
        if (lane < h) o[lane] = 0u;
        const uint32_t nv = (n - h) >> 4;  // whole 16-byte units after the head
        u32x4* ov = reinterpret_cast<u32x4*>(o + h);
        for (uint32_t v = lane; v < nv; v += 64u) ov[v] = u32x4{0u, 0u, 0u, 0u};
        const uint32_t t0 = h + 16u * nv;
        if (t0 + lane < n) o[t0 + lane] = 0u;
    }
}

}  // namespace

hipError_t launch_scrub(const KParams& p, hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    hipLaunchKernelGGL(sg_scrub_kernel, dim3((p.count + 255u) / 256u), dim3(256), 0, s, p);
    return hipGetLastError();
}

static hipError_t launch_keying(const KParams& p, bool open, const KeyJobs& jobs, uint32_t grid, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    if (open)
        hipLaunchKernelGGL((sg_keying_kernel<true>), dim3(grid), dim3(kKeyingThreads), 0, s, p, jobs);
    else
        hipLaunchKernelGGL((sg_keying_kernel<false>), dim3(grid), dim3(kKeyingThreads), 0, s, p, jobs);
    return hipGetLastError();
}

// every record of the batch, by index
static hipError_t launch_keying_all(const KParams& p, bool open, hipStream_t s) {
    KeyJobs jobs = {};
    return launch_keying(p, open, jobs, (p.count + kKeyingThreads - 1u) / kKeyingThreads, s);
}

static hipError_t mark(hipEvent_t ev, hipStream_t s) { return ev ? hipEventRecord(ev, s) : hipSuccess; }

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

// Pinned host buffers for the population readback of mixed batches, shared by
// every calling thread (a thread_local buffer per caller leaked one pinned
// allocation per thread that ever ran a mixed batch).  The pool holds at most
// as many buffers as calls were ever in flight at once; they live as long as
// the process.
std::mutex g_pop_mu;
std::vector<std::pair<uint32_t*, hipEvent_t>> g_pop_free;
struct PinnedPop {
    uint32_t* p = nullptr;
    hipEvent_t ev = nullptr;          // recorded after the readback copy
    hipStream_t copy_s = nullptr;     // set once a copy into p has been enqueued on it
    bool recorded = false;            // ev was recorded after that copy
    hipError_t acquire(size_t bytes) {
        {
            std::lock_guard<std::mutex> lk(g_pop_mu);
            if (!g_pop_free.empty()) {
                p = g_pop_free.back().first;
                ev = g_pop_free.back().second;
                g_pop_free.pop_back();
                return hipSuccess;
            }
        }
        hipError_t e = hipHostMalloc((void**)&p, bytes < 256u ? 256u : bytes, hipHostMallocDefault);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) {
            (void)hipHostFree(p);
            p = nullptr;
            ev = nullptr;
        }
        return e;
    }
    void done() { copy_s = nullptr; }  // the copy has been waited for
    ~PinnedPop() {
        if (!p) return;
        // An error return between the copy and the wait: the buffer goes back to
        // the pool only once the copy into it is known to be done -- by its event
        // when that was recorded, else by the copy's stream.  If neither wait
        // succeeds the buffer is dropped (leaked) rather than handed to another
        // call while a DMA may still write it.
        if (copy_s) {
            const hipError_t w = recorded ? hipEventSynchronize(ev) : hipStreamSynchronize(copy_s);
            if (w != hipSuccess) return;
        }
        std::lock_guard<std::mutex> lk(g_pop_mu);
        g_pop_free.emplace_back(p, ev);
    }
};

// Side streams of mixed batches (per device and priority, pooled like the
// pinned population buffers, created non-blocking with the priority of the
// batch's stream; they live as long as the process).  A pooled stream is
// handed out again only when its last join event reports done, i.e. every
// kernel an earlier batch enqueued on it has finished: the SideStream goes
// back to the pool when launch_aead_t returns, while its keying and bucket
// kernels may still be queued, and a concurrent batch on another caller
// stream must not queue behind them (calls on different streams are
// independent, suruga_gpu.h).  A busy pooled stream is skipped and a new one
// created, up to kSideCap per device and priority (two concurrent mixed
// batches' worth): beyond that the batch runs that part on its own stream
// (the process has four hardware queues, GPU_MAX_HW_QUEUES, and more streams
// share them and serialise anyway; advisor r5).
constexpr int kSideCap = 4;
std::mutex g_side_mu;
struct SidePooled {
    int dev, prio;
    hipStream_t s;
    hipEvent_t done;
};
std::vector<SidePooled> g_side_free;
std::vector<std::pair<std::pair<int, int>, int>> g_side_made;  // (device, priority) -> streams created
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    int dev = -1, prio = 0;
    bool borrowed = false;  // s is the caller's stream (the cap was reached): not pooled, no join
    hipError_t acquire(hipStream_t caller) {
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if ((e = hipStreamGetPriority(caller, &prio)) != hipSuccess) return e;
        {
            std::lock_guard<std::mutex> lk(g_side_mu);
            for (size_t i = 0; i < g_side_free.size(); ++i) {
                const SidePooled& c = g_side_free[i];
                if (c.dev != dev || c.prio != prio || hipEventQuery(c.done) != hipSuccess) continue;
                s = c.s;
                done = c.done;
                g_side_free.erase(g_side_free.begin() + (long)i);
                return hipSuccess;
            }
            int* made = nullptr;
            for (auto& m : g_side_made)
                if (m.first.first == dev && m.first.second == prio) made = &m.second;
            if (!made) {
                g_side_made.push_back({{dev, prio}, 0});
                made = &g_side_made.back().second;
            }
            if (*made >= kSideCap) {
                s = caller;
                borrowed = true;
                return hipSuccess;
            }
            ++*made;
        }
        if ((e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio)) != hipSuccess) {
            s = nullptr;
            return e;
        }
        if ((e = hipEventCreateWithFlags(&done, hipEventDisableTiming)) != hipSuccess) {
            (void)hipStreamDestroy(s);
            s = nullptr;
        }
        return e;
    }
    // the batch's stream s waits for everything enqueued here so far
    hipError_t join_into(hipStream_t t) const {
        if (borrowed) return hipSuccess;
        hipError_t e = hipEventRecord(done, s);
        return e != hipSuccess ? e : hipStreamWaitEvent(t, done, 0);
    }
    ~SideStream() {
        if (!s || borrowed) return;
        std::lock_guard<std::mutex> lk(g_side_mu);
        g_side_free.push_back({dev, prio, s, done});
    }
};
// Every side stream a batch used is joined into its stream on every way out of
// launch_aead_t (the workspace is released on that stream).
struct SideJoin {
    hipStream_t s;
    const SideStream* side[2];
    bool used[2];
    ~SideJoin() {
        for (int i = 0; i < 2; ++i)
            if (used[i]) (void)side[i]->join_into(s);
    }
};

template <bool OPEN>
hipError_t launch_aead_t(const KParams& p, uint32_t max_n, bool uniform, hipStream_t s, uint32_t* over,
                         hipEvent_t ev_keyed, hipEvent_t ev_start) {
    *over = 0;
    hipError_t e;
    if (uniform) {  // every record in one class: keying, then a direct launch
        if ((e = launch_keying_all(p, OPEN, s)) != hipSuccess || (e = mark(ev_keyed, s)) != hipSuccess ||
            (e = mark(ev_start, s)) != hipSuccess)
            return e;
        KParams q = p;
        const uint32_t c = size_class(max_n);
        q.lds_rec_bytes = lds_rec_bytes(c, q.ad_len, max_n);
        return launch_class<OPEN>(c, q, nullptr, nullptr, 0, s);
    }
    uint32_t* const tail = ws_tail(p.ws, p.count);
    uint32_t* const lists = p.ws + (uint64_t)p.count * kWsLists;
    // populations, over-long count and the group / run counters (the keying
    // kernel resets the bucket ones again): one dword fill
    if ((e = hipMemsetD32Async((hipDeviceptr_t)tail, 0, kWsTailWords, s)) != hipSuccess) return e;
    const uint32_t per_wg = kClassifyThreads * kClassifyPerThread;
    hipLaunchKernelGGL(sg_classify_kernel<OPEN>, dim3((p.count + per_wg - 1u) / per_wg), dim3(kClassifyThreads), 0, s,
                       p, lists, tail, max_n);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // Read the list populations back (one host wait per mixed batch) so that
    // the keying kernels run over exactly the listed records and every list
    // on an exact grid; under stream capture the host cannot wait, so every
    // record is keyed and the classes run on persistent grids instead (and the
    // caller leaves p.wpr_mix and p.pack_mix off: the wave-per-record buckets
    // need their populations).
    // (into a pinned buffer from a process-wide pool: a DMA, no staging copy;
    // the buffer goes back to the pool when this call is done with it)
    uint32_t pop[kNumLists + 1];
    hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
    if ((e = hipStreamIsCapturing(s, &cap_status)) != hipSuccess) return e;
    const bool exact = cap_status == hipStreamCaptureStatusNone;
    // Mixed batches run on up to three streams (round 4): the packed launch
    // (its population stays on the device) goes ahead of the host's wait for
    // the readback, so the GPU does not idle while the host waits and
    // launches; the keying launches run on a side stream ks beside the packed
    // launch's tail; the J = 4 and J = 3 buckets follow the keying on ks and on
    // a second side stream, and J = 2 and the size classes on s, so that each
    // persistent bucket grid takes the CU slots that the launches before it
    // free and their tails overlap instead of adding up.
    SideStream side[2];
    SideJoin join{s, {&side[0], &side[1]}, {false, false}};
    hipStream_t ks = s;
    if (exact) {
        PinnedPop pin;
        if ((e = pin.acquire(sizeof pop)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(pin.p, tail, sizeof pop, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        pin.copy_s = s;
        if ((e = hipEventRecord(pin.ev, s)) != hipSuccess) return e;
        pin.recorded = true;
        // the batch's record window starts with the packed launch
        if ((e = mark(ev_keyed, s)) != hipSuccess || (e = mark(ev_start, s)) != hipSuccess) return e;
        ev_keyed = ev_start = nullptr;
        if (p.pack_mix && (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, tail + kPackList,
                                           tail + kTailPackCtr, s)) != hipSuccess)
            return e;
        if ((e = hipEventSynchronize(pin.ev)) != hipSuccess) return e;
        pin.done();
        for (uint32_t i = 0; i <= kNumLists; ++i) pop[i] = pin.p[i];
        *over = pop[kTailOver];
        uint32_t nbuckets = 0;
        for (uint32_t b = 0; b < kWprBuckets; ++b) nbuckets += pop[kNumClasses + b];
        if (((p.pack_mix && pop[kPackList] != 0u) || (p.wpr_mix && nbuckets != 0u)) && side[0].acquire(s) == hipSuccess) {
            ks = side[0].s;
            join.used[0] = true;
            if ((e = hipStreamWaitEvent(ks, pin.ev, 0)) != hipSuccess) return e;  // after classify
        }
        // size-class keying over the class lists only
        KeyJobs jobs = {};
        uint32_t grid = 0;
        for (uint32_t c = 0; c < kNumClasses; ++c) {
            if (pop[c] == 0) continue;
            jobs.list[jobs.njobs] = lists + (uint64_t)c * p.count;
            jobs.count[jobs.njobs] = pop[c];
            jobs.blk0[jobs.njobs] = grid;
            grid += (pop[c] + kKeyingThreads - 1u) / kKeyingThreads;
            ++jobs.njobs;
        }
        if ((e = launch_keying(p, OPEN, jobs, grid, ks)) != hipSuccess) return e;
    } else if ((e = launch_keying_all(p, OPEN, s)) != hipSuccess) {
        return e;
    }
    // wave-per-record buckets (J = 2..4 chunks): their keying records and
    // descriptors are packed by slot in bucket order
    WprList wl[kWprBuckets] = {};
    if (p.wpr_mix && exact) {
        uint64_t base = 0;
        for (uint32_t b = 0; b < kWprBuckets; ++b) {
            const uint32_t nb = pop[kNumClasses + b];
            wl[b].list = lists + (uint64_t)(kNumClasses + b) * p.count;
            wl[b].count = nb;
            wl[b].tab = p.ws + (uint64_t)p.count * kWsWprTab + base * kWprRecWords;
            wl[b].desc = p.ws + (uint64_t)p.count * kWsWprDesc + base * kWprDescWords;
            wl[b].ctr = tail + kTailCtr + b;
            base += nb;
        }
        if ((e = launch_wpr_keying_lists(p, OPEN, wl, ks)) != hipSuccess) return e;
    }
    hipStream_t js[kWprBuckets] = {s, ks, ks};  // bucket b (J = 2 + b)
    if (ks != s) {  // s (J = 2, classes) and the second side stream (J = 3) wait for the keying
        if ((e = side[0].join_into(s)) != hipSuccess) return e;
        if (p.wpr_mix && side[1].acquire(s) == hipSuccess) {
            join.used[1] = true;
            if ((e = hipStreamWaitEvent(side[1].s, side[0].done, 0)) != hipSuccess) return e;
            js[1] = side[1].s;
        }
    }
    if ((e = mark(ev_keyed, s)) != hipSuccess || (e = mark(ev_start, s)) != hipSuccess) return e;
    if (p.wpr_mix && exact) {  // most chunks first
        for (int b = (int)kWprBuckets - 1; b >= 0; --b)
            if ((e = launch_wpr_list(p, OPEN, kWprMinJ + (uint32_t)b, wl[b], js[b])) != hipSuccess) return e;
    }
    // one launch per populated class, largest records first
    KParams q = p;
    for (int c = (int)size_class(max_n); c >= 0; --c) {
        const uint32_t cap = max_n < class_max((uint32_t)c) ? max_n : class_max((uint32_t)c);
        q.lds_rec_bytes = lds_rec_bytes((uint32_t)c, q.ad_len, cap);
        if ((e = launch_class<OPEN>((uint32_t)c, q, lists + (uint64_t)c * p.count, tail + c,
                                    exact ? pop[c] : 0xffffffffu, s)) != hipSuccess)
            return e;
    }
    return hipSuccess;  // (join: s waits for the side streams)
}

hipError_t launch_aead(const KParams& p, bool open, uint32_t max_n, bool uniform, hipStream_t s, uint32_t* over,
                       hipEvent_t ev_keyed, hipEvent_t ev_start) {
    return open ? launch_aead_t<true>(p, max_n, uniform, s, over, ev_keyed, ev_start)
                : launch_aead_t<false>(p, max_n, uniform, s, over, ev_keyed, ev_start);
}

hipError_t launch_frame(const uint8_t* src, uint32_t src_stride, uint8_t* dst, uint32_t pitch, uint32_t count,
                        uint32_t frag, uint32_t last_frag, uint32_t hdr, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint32_t image = (count - 1u) * pitch + SG_HEADER_LEN + last_frag;
    if (image >= (1u << 24) || (src_stride & 3u) || ((uintptr_t)dst & 3u)) return hipErrorInvalidValue;
    const uint64_t rdiv = ((1ull << 40) + pitch - 1u) / pitch;
    uint32_t grid = ((image + 3u) / 4u + 255u) / 256u;
    grid = grid < 4096u ? grid : 4096u;
    hipLaunchKernelGGL(sg_frame_kernel, dim3(grid), dim3(256), 0, s, src, src_stride, dst, pitch, rdiv, count, frag,
                       last_frag, hdr);
    return hipGetLastError();
}

hipError_t launch_copy_out(const uint8_t* src, uint8_t* dst, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if ((uintptr_t)src & 3u) return hipErrorInvalidValue;
    uint64_t grid = (n / 4u + 255u) / 256u;
    grid = grid < 4096u ? (grid ? grid : 1u) : 4096u;
    hipLaunchKernelGGL(sg_copy_out_kernel, dim3((uint32_t)grid), dim3(256), 0, s, src, dst, n);
    return hipGetLastError();
}

hipError_t launch_unframe(const uint8_t* src, uint32_t pitch, uint8_t* dst, uint32_t dst_stride, uint32_t count,
                          uint32_t frag, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if ((dst_stride & 3u) || ((uintptr_t)dst & 3u)) return hipErrorInvalidValue;
    uint32_t grid = (((frag + 3u) / 4u) * count + 255u) / 256u;
    grid = grid < 4096u ? grid : 4096u;
    hipLaunchKernelGGL(sg_unframe_kernel, dim3(grid), dim3(256), 0, s, src, pitch, dst, dst_stride, count, frag);
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

const char* class_kernel_config() {
    return "sg_aead_kernel v9 8 size classes (2..256 lanes per record, one 64-B block per lane, device bucketing, exact class grids), "
           "lane=64B ChaCha block (counter-free round-1 QRs on SALU for wave-uniform records), Poly1305 contiguous-chunk "
           "Horner radix-2^32 (clamped r, unaligned 16-B LDS block loads, folded pad bit) on min(L,64) lanes + per-lane "
           "r^(k(PL-1-t)) scale + DPP sum, tag finalised on the SALU for one-record waves, keying pre-pass";
}

}  // namespace sg
