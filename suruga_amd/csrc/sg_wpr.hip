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
// 2^23; the record's first MFMA starts from a zero accumulator and the
// assembly adds a seed of 2^24 per entry (v_mad_i64_i32 on the signed
// entries), so every 64-bit word is positive.  At the end each lane assembles
// its 16 entries exactly, X = sum_r (D[c_r][q] + 2^24) 2^(8 c_r), reduces it
// mod 2^130 - 5, multiplies by
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
// after the lines (offsets from the line area): 16 zero bytes read past the
// last line, the next record's descriptor (bucket launches), the received tag
constexpr uint32_t kWprDescOff = kWprLines * kWprLineBytes + 16;
constexpr uint32_t kWprRxOff = kWprDescOff + 48;
constexpr uint32_t kWprWaveLds = 2 * kWprChunk + kWprRxOff + 16;  // 10192
// eight waves and the workgroup's next-group slot: two workgroups per CU
constexpr uint32_t kWprWgLds = kWprWaves * kWprWaveLds + 16;
static_assert(2 * kWprWgLds <= 160 * 1024, "two workgroups per CU");
static_assert(kWprDescWords * 4 <= 48, "descriptor slot");
constexpr uint32_t kWprKeyThreads = 64;

// Geometry of the MAC stream ad || le64(|ad|) || ct || le64(n), n a multiple
// of 16 (C1: n = 2^14).  A record of n < 2^14 bytes runs right-aligned in the
// 2^14-byte frame of the kernel (virtual offset 2^14 - n): shifting the
// ciphertext by a multiple of 16 shifts its MAC block indices and the block
// count B alike, so every ciphertext byte keeps its weight r^(B - b) 2^(8 k)
// and the MFMA part of the MAC is the same for every n; only the constant term
// (AD, length and pad blocks, bias) depends on n.
struct WprGeom {
    uint32_t o, sigma, beta, B, rem, delta, m;
};
__device__ __forceinline__ WprGeom wpr_geom(uint32_t adlen, uint32_t n) {
    WprGeom g;
    g.o = adlen + 8u;
    g.sigma = g.o & 15u;
    g.beta = g.o >> 4;
    const uint32_t L = adlen + 16u + n;
    g.B = (L + 15u) >> 4;
    g.rem = L - 16u * (g.B - 1u);
    g.m = n >> 4;                        // 16-byte ciphertext chunks
    g.delta = g.B - g.beta - 1u - g.m;  // 0 or 1
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
// record (sg_internal.h, kW*) stored unit by unit from registers (grouped layout below).
// LIST: lane = slot of a bucket list (record wl.list[slot], any n of the
// bucket), which also writes the slot's descriptor; otherwise slot = record
// and n = 2^14.
// ---------------------------------------------------------------------------
// Table layout in HBM (round 3): the records of eight consecutive slots (a
// record kernel's group) interleaved by 16-byte unit, unit u of slot 8 g + w
// at tab + 1280 g + 4 (u rows + w) words (rows = 8, or count mod 8 in the last
// group).  Each lane stores its own record unit by unit straight from
// registers (non-temporal: the table does not sit dirty in the caches while
// the record kernel streams) and every store instruction still writes whole
// 128-byte lines (a group's row of one unit), so the keying kernel needs no
// LDS staging and runs at the occupancy its registers allow; the record
// kernel's 40 unit reads per record touch lines that the other seven waves of
// its group read at the same time (the same 640 bytes per record from HBM).
__device__ __forceinline__ uint32_t* wpr_tab_unit(const WprList& wl, uint32_t slot, uint32_t u) {
    const uint32_t g = slot >> 3, w = slot & 7u;
    const uint32_t rows = g < (wl.count >> 3) ? 8u : (wl.count & 7u);
    return wl.tab + (uint64_t)g * (8u * kWprRecWords) + 4u * (u * rows + w);
}
// units [U0, U1) of a lane's record (rec: the record's 160 words, registers)
template <uint32_t U0, uint32_t U1>
__device__ __forceinline__ void wpr_store_units(const WprList& wl, uint32_t slot, bool act, const uint32_t* rec) {
    if (!act) return;
#pragma unroll
    for (uint32_t u = U0; u < U1; ++u) {
        const u32x4 val = {rec[4u * u], rec[4u * u + 1u], rec[4u * u + 2u], rec[4u * u + 3u]};
        __builtin_nontemporal_store(val, reinterpret_cast<u32x4*>(wpr_tab_unit(wl, slot, u)));
    }
}

// One launch keys every bucket: job b on blocks [blk0[b], blk0[b + 1]).
struct WprKeyJobs {
    WprList b[kWprBuckets];
    uint32_t blk0[kWprBuckets];
    uint32_t njobs;
};

// (compiled for two waves per SIMD: four and more spill to scratch)
template <bool OPEN, bool LIST>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void sg_wpr_keying_kernel(
    const KParams p, const WprKeyJobs jobs) {
    const uint32_t lane = threadIdx.x;
    WprList wl = jobs.b[0];
    uint32_t b0 = 0;
#pragma unroll
    for (uint32_t i = 1; i < kWprBuckets; ++i)  // (constant indices: the kernarg table stays in SGPRs)
        if (i < jobs.njobs && blockIdx.x >= jobs.blk0[i]) {
            wl = jobs.b[i];
            b0 = jobs.blk0[i];
        }
    const uint32_t slot0 = (blockIdx.x - b0) * kWprKeyThreads;
    const uint32_t slot = slot0 + lane;
    uint32_t rbuf[kWprRecWords];  // the lane's record (registers once unrolled)
#pragma unroll
    for (uint32_t i = 0; i < kWprRecWords; ++i) rbuf[i] = 0u;
    uint32_t* st = rbuf + 80;  // the second half first (offsets below are half-relative)
    const uint32_t adlen = p.tls ? 13u : p.ad_len;
    if (blockIdx.x == b0 && lane == 0u) *wl.ctr = 0u;  // the record kernel's group counter

    const bool act = slot < wl.count;
    const uint32_t rec = LIST ? (act ? wl.list[slot] : 0u) : slot;
    uint32_t n = kWprN;
    if constexpr (LIST) n = act ? p.len[rec] - (OPEN ? 16u : 0u) : kWprN;
    const WprGeom G = wpr_geom(adlen, n);

    F26 r = f26_zero();
    uint32_t s[4] = {0u, 0u, 0u, 0u};
    RecKey rk = {};
    if (act) {
        rk = record_key(p, rec);
        uint32_t ks[16];
        chacha_block(ks, rk.k, 0u, rk.n14, rk.n15);  // block 0 -> poly key (chacha20_poly1305.rs:50,75)
        // r = clamp(pk[0..16]) (poly1305.rs:197-203), s = pk[16..32] (chacha20_poly1305.rs:32-39)
        r = words_to_f26(ks[0] & 0x0fffffffu, ks[1] & 0x0ffffffcu, ks[2] & 0x0ffffffcu, ks[3] & 0x0ffffffcu, 0u);
        s[0] = ks[4]; s[1] = ks[5]; s[2] = ks[6]; s[3] = ks[7];
        if constexpr (LIST) {  // the slot's descriptor: where the record lives, its length and nonce
            const uint64_t io = p.in_off ? p.in_off[rec] : p.in_stride * rec;
            const uint64_t oo = p.out_off ? p.out_off[rec] : p.out_stride * rec;
            uint32_t ki = p.key_index ? p.key_index[rec] : 0u;
            ki = ki < p.num_keys ? ki : p.num_keys - 1u;  // (record_key's clamp)
            uint32_t* d = wl.desc + (uint64_t)slot * kWprDescWords;
            st16(d, u32x4{(uint32_t)io, (uint32_t)(io >> 32), (uint32_t)oo, (uint32_t)(oo >> 32)});
            st16(d + 4, u32x4{n, rec, ki, rk.n14});
            st16(d + 8, u32x4{rk.n15, 0u, 0u, 0u});
        }
    }

    // ---- second half: lo[b] = R^b, hi[h][a] = 2^(32 h) R^(8 a) (R = r^4) ----
    // (LIST: also the pieces of S(c) = sum_{u<c} R^u, c = (n / 64) & 31, see below)
    const uint32_t kq = n >> 6, ca = kq >> 5, cl = kq & 7u, ch = (kq >> 3) & 3u;
    auto sel = [](bool c, const F26& a, const F26& b) {
        return F26{c ? a.v0 : b.v0, c ? a.v1 : b.v1, c ? a.v2 : b.v2, c ? a.v3 : b.v3, c ? a.v4 : b.v4};
    };
    const F26 r2 = fmul(r, r), R = fmul(r2, r2);
    F26 x = f26_one(), sum_lo = f26_zero(), plo = f26_zero(), xlo = f26_one();
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        store_f26(st + (kWLo - 80u) + 5u * b, x);
        sum_lo = f26_add(sum_lo, x);
        if constexpr (LIST) {
            plo = sel((uint32_t)b < cl, f26_add(plo, x), plo);  // sum_{b' < c & 7} R^b'
            xlo = sel((uint32_t)b == cl, x, xlo);               // R^(c & 7)
        }
        x = fmul(x, R);
    }
    const F26 R8 = x;
    F26 y = f26_one(), sum_hi = f26_zero(), phi = f26_zero(), yc = f26_one();
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        store_f26(st + (kWHi - 80u) + 5u * a, y);
        store_f26(st + (kWHi - 80u) + 20u + 5u * a, mul_add(y, 0u, 64u, 0u, 0u, 0u, f26_zero()));  // * 2^32
        sum_hi = f26_add(sum_hi, y);
        if constexpr (LIST) {
            phi = sel((uint32_t)a < ch, f26_add(phi, y), phi);  // sum_{a' < c >> 3} R^(8 a')
            yc = sel((uint32_t)a == ch, y, yc);                 // R^(8 (c >> 3))
        }
        y = fmul(y, R8);
    }
    const F26 T = y;  // R^32 = r^128
    wpr_store_units<20, 40>(wl, slot, act, rbuf);
    st = rbuf;

    // ---- first half: s, ctot, rd[u] = r^(1 + delta + u), tk[k] = T^k ----
    st[kWS + 0] = s[0]; st[kWS + 1] = s[1]; st[kWS + 2] = s[2]; st[kWS + 3] = s[3];
    const F26 r3 = fmul(r2, r), r5 = fmul(R, r), r6 = fmul(R, r2);
    const bool d1 = G.delta != 0u;
    const F26 pw[6] = {r, r2, r3, R, r5, r6};
#pragma unroll
    for (int u = 0; u < 5; ++u) store_f26(st + kWRd + 5u * u, d1 ? pw[u + 1] : pw[u]);
    const F26 rd0 = d1 ? r2 : r;        // r^(1 + delta)
    const F26 rdel = d1 ? r : f26_one();  // r^delta
    F26 t = f26_one(), sum_t = f26_zero(), pta = f26_zero(), ta = f26_one();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        store_f26(st + kWTk + 5u * k, t);
        sum_t = f26_add(sum_t, t);
        if constexpr (LIST) pta = sel((uint32_t)k < ca, f26_add(pta, t), pta);  // sum_{k' < a} T^k'
        t = fmul(t, T);
        if constexpr (LIST) ta = sel((uint32_t)k + 1u == ca, t, ta);            // T^a
    }
    wpr_store_units<3, 20>(wl, slot, act, rbuf);  // rd and tk now; s and ctot (units 0-2) at the end

    // geometric sums: SW = sum_{u<32} R^u; g = G(m) = sum_{i=1..m} r^i and rm = r^m
    // (m = n / 16: for n = 2^14, G(1024) = (r + r^2 + r^3 + r^4) SW sum_k T^k, r^1024 = T^8).
    // Bucket records (LIST) have n = 64 k', k' = 32 a + c (a = 2..8, c < 32), so from the
    // tables: G(4 k') = G4 S(k'), S(k') = sum_{u<k'} R^u = SW sum_{k<a} T^k + T^a S(c),
    // S(c) = sum_{a'<c>>3} R^(8 a') sum_lo + R^(8 (c>>3)) sum_{b<c&7} R^b, r^m = T^a R^(8 (c>>3)) R^(c&7)
    // (7 products instead of the ~25 of a square-and-multiply geometric sum)
    const F26 SW = fmul(carry1(sum_hi), carry1(sum_lo));
    const F26 G4 = carry1(f26_add(f26_add(r, r2), f26_add(r3, R)));
    F26 g, rm;
    if constexpr (LIST) {
        const F26 Sc = fmul_add(yc, carry1(plo), fmul(carry1(phi), carry1(sum_lo)));
        const F26 Sk = fmul_add(SW, carry1(pta), fmul(ta, Sc));
        g = fmul(G4, Sk);
        rm = fmul(ta, fmul(yc, xlo));
    } else {
        g = fmul(fmul(G4, SW), carry1(sum_t));
        rm = t;
    }
    // pads (poly1305.rs:224-225): 2^128 sum_{b < B-1} r^(B-b) + 2^(8 rem) r
    //   = 2^128 G(B) + (2^(8 rem) + p - 2^128) r,  G(B) = G(m) + r^m G(B - m)
    const F26 GB = fmul_add(rm, geo_sum(r, G.B - G.m), g);
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
    //   = r^delta G(m) (A1 r + A2),  A1 = sum_{k=sigma}^{15} 128 2^(8k),  A2 = sum_{k<sigma} 128 2^(8k)
    F26 bias;
    {
        uint32_t a1[4], a2[4];
#pragma unroll
        for (uint32_t w = 0; w < 4; ++w) {
            const uint32_t mk = bytes_from(w, G.sigma);
            a1[w] = 0x80808080u & mk;
            a2[w] = 0x80808080u & ~mk;
        }
        const F26 A1 = words_to_f26(a1[0], a1[1], a1[2], a1[3], 0u);
        const F26 A2 = words_to_f26(a2[0], a2[1], a2[2], a2[3], 0u);
        bias = fmul(fmul(g, fmul_add(A1, r, A2)), rdel);
    }
    // accumulator seed: -(2^24 sum_c 2^(8c)) SW (every column, the idle lanes' too)
    const F26 seed = mul_add(SW, kCJ0, kCJ1, kCJ2, kCJ3, kCJ4, f26_zero());
    // prefix ad || le64(|ad|) (stream bytes < o) as blocks 0..beta: Horner, then r^(B - beta) = r^m r^(1 + delta)
    F26 hp = f26_zero();
    if (act) {
        for (uint32_t b = 0; b <= G.beta; ++b) {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (uint32_t i = 0; i < 16u; ++i) {
                const uint32_t pos = 16u * b + i;
                if (pos < G.o) w[i >> 2] |= (uint32_t)prefix_byte(p, rec, rk.seq, n, adlen, pos) << (8u * (i & 3u));
            }
            hp = fmul_add(hp, r, words_to_f26(w[0], w[1], w[2], w[3], 0u));
        }
    }
    const F26 prefix = fmul(fmul(hp, rm), rd0);
    // suffix le64(n) at stream offset o + n = 16 (beta + m) + sigma: n 2^(8 sigma) split at 2^128
    F26 suffix;
    {
        const uint32_t wi = G.sigma >> 2, bs = 8u * (G.sigma & 3u);
        const uint64_t v = (uint64_t)n << bs;
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
    wpr_store_units<0, 3>(wl, slot, act, rbuf);
}

// ---------------------------------------------------------------------------
// The record kernel.
// ---------------------------------------------------------------------------
// a * b + c mod 2^64 (a signed, b a wave-uniform multiplier) in one
// v_mad_i64_i32; the _1 form: a + c with c uniform.  The compiler does not see
// these as instructions: the first use of an MFMA result goes through
// mfma_result_fence() (the XDL-write -> VALU-read wait states), and the asm is
// volatile so that it stays behind the fence.
__device__ __forceinline__ void mfma_result_fence() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
__device__ __forceinline__ uint64_t mad_i64_i32(int32_t a, uint32_t b, uint64_t c) {
    uint64_t d, cc;
    asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=&v"(d), "=s"(cc) : "v"(a), "s"(b), "v"(c));
    return d;
}
// a * b + c (unsigned 32 x 32 + 64 bits, b wave-uniform) in one v_mad_u64_u32
// (a power-of-two b would otherwise become a 64-bit shift and an add)
__device__ __forceinline__ uint64_t mad_u64_u32(uint32_t a, uint32_t b, uint64_t c) {
    uint64_t d, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(d), "=s"(cc) : "v"(a), "s"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint64_t mad_i64_i32_1(int32_t a, uint64_t c) {
    uint64_t d, cc;
    asm volatile("v_mad_i64_i32 %0, %1, %2, 1, %3" : "=&v"(d), "=s"(cc) : "v"(a), "s"(c));
    return d;
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
#if SG_WPR_PROFILE
constexpr uint32_t kProfPhases = 10, kProfWaves = 4096;
__device__ unsigned long long g_wpr_prof[kProfWaves][kProfPhases];
#define SG_TICK(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define SG_ACC(k, a, b) prof[k] += (b) - (a)
#else
#define SG_TICK(v)
#define SG_ACC(k, a, b)
#endif

// The double-round body: grouped ARX with an s_barrier after every rotate group
#define SG_WPR_DR_ASM SG_CHACHA_DR_NB1_BAR1

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
typedef const __attribute__((address_space(3))) uint32_t* lu32p;
__device__ __forceinline__ uint32_t cload(const void* base, uint64_t word) {
    return ((cu32p)(uintptr_t)base)[word];
}

// One 16-byte LDS-DMA per lane: LDS [l0 + 16 lane, +16) <- g (lanes with exec set).
// The same with a wave-uniform base address in SGPRs and the lane's 32-bit
// offset in a VGPR (global_load_lds_dwordx4 saddr form): one VGPR per lane for
// every DMA of the kernel instead of a 64-bit address per instruction.
__device__ __forceinline__ void dma_sv(uint32_t l0, const void* sbase, uint32_t voff) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" SG_DMA_POL "\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(l0)
                 : "memory");
}

// Address forms of the output path (round 4): the staged
// output is read from LDS through one VGPR base (the lane's swizzled unit in
// the wave's slice) with the buffer and piece as immediate offsets, and stored
// with the saddr form of global_store (record base in SGPRs, the lane's 16-byte
// offset in a VGPR, the piece as the instruction offset), so that no VALU
// address arithmetic runs per piece.  The stores are asm: their vmcnt is
// counted by the kernel's own waits like the DMAs' (s_nop: no VALU may
// overwrite the data registers of a >64-bit store in the next cycle).
typedef const __attribute__((address_space(3))) u32x4* lu128p;
template <uint32_t OFF>
__device__ __forceinline__ void gst16_s(const void* sbase, uint32_t voff, const u32x4& v) {
    static_assert(OFF < 4096u, "global instruction offset");
    asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3" SG_DMA_POL "\n\ts_nop 0"
                 :
                 : "v"(voff), "v"(v), "s"(sbase), "i"(OFF)
                 : "memory");
}

__device__ __forceinline__ void dma_one(uint32_t l0, const void* g) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(l0)
                 : "memory");
}

// Where a record lives and what keys it (uniform per wave).  Uniform batches
// derive it from the record index; bucket launches read the slot's descriptor.
struct RecDesc {
    uint64_t io, oo;    // byte offsets of the input / output record
    uint32_t n;         // plaintext length
    uint32_t rec;       // record index (status, key index, sequence number)
    uint32_t ki, n14, n15;
};

template <bool OPEN, bool TLS, uint32_t J, bool LIST>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void sg_wpr_kernel(const KParams p,
                                                                                               const WprList wl) {
    static_assert(J >= 1u && J <= 4u && (LIST || J == 4u), "uniform launches are full 16 KiB records");
    constexpr uint32_t j0 = 4u - J;  // the first chunk of the right-aligned record in the 16 KiB frame
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    uint8_t* buf = lds + wave * kWprWaveLds;
    uint8_t* lines = buf + kWprLinesOff;  // also the landing area of the record's keying table
    const uint32_t lds_wave = uniform((uint32_t)(uintptr_t)buf);
    const uint32_t lds_lines = uniform(lds_wave + kWprLinesOff);
    const uint32_t lds_desc = uniform(lds_lines + kWprDescOff);
    const uint32_t lds_rxs = uniform(lds_lines + kWprRxOff);
    const uint32_t hh = lane >> 5, q = lane & 31u;
    const uint32_t adlen = TLS ? 13u : p.ad_len;
    const uint32_t sigma = (adlen + 8u) & 15u;
    // T fragment byte a' comes from the V window for a' < 16 - sigma, else from P
    const uint32_t nv = 16u - sigma;
    const u32x4 vmask = {~bytes_from(0u, nv), ~bytes_from(1u, nv), ~bytes_from(2u, nv), ~bytes_from(3u, nv)};
    // LDS swizzle: 16-byte unit 4 t + c of a chunk lives at 4 t + (c ^ f(t)),
    // f(t) = (t ^ (t >> 2)) & 3.  Conflict-free for all three
    // accesses under the gfx950 banking rules (tests/test_lds_swizzle.py): the
    // lanes' ds_read_b128 of their own block (16-lane groups, 64 banks), the
    // staging ds_write_b128 (8 contiguous lanes, 32 banks: f is a bijection of
    // t's bits 1-2 for each t bit 0) and the lane-contiguous read-out.  (Round 4's f = (t >> 2) & 3
    // put lanes 8m and 8m + 2 of every write group on one bank slot: 8 conflict
    // cycles per write, 128 per record, SQ_LDS_BANK_CONFLICT = 2^27 per launch.)
    const uint32_t wunit = (lane & ~3u) | ((lane ^ (lane >> 2) ^ (lane >> 4)) & 3u);  // unit of global position 64 k + lane
    const uint32_t xq = (lane ^ (lane >> 2)) & 3u;
    // the lane's MAC window base (line 5 (1 - hh), dword of byte 47 - q) and shift
    const uint8_t* mac_base = lines + 240u * (1u - hh) + 4u * ((47u - q) >> 2);
    const uint32_t mac_shift = (47u - q) & 3u;
    // window bases of steps jj >= 2 (mac_lo) and jj < 2 (mac_hi), 64 bytes before
    // the P window of the step's largest offset
    uint32_t mac_lo_a = (uint32_t)(uintptr_t)(mac_base - 64), mac_hi_a = (uint32_t)(uintptr_t)(mac_base + 960 - 64);
    asm volatile("" : "+v"(mac_lo_a), "+v"(mac_hi_a));
    const lu32p mac_lo = (lu32p)(uintptr_t)mac_lo_a, mac_hi = (lu32p)(uintptr_t)mac_hi_a;
    // output read-out base (the lane's swizzled unit of the wave's slice) and the
    // lane's byte offset of a lane-contiguous 1 KiB piece
    // (uniform 16 KiB launches only: the bucket kernels have no VGPRs to spare)
    constexpr bool kAddr = !LIST;
    uint32_t ob_a = (uint32_t)(uintptr_t)(buf + 16u * wunit), lane16 = 16u * lane;
    if constexpr (kAddr) asm volatile("" : "+v"(ob_a), "+v"(lane16));
    const lu128p ob_base = (lu128p)(uintptr_t)ob_a;
    const uint32_t cnt = wl.count;
    const uint32_t ngroups = (cnt + kWprWaves - 1u) / kWprWaves;

    // The record of slot `slot` (slot < cnt): uniform batches from the strides,
    // bucket launches from the descriptor the keying kernel wrote.
    auto desc_of_slot = [&](uint32_t slot) {
        RecDesc d;
        if constexpr (LIST) {
            const uint32_t* dw = wl.desc + (uint64_t)slot * kWprDescWords;
            d.io = (uint64_t)cload(dw, 0) | ((uint64_t)cload(dw, 1) << 32);
            d.oo = (uint64_t)cload(dw, 2) | ((uint64_t)cload(dw, 3) << 32);
            d.n = cload(dw, 4);
            d.rec = cload(dw, 5);
            d.ki = cload(dw, 6);
            d.n14 = cload(dw, 7);
            d.n15 = cload(dw, 8);
        } else {
            d.rec = slot;
            d.io = p.in_stride * slot;
            d.oo = p.out_stride * slot;
            d.n = kWprN;
            d.ki = p.key_index ? cload(p.key_index, slot) : 0u;
            d.ki = d.ki < p.num_keys ? d.ki : p.num_keys - 1u;  // (record_key's clamp)
            // nonce (chacha20.rs:25-51; TLS: be64(seq), tls.rs:103)
            if constexpr (TLS) {
                uint64_t seq = p.seq0 + slot;
                if (p.seq) seq = (uint64_t)cload(p.seq, 2ull * slot) | ((uint64_t)cload(p.seq, 2ull * slot + 1u) << 32);
                d.n14 = sbswap32((uint32_t)(seq >> 32));  // (on the SALU: the chain below stays scalar)
                d.n15 = sbswap32((uint32_t)seq);
            } else {
                d.n14 = cload(p.nonces, 2ull * slot);
                d.n15 = cload(p.nonces, 2ull * slot + 1u);
            }
        }
        return d;
    };
    // the next record's descriptor, landed in the wave's LDS descriptor slot
    auto desc_from_lds = [&]() {
        const uint32_t* dl = reinterpret_cast<const uint32_t*>(lines + kWprDescOff);
        RecDesc d;
        d.io = (uint64_t)uniform(dl[0]) | ((uint64_t)uniform(dl[1]) << 32);
        d.oo = (uint64_t)uniform(dl[2]) | ((uint64_t)uniform(dl[3]) << 32);
        d.n = uniform(dl[4]);
        d.rec = uniform(dl[5]);
        d.ki = uniform(dl[6]);
        d.n14 = uniform(dl[7]);
        d.n15 = uniform(dl[8]);
        return d;
    };

    // Chunk c of a record is fetched by LDS-DMA into the wave buffer that the
    // previous chunk does not occupy, one chunk ahead: lane l of DMA piece k
    // lands at LDS unit 64 k + l and reads global unit 64 k + wunit(l), so LDS
    // unit phi(g) holds global unit g (phi = wunit within each 64-unit piece,
    // an involution: f depends only on the lane bits wunit keeps).  The record sits right-aligned in the 16 KiB frame:
    // frame byte v is record byte v - vs (vs = 2^14 - n), so the first chunk
    // j0 of a shorter record starts with lo = 4096 J - n bytes that belong to
    // no record; their lanes neither load nor store.  The record's keying
    // table (640 B) is fetched into the line area the same way.  The only
    // vector-memory operations of the kernel are these DMAs, the descriptor
    // DMA and the output stores, so the waits below count exactly.
    auto dma_piece_of = [&](uint32_t ldsb, const uint8_t* chunk_base, uint32_t k, uint32_t lo) {
        // chunk_base: the record's frame chunk start in real addresses (may lie before the record)
        if (!LIST || 1024u * k + 16u * wunit >= lo) dma_sv(uniform(ldsb + 1024u * k), chunk_base + 1024u * k, 16u * wunit);
    };
    auto dma_table_of = [&](uint32_t slot) {  // into the line area, lane u: unit u
        if (lane < kWprRecWords / 4u) {
            dma_one(lds_lines, wpr_tab_unit(wl, slot, lane));
        }
    };
    auto dma_desc_of = [&](uint32_t slot) {  // LIST: into the descriptor slot
        if (lane < kWprDescWords / 4u) dma_one(lds_desc, wl.desc + (uint64_t)slot * kWprDescWords + 4u * lane);
    };
    // Record groups are handed out dynamically: the first ones are static, every
    // later one comes from a device counter (zeroed by the keying kernel),
    // fetched by wave 0 during a group and passed to the other waves through
    // LDS.  The two workgroups sharing a CU do not progress at the same rate (a
    // static g += gridDim.x split left the fastest waves idle for the last 40 %
    // of the launch).  Uniform launches fetch one group ahead (the next
    // record's first chunk is addressed from its index); bucket launches two
    // groups ahead, so that the next record's descriptor can be fetched a whole
    // record before its first chunk.
    uint32_t* const ctr = wl.ctr;
    uint32_t* const gslot = reinterpret_cast<uint32_t*>(lds + kWprWaves * kWprWaveLds);
    uint32_t g = blockIdx.x;
    uint32_t gnx = LIST ? blockIdx.x + gridDim.x : ngroups;  // LIST: the next group, known a record ahead
    constexpr uint32_t kStatic = LIST ? 2u : 1u;            // groups handed out statically per workgroup
    RecDesc cd = {};                                        // the current record
    uint32_t par = 0u;  // LIST, J odd: the buffer of the record's first chunk alternates
    if (g < ngroups && g * kWprWaves + wave < cnt) {
        const uint32_t slot = g * kWprWaves + wave;
        cd = desc_of_slot(slot);
        const uint32_t vs = kWprN - cd.n, lo = kWprChunk * J - cd.n;
        const uint8_t* cb0 = p.in + cd.io + kWprChunk * j0 - vs;
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) dma_piece_of(lds_wave, cb0, k, lo);
        dma_table_of(slot);
    }
    bool first = true;
    // the previous chunk's output waits in its LDS buffer and leaves during
    // the next chunk's first double rounds (pend: it belongs to an active record)
    bool pend = false;
    uint8_t* pend_dst = p.out;
    uint32_t pend_lo = 0u;  // bytes of the pending chunk before the record (LIST: the first chunk)
    uint32_t lastb = 0u;    // the buffer of the last chunk

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
        const uint32_t slot = g * kWprWaves + wave;
        const bool active = slot < cnt;  // an inactive wave still runs every round and barrier
        // (an inactive wave takes any record: its results are not stored)
        if constexpr (!LIST) cd = desc_of_slot(active ? slot : cnt - 1u);
        else if (!active) cd = desc_of_slot(cnt - 1u);
        const uint32_t n = LIST ? cd.n : kWprN;
        const uint32_t vs = kWprN - n;                             // frame offset of the record
        const uint32_t lo = LIST ? kWprChunk * J - n : 0u;         // idle bytes of chunk j0
        // the lanes of chunk j0 that hold record bytes (the others sit out its rounds)
        const uint64_t live0 = LIST ? __builtin_amdgcn_ballot_w64(64u * lane >= lo) : ~0ull;
        const uint8_t* inb = p.in + cd.io;
        uint8_t* outb = p.out + cd.oo;
        uint32_t gn = ngroups, gnn = ngroups;  // the next group (uniform launches: known from iteration 3 on)
        if constexpr (LIST) gn = gnx;
        RecDesc nd = {};                       // the next record (LIST: from iteration j0 + 1 on)
        bool next = false;
        uint32_t kw[8];
#pragma unroll
        for (uint32_t i = 0; i < 8u; ++i) kw[i] = cload(p.keys, 8ull * cd.ki + i);
        const uint32_t n14 = cd.n14, n15 = cd.n15;
        // The column quarter rounds 1-3 of the first double round see no block
        // counter (word 13 is 0, chacha20.rs:114-121): the same for every lane
        // and chunk of the record, so they run once per record on the SALU.
        uint32_t u[16] = {kSigma0, kSigma1, kSigma2, kSigma3, kw[0], kw[1], kw[2], kw[3],
                          kw[4],   kw[5],   kw[6],   kw[7],   0u,    0u,    n14,   n15};
        SG_QR_S(u[1], u[5], u[9], u[13]) SG_QR_S(u[2], u[6], u[10], u[14]) SG_QR_S(u[3], u[7], u[11], u[15])
        // and the steps of the double round whose operands are all uniform
        // (tools/gen_chacha_grp.py, SG_CHACHA_DR1S_*; tests/test_chacha_asm_model.py)
        const uint32_t S0 = u[0] + u[4], T1 = u[1] + u[6], T2 = u[2] + u[7];
        const uint32_t T13 = srotl32(u[13] ^ T2, 16);

        // ---- the keying table has landed (it was followed only by the previous
        // record's tag / status store; the chunk-0 DMA is older)
        if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        first = false;
        wave_lds_sync();
        uint32_t fetched = 0u;
        if (wave == 0u && lane == 0u)
            fetched = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (LIST) {  // the next record's descriptor, a record ahead of its first chunk
            if (gn < ngroups && gn * kWprWaves + wave < cnt) dma_desc_of(gn * kWprWaves + wave);
        }
        // open: the received tag (chacha20_poly1305.rs:72-73) into the wave's tag
        // slot by LDS-DMA; it is read in the epilogue (a scalar load here would
        // hold up the table reads below until it returned)
        if (OPEN && lane == 0u) dma_one(lds_rxs, inb + n);
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
            const uint32_t k = lane / 5u, uu = lane - 5u * k;
            lv = fmul(load_f26(tab + kWRd + 5u * uu), load_f26(tab + kWTk + 5u * k));
        }
        wave_lds_sync();  // every table read is done before the lines overwrite it
        if (lane < kWprLines) {
            // any representative below 2^135 of r^e works (the MAC is exact mod p),
            // so the product's limbs (v0, v2..v4 < 2^26, v1 < 2^26 + 2^9) are
            // summed straight into 32-bit words, X = sum v_i 2^(26 i) < 2^131:
            // four v_mad_u64_u32, no carry ripple, no reduction (round 4; the
            // ripple_full form took ~35 more VALU per record)
            uint32_t c;  // digits = the bytes of X + 0x80..80, each ^ 0x80
            uint32_t d[5];
            uint64_t t = mad_u64_u32(lv.v1, 1u << 26, (uint64_t)lv.v0);
            const uint32_t x0 = (uint32_t)t;
            t = mad_u64_u32(lv.v2, 1u << 20, t >> 32);
            const uint32_t x1 = (uint32_t)t;
            t = mad_u64_u32(lv.v3, 1u << 14, t >> 32);
            const uint32_t x2 = (uint32_t)t;
            t = mad_u64_u32(lv.v4, 1u << 8, t >> 32);
            d[0] = addc(x0, 0x80808080u, 0u, &c) ^ 0x80808080u;
            d[1] = addc(x1, 0x80808080u, c, &c) ^ 0x80808080u;
            d[2] = addc(x2, 0x80808080u, c, &c) ^ 0x80808080u;
            d[3] = addc((uint32_t)t, 0x80808080u, c, &c) ^ 0x80808080u;
            d[4] = ((uint32_t)(t >> 32) + 0x80u + c) ^ 0x80u;
            uint8_t* ln = lines + kWprLineBytes * lane;
            const u32x4 z = zero4();
            if constexpr (TLS) {
                // sigma = 5: line byte b = digit 42 - b (b = 26..42), i.e. the
                // byte-reversed digit words R[k] = bswap(d[4 - k]) (digits 19 - 4k
                // .. 16 - 4k, 17..19 zero) laid from byte 23 on: three 16-byte
                // stores instead of 17 byte stores
                uint32_t R[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) R[k] = __builtin_bswap32(d[4 - k]);
                st16(ln, z);
                st16(ln + 16, u32x4{0u, R[0] << 24, __builtin_amdgcn_alignbyte(R[1], R[0], 1),
                                    __builtin_amdgcn_alignbyte(R[2], R[1], 1)});
                st16(ln + 32, u32x4{__builtin_amdgcn_alignbyte(R[3], R[2], 1), __builtin_amdgcn_alignbyte(R[4], R[3], 1),
                                    R[4] >> 8, 0u});
            } else {
                st16(ln, z);
                st16(ln + 16, z);
                st16(ln + 32, z);
#pragma unroll
                for (uint32_t i = 0; i < 17u; ++i) ln[47u - sigma - i] = (uint8_t)(d[i >> 2] >> (8u * (i & 3u)));
            }
        } else if (lane == kWprLines) {
            st16(lines + kWprLines * kWprLineBytes, zero4());
        }
        wave_lds_sync();
        SG_TICK(t_pl);
        SG_ACC(1, t_tw, t_pl);  // W and the digit lines

        // The first MFMA of the record starts from a zero accumulator (srcC = 0,
        // no per-record register initialisation); the 2^24 seed of every entry
        // is added at the assembly below.
        i32x16 acc = {};

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
            // from one of two opaque bases, so that every offset fits ds_read2_b32
            // (< 1 KiB) and no address is computed on the VALU
            const uint32_t off = 480u * ((3u - jj) & 1u) + 48u * (4u - i);
            const lu32p pb = (jj >= 2u ? mac_lo : mac_hi) + off / 4u;
            const lu32p vb = pb + 16;
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
        auto mac_mfma_f = [&](const u32x4& f, const u32x4& a, bool first = false) {
            const i32x16 c0 = {};
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, f),
                                                         __builtin_bit_cast(i32x4, a ^ 0x80808080u), first ? c0 : acc,
                                                         0, 0, 0);
        };
        auto mac_mfma = [&](const MacRaw& R, const u32x4& a, bool first = false) { mac_mfma_f(mac_frag(R), a, first); };
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
    // chunk j0 of a shorter record: the double rounds run with EXEC limited to
    // its live lanes (restored in the same statement; s_barrier ignores EXEC)
#define SG_DR_LIVE()                                                                                              \
    do {                                                                                                          \
        uint64_t sv;                                                                                              \
        asm volatile("s_and_saveexec_b64 %16, %17\n" SG_WPR_DR_ASM "s_mov_b64 exec, %16\n"                       \
                     : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),          \
                       "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),       \
                       "+v"(x[14]), "+v"(x[15]), "=&s"(sv)                                                          \
                     : "s"(live0)                                                                                 \
                     : "scc");                                                                                    \
    } while (0)

#pragma unroll
        for (uint32_t j = j0; j < 4u; ++j) {
            SG_TICK(t_js);
            // chunk j has landed (j > j0: its DMA was the last memory operation
            // of iteration j - 1; j = j0: waited for with the table), and so has
            // the next record's descriptor (LIST)
            if (j > j0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (j == j0 + 1u && wave == 0u && lane == 0u) *gslot = kStatic * gridDim.x + fetched;  // the atomic has returned
            wave_lds_sync();
            if constexpr (LIST) {
                if (j == j0 + 1u && gn < ngroups && gn * kWprWaves + wave < cnt) {
                    nd = desc_from_lds();
                    next = true;
                }
            } else if (j == 3u) {  // wave 0 published it before the barriers of iterations 1 and 2
                gn = uniform(*gslot);
                next = gn < ngroups && gn * kWprWaves + wave < cnt;
                nd.io = p.in_stride * (gn * kWprWaves + wave);  // only the address: the rest at its start
            }
            SG_TICK(t_jw);
            SG_ACC(2, t_js, t_jw);  // wait for the chunk
            // buffers: chunk j in bj, the pending output in the other one
            const uint32_t bj = ((j - j0) + par) & 1u;
            uint8_t* cb = buf + kWprChunk * bj;
            uint8_t* pb = buf + kWprChunk * (bj ^ 1u);
            const uint32_t plo = pend_lo;

            // keystream block 64 j + lane + 1 of the frame = block 64 j + lane + 1 - vs / 64 of the
            // record (chacha20_poly1305.rs:52), lock-step rounds
            const uint32_t bctr = 64u * j + lane + 1u - (vs >> 6);
            uint32_t x[16];
            x[12] = bctr;
            u32x4 D[4];
            SG_PIN();
            // first double round: every word but the counter enters from SGPRs
            // (EXEC limited to the live lanes in chunk j0 of a shorter record; the
            // rounds run at full EXEC, restored at the end of each statement, and
            // the live mask is the last operand so that the macros' numbering holds)
            const uint64_t live = (LIST && j == j0) ? live0 : ~0ull;
            asm volatile("s_mov_b64 exec, %7\n" SG_CHACHA_DR1S_COL "s_mov_b64 exec, -1\n"
                         : "=v"(x[0]), "=v"(x[4]), "=v"(x[8]), "+v"(x[12])
                         : "s"(S0), "s"(kw[0]), "s"(kw[4]), "s"(live));
            asm volatile("s_mov_b64 exec, %28\n" SG_CHACHA_DR1S_DIAG "s_mov_b64 exec, -1\n"
                         : "+v"(x[0]), "+v"(x[4]), "+v"(x[8]), "+v"(x[12]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]),
                           "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[13]),
                           "=v"(x[14]), "=v"(x[15])
                         : "s"(u[5]), "s"(u[15]), "s"(T1), "s"(u[3]), "s"(u[14]), "s"(u[10]), "s"(u[11]), "s"(T13),
                           "s"(u[9]), "s"(u[6]), "s"(u[7]), "s"(T2), "s"(live));
            SG_PIN();
            // The previous chunk's output leaves lane-contiguously one 1 KiB piece
            // per double round (read from LDS one gap ahead of its store), and
            // piece k of the next chunk's DMA follows the store of output piece k
            // (the same LDS range): the stores and DMAs of the 16 waves of a CU
            // spread over five gaps instead of queueing behind each other.
            auto out_piece = [&](uint32_t k) {
                if constexpr (kAddr) return ob_base[(kWprChunk * (bj ^ 1u) + 1024u * k) / 16u];
                return ld16(pb + 1024u * k + 16u * wunit);
            };
            auto store_piece = [&](uint32_t k, const u32x4& v) {
                if (!LIST || 1024u * k + 16u * lane >= plo) {
                    if constexpr (kAddr) {
                        switch (k) {
                            case 0: gst16_s<0u>(pend_dst, lane16, v); break;
                            case 1: gst16_s<1024u>(pend_dst, lane16, v); break;
                            case 2: gst16_s<2048u>(pend_dst, lane16, v); break;
                            default: gst16_s<3072u>(pend_dst, lane16, v); break;
                        }
                    } else {
                        gst16(pend_dst + 1024u * k + 16u * lane, v);
                    }
                }
            };
            auto dma_piece = [&](uint32_t k) {
                const uint32_t ldsb = lds_wave + kWprChunk * (bj ^ 1u);
                if (j < 3u) {
                    if (active) dma_piece_of(ldsb, inb + kWprChunk * (j + 1u) - vs, k, 0u);
                } else if (next) {
                    const uint32_t nvs = kWprN - (LIST ? nd.n : kWprN);
                    dma_piece_of(ldsb, p.in + nd.io + kWprChunk * j0 - nvs, k, LIST ? kWprChunk * J - nd.n : 0u);
                }
            };
            u32x4 oa = {}, ob = {};
            if (j > j0) mac_load(j - 1u, 0u, R0);
            if (pend) oa = out_piece(0u);
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            if (LIST && j == 3u) {  // wave 0 published it at the start of iteration j0 + 1 (LIST: J >= 2)
                gnn = uniform(*gslot);
            }
            if (j > j0) {
                mac_mfma(R0, A[0], j == j0 + 1u);
                mac_load(j - 1u, 1u, R1);
            }
            if (pend) {
                store_piece(0u, oa);
                ob = out_piece(1u);
            }
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            if (j > j0) {
                mac_mfma(R1, A[1]);
                mac_load(j - 1u, 2u, R0);
            }
            if (pend) {
                store_piece(1u, ob);
                oa = out_piece(2u);
            }
            dma_piece(0u);
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            if (j > j0) {
                mac_mfma(R0, A[2]);
                mac_load(j - 1u, 3u, R1);
            }
            if (pend) {
                store_piece(2u, oa);
                ob = out_piece(3u);
            }
            dma_piece(1u);
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            if (j > j0) mac_mfma(R1, A[3]);
            if (pend) store_piece(3u, ob);
            dma_piece(2u);
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            dma_piece(3u);
            if (j == 3u) {
                mac_load(3u, 0u, R0);
                mac_load(3u, 1u, R1);
            }
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            if (j == 3u) {
                F3[0] = mac_frag(R0);
                F3[1] = mac_frag(R1);
                mac_load(3u, 2u, R0);
                mac_load(3u, 3u, R1);
            }
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            if (j == 3u) {
                F3[2] = mac_frag(R0);
                F3[3] = mac_frag(R1);
            }
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) D[i] = ld16(cb + 16u * (4u * lane + (i ^ xq)));
            SG_PIN();
            if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();
            SG_PIN();
            SG_TICK(t_jr);
            SG_ACC(3, t_jw, t_jr);  // rounds (+ MAC of the previous chunk)
            if (j == 3u && next) {  // the line area is read out: the next record's table lands there
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                dma_table_of(gn * kWprWaves + wave);
            }
            // feed-forward (chacha20.rs:104-106) and XOR (chacha20.rs:143-153)
            u32x4 O[4];
            O[0] = D[0] ^ u32x4{x[0] + kSigma0, x[1] + kSigma1, x[2] + kSigma2, x[3] + kSigma3};
            O[1] = D[1] ^ u32x4{x[4] + kw[0], x[5] + kw[1], x[6] + kw[2], x[7] + kw[3]};
            O[2] = D[2] ^ u32x4{x[8] + kw[4], x[9] + kw[5], x[10] + kw[6], x[11] + kw[7]};
            O[3] = D[3] ^ u32x4{x[12] + bctr, x[13], x[14] + n14, x[15] + n15};
            // the MAC reads the ciphertext: received (open) or just produced (seal);
            // the lanes of the frame before the record contribute nothing (i8 0)
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) A[i] = OPEN ? D[i] : O[i];
            if (LIST && j == j0 && 64u * lane < lo) {
#pragma unroll
                for (uint32_t i = 0; i < 4u; ++i) A[i] = u32x4{0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};
            }
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
            pend_dst = outb + kWprChunk * j - vs;
            pend_lo = j == j0 ? lo : 0u;
            lastb = bj;
            SG_TICK(t_je);
            SG_ACC(4, t_jr, t_je);  // feed-forward, XOR, staging, stores
#if SG_WPR_PROFILE
            t_prev = t_je;
#endif
        }
#undef SG_DR
#undef SG_PIN

        // ---- assemble X = sum_r (D[c_r][q] + 2^24) 2^(8 c_r - 32 hh), c_r = (r & 3) + 8 (r >> 2) + 4 hh
        // (|D| < 2^23 signed; the seed 2^24 per entry makes every 64-bit word positive)
        uint32_t xw[8];
        constexpr uint64_t kSeed = (1ull << 24) + (1ull << 32) + (1ull << 40) + (1ull << 48);
        mfma_result_fence();
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint64_t yv = mad_i64_i32_1(acc[4 * m], kSeed);  // exact mod 2^64: the sum is positive
            yv = mad_i64_i32(acc[4 * m + 1], 256u, yv);
            yv = mad_i64_i32(acc[4 * m + 2], 65536u, yv);
            yv = mad_i64_i32(acc[4 * m + 3], 16777216u, yv);
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
                st16(outb + n, u32x4{tw[0], tw[1], tw[2], tw[3]});  // ct || tag (chacha20_poly1305.rs:55)
            } else {
                // constant-time compare: diff |= a ^ b over all 16 bytes (chacha20_poly1305.rs:84-87)
                const uint32_t* rxl = reinterpret_cast<const uint32_t*>(lines + kWprRxOff);
                const uint32_t diff = (rxl[0] ^ tw[0]) | (rxl[1] ^ tw[1]) | (rxl[2] ^ tw[2]) | (rxl[3] ^ tw[3]);
                p.status[cd.rec] = diff != 0u ? 1u : 0u;
            }
        }
        g = gn;
        if constexpr (LIST) {
            gnx = gnn;
            par ^= J & 1u;
        }
        if constexpr (LIST) cd = nd;
    }
    if (pend) {  // the last record's last chunk
        wave_lds_sync();
        const uint8_t* pb = buf + kWprChunk * lastb;
        // the lane index recomputed here (mbcnt) rather than kept live across the
        // record loop: at 128 VGPRs a value held from the prologue to this tail
        // is what the allocator spills first
        const uint32_t ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k)
            if (!LIST || 1024u * k + 16u * ln >= pend_lo)
                gst16(pend_dst + 1024u * k + 16u * ln, ld16(pb + 1024u * k + 16u * wunit));
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

hipError_t device_cus(int* cus) {
    int dev = 0;
    hipError_t e;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    *cus = dev >= 0 && dev < 64 ? __atomic_load_n(&g_cus[dev], __ATOMIC_RELAXED) : 0;
    if (*cus <= 0) {
        if ((e = hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        if (dev >= 0 && dev < 64) __atomic_store_n(&g_cus[dev], *cus, __ATOMIC_RELAXED);
    }
    return hipSuccess;
}

// persistent grid: two workgroups (16 waves) per CU, at most one per record group
static uint32_t wpr_grid(int cus, uint32_t count) {
    const uint32_t ngroups = (count + kWprWaves - 1u) / kWprWaves;
    const uint32_t grid = 2u * (uint32_t)cus;
    return grid < ngroups ? grid : ngroups;
}

hipError_t launch_wpr(const KParams& p, bool open, hipStream_t s, hipEvent_t ev_keyed, hipEvent_t ev_start) {
    WprList wl;
    wl.list = nullptr;
    wl.count = p.count;
    wl.tab = p.ws + (uint64_t)p.count * kWsWprTab;
    wl.desc = nullptr;
    wl.ctr = ws_tail(p.ws, p.count) + kTailCtr + kWprBuckets;
    WprKeyJobs jobs = {};
    jobs.b[0] = wl;
    jobs.njobs = 1;
    const uint32_t kgrid = (p.count + kWprKeyThreads - 1u) / kWprKeyThreads;
    if (open)
        hipLaunchKernelGGL((sg_wpr_keying_kernel<true, false>), dim3(kgrid), dim3(kWprKeyThreads), 0, s, p, jobs);
    else
        hipLaunchKernelGGL((sg_wpr_keying_kernel<false, false>), dim3(kgrid), dim3(kWprKeyThreads), 0, s, p, jobs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ev_keyed && (e = hipEventRecord(ev_keyed, s)) != hipSuccess) return e;
    if (ev_start && (e = hipEventRecord(ev_start, s)) != hipSuccess) return e;
    int cus = 0;
    if ((e = device_cus(&cus)) != hipSuccess) return e;
    const uint32_t grid = wpr_grid(cus, p.count);
#define SG_WPR_LAUNCH(O, T) hipLaunchKernelGGL((sg_wpr_kernel<O, T, 4, false>), dim3(grid), dim3(512), kWprWgLds, s, p, wl)
    if (open) {
        if (p.tls) SG_WPR_LAUNCH(true, true); else SG_WPR_LAUNCH(true, false);
    } else {
        if (p.tls) SG_WPR_LAUNCH(false, true); else SG_WPR_LAUNCH(false, false);
    }
#undef SG_WPR_LAUNCH
    return hipGetLastError();
}

hipError_t launch_wpr_keying_lists(const KParams& p, bool open, const WprList* wl, hipStream_t s) {
    if (!p.tls) return hipErrorInvalidValue;  // buckets are TLS records
    WprKeyJobs jobs = {};
    uint32_t grid = 0;
    for (uint32_t b = 0; b < kWprBuckets; ++b) {
        if (wl[b].count == 0) continue;
        jobs.b[jobs.njobs] = wl[b];
        jobs.blk0[jobs.njobs] = grid;
        grid += (wl[b].count + kWprKeyThreads - 1u) / kWprKeyThreads;
        ++jobs.njobs;
    }
    if (grid == 0) return hipSuccess;
    if (open)
        hipLaunchKernelGGL((sg_wpr_keying_kernel<true, true>), dim3(grid), dim3(kWprKeyThreads), 0, s, p, jobs);
    else
        hipLaunchKernelGGL((sg_wpr_keying_kernel<false, true>), dim3(grid), dim3(kWprKeyThreads), 0, s, p, jobs);
    return hipGetLastError();
}

hipError_t launch_wpr_list(const KParams& p, bool open, uint32_t J, const WprList& wl, hipStream_t s) {
    if (wl.count == 0) return hipSuccess;
    if (!p.tls || J < kWprMinJ || J > 4u) return hipErrorInvalidValue;  // buckets are TLS records of 2..4 chunks
    hipError_t e;
    int cus = 0;
    if ((e = device_cus(&cus)) != hipSuccess) return e;
    const uint32_t grid = wpr_grid(cus, wl.count);
#define SG_WPR_LAUNCH(O, JJ) hipLaunchKernelGGL((sg_wpr_kernel<O, true, JJ, true>), dim3(grid), dim3(512), kWprWgLds, s, p, wl)
    switch (J) {
        case 2: if (open) SG_WPR_LAUNCH(true, 2); else SG_WPR_LAUNCH(false, 2); break;
        case 3: if (open) SG_WPR_LAUNCH(true, 3); else SG_WPR_LAUNCH(false, 3); break;
        default: if (open) SG_WPR_LAUNCH(true, 4); else SG_WPR_LAUNCH(false, 4); break;
    }
#undef SG_WPR_LAUNCH
    return hipGetLastError();
}

static int g_wpr = -1;  // -1: not read from the environment yet
bool wpr_enabled() {
    if (__atomic_load_n(&g_wpr, __ATOMIC_ACQUIRE) < 0) {
        const char* e = getenv("SG_LOCKSTEP");
        int expect = -1;
        __atomic_compare_exchange_n(&g_wpr, &expect, e ? (e[0] == '1' ? 1 : 0) : 1, false,
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
    return "sg_wpr_kernel v17: full 16 KiB records, one wave per record (8 per 512-thread workgroup, persistent "
           "2 per CU, record groups handed out by a device counter), 4 KiB chunks LDS-DMA prefetched lane-contiguously into an XOR-swizzled LDS slice, output "
           "read out during the next chunk's first double rounds, lock-step grouped ChaCha20 rounds (s_barrier per "
           "rotate group; the first double round takes its uniform words from SGPRs, the counter-free steps once "
           "per record on the SALU), non-temporal record stream (nt LDS-DMA loads and stores), Poly1305 as 16 "
           "v_mfma_i32_32x32x32_i8 per record fed from the ciphertext registers one chunk behind (Toeplitz digit "
           "lines of r^(128k+d) in LDS, read as aligned dwords + v_alignbyte), exact per-lane assembly, "
           "W = r^(4(31-q)) scaling, DPP sum; keying pre-pass with the constant term; bucket records: the idle lanes "
           "of the first chunk sit out its rounds (EXEC)";
}

}  // namespace sg
