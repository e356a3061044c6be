// sg_pack.hip -- gfx950 packed ChaCha20-Poly1305 for the small records of a
// mixed TLS batch (klutzy/suruga src/cipher/chacha20_poly1305.rs:48-94 on
// records of 64 B .. 4 KiB, a multiple of 64 bytes: the C2 sizes below the
// wave-per-record buckets of sg_wpr.hip).
//
// The size-class kernels (sg_kernels.hip) give every record a power-of-two
// number of lanes, so a record of 33 blocks occupies a 64-lane wave, and they
// need a keying pre-pass whose 352-byte record per record goes through HBM.
// Here a 512-thread workgroup takes a run of 128 consecutive records of the
// list and lays their 64-byte blocks end to end: chunk c of the run is blocks
// 64 c .. 64 c + 63, lane t of the chunk computes keystream block j + 1 of the
// record that owns run block 64 c + t (j its block index in the record,
// chacha20.rs:111-135), and wave w takes chunks w, w + 8, ..., so no lane
// idles except in the run's last chunk and the last round.  The eight waves
// run the rounds in lock-step (grouped ARX asm with an s_barrier per rotate
// group, sg_chacha_grp.inc, as the wave-per-record kernel): the two waves of
// a SIMD then issue their full-rate add / xor back to back.  Lanes without a
// block (a round with no chunk for the wave, the tail of the last chunk) run
// the rounds with EXEC off, which saves power (the launch is power-capped).
// The grid is persistent (three workgroups per CU) and takes runs from a
// device counter until the list's population, read from the workspace, is
// used up: the host launches it before it has read the populations back
// (sg_kernels.hip, launch_aead_t), so the GPU runs it while the host waits.
//
//   setup (waves 0-1, one lane per record): keystream block 0 -> r, s
//     (chacha20_poly1305.rs:50-52, poly1305.rs:197-203), the powers
//     hi[a] = r^(1 + 32 a) and lo[b] = r^(4 b) (a, b < 8), the record's
//     constant term, its first run block and the start bitmap of the run;
//   chunks (all waves): XOR the record bytes, store, and add the lane's
//     Poly1305 term into the record's LDS accumulator;
//   finish (waves 0-1, one lane per record): tag = (acc + constant) + s,
//     appended (seal, :55) or compared in constant time (open, :84-93).
//
// MAC (poly1305.rs:207-228 over ad || le64(13) || ct || le64(n),
// chacha20_poly1305.rs:19-42).  With the 13-byte TLS AD the ciphertext starts
// at stream byte 21 = 16 + 5, and with n = 64 nb the stream has B = 4 nb + 2
// blocks, the last one 13 bytes long.  Lane j's 64 ciphertext bytes are the
// last 11 bytes of block 4 j + 1, blocks 4 j + 2 .. 4 j + 4 whole and the
// first 5 bytes of block 4 j + 5; as values v1..v5 (the lane's bytes at their
// positions in the blocks) its share of h is
//   Q_j r^(1 + 4 (nb - 1 - j)),  Q_j = sum_k (v_k + [k < 5] 2^128) r^(5 - k),
// every full block's pad 2^128 counted by the lane that holds the block's last
// byte.  Q_j is a four-step Horner with the clamped r in radix 2^32 (as the
// size-class kernels), the weight W = hi[i >> 3] lo[i & 7] (i = nb - 1 - j)
// one radix-2^26 product.  What no lane holds -- block 0 (AD bytes 0-12,
// le64(13) bytes 0-2) with its pad, and the last block's le64(n) and pad --
// is the constant term
//   (block0 + 2^128) r^B + (n 2^40 + 2^104) r
// (block 1 starts with le64(13) bytes 3-7, which are zero).  The terms go
// into the record's LDS accumulator with their limbs below 2^26 (limb 1: below
// 2^26 + 2^7, summed as 64 bits), so the at most 64 terms of a record never
// overflow a word; every step is exact mod 2^130 - 5 and the tag is the
// reference's bit for bit.
#include "sg_internal.h"
#include "sg_device.h"
#include "sg_chacha_grp.inc"  // grouped ChaCha20 double round (tools/gen_chacha_grp.py --product)

// Barriers per double round of the grouped asm (generated next to the macro)
// and a compile-time count of the macro text itself: the idle waves of a
// packed round execute exactly ten double rounds' worth of s_barrier.
#define SG_PACK_XSTR(x) #x
#define SG_PACK_STR(x) SG_PACK_XSTR(x)
#define SG_PACK_IDLE_BARS (10 * SG_CHACHA_DR_NB1_BAR1_BARRIERS)
namespace {
constexpr unsigned count_barriers(const char* s) {
    unsigned n = 0;
    for (; *s; ++s) {
        const char* b = "s_barrier";
        const char* t = s;
        while (*b && *t == *b) ++t, ++b;
        if (!*b) ++n;
    }
    return n;
}
static_assert(count_barriers(SG_CHACHA_DR_NB1_BAR1) == SG_CHACHA_DR_NB1_BAR1_BARRIERS,
              "barrier count of the double-round asm");
}  // namespace

#include <stdint.h>
#include <stdlib.h>

namespace sg {
namespace {

using namespace dev;

// the packed kernel's lanes each move their own 64-byte block: default cache
// policy (the non-temporal one measured -1.3 % on C2, round 3)
__device__ __forceinline__ u32x4 pld16(const void* p) { return ld16(p); }
__device__ __forceinline__ void pst16(void* p, u32x4 v) { st16(p, v); }

constexpr uint32_t kPackRecs = 128;                // records per workgroup run
constexpr uint32_t kPackWaves = 8;                 // two per SIMD: lock-step pairs
constexpr uint32_t kPackThreads = 64u * kPackWaves;
constexpr uint32_t kPackBlocks = kPackRecs * 64u;  // run blocks at most (nb <= 64)
constexpr uint32_t kPackChunks = kPackBlocks / 64u;
constexpr uint32_t kSlotWords = 30;                // record slot stride (ds_read_b64, bank spread)
// weight tables hi[8] lo[8] (entry e: hi[e], lo[e - 8]) as 128-bit words, the
// top two bits of entry e at bit 2 e of word 64 (odd stride: bank spread), so
// that three workgroups fit a CU's LDS
constexpr uint32_t kTabWords = 65;
constexpr uint32_t kTabTop = 64;
// slot layout (u32 words)
constexpr uint32_t kSKey = 0;     // key[8]
constexpr uint32_t kSN14 = 8, kSN15 = 9;
constexpr uint32_t kSR = 10;      // r0..r3 (clamped, radix 2^32)
constexpr uint32_t kSIn = 14;     // in_off lo, hi
constexpr uint32_t kSOut = 16;    // out_off lo, hi
constexpr uint32_t kSS = 18;      // s[4]
constexpr uint32_t kSCtot = 22;   // constant term (5 limbs)
constexpr uint32_t kSNb = 27, kSStart = 28, kSRec = 29;
static_assert(kSRec < kSlotWords, "slot layout");

// Per-record MAC accumulator: the lane terms
// fmul(Q, W) go in unreduced -- limbs 0, 2, 3, 4 < 2^26 (64 of them stay below
// 2^32), limb 1 < 2^26 + 2^7 summed as 64 bits -- instead of through a full
// carry ripple per lane (~30 VALU per chunk; round 4).  Three 64-bit LDS
// atomics per lane: (v0, v2) and (v3, v4) as the two halves of one u64 each
// (a half never carries into the other: its sum stays below 2^32) and v1;
// same-address atomics of the lanes of one record serialise, so fewer
// instructions cost fewer conflict cycles (five u32 atomics measured 0.7 %
// slower on C2, r04u).
constexpr uint32_t kAccWords = 6u;  // (v0, v2) u64 | (v3, v4) u64 | v1 u64
struct PackLds {
    uint32_t slot[kPackRecs * kSlotWords];
    uint32_t tab[kPackRecs * kTabWords];
    alignas(8) uint32_t acc[kPackRecs * kAccWords];
    uint32_t bits[kPackBlocks / 32];  // run block b starts a record
    uint32_t base[kPackChunks];       // first-chunk histogram, then records starting before chunk c
    uint32_t wtot;                    // wave 0's blocks (setup scan)
    uint32_t nchunks, total;
    uint32_t run;
};
static_assert(sizeof(PackLds) <= 65536, "static LDS");
static_assert(3 * sizeof(PackLds) <= 160 * 1024, "three workgroups per CU");

// table entry e <- x (fully reduced first; top bits collected by the caller)
__device__ __forceinline__ uint32_t tab_put(uint32_t* tb, uint32_t e, F26 x) {
    x = ripple_full(x);  // limbs < 2^26: x < 2^130
    tb[4u * e + 0] = x.v0 | (x.v1 << 26);
    tb[4u * e + 1] = (x.v1 >> 6) | (x.v2 << 20);
    tb[4u * e + 2] = (x.v2 >> 12) | (x.v3 << 14);
    tb[4u * e + 3] = (x.v3 >> 18) | (x.v4 << 8);
    return (x.v4 >> 24) << (2u * e);
}
__device__ __forceinline__ F26 tab_get(const uint32_t* tb, uint32_t e, uint32_t top) {
    return words_to_f26(tb[4u * e], tb[4u * e + 1], tb[4u * e + 2], tb[4u * e + 3], (top >> (2u * e)) & 3u);
}
// W(i) = r^(1 + 4 i) = hi[i >> 3] lo[i & 7]
__device__ __forceinline__ F26 tab_weight(const uint32_t* tb, uint32_t i) {
    const uint32_t top = tb[kTabTop];
    return fmul(tab_get(tb, i >> 3, top), tab_get(tb, 8u + (i & 7u), top));
}

// inclusive prefix sum over the 64 lanes of a wave
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
#pragma unroll
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// The record's 64-byte block d[16] (ciphertext words) as the Poly1305 values
// v1..v5 of the header comment, the MAC stream shifted by 5 bytes:
// stream word w of the lane is alignbyte(d[w - 1], d[w - 2], 3).
__device__ __forceinline__ void lane_mac(H32& h, const uint32_t d[16], uint32_t r0, uint32_t r1, uint32_t r2,
                                         uint32_t r3, uint32_t s1, uint32_t s2, uint32_t s3) {
    uint32_t e[18];
    e[0] = 0u;
    e[1] = d[0] << 8;
#pragma unroll
    for (int w = 2; w < 17; ++w) e[w] = __builtin_amdgcn_alignbyte(d[w - 1], d[w - 2], 3);
    e[17] = d[15] >> 24;
    h = H32{0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k)  // (h + v_k + 2^128) r
        horner_step(h, e[4 * k], e[4 * k + 1], e[4 * k + 2], e[4 * k + 3], 1u, r0, r1, r2, r3, s1, s2, s3);
    uint32_t c;  // + v5 (no pad: block 4 j + 5 ends in the next lane or is the last block)
    h.h0 = addc(h.h0, e[16], 0u, &c);
    h.h1 = addc(h.h1, e[17], c, &c);
    h.h2 = addc(h.h2, 0u, c, &c);
    h.h3 = addc(h.h3, 0u, c, &c);
    h.h4 += c;
}

// Phase timing (experiment builds only, -DSG_PACK_PROFILE=1; output
// unchanged): s_memtime stamps of waves 0 and 7 of the first kProfWgs
// workgroups, read back by tools/pack_phase.py through sg_pack_profile_read.
#ifndef SG_PACK_PROFILE
#define SG_PACK_PROFILE 0
#endif
#if SG_PACK_PROFILE
constexpr uint32_t kProfWgs = 8192, kProfStamps = 12;
__device__ unsigned long long g_pack_prof[kProfWgs][kProfStamps];
#define SG_STAMP(w, k)                                                                              \
    do {                                                                                            \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                           \
        if (wave == (w) && lane == 0u && blockIdx.x < kProfWgs) g_pack_prof[blockIdx.x][k] = t_;     \
    } while (0)
#else
#define SG_STAMP(w, k)
#endif

// One run: records first .. first + nrec - 1 of the packed list.
template <bool OPEN>
__device__ __forceinline__ void pack_run(const KParams& p, const uint32_t* __restrict__ list, const uint32_t first,
                                         const uint32_t nrec, PackLds& L, const uint32_t tid, const uint32_t lane,
                                         const uint32_t wave) {

    SG_STAMP(0u, 0);
    for (uint32_t i = tid; i < kPackBlocks / 32u; i += kPackThreads) L.bits[i] = 0u;
    for (uint32_t i = tid; i < kPackRecs * kAccWords; i += kPackThreads) L.acc[i] = 0u;
    if (tid < kPackChunks) L.base[tid] = 0u;

    // ---- setup: lane m of waves 0-1 keys record m of the run ---------------------
    // (a) everything but the record's place in the run: the loads first, as
    // three levels (list -> per-record arrays -> key words), then block 0, the
    // powers and the constant term
    const uint32_t m0 = tid;  // waves 0-1
    const bool act = m0 < nrec;
    uint32_t nb = 0u, start = 0u;
    if (wave < 2u) {
        const uint32_t rec = act ? list[first + m0] : 0u;
        uint32_t* sl = L.slot + m0 * kSlotWords;
        uint32_t* tb = L.tab + m0 * kTabWords;
        if (act) {
            const uint32_t len = record_len(p, rec);
            const uint64_t io = p.in_off ? p.in_off[rec] : p.in_stride * rec;
            const uint64_t oo = p.out_off ? p.out_off[rec] : p.out_stride * rec;
            const RecKey rk = record_key(p, rec);
            const uint32_t n = OPEN ? len - 16u : len;  // listed records: 64 <= n <= 4096, n % 64 == 0
            nb = n >> 6;
#if SG_PACK_PROFILE
            if (rk.k[0] == 0x12345678u && rk.seq == 1u) g_pack_prof[0][11] = io + oo;  // wait for the loads
#endif
            SG_STAMP(0u, 8);
            uint32_t ks[16];
            chacha_block(ks, rk.k, 0u, rk.n14, rk.n15);  // block 0 -> poly key (chacha20_poly1305.rs:50,75)
            // r = clamp(pk[0..16]) (poly1305.rs:197-203), s = pk[16..32] (chacha20_poly1305.rs:32-39)
            const uint32_t r0 = ks[0] & 0x0fffffffu, r1 = ks[1] & 0x0ffffffcu;
            const uint32_t r2w = ks[2] & 0x0ffffffcu, r3 = ks[3] & 0x0ffffffcu;
            SG_STAMP(0u, 9);
#pragma unroll
            for (int i = 0; i < 8; ++i) sl[kSKey + i] = rk.k[i];
            sl[kSN14] = rk.n14;
            sl[kSN15] = rk.n15;
            sl[kSR + 0] = r0; sl[kSR + 1] = r1; sl[kSR + 2] = r2w; sl[kSR + 3] = r3;
            sl[kSIn] = (uint32_t)io; sl[kSIn + 1] = (uint32_t)(io >> 32);
            sl[kSOut] = (uint32_t)oo; sl[kSOut + 1] = (uint32_t)(oo >> 32);
            sl[kSS + 0] = ks[4]; sl[kSS + 1] = ks[5]; sl[kSS + 2] = ks[6]; sl[kSS + 3] = ks[7];
            sl[kSNb] = nb;
            sl[kSRec] = rec;
            // hi[a] = r^(1 + 32 a), lo[b] = R^b (R = r^4), two product chains
            const F26 r = words_to_f26(r0, r1, r2w, r3, 0u);
            const F26 r2 = fmul(r, r), R = fmul(r2, r2);
            F26 y = f26_one();
            uint32_t top = 0u;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                top |= tab_put(tb, 8u + b, y);
                y = fmul(y, R);
            }
            const F26 R8 = y;  // r^32
            F26 z = r;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                top |= tab_put(tb, a, z);
                if (a < 7) z = fmul(z, R8);
            }
            tb[kTabTop] = top;
            SG_STAMP(0u, 10);
            // constant term (header comment): r^B = r^(4 nb + 2) = W(nb - 1) R r
            const uint32_t il = nb - 1u;
            const F26 wl = tab_weight(tb, il);
            const F26 rB = fmul(fmul(wl, R), r);
            // block 0: be64(seq) || type || major || minor || be16(n) || le64(13)[0..3] (tls.rs:103-112)
            const uint32_t w2 = (p.tls_hdr & 0x00ffffffu) | (((n >> 8) & 0xffu) << 24);
            const uint32_t w3 = (n & 0xffu) | (13u << 8);
            const F26 blk0 = words_to_f26(rk.n14, rk.n15, w2, w3, 1u);   // + the pad 2^128
            const F26 sfx = words_to_f26(0u, n << 8, 0u, 256u, 0u);      // n 2^40 + 2^104
            store_f26(sl + kSCtot, fmul_add(blk0, rB, fmul(sfx, r)));
        }
        const uint32_t incl = wave_incl_scan(nb, lane);
        start = incl - nb;
        if (wave == 0u && lane == 63u) L.wtot = incl;
    }
    SG_STAMP(0u, 1);
    __syncthreads();
    // (b) the record's first run block: the start bitmap and first-chunk histogram
    if (wave < 2u) {
        if (wave == 1u) start += L.wtot;
        if (act) {
            L.slot[m0 * kSlotWords + kSStart] = start;
            atomicOr(&L.bits[start >> 5], 1u << (start & 31u));
            atomicAdd(&L.base[start >> 6], 1u);
        }
    }
    __syncthreads();
    // (c) base[c]: records whose first block lies before chunk c (exclusive scan
    // of the first-chunk histogram, two chunks per lane)
    if (wave == 0u) {
        const uint32_t h0 = L.base[2u * lane], h1 = L.base[2u * lane + 1u];
        const uint32_t incl = wave_incl_scan(h0 + h1, lane);
        L.base[2u * lane] = incl - h0 - h1;
        L.base[2u * lane + 1u] = incl - h1;
    }
    if (wave == 1u && lane == 63u) {
        const uint32_t total = start + nb;  // the run's last record (or an empty lane) ends the run
        L.total = total;
        L.nchunks = (total + 63u) >> 6;
    }
    __syncthreads();

    // ---- chunk rounds: wave w takes chunk 8 k + w in round k --------------------
    // Every wave runs every round's ChaCha20 double rounds (grouped by kind,
    // s_barrier after each rotate group: the two waves of a SIMD issue their
    // full-rate add / xor back to back, sg_chacha_grp.inc), also in a round with
    // no chunk for it, so that all waves meet the same barriers.
    SG_STAMP(0u, 2);
    SG_STAMP(7u, 6);
    // (scalar: the idle-round branch below must be wave-uniform, or working and
    // idle waves would meet different barrier counts)
    const uint32_t total = L.total, nchunks = __builtin_amdgcn_readfirstlane(L.nchunks);
    const uint32_t nrounds = (nchunks + kPackWaves - 1u) / kPackWaves;
    // Chunk order within a round: SIMD pairs first (waves w and w + 4 share a
    // SIMD), so that in the last, partial round the chunks go to whole pairs
    // and the waves without one only keep the barrier count (s_barrier, no
    // VALU): their issue slots go to the CU's other workgroups, and the working
    // waves stay paired (round 2 measured that idle waves running the rounds
    // with EXEC off save only power).
    const uint32_t pos = 2u * (wave & 3u) + (wave >> 2);
    for (uint32_t k = 0; k < nrounds; ++k) {
        const uint32_t c = kPackWaves * k + pos;
        if (c >= nchunks) {  // (wave-uniform) no chunk in this round
            // as many barriers as the ten double rounds of a working wave
            asm volatile(".rept " SG_PACK_STR(SG_PACK_IDLE_BARS) "\ns_barrier\n.endr" ::: "memory");
            continue;
        }
        const uint32_t b = 64u * c + lane;
        const bool valid = c < nchunks && b < total;
        // the record of run block b: the starts at or before it
        uint32_t m = 0u;
        if (c < nchunks) {
            const uint32_t mlo = L.bits[2u * c], mhi = L.bits[2u * c + 1u];
            const uint32_t below = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
            const uint32_t own = ((lane < 32u ? mlo >> lane : mhi >> (lane - 32u)) & 1u);
            m = L.base[c] + below + own - 1u;
        }
        if (!valid) m = 0u;
        const uint32_t* sl = L.slot + m * kSlotWords;
        const uint32_t j = b - sl[kSStart];
        const uint64_t io = (uint64_t)sl[kSIn] | ((uint64_t)sl[kSIn + 1] << 32);
        const uint64_t oo = (uint64_t)sl[kSOut] | ((uint64_t)sl[kSOut + 1] << 32);
        u32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
        if (valid) {
            const uint8_t* src = p.in + io + 64u * j;
            // (plain policy: the nontemporal one measured -1.3 % on C2 for this
            // kernel's 64-byte lane stride, round 3)
            d0 = pld16(src); d1 = pld16(src + 16); d2 = pld16(src + 32); d3 = pld16(src + 48);
        }
        uint32_t kw[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = sl[kSKey + i];
        const uint32_t ctr = j + 1u, n14 = sl[kSN14], n15 = sl[kSN15];  // data uses blocks 1.. (chacha20_poly1305.rs:52)
        uint32_t x[16] = {kSigma0, kSigma1, kSigma2, kSigma3, kw[0], kw[1], kw[2], kw[3],
                          kw[4],   kw[5],   kw[6],   kw[7],   ctr,     0u,    n14,   n15};
        // EXEC limited to the lanes with a block (none in a round without a
        // chunk for this wave; s_barrier ignores EXEC, so all waves still meet)
        const uint64_t live = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
        for (int dr = 0; dr < 10; ++dr) {
            uint64_t sv;
            asm volatile("s_and_saveexec_b64 %16, %17\n" SG_CHACHA_DR_NB1_BAR1 "s_mov_b64 exec, %16\n"
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                           "+v"(x[14]), "+v"(x[15]), "=&s"(sv)
                         : "s"(live)
                         : "scc");
        }
        if (valid) {
            // feed-forward (chacha20.rs:104-106) and XOR (chacha20.rs:143-153)
            const u32x4 o0 = d0 ^ u32x4{x[0] + kSigma0, x[1] + kSigma1, x[2] + kSigma2, x[3] + kSigma3};
            const u32x4 o1 = d1 ^ u32x4{x[4] + kw[0], x[5] + kw[1], x[6] + kw[2], x[7] + kw[3]};
            const u32x4 o2 = d2 ^ u32x4{x[8] + kw[4], x[9] + kw[5], x[10] + kw[6], x[11] + kw[7]};
            const u32x4 o3 = d3 ^ u32x4{x[12] + ctr, x[13], x[14] + n14, x[15] + n15};
            uint8_t* dst = p.out + oo + 64u * j;
            pst16(dst, o0);
            pst16(dst + 16, o1);
            pst16(dst + 32, o2);
            pst16(dst + 48, o3);
            // the MAC reads the ciphertext: received (open) or produced (seal)
            const u32x4 a0 = OPEN ? d0 : o0, a1 = OPEN ? d1 : o1, a2 = OPEN ? d2 : o2, a3 = OPEN ? d3 : o3;
            const uint32_t cw[16] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3],
                                     a2[0], a2[1], a2[2], a2[3], a3[0], a3[1], a3[2], a3[3]};
            const uint32_t r0 = sl[kSR + 0], r1 = sl[kSR + 1], r2 = sl[kSR + 2], r3 = sl[kSR + 3];
            H32 h;
            lane_mac(h, cw, r0, r1, r2, r3, r1 + (r1 >> 2), r2 + (r2 >> 2), r3 + (r3 >> 2));
            const F26 Q = words_to_f26(h.h0, h.h1, h.h2, h.h3, h.h4);
            const uint32_t i = sl[kSNb] - 1u - j;
            const uint32_t* tb = L.tab + m * kTabWords;
            const F26 W = tab_weight(tb, i);
            uint32_t* ac = L.acc + kAccWords * m;
            const F26 t = fmul(Q, W);
            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 0),
                      (unsigned long long)t.v0 | ((unsigned long long)t.v2 << 32));
            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 2),
                      (unsigned long long)t.v3 | ((unsigned long long)t.v4 << 32));
            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);
        }
    }
    SG_STAMP(0u, 3);
    SG_STAMP(7u, 7);
    __syncthreads();
    SG_STAMP(0u, 4);

    // ---- finish: one lane per record (waves 0-1) --------------------------------
    if (act) {
        const uint32_t* sl = L.slot + m0 * kSlotWords;
        const uint32_t n = 64u * sl[kSNb], rec = sl[kSRec];
        const uint32_t* ac = L.acc + kAccWords * m0;
        // (v1 = lo + hi 2^32 -> hi 2^58 = (hi << 6) 2^52 joins limb 2 after the
        // first carry pass: limb 2's raw sum can reach 2^32 - 64, and hi <= 1)
        F26 f = carry1(F26{ac[0], ac[4], ac[1], ac[2], ac[3]});
        f.v2 += ac[5] << 6;
        f = carry1(f26_add(f, load_f26(sl + kSCtot)));
        const uint32_t s[4] = {sl[kSS + 0], sl[kSS + 1], sl[kSS + 2], sl[kSS + 3]};
        uint32_t tw[4];
        tag_words(f, s, tw);
        const uint64_t io = (uint64_t)sl[kSIn] | ((uint64_t)sl[kSIn + 1] << 32);
        const uint64_t oo = (uint64_t)sl[kSOut] | ((uint64_t)sl[kSOut + 1] << 32);
        if constexpr (!OPEN) {
            st16(p.out + oo + n, u32x4{tw[0], tw[1], tw[2], tw[3]});  // ct || tag (chacha20_poly1305.rs:55)
        } else {
            // constant-time compare: diff |= a ^ b over all 16 bytes (chacha20_poly1305.rs:84-87)
            const u32x4 rx = ld16(p.in + io + n);
            const uint32_t diff = (rx[0] ^ tw[0]) | (rx[1] ^ tw[1]) | (rx[2] ^ tw[2]) | (rx[3] ^ tw[3]);
            p.status[rec] = diff != 0u ? 1u : 0u;
        }
    }
    SG_STAMP(0u, 5);
}

// Persistent grid (three workgroups per CU, the LDS bound): the packed list's
// population is read from the workspace tail (the host does not need it, so
// the launch goes ahead of the population readback) and the 128-record runs
// come from a device counter, so that the runs' different lengths even out.
template <bool OPEN>
__global__ __launch_bounds__(kPackThreads) __attribute__((amdgpu_waves_per_eu(6)))
void sg_pack_kernel(const KParams p, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt, uint32_t* ctr) {
    __shared__ PackLds L;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uniform(tid >> 6);
    const uint32_t count = __builtin_amdgcn_readfirstlane(*cnt);
    const uint32_t nruns = (count + kPackRecs - 1u) / kPackRecs;
    for (;;) {
        if (tid == 0u) L.run = atomicAdd(ctr, 1u);
        __syncthreads();
        const uint32_t run = __builtin_amdgcn_readfirstlane(L.run);
        if (run >= nruns) break;  // (workgroup-uniform)
        const uint32_t first = run * kPackRecs;
        pack_run<OPEN>(p, list, first, count - first < kPackRecs ? count - first : kPackRecs, L, tid, lane, wave);
        __syncthreads();  // the finish read the slots that the next run's setup rewrites, and L.run
    }
}

}  // namespace

hipError_t launch_pack(const KParams& p, bool open, const uint32_t* list, const uint32_t* count, uint32_t* ctr,
                       hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    if (!p.tls) return hipErrorInvalidValue;  // the MAC geometry is the 13-byte TLS AD's
    int cus = 0;
    hipError_t e;
    if ((e = device_cus(&cus)) != hipSuccess) return e;
    const uint32_t most = (p.count + kPackRecs - 1u) / kPackRecs;
    const uint32_t grid = 3u * (uint32_t)cus < most ? 3u * (uint32_t)cus : most;  // three workgroups per CU
    if (open)
        hipLaunchKernelGGL((sg_pack_kernel<true>), dim3(grid), dim3(kPackThreads), 0, s, p, list, count, ctr);
    else
        hipLaunchKernelGGL((sg_pack_kernel<false>), dim3(grid), dim3(kPackThreads), 0, s, p, list, count, ctr);
    return hipGetLastError();
}

#if SG_PACK_PROFILE
extern "C" int sg_pack_profile_read(unsigned long long* host, size_t n) {
    const size_t bytes = sizeof(g_pack_prof);
    if (n * sizeof(unsigned long long) < bytes) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pack_prof), bytes) != hipSuccess) return -2;
    return (int)(bytes / sizeof(unsigned long long));
}
#endif

static int g_pack = -1;  // -1: not read from the environment yet
bool pack_enabled() {
    if (__atomic_load_n(&g_pack, __ATOMIC_ACQUIRE) < 0) {
        const char* e = getenv("SG_PACK");
        int expect = -1;
        __atomic_compare_exchange_n(&g_pack, &expect, e ? (e[0] == '1' ? 1 : 0) : 1, false,
                                    __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
    }
    return __atomic_load_n(&g_pack, __ATOMIC_ACQUIRE) == 1;
}
int set_pack(int enable) {
    const int prev = pack_enabled() ? 1 : 0;
    if (enable >= 0) __atomic_store_n(&g_pack, enable ? 1 : 0, __ATOMIC_RELEASE);
    return prev;
}

const char* pack_kernel_config() {
    return "sg_pack_kernel v5: mixed-batch TLS records of 64 B-4 KiB (multiples of 64 B) packed 64-byte block per lane "
           "across 128-record runs (512-thread workgroups on a persistent grid taking runs from a device counter, launched "
           "ahead of the population readback; chunk rounds, lock-step grouped ChaCha20 rounds with EXEC limited "
           "to the lanes holding a block; chunks to SIMD pairs first, waves without a chunk in the last round keep "
           "only the barriers), keying in the same kernel "
           "(block 0, r^(1+32a) and r^(4b) tables in LDS), per-lane Poly1305 share as a 4-step radix-2^32 Horner times "
           "r^(1+4i), unreduced into the record accumulator by three 64-bit LDS atomics, constant term for AD / length / pads";
}

}  // namespace sg
