/*
 * suruga_oracle.c -- CPU restatement of suruga's ChaCha20-Poly1305 record AEAD.
 *
 * TEST INFRASTRUCTURE ONLY (see suruga_oracle.h): the parity checker and the
 * bench's CPU baseline ("port"), never linked into the product library.
 *
 * Every function follows the reference's algorithm step for step, including
 * its radix-2^26 limb arithmetic with three carry passes and its constant-time
 * normalize/choose, so that intermediate states (not just final tags) match.
 * Reference file:line citations are relative to klutzy/suruga.
 */
#include "suruga_oracle.h"
#include "so_pool.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#ifdef SO_DEBUG
#include <assert.h>
#define SO_DEBUG_ASSERT(x) assert(x)
#else
#define SO_DEBUG_ASSERT(x) ((void)0)
#endif

/* ------------------------------------------------------------------------ */
/* util.rs                                                                   */
/* ------------------------------------------------------------------------ */

/* util.rs:43-45 -- mem::transmute(x.to_be()) */
void so_u64_be(uint64_t x, uint8_t out[8]) {
    for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(x >> (56 - 8 * i));
}

/* util.rs:47-49 -- mem::transmute(x.to_le()) */
void so_u64_le(uint64_t x, uint8_t out[8]) {
    for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(x >> (8 * i));
}

/* tls.rs:103-112 (writer) / :250-265 (reader) */
void so_tls_ad(uint64_t seq, uint8_t content_type, uint8_t major, uint8_t minor,
               uint16_t frag_len, uint8_t ad[13]) {
    so_u64_be(seq, ad);
    ad[8] = content_type;
    ad[9] = major;
    ad[10] = minor;
    ad[11] = (uint8_t)(frag_len >> 8);
    ad[12] = (uint8_t)frag_len;
}

/* ------------------------------------------------------------------------ */
/* chacha20.rs                                                               */
/* ------------------------------------------------------------------------ */

/* chacha20.rs:7-16 to_le_u32! */
static uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}

int so_chacha20_new(so_chacha20* st, const uint8_t* key, size_t key_len,
                    const uint8_t* nonce, size_t nonce_len) {
    if (key_len != 32 || nonce_len != 8) return -1; /* :26-27 assert_eq! */
    /* "expand 32-byte k"  :32-35 */
    st->vals[0] = 0x61707865u;
    st->vals[1] = 0x3320646eu;
    st->vals[2] = 0x79622d32u;
    st->vals[3] = 0x6b206574u;
    for (int i = 0; i < 8; ++i) st->vals[4 + i] = le32(key + 4 * i); /* :37-39 */
    st->vals[12] = 0; /* counter :42-43 */
    st->vals[13] = 0;
    st->vals[14] = le32(nonce);     /* :45 */
    st->vals[15] = le32(nonce + 4); /* :46 */
    return 0;
}

/* chacha20.rs:55-61 rot! (Wrapping<u32> shifts) */
static uint32_t rotl(uint32_t a, unsigned e) { return (a << e) | (a >> (32 - e)); }

/* chacha20.rs:63-81 quarter_round! */
#define SO_QR(v, a, b, c, d)                                \
    do {                                                    \
        v[a] += v[b]; v[d] ^= v[a]; v[d] = rotl(v[d], 16);  \
        v[c] += v[d]; v[b] ^= v[c]; v[b] = rotl(v[b], 12);  \
        v[a] += v[b]; v[d] ^= v[a]; v[d] = rotl(v[d], 8);   \
        v[c] += v[d]; v[b] ^= v[c]; v[b] = rotl(v[b], 7);   \
    } while (0)

/* chacha20.rs:53-109 round20 */
static void round20(const uint32_t in[16], uint32_t out[16]) {
    uint32_t v[16];
    memcpy(v, in, sizeof v);
    for (int r = 0; r < 10; ++r) {
        /* column round :91-95 */
        SO_QR(v, 0, 4, 8, 12);
        SO_QR(v, 1, 5, 9, 13);
        SO_QR(v, 2, 6, 10, 14);
        SO_QR(v, 3, 7, 11, 15);
        /* diagonal round :97-101 */
        SO_QR(v, 0, 5, 10, 15);
        SO_QR(v, 1, 6, 11, 12);
        SO_QR(v, 2, 7, 8, 13);
        SO_QR(v, 3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) out[i] = v[i] + in[i]; /* :104-106 */
}

/* chacha20.rs:111-135 */
void so_chacha20_next(so_chacha20* st, uint8_t out[64]) {
    uint32_t next[16];
    round20(st->vals, next);
    st->vals[12] += 1u; /* :116 -- word 13 never changes */
    for (int i = 0; i < 16; ++i) {
        out[4 * i + 0] = (uint8_t)next[i];
        out[4 * i + 1] = (uint8_t)(next[i] >> 8);
        out[4 * i + 2] = (uint8_t)(next[i] >> 16);
        out[4 * i + 3] = (uint8_t)(next[i] >> 24);
    }
}

/* chacha20.rs:143-153 */
void so_chacha20_encrypt(so_chacha20* st, const uint8_t* in, size_t n, uint8_t* out) {
    uint8_t ks[64];
    for (size_t off = 0; off < n; off += 64) {
        size_t chunk = n - off < 64 ? n - off : 64;
        so_chacha20_next(st, ks);
        for (size_t j = 0; j < chunk; ++j) out[off + j] = in[off + j] ^ ks[j];
    }
}

/* ------------------------------------------------------------------------ */
/* poly1305.rs                                                               */
/* ------------------------------------------------------------------------ */

/* poly1305.rs:35-49 -- limb-wise, no reduction */
so_int1305 so_int1305_add(so_int1305 a, so_int1305 b) {
    so_int1305 r;
    for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i];
    return r;
}

/* poly1305.rs:51-128 */
so_int1305 so_int1305_mult(so_int1305 a, so_int1305 b) {
    const uint32_t b5[5] = {b.v[0] * 5u, b.v[1] * 5u, b.v[2] * 5u, b.v[3] * 5u, b.v[4] * 5u};
#define M(i, j) ((uint64_t)a.v[i] * (uint64_t)b.v[j])
#define M5(i, j) ((uint64_t)a.v[i] * (uint64_t)b5[j])
    uint64_t v[5] = {
        M(0, 0) + M5(1, 4) + M5(2, 3) + M5(3, 2) + M5(4, 1),
        M(0, 1) + M(1, 0) + M5(2, 4) + M5(3, 3) + M5(4, 2),
        M(0, 2) + M(1, 1) + M(2, 0) + M5(3, 4) + M5(4, 3),
        M(0, 3) + M(1, 2) + M(2, 1) + M(3, 0) + M5(4, 4),
        M(0, 4) + M(1, 3) + M(2, 2) + M(3, 1) + M(4, 0),
    };
#undef M
#undef M5
    uint64_t carry = 0;
/* debug_assert_eq!(v[i] >> 32, 0) for every limb (poly1305.rs:87-91, 103-107, 119-123) */
#define LIMBS_FIT_32()                                                              \
    do {                                                                            \
        for (int i_ = 0; i_ < 5; ++i_) SO_DEBUG_ASSERT((v[i_] >> 32) == 0);         \
    } while (0)
#define REDUCE_DIGIT(i)           \
    do {                          \
        v[i] += carry;            \
        carry = v[i] >> 26;       \
        v[i] &= (1ull << 26) - 1; \
    } while (0)
    /* pass 1 :81-85, then the limb and carry bounds of :87-93 */
    REDUCE_DIGIT(0); REDUCE_DIGIT(1); REDUCE_DIGIT(2); REDUCE_DIGIT(3); REDUCE_DIGIT(4);
    LIMBS_FIT_32();
    SO_DEBUG_ASSERT(carry <= 25ull * ((1ull << 26) - 1));
    carry *= 5; /* :95 */
    /* pass 2 :97-101, bounds :103-109 */
    REDUCE_DIGIT(0); REDUCE_DIGIT(1); REDUCE_DIGIT(2); REDUCE_DIGIT(3); REDUCE_DIGIT(4);
    LIMBS_FIT_32();
    SO_DEBUG_ASSERT(carry <= 1);
    carry *= 5; /* :111 */
    /* pass 3 :113-117, bounds :119-125 */
    REDUCE_DIGIT(0); REDUCE_DIGIT(1); REDUCE_DIGIT(2); REDUCE_DIGIT(3); REDUCE_DIGIT(4);
    LIMBS_FIT_32();
    SO_DEBUG_ASSERT(carry == 0);
#undef LIMBS_FIT_32
#undef REDUCE_DIGIT
    so_int1305 r = {{(uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3],
                     (uint32_t)v[4]}};
    return r;
}

/* poly1305.rs:130-162 -- 26-bit slices of 16 little-endian bytes */
so_int1305 so_int1305_from_bytes(const uint8_t m[16]) {
#define B4(i, n)                                                     \
    (((uint32_t)m[i] >> (n)) | ((uint32_t)m[(i) + 1] << (8 - (n))) | \
     ((uint32_t)m[(i) + 2] << (16 - (n))) |                          \
     (((uint32_t)m[(i) + 3] & ((1u << (2 + (n))) - 1)) << (24 - (n))))
#define B3(i, n)                                                     \
    (((uint32_t)m[i] >> (n)) | ((uint32_t)m[(i) + 1] << (8 - (n))) | \
     ((uint32_t)m[(i) + 2] << (16 - (n))))
    so_int1305 r = {{B4(0, 0), B4(3, 26 * 1 - 8 * 3), B4(6, 26 * 2 - 8 * 6),
                     B4(9, 26 * 3 - 8 * 9), B3(13, 0)}};
#undef B4
#undef B3
    for (int i = 0; i < 5; ++i) SO_DEBUG_ASSERT((r.v[i] >> 26) == 0);
    return r;
}

/* poly1305.rs:5-19, :31 choose: flag ? b : a, branch-free */
static so_int1305 choose(uint32_t flag, so_int1305 a, so_int1305 b) {
    so_int1305 r;
    for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] ^ (flag * (a.v[i] ^ b.v[i]));
    return r;
}

/* poly1305.rs:165-192 */
so_int1305 so_int1305_normalize(so_int1305 a) {
    static const uint64_t P5[5] = {5, 0, 0, 0, ((1ull << 6) - 1) << 26};
    so_int1305 ret_b = {{0, 0, 0, 0, 0}};
    uint64_t carry = 0;
    for (int i = 0; i < 4; ++i) {
        uint64_t v = (uint64_t)a.v[i] + P5[i] + carry;
        carry = v >> 26;
        ret_b.v[i] = (uint32_t)(v & ((1ull << 26) - 1));
    }
    ret_b.v[4] = (uint32_t)((uint64_t)a.v[4] + P5[4] + carry);
    uint32_t is_case_b = ret_b.v[4] >> 31;
    return choose(is_case_b, ret_b, a);
}

/* poly1305.rs:195-315 */
void so_poly1305_authenticate(const uint8_t* msg, size_t len, const uint8_t r_in[16],
                              const uint8_t aes[16], uint8_t tag[16]) {
    uint8_t rb[16];
    memcpy(rb, r_in, 16);
    /* clamp :197-203 */
    rb[3] &= 15; rb[4] &= 252; rb[7] &= 15; rb[8] &= 252;
    rb[11] &= 15; rb[12] &= 252; rb[15] &= 15;
    const so_int1305 r = so_int1305_from_bytes(rb);

    so_int1305 h = {{0, 0, 0, 0, 0}};
    const size_t chunks = (len + 15) / 16;
    for (size_t i = 0; i < chunks; ++i) { /* :213-228 */
        uint8_t m[16] = {0};
        size_t m_len = i < chunks - 1 ? 16 : len - 16 * i;
        memcpy(m, msg + 16 * i, m_len);
        so_int1305 c = so_int1305_from_bytes(m);
        size_t flag_pos = m_len * 8; /* append 1 :224-225 */
        c.v[flag_pos / 26] |= 1u << (flag_pos % 26);
        h = so_int1305_mult(so_int1305_add(c, h), r);
    }

    h = so_int1305_normalize(h); /* :230 */
    /* serialize mod 2^128 :231-264 */
    const uint32_t* v = h.v;
    uint8_t hb[16] = {
        (uint8_t)(v[0]), (uint8_t)(v[0] >> 8), (uint8_t)(v[0] >> 16),
        (uint8_t)((v[0] >> 24) | ((v[1] & 63u) << 2)),
        (uint8_t)(v[1] >> 6), (uint8_t)(v[1] >> 14),
        (uint8_t)((v[1] >> 22) | ((v[2] & 15u) << 4)),
        (uint8_t)(v[2] >> 4), (uint8_t)(v[2] >> 12),
        (uint8_t)((v[2] >> 20) | ((v[3] & 3u) << 6)),
        (uint8_t)(v[3] >> 2), (uint8_t)(v[3] >> 10), (uint8_t)(v[3] >> 18),
        (uint8_t)(v[4]), (uint8_t)(v[4] >> 8), (uint8_t)(v[4] >> 16),
    };
    /* h + aes (mod 2^128) with a 32-bit carry chain :266-312 */
    uint64_t carry = 0;
    for (int w = 0; w < 4; ++w) {
        uint64_t sum = (uint64_t)le32(hb + 4 * w) + (uint64_t)le32(aes + 4 * w) + carry;
        uint32_t rw = (uint32_t)sum;
        carry = sum >> 32;
        tag[4 * w + 0] = (uint8_t)rw;
        tag[4 * w + 1] = (uint8_t)(rw >> 8);
        tag[4 * w + 2] = (uint8_t)(rw >> 16);
        tag[4 * w + 3] = (uint8_t)(rw >> 24);
    }
}

/* ------------------------------------------------------------------------ */
/* chacha20_poly1305.rs                                                      */
/* ------------------------------------------------------------------------ */

/* :19-42 -- msg = ad || le64(|ad|) || ct || le64(|ct|), no padding
 * (draft-agl-tls-chacha20poly1305-04 "data first, length later") */
void so_compute_mac(const uint8_t poly_key[32], const uint8_t* ct, size_t n,
                    const uint8_t* ad, size_t adlen, uint8_t tag[16]) {
    size_t len = adlen + 8 + n + 8;
    uint8_t* msg = (uint8_t*)malloc(len);
    if (adlen) memcpy(msg, ad, adlen);
    so_u64_le((uint64_t)adlen, msg + adlen);
    if (n) memcpy(msg + adlen + 8, ct, n);
    so_u64_le((uint64_t)n, msg + adlen + 8 + n);
    /* r = pk[0..16], s = pk[16..32] (:32-39) */
    so_poly1305_authenticate(msg, len, poly_key, poly_key + 16, tag);
    free(msg);
}

/* :48-59 */
void so_seal(const uint8_t key[32], const uint8_t nonce[8], const uint8_t* pt, size_t n,
             const uint8_t* ad, size_t adlen, uint8_t* out) {
    so_chacha20 st;
    uint8_t pk[64];
    so_chacha20_new(&st, key, 32, nonce, 8);
    so_chacha20_next(&st, pk);            /* block 0 = poly1305 key */
    so_chacha20_encrypt(&st, pt, n, out); /* blocks 1.. */
    so_compute_mac(pk, out, n, ad, adlen, out + n);
}

/* :65-94 */
int so_open(const uint8_t key[32], const uint8_t nonce[8], const uint8_t* in, size_t in_len,
            const uint8_t* ad, size_t adlen, uint8_t* out) {
    if (in_len < SO_MAC_LEN) return SO_SHORT; /* :68-70 */
    size_t n = in_len - SO_MAC_LEN;
    so_chacha20 st;
    uint8_t pk[64], mac[16];
    so_chacha20_new(&st, key, 32, nonce, 8);
    so_chacha20_next(&st, pk);
    so_compute_mac(pk, in, n, ad, adlen, mac);
    so_chacha20_encrypt(&st, in, n, out); /* always decrypt :80-82 */
    uint8_t diff = 0;                     /* constant-time OR of XORs :84-87 */
    for (int i = 0; i < SO_MAC_LEN; ++i) diff |= mac[i] ^ in[n + i];
    return diff != 0 ? SO_BAD_MAC : SO_OK;
}

/* ------------------------------------------------------------------------ */
/* synthetic workload + batch driver                                         */
/* ------------------------------------------------------------------------ */

uint64_t so_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void so_fill_record(uint64_t seed, uint64_t j, uint8_t* buf, size_t n) {
    for (size_t i = 0; i < n; i += 8) {
        uint64_t w = so_splitmix64(seed ^ (j << 32) ^ (uint64_t)(i / 8));
        for (size_t b = 0; b < 8 && i + b < n; ++b) buf[i + b] = (uint8_t)(w >> (8 * b));
    }
}

/* The batch drivers below run on the persistent pool of so_pool.h (one
 * contiguous record range per thread); the reference itself is single-threaded
 * per connection (cipher/mod.rs:18-23), so threads stand for independent
 * connections/records. */
typedef struct {
    const uint8_t* key;
    uint64_t seq0;
    const uint8_t* in;
    uint8_t* out;
    uint8_t* status;
    size_t n, count;
    size_t bad[SP_MAX_THREADS];
    int open;
} so_job;

static void so_batch_task(void* arg, int t, int nt) {
    so_job* j = (so_job*)arg;
    uint8_t nonce[8], ad[13];
    size_t begin, end, bad = 0;
    sp_range(j->count, t, nt, &begin, &end);
    for (size_t i = begin; i < end; ++i) {
        uint64_t seq = j->seq0 + i;
        so_u64_be(seq, nonce); /* tls.rs:103 */
        so_tls_ad(seq, 23, 3, 3, (uint16_t)j->n, ad);
        if (!j->open) {
            so_seal(j->key, nonce, j->in + i * j->n, j->n, ad, 13, j->out + i * (j->n + 16));
        } else {
            int st = so_open(j->key, nonce, j->in + i * (j->n + 16), j->n + 16, ad, 13,
                             j->out + i * j->n);
            if (j->status) j->status[i] = (uint8_t)st;
            if (st != SO_OK) bad++;
        }
    }
    j->bad[t] = bad;
}

static size_t so_run(const uint8_t key[32], uint64_t seq0, const uint8_t* in, size_t n,
                     size_t count, uint8_t* out, uint8_t* status, int threads, int open) {
    if (threads < 1) threads = 1;
    if (count > 0 && (size_t)threads > count) threads = (int)count;
    if (threads > SP_MAX_THREADS) threads = SP_MAX_THREADS;
    so_job* j = (so_job*)calloc(1, sizeof(so_job));
    j->key = key; j->seq0 = seq0; j->in = in; j->out = out; j->status = status;
    j->n = n; j->count = count; j->open = open;
    sp_run(so_batch_task, j, threads);
    size_t bad = 0;
    for (int t = 0; t < threads; ++t) bad += j->bad[t];
    free(j);
    return bad;
}

void so_seal_batch_tls(const uint8_t key[32], uint64_t seq0, const uint8_t* pt, size_t n,
                       size_t count, uint8_t* ct, int threads) {
    so_run(key, seq0, pt, n, count, ct, NULL, threads, 0);
}

size_t so_open_batch_tls(const uint8_t key[32], uint64_t seq0, const uint8_t* ct, size_t n,
                         size_t count, uint8_t* pt, uint8_t* status, int threads) {
    return so_run(key, seq0, ct, n, count, pt, status, threads, 1);
}

/* Mixed TLS batch (C2 shape): record i = in[in_off[i], + lens[i]) (seal: the
 * plaintext; open: ct || tag, lens[i] >= 16 counting the tag) with key
 * keys[32 key_index[i]] and sequence number seq[i], output at out + out_off[i].
 * Returns the number of records whose open status != SO_OK (open only). */
typedef struct {
    const uint8_t* keys;
    const uint32_t* key_index;
    const uint64_t* seq;
    const uint32_t* lens;
    const uint64_t* in_off;
    const uint64_t* out_off;
    const uint8_t* in;
    uint8_t* out;
    uint8_t* status;
    size_t count;
    size_t bad[SP_MAX_THREADS];
    int open;
} so_mjob;

static void so_mixed_task(void* arg, int t, int nt) {
    so_mjob* j = (so_mjob*)arg;
    uint8_t nonce[8], ad[13];
    size_t begin, end, bad = 0;
    sp_range(j->count, t, nt, &begin, &end);
    for (size_t i = begin; i < end; ++i) {
        const uint8_t* key = j->keys + 32u * j->key_index[i];
        const size_t len = j->lens[i];
        so_u64_be(j->seq[i], nonce);
        if (!j->open) {
            so_tls_ad(j->seq[i], 23, 3, 3, (uint16_t)len, ad);
            so_seal(key, nonce, j->in + j->in_off[i], len, ad, 13, j->out + j->out_off[i]);
        } else {
            so_tls_ad(j->seq[i], 23, 3, 3, (uint16_t)(len >= 16 ? len - 16 : 0), ad);
            int st = so_open(key, nonce, j->in + j->in_off[i], len, ad, 13, j->out + j->out_off[i]);
            if (j->status) j->status[i] = (uint8_t)st;
            if (st != SO_OK) bad++;
        }
    }
    j->bad[t] = bad;
}

size_t so_batch_mixed(int open, const uint8_t* keys, const uint32_t* key_index, const uint64_t* seq,
                      const uint32_t* lens, const uint64_t* in_off, const uint64_t* out_off, const uint8_t* in,
                      uint8_t* out, uint8_t* status, size_t count, int threads) {
    if (threads < 1) threads = 1;
    if (count > 0 && (size_t)threads > count) threads = (int)count;
    if (threads > SP_MAX_THREADS) threads = SP_MAX_THREADS;
    so_mjob* j = (so_mjob*)calloc(1, sizeof(so_mjob));
    j->keys = keys; j->key_index = key_index; j->seq = seq; j->lens = lens; j->in_off = in_off;
    j->out_off = out_off; j->in = in; j->out = out; j->status = status; j->count = count; j->open = open;
    sp_run(so_mixed_task, j, threads);
    size_t bad = 0;
    for (int t = 0; t < threads; ++t) bad += j->bad[t];
    free(j);
    return bad;
}

/* XOR-fold of the tags of `count` TLS records sealed with seq = seq0 + i and
 * plaintext record j0 + i of the fill rule (so_fill_record), computed without
 * materialising the batch: the checker of a full-size device run (bench.py
 * folds the device's tags the same way).  Test infrastructure only. */
typedef struct {
    const uint8_t* key;
    uint64_t seq0, seed, j0;
    size_t n, count;
    uint8_t fold[SP_MAX_THREADS][16];
} so_fold_job;

static void so_fold_task(void* arg, int t, int nt) {
    so_fold_job* j = (so_fold_job*)arg;
    uint8_t* pt = (uint8_t*)malloc(j->n ? j->n : 1);
    uint8_t* ct = (uint8_t*)malloc(j->n + 16);
    uint8_t nonce[8], ad[13];
    size_t begin, end;
    sp_range(j->count, t, nt, &begin, &end);
    memset(j->fold[t], 0, 16);
    for (size_t i = begin; i < end; ++i) {
        uint64_t seq = j->seq0 + i;
        so_fill_record(j->seed, j->j0 + i, pt, j->n);
        so_u64_be(seq, nonce);
        so_tls_ad(seq, 23, 3, 3, (uint16_t)j->n, ad);
        so_seal(j->key, nonce, pt, j->n, ad, 13, ct);
        for (int b = 0; b < 16; ++b) j->fold[t][b] ^= ct[j->n + b];
    }
    free(pt);
    free(ct);
}

void so_tag_fold_tls(const uint8_t key[32], uint64_t seq0, uint64_t seed, uint64_t j0, size_t n, size_t count,
                     int threads, uint8_t out[16]) {
    if (threads < 1) threads = 1;
    if (count > 0 && (size_t)threads > count) threads = (int)count;
    if (threads > SP_MAX_THREADS) threads = SP_MAX_THREADS;
    so_fold_job* j = (so_fold_job*)calloc(1, sizeof(so_fold_job));
    j->key = key; j->seq0 = seq0; j->seed = seed; j->j0 = j0; j->n = n; j->count = count;
    sp_run(so_fold_task, j, threads);
    memset(out, 0, 16);
    for (int t = 0; t < threads; ++t)
        for (int b = 0; b < 16; ++b) out[b] ^= j->fold[t][b];
    free(j);
}

/* XOR-fold of the tags of a mixed TLS batch (C2 shape): record i is
 * pt[in_off[i] .. + lens[i]) sealed with key keys[key_index[i]] and sequence
 * number seq[i] (tls.rs:103-112, chacha20_poly1305.rs:48-59).  The checker of
 * bench.py's full-size C2 run.  Test infrastructure only. */
typedef struct {
    const uint8_t* keys;
    const uint32_t* key_index;
    const uint64_t* seq;
    const uint32_t* lens;
    const uint64_t* in_off;
    const uint8_t* pt;
    size_t count;
    uint8_t fold[SP_MAX_THREADS][16];
} so_mfold_job;

static void so_mfold_task(void* arg, int t, int nt) {
    so_mfold_job* j = (so_mfold_job*)arg;
    uint8_t* ct = (uint8_t*)malloc(65536 + 16);
    uint8_t nonce[8], ad[13];
    size_t begin, end;
    sp_range(j->count, t, nt, &begin, &end);
    memset(j->fold[t], 0, 16);
    for (size_t i = begin; i < end; ++i) {
        const size_t n = j->lens[i];
        so_u64_be(j->seq[i], nonce);
        so_tls_ad(j->seq[i], 23, 3, 3, (uint16_t)n, ad);
        so_seal(j->keys + 32u * j->key_index[i], nonce, j->pt + j->in_off[i], n, ad, 13, ct);
        for (int b = 0; b < 16; ++b) j->fold[t][b] ^= ct[n + b];
    }
    free(ct);
}

void so_tag_fold_mixed(const uint8_t* keys, const uint32_t* key_index, const uint64_t* seq, const uint32_t* lens,
                       const uint64_t* in_off, const uint8_t* pt, size_t count, int threads, uint8_t out[16]) {
    if (threads < 1) threads = 1;
    if (count > 0 && (size_t)threads > count) threads = (int)count;
    if (threads > SP_MAX_THREADS) threads = SP_MAX_THREADS;
    so_mfold_job* j = (so_mfold_job*)calloc(1, sizeof(so_mfold_job));
    j->keys = keys; j->key_index = key_index; j->seq = seq; j->lens = lens; j->in_off = in_off; j->pt = pt;
    j->count = count;
    sp_run(so_mfold_task, j, threads);
    memset(out, 0, 16);
    for (int t = 0; t < threads; ++t)
        for (int b = 0; b < 16; ++b) out[b] ^= j->fold[t][b];
    free(j);
}
