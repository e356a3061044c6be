/*
 * ossl_aead.c -- an OPTIMISED-CPU comparison line for bench.py (SURVEY.md 8d,
 * "optional second CPU reference line"): suruga's AEAD composed from OpenSSL
 * 3.0 libcrypto primitives.  TEST / BENCHMARK INFRASTRUCTURE ONLY: the product
 * never links it, and parity is still judged against suruga_oracle.c.
 *
 *   keystream: EVP_chacha20 with the 16-byte IV le32(counter) || 0^4 || nonce8
 *              reproduces suruga's state (counter in word 12, word 13 = 0,
 *              nonce in words 14-15; chacha20.rs:25-51).  Counter 0 gives the
 *              Poly1305 key (chacha20_poly1305.rs:50), data uses 1.. (:52).
 *   MAC:       EVP_MAC "POLY1305" keyed with pk[0..32] over
 *              ad || le64(|ad|) || ct || le64(|ct|) (chacha20_poly1305.rs:19-42).
 *   open:      always decrypts, then compares the tag (:65-94).
 * OpenSSL's own EVP_chacha20_poly1305 is the RFC 7539 construction and does
 * NOT match suruga; it is not used.
 */
#include <openssl/core_names.h>
#include <openssl/evp.h>
#include <pthread.h>

#include "so_pool.h"
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    EVP_CIPHER_CTX* c;
    EVP_MAC_CTX* m;
} ossl_ctx;

/* Every thread keeps one cipher and one MAC context for its whole slice,
 * re-keyed per record with init only.  (Round 2 re-initialised with
 * EVP_chacha20() per record: an implicit fetch on OpenSSL 3's global store
 * whose lock serialised the threads.)  Round 4: the cipher and MAC methods are
 * fetched from a library context of the thread's own (created once per pool
 * thread).  With one shared fetch, every EVP_EncryptInit_ex2 re-key touched
 * the same method object: 0.26 us per 64-byte re-key on one thread but 1.67 us
 * per thread with 8 threads (cache-line ping-pong on its shared state), which
 * capped the C2 line (small records: ~2 inits per record) at 0.17 scaling
 * efficiency; per-thread library contexts measured 0.26 -> 0.30 us. */
typedef struct {
    OSSL_LIB_CTX* lib;
    EVP_CIPHER* cipher;
    EVP_MAC* mac;
} tl_methods;
static __thread tl_methods tl_m;

/* The thread's contexts are freed when the thread exits (pthread key
 * destructor): the pool threads live as long as the process, but every other
 * thread that calls in (thread 0 of a batch is the caller) would otherwise
 * leak one library context. */
static pthread_key_t tl_key;
static pthread_once_t tl_key_once = PTHREAD_ONCE_INIT;
static void tl_free(void* v) {
    tl_methods* m = (tl_methods*)v;
    EVP_CIPHER_free(m->cipher);
    EVP_MAC_free(m->mac);
    OSSL_LIB_CTX_free(m->lib);
    m->cipher = NULL;
    m->mac = NULL;
    m->lib = NULL;
}
static void tl_key_make(void) { (void)pthread_key_create(&tl_key, tl_free); }

static int tl_fetch(void) {
    if (tl_m.lib == NULL) {
        pthread_once(&tl_key_once, tl_key_make);
        tl_m.lib = OSSL_LIB_CTX_new();
        if (tl_m.lib == NULL) return 0;
        tl_m.cipher = EVP_CIPHER_fetch(tl_m.lib, "ChaCha20", NULL);
        tl_m.mac = EVP_MAC_fetch(tl_m.lib, "POLY1305", NULL);
        (void)pthread_setspecific(tl_key, &tl_m);
    }
    return tl_m.cipher != NULL && tl_m.mac != NULL;
}

static int ossl_init(ossl_ctx* x, EVP_CIPHER* cipher, EVP_MAC* mac) {
    x->c = EVP_CIPHER_CTX_new();
    x->m = EVP_MAC_CTX_new(mac);
    return x->c && x->m && EVP_EncryptInit_ex2(x->c, cipher, NULL, NULL, NULL) == 1;
}

static void ossl_free(ossl_ctx* x) {
    EVP_CIPHER_CTX_free(x->c);
    EVP_MAC_CTX_free(x->m);
}

static void keystream_xor(ossl_ctx* x, const uint8_t key[32], const uint8_t nonce[8], uint32_t ctr,
                          const uint8_t* in, size_t n, uint8_t* out) {
    uint8_t iv[16] = {(uint8_t)ctr, (uint8_t)(ctr >> 8), (uint8_t)(ctr >> 16), (uint8_t)(ctr >> 24), 0, 0, 0, 0};
    memcpy(iv + 8, nonce, 8);
    int len = 0;
    EVP_EncryptInit_ex2(x->c, NULL, key, iv, NULL);  /* same cipher, new key / IV */
    EVP_EncryptUpdate(x->c, out, &len, in, (int)n);
}

static void le64(uint64_t v, uint8_t o[8]) {
    for (int i = 0; i < 8; ++i) o[i] = (uint8_t)(v >> (8 * i));
}

static void mac(ossl_ctx* x, const uint8_t pk[32], const uint8_t* ad, size_t adlen, const uint8_t* ct, size_t n,
                uint8_t tag[16]) {
    uint8_t l[8];
    size_t outl = 0;
    EVP_MAC_init(x->m, pk, 32, NULL);
    EVP_MAC_update(x->m, ad, adlen);
    le64(adlen, l);
    EVP_MAC_update(x->m, l, 8);
    if (n) EVP_MAC_update(x->m, ct, n);
    le64(n, l);
    EVP_MAC_update(x->m, l, 8);
    EVP_MAC_final(x->m, tag, &outl, 16);
}

static void tls_nonce_ad(uint64_t seq, size_t n, uint8_t nonce[8], uint8_t ad[13]) {
    for (int i = 0; i < 8; ++i) nonce[i] = (uint8_t)(seq >> (56 - 8 * i)); /* tls.rs:103 */
    memcpy(ad, nonce, 8);
    ad[8] = 23;
    ad[9] = 3;
    ad[10] = 3;
    ad[11] = (uint8_t)(n >> 8);
    ad[12] = (uint8_t)n;
}

static const uint8_t kZero[64];

int ossl_seal(ossl_ctx* x, const uint8_t key[32], const uint8_t nonce[8], const uint8_t* pt, size_t n,
              const uint8_t* ad, size_t adlen, uint8_t* out) {
    uint8_t pk[64];
    keystream_xor(x, key, nonce, 0, kZero, 64, pk);
    keystream_xor(x, key, nonce, 1, pt, n, out);
    mac(x, pk, ad, adlen, out, n, out + n);
    return 0;
}

int ossl_open(ossl_ctx* x, const uint8_t key[32], const uint8_t nonce[8], const uint8_t* in, size_t in_len,
              const uint8_t* ad, size_t adlen, uint8_t* out) {
    if (in_len < 16) return 2;
    const size_t n = in_len - 16;
    uint8_t pk[64], tag[16];
    keystream_xor(x, key, nonce, 0, kZero, 64, pk);
    mac(x, pk, ad, adlen, in, n, tag);
    keystream_xor(x, key, nonce, 1, in, n, out);
    uint8_t diff = 0;
    for (int i = 0; i < 16; ++i) diff |= (uint8_t)(tag[i] ^ in[n + i]);
    return diff ? 1 : 0;
}

/* One batch: uniform TLS records (lens == NULL: record i at in + i * stride_in,
 * n bytes) or a mixed batch (record i at in + in_off[i], lens[i] bytes, key
 * keys[32 key_index[i]], seq[i]). */
typedef struct {
    const uint8_t* keys;
    const uint32_t* key_index;
    const uint64_t* seq;
    const uint32_t* lens;
    const uint64_t* in_off;
    const uint64_t* out_off;
    uint64_t seq0;
    const uint8_t* in;
    uint8_t* out;
    size_t n, count;
    int open;
    EVP_CIPHER* cipher;
    EVP_MAC* mac;
    size_t bad[SP_MAX_THREADS];
} job;

static void task(void* arg, int t, int nt) {
    job* j = (job*)arg;
    size_t begin, end, bad = 0;
    sp_range(j->count, t, nt, &begin, &end);
    ossl_ctx x = {NULL, NULL};
    if (!tl_fetch() || !ossl_init(&x, tl_m.cipher, tl_m.mac)) {
        ossl_free(&x);
        j->bad[t] = (size_t)-1;
        return;
    }
    uint8_t nonce[8], ad[13];
    for (size_t i = begin; i < end; ++i) {
        const uint8_t* key = j->lens ? j->keys + 32u * j->key_index[i] : j->keys;
        const uint64_t seq = j->lens ? j->seq[i] : j->seq0 + i;
        const size_t len = j->lens ? j->lens[i] : (j->open ? j->n + 16 : j->n);
        const uint8_t* src = j->lens ? j->in + j->in_off[i] : j->in + i * (j->open ? j->n + 16 : j->n);
        uint8_t* dst = j->lens ? j->out + j->out_off[i] : j->out + i * (j->open ? j->n : j->n + 16);
        const size_t n = j->open ? (len >= 16 ? len - 16 : 0) : len;
        tls_nonce_ad(seq, n, nonce, ad);
        if (!j->open)
            ossl_seal(&x, key, nonce, src, n, ad, 13, dst);
        else if (ossl_open(&x, key, nonce, src, len, ad, 13, dst))
            bad++;
    }
    ossl_free(&x);
    j->bad[t] = bad;
}

static size_t run(job* j, int threads) {
    /* availability check on the default context; the threads use their own */
    j->mac = EVP_MAC_fetch(NULL, "POLY1305", NULL);
    j->cipher = EVP_CIPHER_fetch(NULL, "ChaCha20", NULL);
    size_t bad = 0;
    if (!j->mac || !j->cipher) {
        bad = (size_t)-1;
    } else {
        if (threads < 1) threads = 1;
        if (j->count > 0 && (size_t)threads > j->count) threads = (int)j->count;
        if (threads > SP_MAX_THREADS) threads = SP_MAX_THREADS;
        sp_run(task, j, threads);
        for (int t = 0; t < threads; ++t) {
            if (j->bad[t] == (size_t)-1) bad = (size_t)-1;
            else if (bad != (size_t)-1) bad += j->bad[t];
        }
    }
    EVP_MAC_free(j->mac);
    EVP_CIPHER_free(j->cipher);
    return bad;
}

/* TLS-mode batch (same layout and nonce/AD rules as so_*_batch_tls).  Returns
 * the number of records that failed to open (open), or (size_t)-1 when
 * libcrypto cannot provide ChaCha20 / POLY1305. */
size_t ossl_batch_tls(int open, const uint8_t key[32], uint64_t seq0, const uint8_t* in, size_t n, size_t count,
                      uint8_t* out, int threads) {
    job* j = (job*)calloc(1, sizeof(job));
    j->keys = key; j->seq0 = seq0; j->in = in; j->out = out; j->n = n; j->count = count; j->open = open;
    const size_t bad = run(j, threads);
    free(j);
    return bad;
}

/* Mixed TLS batch (same layout as so_batch_mixed). */
size_t ossl_batch_mixed(int open, const uint8_t* keys, const uint32_t* key_index, const uint64_t* seq,
                        const uint32_t* lens, const uint64_t* in_off, const uint64_t* out_off, const uint8_t* in,
                        uint8_t* out, size_t count, int threads) {
    job* j = (job*)calloc(1, sizeof(job));
    j->keys = keys; j->key_index = key_index; j->seq = seq; j->lens = lens; j->in_off = in_off;
    j->out_off = out_off; j->in = in; j->out = out; j->count = count; j->open = open;
    const size_t bad = run(j, threads);
    free(j);
    return bad;
}
