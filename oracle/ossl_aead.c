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
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    EVP_CIPHER_CTX* c;
    EVP_MAC_CTX* m;
} ossl_ctx;

static int ossl_init(ossl_ctx* x, EVP_MAC* mac) {
    x->c = EVP_CIPHER_CTX_new();
    x->m = EVP_MAC_CTX_new(mac);
    return x->c && x->m;
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
    EVP_EncryptInit_ex(x->c, EVP_chacha20(), NULL, key, iv);
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

typedef struct {
    const uint8_t* key;
    uint64_t seq0;
    const uint8_t* in;
    uint8_t* out;
    size_t n, begin, end, bad;
    int open;
    EVP_MAC* mac;
} job;

static void* worker(void* arg) {
    job* j = (job*)arg;
    ossl_ctx x;
    if (!ossl_init(&x, j->mac)) {
        j->bad = (size_t)-1;
        return NULL;
    }
    uint8_t nonce[8], ad[13];
    for (size_t i = j->begin; i < j->end; ++i) {
        tls_nonce_ad(j->seq0 + i, j->n, nonce, ad);
        if (!j->open)
            ossl_seal(&x, j->key, nonce, j->in + i * j->n, j->n, ad, 13, j->out + i * (j->n + 16));
        else if (ossl_open(&x, j->key, nonce, j->in + i * (j->n + 16), j->n + 16, ad, 13, j->out + i * j->n))
            j->bad++;
    }
    ossl_free(&x);
    return NULL;
}

/* TLS-mode batch (same layout and nonce/AD rules as so_*_batch_tls).  Returns
 * the number of records that failed to open (open), or (size_t)-1 when
 * libcrypto cannot provide POLY1305. */
size_t ossl_batch_tls(int open, const uint8_t key[32], uint64_t seq0, const uint8_t* in, size_t n, size_t count,
                      uint8_t* out, int threads) {
    EVP_MAC* m = EVP_MAC_fetch(NULL, "POLY1305", NULL);
    if (!m) return (size_t)-1;
    if (threads < 1) threads = 1;
    if (count > 0 && (size_t)threads > count) threads = (int)count;
    job* jobs = (job*)calloc((size_t)threads, sizeof(job));
    pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    size_t per = (count + (size_t)threads - 1) / (size_t)threads, bad = 0;
    for (int t = 0; t < threads; ++t) {
        job* j = &jobs[t];
        j->key = key; j->seq0 = seq0; j->in = in; j->out = out; j->n = n; j->open = open; j->mac = m;
        j->begin = (size_t)t * per < count ? (size_t)t * per : count;
        j->end = j->begin + per < count ? j->begin + per : count;
        if (threads == 1) worker(j);
        else pthread_create(&tids[t], NULL, worker, j);
    }
    for (int t = 0; t < threads; ++t) {
        if (threads > 1) pthread_join(tids[t], NULL);
        if (jobs[t].bad == (size_t)-1) bad = (size_t)-1;
        else if (bad != (size_t)-1) bad += jobs[t].bad;
    }
    free(jobs);
    free(tids);
    EVP_MAC_free(m);
    return bad;
}
