/*
 * suruga_oracle.h -- CPU restatement of suruga's record-layer AEAD.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X path,
 * never the product: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The shipped library (libsuruga_gpu.so) does
 * not link it and has no CPU fallback.
 *
 * Restates, limb for limb, the reference (klutzy/suruga, Rust):
 *   src/crypto/chacha20.rs:25-153      ChaCha20 (state, round20, next, encrypt)
 *   src/crypto/poly1305.rs:25-315      Int1305 radix-2^26 + authenticate
 *   src/cipher/chacha20_poly1305.rs    compute_mac / encrypt / decrypt
 *   src/tls.rs:103-112, 250-265        nonce = be64(seq), 13-byte AD
 *   src/util.rs:43-49                  u64_be_array / u64_le_array
 *
 * Pinned by the reference's own known-answer tests (chacha20.rs:169-228,
 * poly1305.rs:354-458), committed under tests/golden/, and cross-checked
 * against OpenSSL libcrypto primitives by tests/golden/make_golden.py.
 */
#ifndef SURUGA_ORACLE_H
#define SURUGA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- ChaCha20 (chacha20.rs) ------------------------------------------- */
typedef struct { uint32_t vals[16]; } so_chacha20;

/* chacha20.rs:25-51.  key 32 B, nonce 8 B (returns -1 on bad lengths where
 * the reference would panic, :26-27). */
int  so_chacha20_new(so_chacha20* st, const uint8_t* key, size_t key_len,
                     const uint8_t* nonce, size_t nonce_len);
/* chacha20.rs:111-135: one 64-byte keystream block, then vals[12] += 1
 * (mod 2^32, no carry into vals[13]). */
void so_chacha20_next(so_chacha20* st, uint8_t out[64]);
/* chacha20.rs:143-153: XOR data with the stream in 64-byte chunks; the
 * surplus keystream of a partial chunk is discarded. */
void so_chacha20_encrypt(so_chacha20* st, const uint8_t* in, size_t n, uint8_t* out);

/* ---- Poly1305 (poly1305.rs) ------------------------------------------- */
typedef struct { uint32_t v[5]; } so_int1305;
so_int1305 so_int1305_add(so_int1305 a, so_int1305 b);        /* :35-49   */
so_int1305 so_int1305_mult(so_int1305 a, so_int1305 b);       /* :51-128  */
so_int1305 so_int1305_from_bytes(const uint8_t m[16]);        /* :130-162 */
so_int1305 so_int1305_normalize(so_int1305 a);                /* :165-192 */
/* :195-315 */
void so_poly1305_authenticate(const uint8_t* msg, size_t len, const uint8_t r[16],
                              const uint8_t s[16], uint8_t tag[16]);

/* ---- AEAD (chacha20_poly1305.rs) --------------------------------------- */
#define SO_KEY_LEN 32
#define SO_MAC_LEN 16
#define SO_OK 0
#define SO_BAD_MAC 1   /* "wrong mac"          chacha20_poly1305.rs:89-90 */
#define SO_SHORT 2     /* "message too short"  chacha20_poly1305.rs:68-70 */

/* :19-42 */
void so_compute_mac(const uint8_t poly_key[32], const uint8_t* ct, size_t n,
                    const uint8_t* ad, size_t adlen, uint8_t tag[16]);
/* :48-59  out must hold n + 16 bytes (ct || tag). */
void so_seal(const uint8_t key[32], const uint8_t nonce[8], const uint8_t* pt, size_t n,
             const uint8_t* ad, size_t adlen, uint8_t* out);
/* :65-94  in = ct || tag (in_len >= 16); out holds in_len - 16 bytes and is
 * ALWAYS written (the reference decrypts before comparing, :80-82).
 * Returns SO_OK, SO_BAD_MAC or SO_SHORT. */
int  so_open(const uint8_t key[32], const uint8_t nonce[8], const uint8_t* in, size_t in_len,
             const uint8_t* ad, size_t adlen, uint8_t* out);

/* ---- TLS record-layer contract (tls.rs, util.rs) ----------------------- */
void so_u64_be(uint64_t x, uint8_t out[8]);                           /* util.rs:43-45 */
void so_u64_le(uint64_t x, uint8_t out[8]);                           /* util.rs:47-49 */
/* tls.rs:103-112 (write) and :250-265 (read): be64(seq) || type || major ||
 * minor || be16(frag_len). */
void so_tls_ad(uint64_t seq, uint8_t content_type, uint8_t major, uint8_t minor,
               uint16_t frag_len, uint8_t ad[13]);

/* ---- synthetic workload generator shared with the GPU bench ------------ */
/* byte i of record j = byte (i mod 8) of splitmix64(seed ^ (j << 32) ^ (i / 8)). */
uint64_t so_splitmix64(uint64_t x);
void so_fill_record(uint64_t seed, uint64_t j, uint8_t* buf, size_t n);

/* ---- multi-threaded batch driver (CPU baseline) ------------------------ */
/* TLS mode batch over `count` records of `n` bytes each, laid out densely
 * (pt stride n, ct stride n + 16).  Record i uses key, seq = seq0 + i,
 * AD = so_tls_ad(seq, 23, 3, 3, n).  Returns the number of records whose
 * open status != SO_OK (open only). */
void   so_seal_batch_tls(const uint8_t key[32], uint64_t seq0, const uint8_t* pt,
                         size_t n, size_t count, uint8_t* ct, int threads);
size_t so_open_batch_tls(const uint8_t key[32], uint64_t seq0, const uint8_t* ct,
                         size_t n, size_t count, uint8_t* pt, uint8_t* status, int threads);

/* Mixed TLS batch (C2 shape, the CPU baseline of bench.py --workload c2):
 * record i = in[in_off[i], + lens[i]) (open: ct || tag, lens[i] counting the
 * tag), key keys[32 key_index[i]], sequence number seq[i], output at
 * out + out_off[i].  Returns the number of failed opens. */
size_t so_batch_mixed(int open, const uint8_t* keys, const uint32_t* key_index, const uint64_t* seq,
                      const uint32_t* lens, const uint64_t* in_off, const uint64_t* out_off, const uint8_t* in,
                      uint8_t* out, uint8_t* status, size_t count, int threads);

/* XOR-fold of the tags of count TLS records (seq = seq0 + i, plaintext =
 * fill-rule record j0 + i) without materialising them. */
void so_tag_fold_tls(const uint8_t key[32], uint64_t seq0, uint64_t seed, uint64_t j0, size_t n, size_t count,
                     int threads, uint8_t out[16]);
/* XOR-fold of the tags of a mixed batch: record i = pt[in_off[i], + lens[i]),
 * key keys[32 key_index[i]], sequence number seq[i] (TLS nonce and AD). */
void so_tag_fold_mixed(const uint8_t* keys, const uint32_t* key_index, const uint64_t* seq, const uint32_t* lens,
                       const uint64_t* in_off, const uint8_t* pt, size_t count, int threads, uint8_t out[16]);

#ifdef __cplusplus
}
#endif

#endif
