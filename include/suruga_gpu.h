/*
 * suruga_gpu.h -- C ABI of the MI355X (gfx950) ChaCha20-Poly1305 record AEAD.
 *
 * This is the drop-in boundary for suruga's cipher plugin interface
 * (klutzy/suruga src/cipher/mod.rs:14-32).  Every entry point below replaces
 * one item of that interface; the reference-side bindings a maintainer would
 * add are shown in INTEGRATION.md.
 *
 *   Aead::key_size / fixed_iv_len / mac_len      mod.rs:15-17
 *       -> sg_key_size / sg_fixed_iv_len / sg_mac_len
 *          (values from chacha20_poly1305.rs:15-17, 102-119)
 *   Aead::new_encryptor / new_decryptor           mod.rs:18-19, chacha20_poly1305.rs:121-134
 *       -> sg_ctx_new (one context per direction, key moved in) / sg_ctx_free
 *   Encryptor::encrypt(nonce, plain, ad) -> Vec   mod.rs:22-24, chacha20_poly1305.rs:48-59
 *       -> sg_seal   (caller-provided out of n + 16 bytes: ct || tag)
 *   Decryptor::decrypt(nonce, encrypted, ad)      mod.rs:28-31, chacha20_poly1305.rs:65-94
 *       -> sg_open   (returns SG_E_BAD_MAC / SG_E_SHORT where the reference
 *                     returns Err(TlsError{kind: BadRecordMac, ..}))
 *   Decryptor::mac_len                            mod.rs:31, chacha20_poly1305.rs:96-99
 *       -> sg_mac_len
 *   TlsWriter::write_data chunk loop / TlsReader::read_record (tls.rs:99-147,217-281)
 *       -> sg_seal_batch / sg_open_batch: many records per call, nonce and the
 *          13-byte additional data built on the device from the record-layer
 *          rules (tls.rs:103-112, 250-265) in SG_BATCH_TLS mode.
 *
 * Construction: draft-agl-tls-chacha20poly1305-04 as implemented by suruga
 * (64-bit nonce, 32-bit block counter in state word 12 only, Poly1305 key =
 * keystream block 0, MAC over ad || le64(|ad|) || ct || le64(|ct|) with no
 * padding).  NOT RFC 7539.
 *
 * Plain C types only: no HIP or torch types cross this boundary.  Device
 * pointers are passed as plain pointers; a HIP stream as void*.
 */
#ifndef SURUGA_GPU_H
#define SURUGA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
#define SG_OK          0
#define SG_E_BAD_MAC   1   /* tag mismatch: TlsErrorKind::BadRecordMac "wrong mac"
                              (chacha20_poly1305.rs:89-90)                        */
#define SG_E_SHORT     2   /* input shorter than the tag: BadRecordMac "message too
                              short" (chacha20_poly1305.rs:68-70)                 */
#define SG_E_ARG      -1   /* bad argument (lengths, NULL pointers, limits); the
                              reference panics here (chacha20.rs:26-27)           */
#define SG_E_HIP      -2   /* HIP runtime error                                  */
#define SG_E_NODEV    -3   /* no usable gfx950 device                            */

/* ---- limits ------------------------------------------------------------ */
#define SG_KEY_LEN         32u
#define SG_NONCE_LEN        8u
#define SG_MAC_LEN         16u
#define SG_MAX_AD_LEN     255u
/* The size-class kernels (every batch that is not uniform 16 KiB records or
 * a mixed TLS batch of 64-byte multiples) stage a record's MAC stream in LDS,
 * which bounds a record at 32 KiB; the wave-per-record and packed kernels
 * stream their records.  TLS records are at most 2^14 (+2048 expansion) bytes
 * (tls.rs:32-35). */
#define SG_MAX_RECORD_LEN 32768u

/* ---- Aead constants (chacha20_poly1305.rs:15-17, 104-119) --------------- */
size_t sg_key_size(void);     /* 32 */
size_t sg_fixed_iv_len(void); /* 0  */
size_t sg_mac_len(void);      /* 16 */
int    sg_abi_version(void);  /* SG_ABI_VERSION */

/* ---- per-direction context (Aead::new_encryptor / new_decryptor) -------- */
typedef struct sg_ctx sg_ctx;

/* Copies the 32-byte key to device `device` (HIP ordinal).  Returns NULL on
 * failure (sg_last_error() says why). */
sg_ctx* sg_ctx_new(const uint8_t key[32], int device);
void    sg_ctx_free(sg_ctx* ctx);

/* Encryptor::encrypt.  Host pointers.  out receives n + 16 bytes (ct || tag).
 * nonce is 8 bytes (TLS: be64(seq), tls.rs:103).  Returns SG_OK or < 0. */
int sg_seal(sg_ctx* ctx, const uint8_t* nonce, size_t nonce_len,
            const uint8_t* pt, size_t n, const uint8_t* ad, size_t adlen, uint8_t* out);

/* Decryptor::decrypt.  Host pointers.  in = ct || tag (in_len bytes); out
 * receives in_len - 16 bytes of plaintext on SG_OK.  On SG_E_BAD_MAC the
 * plaintext is withheld (out is zero-filled), as the reference returns no
 * plaintext with its Err (chacha20_poly1305.rs:89-93); the decryption itself
 * always runs (:80-82).  Returns SG_OK, SG_E_BAD_MAC, SG_E_SHORT or < 0. */
int sg_open(sg_ctx* ctx, const uint8_t* nonce, size_t nonce_len,
            const uint8_t* in, size_t in_len, const uint8_t* ad, size_t adlen, uint8_t* out);

/* ---- batch interface (record-layer batching point, tls.rs:140) --------- */
#define SG_BATCH_TLS  0x1u  /* nonce = be64(seq_i); ad = be64(seq_i) || content_type ||
                               ver_major || ver_minor || be16(n_i)  (tls.rs:103-112,
                               250-265); `nonces`/`ads` are ignored               */
#define SG_BATCH_KEEP_FAILED 0x2u  /* open: leave the (unauthenticated) plaintext of
                                      records whose status is SG_E_BAD_MAC in `out`.
                                      By default it is zero-filled after the batch, as
                                      the reference hands out no plaintext with its
                                      Err (chacha20_poly1305.rs:89-93; the decryption
                                      itself always runs, :80-82).                   */

typedef struct sg_batch {
    uint32_t count;            /* number of records                                 */
    uint32_t flags;            /* SG_BATCH_*                                        */

    /* keys: key table [num_keys][32] in device memory; record i uses
     * key_index[i] (device array) or key 0 when key_index is NULL.  Indices
     * must be < num_keys; the kernels clamp a larger one to num_keys - 1, so
     * it never reads outside the table (that record's output is meaningless). */
    const uint8_t*  keys;
    uint32_t        num_keys;
    const uint32_t* key_index;

    /* TLS mode: seq_i = seq ? seq[i] : seq0 + i   (device array)            */
    const uint64_t* seq;
    uint64_t        seq0;
    uint8_t         content_type;   /* 23 = application_data (tls.rs:26)     */
    uint8_t         ver_major;      /* 3                                     */
    uint8_t         ver_minor;      /* 3                                     */
    uint8_t         _pad0;

    /* explicit mode: nonce_i = nonces + 8*i; ad_i = ads + ad_stride*i, ad_len
     * bytes (device memory)                                                   */
    const uint8_t*  nonces;
    const uint8_t*  ads;
    uint32_t        ad_len;
    uint32_t        ad_stride;

    /* record layout (device memory).  Record i reads in + in_off_i and writes
     * out + out_off_i, where off_i = off ? off[i] : stride * i.
     *   seal: input = plaintext of len_i bytes, output = ct || tag (len_i + 16)
     *   open: input = ct || tag of len_i bytes (len_i >= 16 else status
     *         SG_E_SHORT), output = plaintext (len_i - 16)
     * len_i = len ? len[i] : uniform_len.  max_len >= every len_i is required
     * when len != NULL (it sizes the LDS staging of one record); a longer
     * record is skipped and the call returns SG_E_ARG once every other record
     * is done (on a NULL stream: after the device work has finished; under
     * stream capture it is skipped silently).                                  */
    const uint8_t*  in;
    const uint64_t* in_off;
    uint64_t        in_stride;
    uint8_t*        out;
    const uint64_t* out_off;
    uint64_t        out_stride;
    const uint32_t* len;
    uint32_t        uniform_len;
    uint32_t        max_len;

    /* open: per-record status, device: SG_OK / SG_E_BAD_MAC / SG_E_SHORT, or
     * SG_STATUS_SKIPPED for a record longer than max_len (not processed, its
     * output left untouched).  The output of an SG_E_BAD_MAC record is zeroed
     * unless flags has SG_BATCH_KEEP_FAILED: it is never authenticated
     * plaintext.                                                             */
    uint8_t*        status;

    /* HIP stream (hipStream_t).  Non-NULL: the call is asynchronous on that
     * stream, except that a mixed-size batch (len != NULL, records in more
     * than one size class) waits once for its classification so that every
     * class runs on an exact grid; under stream capture it does not wait
     * (persistent class grids), so the whole call is graph-capturable with a
     * caller workspace.  A mixed TLS batch also runs its keying and two of its
     * record launches on library-owned side streams, which wait for this
     * stream's earlier work and are joined back into it before the call
     * returns.  NULL: the null (default) stream -- ordered after the
     * caller's earlier work on it -- and the call returns when the batch is
     * done.  No library lock is held while a call waits, so calls on
     * different streams (e.g. a writer and a reader thread, client.rs:19-24)
     * run concurrently on the device. */
    void*           stream;

    /* scratch of >= sg_workspace_size(count) bytes of 16-byte aligned device
     * memory, or NULL to use a library-owned cache: each call takes a buffer
     * no other call is enqueuing on and orders its reuse on the device with an
     * event, so asynchronous calls on different streams never share scratch.
     * A call under stream capture must pass a workspace. */
    void*           workspace;
    size_t          workspace_size;
} sg_batch;

#define SG_STATUS_SKIPPED 3  /* open status of a record with len_i > max_len;
                                sg_*_batch then returns SG_E_ARG            */

size_t sg_workspace_size(uint32_t count);

/* Batch seal / open on device-resident records.  Records are independent
 * (one wave each for 4-16 KiB records, 64-byte blocks of many small records
 * packed into one wave, or 2-256 lanes per record in the size classes).
 * Returns SG_OK or < 0 for argument/HIP errors; per-record MAC results of
 * open land in b->status. */
int sg_seal_batch(const sg_batch* b);
int sg_open_batch(const sg_batch* b);

/* ---- batched record layer over host memory ------------------------------
 * The throughput form of TlsWriter / TlsReader (tls.rs:68-380): many records
 * per call, pipelined inside the library, up to four chunks of 256 records in
 * flight.  Unregistered (pageable) buffers: the records are framed through
 * pinned staging that the kernels read and write over the host link
 * themselves.  Registered buffers (sg_host_register): host<->device copies
 * straight from and into them, each step (copy in, kernels, copy out)
 * enqueued by the calling thread once the step before it has completed, so
 * that a reader and a writer on two contexts never queue behind each other's
 * unfinished work.  Wire format exactly as the reference writes and parses it:
 *   header = content_type || major || minor || be16(fragment length)
 *   (tls.rs:126-130, 218-236) followed by the fragment (ct || tag).        */
#define SG_RECORD_MAX_LEN      16384u              /* RECORD_MAX_LEN      tls.rs:32 */
#define SG_ENC_RECORD_MAX_LEN  (16384u + 2048u)    /* ENC_RECORD_MAX_LEN  tls.rs:35 */
#define SG_HEADER_LEN          5u
/* record-layer error codes (TlsErrorKind, tls_result.rs:5-20) */
#define SG_E_UNEXPECTED_MESSAGE 3  /* unknown content type (tls.rs:218-225)          */
#define SG_E_RECORD_OVERFLOW    4  /* fragment > 2^14 + 2048 (tls.rs:232-234), or a
                                      decrypted fragment > 2^14 (tls.rs:269-272,
                                      where the reference panics)                  */

/* Caller buffers for the record layer's zero-copy path: page-locks [p, p+len)
 * (hipHostRegister) and records the range.  When sg_write_records' `data` and
 * `wire`, or sg_read_records' `wire` and `out`, both lie inside registered
 * ranges, the record bytes move by DMA straight between those buffers and the
 * device -- no framing copy through the library's pinned staging
 * (sg_write_records builds each chunk's wire image, headers included, in HBM;
 * sg_read_records parses the headers on the host, takes the zero-copy path for
 * chunks of equal, back-to-back records, whose wire image it takes apart in
 * HBM, and clears the plaintext of a failed record and of every record after
 * it in `out`, as it delivers none of them).  Unregister only when no call uses the range.
 * SG_ZERO_COPY=0 in the environment disables the path.  SG_OK or SG_E_ARG /
 * SG_E_HIP. */
int sg_host_register(void* p, size_t len);
int sg_host_unregister(void* p);

/* Upper bound of the wire bytes sg_write_records produces for len bytes. */
size_t sg_wire_bound(size_t len);

/* TlsWriter::write_data (tls.rs:137-147) + write_record (:99-135) for a whole
 * buffer: `data` is cut into ceil(len / 2^14) fragments (len == 0 writes no
 * record, as the reference's chunks() loop yields none), record i is sealed with
 * seq = seq0 + i (nonce be64(seq), AD be64(seq)||type||major||minor||be16(n)),
 * and its wire image is appended to `wire`.  Host memory in and out.
 * Returns the number of records written (the caller adds it to its
 * write_count, tls.rs:132) or < 0; *wire_len = bytes written. */
int64_t sg_write_records(sg_ctx* ctx, uint64_t seq0, uint8_t content_type, uint8_t ver_major,
                         uint8_t ver_minor, const uint8_t* data, size_t len, uint8_t* wire,
                         size_t wire_cap, size_t* wire_len);

/* TlsReader::read_record (tls.rs:217-281) for every COMPLETE record at the
 * start of `wire`: header checks in the reference's order (unknown type ->
 * SG_E_UNEXPECTED_MESSAGE, length > 2^14+2048 -> SG_E_RECORD_OVERFLOW,
 * length < 16 -> SG_E_SHORT), AD = be64(seq)||type||major||minor||be16(len-16)
 * with seq = seq0 + i, open, and append the plaintext fragments to `out`.
 * Processing stops at the first failing record; the records before it are
 * delivered.  Per-record content types / plaintext lengths go to `types` /
 * `frag_lens` (capacity max_records, either may be NULL). */
typedef struct sg_read_result {
    uint64_t records;    /* records opened successfully (the caller adds this to read_count) */
    uint64_t consumed;   /* wire bytes of those records                                     */
    uint64_t out_len;    /* plaintext bytes written to out                                  */
    int32_t  error;      /* SG_OK, or the status of record number `records`                 */
    uint32_t _pad;
} sg_read_result;
int sg_read_records(sg_ctx* ctx, uint64_t seq0, const uint8_t* wire, size_t wire_len, uint8_t* out,
                    size_t out_cap, uint8_t* types, uint32_t* frag_lens, size_t max_records,
                    sg_read_result* res);

/* The header checks of sg_read_records alone (TlsReader::read_record,
 * tls.rs:217-238, 258-262, 269-272), host only -- no context, no GPU: the
 * complete records at the start of `wire` (at most max_records) go to `recs`
 * (offset of the fragment after its 5-byte header, fragment length, type,
 * version), *count of them; *error = SG_OK, or the error of the first bad
 * header (SG_E_UNEXPECTED_MESSAGE, SG_E_RECORD_OVERFLOW, SG_E_SHORT) that
 * stopped the parse.  An incomplete record at the end is not an error.
 * Returns SG_OK or SG_E_ARG. */
typedef struct sg_wire_record {
    uint64_t offset;
    uint32_t frag_len;
    uint8_t  type, ver_major, ver_minor, _pad;
} sg_wire_record;
int sg_parse_records(const uint8_t* wire, size_t wire_len, size_t max_records, sg_wire_record* recs,
                     size_t* count, int32_t* error);

/* Time (ms) spent by the last sg_write_records / sg_read_records call of this
 * thread in host->device copies, kernels and device->host copies (HIP events;
 * summed over the pipelined chunks; with unregistered buffers the kernels move
 * the bytes over the host link themselves and all device time counts as
 * kernels) and in host-side framing memcpy. */
int sg_record_timing(double* h2d_ms, double* kernel_ms, double* d2h_ms, double* host_ms);

/* ---- TLS 1.2 key schedule on the host (cipher/prf.rs, client.rs:130-225) --
 * Produces the per-connection key tables the batch calls take.  CPU only
 * (no device needed); the reference's hmac_sha256 panics for keys longer than
 * 64 bytes (prf.rs:11-14): SG_E_ARG here. */
void sg_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);          /* crypto/sha2.rs:18-116 */
int  sg_hmac_sha256(const uint8_t* key, size_t key_len, const uint8_t* msg, size_t len,
                    uint8_t out[32]);                                     /* prf.rs:8-29          */
typedef struct sg_prf sg_prf;                                             /* prf.rs:31-36 Prf     */
sg_prf* sg_prf_new(const uint8_t* secret, size_t secret_len,
                   const uint8_t* seed, size_t seed_len);                 /* prf.rs:38-48         */
int  sg_prf_get_bytes(sg_prf* prf, uint8_t* out, size_t n);               /* prf.rs:60-89         */
void sg_prf_free(sg_prf* prf);
/* client.rs:130-163 for `count` connections (threads >= 1):
 *   master_secret_i = PRF(pre_master_i, "master secret" || client_random_i || server_random_i)[0..48]
 *   key block = PRF(master_secret_i, "key expansion" || server_random_i || client_random_i)
 *   client_write_key_i = key block[0..32] (the client's encryptor key, client.rs:152-154)
 *   server_write_key_i = key block[32..64] (the client's decryptor key, :157)
 * pre_master_i = pre_master + pm_stride*i (pm_len bytes); randoms are [count][32];
 * master_secret ([count][48]) may be NULL. */
int  sg_derive_keys(uint32_t count, const uint8_t* pre_master, size_t pm_len, size_t pm_stride,
                    const uint8_t* client_random, const uint8_t* server_random, uint8_t* master_secret,
                    uint8_t* client_write_keys, uint8_t* server_write_keys, int threads);
/* client.rs:184-192 (server = 0, "client finished") / :213-221 (server = 1,
 * "server finished"): PRF(master_secret, label || handshake_hash)[0..12]. */
int  sg_finished_verify_data(const uint8_t master_secret[48], int server,
                             const uint8_t handshake_hash[32], uint8_t out[12]);

/* ---- synthetic workload helpers (bench / tests) ------------------------ */
/* Fills records on the device: byte i of record j =
 * byte (i mod 8) of splitmix64(seed ^ ((j0 + j) << 32) ^ (i / 8)).
 * Records are len bytes each at buf + stride * j.                         */
int sg_fill_records(uint8_t* buf, uint64_t stride, uint32_t len, uint32_t count,
                    uint64_t seed, uint64_t j0, void* stream);
/* Byte-compares a[j] and b[j] (len bytes at stride_a / stride_b); adds the
 * number of mismatching records to *mismatches (device uint64).            */
int sg_compare_records(const uint8_t* a, uint64_t stride_a, const uint8_t* b,
                       uint64_t stride_b, uint32_t len, uint32_t count,
                       unsigned long long* mismatches, void* stream);

/* ---- diagnostics -------------------------------------------------------- */
const char* sg_last_error(void);       /* thread-local message of the last failure */
const char* sg_build_info(void);       /* arch + kernel configuration string       */
const char* sg_source_hash(void);      /* hash of the sources the library was built
                                          from (16 hex digits; suruga_amd/_build.py) */
/* Kernel timing with HIP events recorded on the launch stream.  While timing
 * is enabled every batch call brackets its keying kernel and its seal/open
 * kernel with events; sg_timing_read synchronises on them and returns the
 * average duration (ms) per launch of each kind and the launch counts.
 * sg_set_timing(1) resets the accumulators; sg_set_timing(0) stops them. */
int sg_set_timing(int enable);
int sg_timing_read(double* seal_ms, double* open_ms, double* keying_ms,
                   uint32_t* n_seal, uint32_t* n_open, uint32_t* n_keying);

/* Kernel form for uniform batches of full 16 KiB records (n = 2^14, the
 * size TlsWriter::write_data gives every record but a stream's tail; C1):
 * 1 = the wave-per-record kernel (one wave per record, lock-step ChaCha20
 * rounds, Poly1305 on the matrix cores fed from the ciphertext registers),
 * 0 = the size-class kernel used for every other batch.  Both are bit-exact;
 * the switch exists for A/B measurement and for tests that cover both.
 * Initial value: environment SG_LOCKSTEP ("0"/"1"), else 1.  Returns the
 * previous setting; a negative argument only queries. */
int sg_set_lockstep(int enable);

/* Kernel form for the small records of mixed TLS batches (64 B .. 4 KiB, a
 * multiple of 64 bytes, 16-byte aligned; C2): 1 = the packed kernel (the
 * 64-byte blocks of runs of 128 records of the packed list laid end to end
 * over the lanes of a 512-thread workgroup, keyed in the same kernel), 0 = the
 * size-class kernels.  Both are
 * bit-exact; A/B and test switch like sg_set_lockstep.  Initial value:
 * environment SG_PACK ("0"/"1"), else 1.  Returns the previous setting; a
 * negative argument only queries. */
int sg_set_packed(int enable);

#ifdef __cplusplus
}
#endif
#endif /* SURUGA_GPU_H */
