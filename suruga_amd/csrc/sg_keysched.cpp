// sg_keysched.cpp -- TLS 1.2 key schedule on the host (SURVEY.md section 8f,
// rank 4): SHA-256, HMAC-SHA256 and the P_SHA256 PRF of suruga
// (src/crypto/sha2.rs, src/cipher/prf.rs) and the client's derivation of the
// per-direction AEAD keys (src/client.rs:130-163) and Finished verify data
// (client.rs:184-225).  It produces the key tables that sg_seal_batch /
// sg_open_batch consume; it is a few microseconds of CPU per connection, so
// it stays on the CPU as the survey ranks it, threaded over connections.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/suruga_gpu.h"
#include "sg_err.h"  // host only: no HIP (tests/cpp/test_host_san.cpp builds it with g++ under sanitizers)

namespace sg {
namespace {

// ---- SHA-256 (FIPS 180-4; the algorithm of crypto/sha2.rs:18-116) ----------
constexpr uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct Sha256 {
    uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint8_t blk[64];
    size_t fill = 0;
    uint64_t total = 0;

    void compress(const uint8_t* p) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    void update(const uint8_t* p, size_t n) {
        total += n;
        while (n) {
            const size_t k = std::min(n, (size_t)64 - fill);
            std::memcpy(blk + fill, p, k);
            fill += k;
            p += k;
            n -= k;
            if (fill == 64) {
                compress(blk);
                fill = 0;
            }
        }
    }
    void finish(uint8_t out[32]) {
        const uint64_t bits = total * 8;
        const uint8_t pad = 0x80;
        update(&pad, 1);
        const uint8_t zero[64] = {0};
        update(zero, (fill <= 56 ? 56 : 120) - fill);
        uint8_t len[8];
        for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(len, 8);
        for (int i = 0; i < 8; ++i) {
            out[4 * i] = (uint8_t)(h[i] >> 24);
            out[4 * i + 1] = (uint8_t)(h[i] >> 16);
            out[4 * i + 2] = (uint8_t)(h[i] >> 8);
            out[4 * i + 3] = (uint8_t)h[i];
        }
    }
};

// prf.rs:8-29: ipad/opad with the key XORed in; keys longer than the block
// are unimplemented!() in the reference.
void hmac(const uint8_t* key, size_t key_len, const uint8_t* m1, size_t n1, const uint8_t* m2, size_t n2,
          uint8_t out[32]) {
    uint8_t ipad[64], opad[64];
    std::memset(ipad, 0x36, 64);
    std::memset(opad, 0x5c, 64);
    for (size_t i = 0; i < key_len; ++i) {
        ipad[i] ^= key[i];
        opad[i] ^= key[i];
    }
    uint8_t inner[32];
    Sha256 hi;
    hi.update(ipad, 64);
    hi.update(m1, n1);
    if (n2) hi.update(m2, n2);
    hi.finish(inner);
    Sha256 ho;
    ho.update(opad, 64);
    ho.update(inner, 32);
    ho.finish(out);
}

}  // namespace

// prf.rs:31-89: A(1) = HMAC(secret, seed); block i = HMAC(secret, A(i) || seed);
// A(i+1) = HMAC(secret, A(i)); get_bytes hands out the stream in order, keeping
// the unused tail of the last block.
struct Prf {
    std::vector<uint8_t> secret, seed;
    uint8_t a[32];
    uint8_t buf[32];
    size_t buf_len = 0, buf_off = 0;

    Prf(const uint8_t* s, size_t sl, const uint8_t* sd, size_t sdl) : secret(s, s + sl), seed(sd, sd + sdl) {
        hmac(secret.data(), secret.size(), seed.data(), seed.size(), nullptr, 0, a);
    }
    void next_block(uint8_t out[32]) {
        hmac(secret.data(), secret.size(), a, 32, seed.data(), seed.size(), out);
        uint8_t na[32];
        hmac(secret.data(), secret.size(), a, 32, nullptr, 0, na);
        std::memcpy(a, na, 32);
    }
    void get_bytes(uint8_t* out, size_t n) {
        while (n) {
            if (buf_off == buf_len) {
                next_block(buf);
                buf_len = 32;
                buf_off = 0;
            }
            const size_t k = std::min(n, buf_len - buf_off);
            std::memcpy(out, buf + buf_off, k);
            buf_off += k;
            out += k;
            n -= k;
        }
    }
};

namespace {
constexpr size_t kMaxHmacKey = 64;

void derive_one(const uint8_t* pm, size_t pm_len, const uint8_t* cr, const uint8_t* sr, uint8_t* ms_out,
                uint8_t* cwk, uint8_t* swk) {
    // client.rs:130-137: master_secret = PRF(pre_master, "master secret" || client_random || server_random)[..48]
    uint8_t seed[13 + 64];
    std::memcpy(seed, "master secret", 13);
    std::memcpy(seed + 13, cr, 32);
    std::memcpy(seed + 45, sr, 32);
    uint8_t ms[48];
    Prf(pm, pm_len, seed, 77).get_bytes(ms, 48);
    // client.rs:142-160: key block = PRF(master, "key expansion" || server_random || client_random);
    // client write key first, then the read (server write) key; no MAC keys, no IVs (AEAD, fixed_iv_len 0)
    std::memcpy(seed, "key expansion", 13);
    std::memcpy(seed + 13, sr, 32);
    std::memcpy(seed + 45, cr, 32);
    Prf kb(ms, 48, seed, 77);
    kb.get_bytes(cwk, SG_KEY_LEN);
    kb.get_bytes(swk, SG_KEY_LEN);
    if (ms_out) std::memcpy(ms_out, ms, 48);
}
}  // namespace
}  // namespace sg

using sg::fail;

extern "C" {

void sg_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
    sg::Sha256 h;
    if (len) h.update(msg, len);
    h.finish(out);
}

int sg_hmac_sha256(const uint8_t* key, size_t key_len, const uint8_t* msg, size_t len, uint8_t out[32]) {
    if (key_len > sg::kMaxHmacKey) return fail(SG_E_ARG, "HMAC key longer than 64 bytes (unimplemented in prf.rs:11-14)%s");
    if ((key_len && !key) || (len && !msg) || !out) return fail(SG_E_ARG, "NULL argument%s");
    sg::hmac(key, key_len, msg, len, nullptr, 0, out);
    return SG_OK;
}

sg_prf* sg_prf_new(const uint8_t* secret, size_t secret_len, const uint8_t* seed, size_t seed_len) {
    if (secret_len > sg::kMaxHmacKey || (secret_len && !secret) || (seed_len && !seed)) {
        fail(SG_E_ARG, "bad PRF secret/seed%s");
        return nullptr;
    }
    return reinterpret_cast<sg_prf*>(new sg::Prf(secret, secret_len, seed, seed_len));
}

int sg_prf_get_bytes(sg_prf* prf, uint8_t* out, size_t n) {
    if (!prf || (n && !out)) return fail(SG_E_ARG, "NULL argument%s");
    reinterpret_cast<sg::Prf*>(prf)->get_bytes(out, n);
    return SG_OK;
}

void sg_prf_free(sg_prf* prf) { delete reinterpret_cast<sg::Prf*>(prf); }

int sg_derive_keys(uint32_t count, const uint8_t* pre_master, size_t pm_len, size_t pm_stride,
                   const uint8_t* client_random, const uint8_t* server_random, uint8_t* master_secret,
                   uint8_t* client_write_keys, uint8_t* server_write_keys, int threads) {
    if (!count) return SG_OK;
    if (!pre_master || !client_random || !server_random || !client_write_keys || !server_write_keys)
        return fail(SG_E_ARG, "NULL argument%s");
    if (pm_len > sg::kMaxHmacKey || pm_stride < pm_len) return fail(SG_E_ARG, "bad pre-master length/stride%s");
    const uint32_t nt = (uint32_t)std::max(1, std::min<int>(threads, (int)count));
    auto work = [&](uint32_t t) {
        for (uint32_t i = t; i < count; i += nt)
            sg::derive_one(pre_master + (size_t)pm_stride * i, pm_len, client_random + 32ull * i,
                           server_random + 32ull * i, master_secret ? master_secret + 48ull * i : nullptr,
                           client_write_keys + 32ull * i, server_write_keys + 32ull * i);
    };
    if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (uint32_t t = 0; t < nt; ++t) pool.emplace_back(work, t);
        for (auto& th : pool) th.join();
    }
    return SG_OK;
}

int sg_finished_verify_data(const uint8_t master_secret[48], int server, const uint8_t handshake_hash[32],
                            uint8_t out[12]) {
    if (!master_secret || !handshake_hash || !out) return fail(SG_E_ARG, "NULL argument%s");
    // client.rs:184-192 / 213-221: PRF(master, "client finished"|"server finished" || sha256(msgs))[..12]
    uint8_t seed[15 + 32];
    std::memcpy(seed, server ? "server finished" : "client finished", 15);
    std::memcpy(seed + 15, handshake_hash, 32);
    sg::Prf(master_secret, 48, seed, sizeof seed).get_bytes(out, 12);
    return SG_OK;
}

}  // extern "C"
