// test_host_san.cpp -- the library's host-only code under AddressSanitizer and
// UndefinedBehaviorSanitizer ("race detection /
// sanitizers"), built with g++ -fsanitize=address,undefined
// by tests/test_sanitizers.py from the product sources themselves:
//
//   * suruga_amd/csrc/sg_wire.cpp -- the TLS record header parser that
//     sg_read_records runs on bytes a peer controls (tls.rs:217-238, 258-262,
//     269-272), fed valid streams, every truncation of them, every content-type
//     byte, every length class at its edges and a deterministic random corpus,
//     with the exact expected outcome computed by an independent model below;
//   * suruga_amd/csrc/sg_keysched.cpp -- SHA-256 / HMAC-SHA256 / the P_SHA256
//     PRF / the key block, on the FIPS 180-4 and RFC 4231 vectors, the PRF's
//     split-read invariance (prf.rs:135-162) and a threaded key derivation.
//
// No GPU: neither file includes a HIP header.  Exit code 0 = every check
// passed; a sanitizer report aborts the program (halt_on_error).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/suruga_gpu.h"
#include "../../suruga_amd/csrc/sg_err.h"

// sg_capi.cpp owns the thread-local message; this program only needs the code
int sg::fail(int code, const char*, const char*) { return code; }

static int g_fail = 0;
#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                          \
        }                                                                      \
    } while (0)

static uint64_t g_rng = 0x5341'4e49'5449'5a45ull;  // deterministic corpus
static uint64_t rnd() {
    g_rng += 0x9E3779B97F4A7C15ull;
    uint64_t z = g_rng;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---- the parser ------------------------------------------------------------
struct Expect {
    std::vector<sg_wire_record> recs;
    int32_t error = SG_OK;
};

// An independent statement of TlsReader::read_record's header checks, one
// record at a time (tls.rs:218-238: type, then length > ENC_RECORD_MAX_LEN,
// then the fragment must be complete; :258-262 < mac_len; :269-272 > 2^14).
static Expect model(const std::vector<uint8_t>& w, size_t max_records) {
    Expect e;
    size_t pos = 0;
    while (e.recs.size() < max_records) {
        if (w.size() < pos + 5) break;
        const uint8_t t = w[pos];
        if (!(t == 20 || t == 21 || t == 22 || t == 23)) { e.error = SG_E_UNEXPECTED_MESSAGE; break; }
        const size_t len = (size_t)w[pos + 3] * 256 + w[pos + 4];
        if (len > 16384 + 2048) { e.error = SG_E_RECORD_OVERFLOW; break; }
        if (w.size() < pos + 5 + len) break;
        if (len < 16) { e.error = SG_E_SHORT; break; }
        if (len - 16 > 16384) { e.error = SG_E_RECORD_OVERFLOW; break; }
        e.recs.push_back({(uint64_t)(pos + 5), (uint32_t)len, t, w[pos + 1], w[pos + 2], 0});
        pos += 5 + len;
    }
    return e;
}

// The parser on an exact-size heap copy of the bytes (ASan flags any read past it).
static void check_parse(const std::vector<uint8_t>& w, size_t max_records = 1u << 20) {
    uint8_t* buf = w.empty() ? nullptr : static_cast<uint8_t*>(std::malloc(w.size()));
    if (buf) std::memcpy(buf, w.data(), w.size());
    const size_t cap = max_records < 4096 ? max_records : 4096;
    std::vector<sg_wire_record> recs(cap ? cap : 1);
    size_t count = 12345;
    int32_t error = 777;
    const int rc = sg_parse_records(buf, w.size(), cap, recs.data(), &count, &error);
    std::free(buf);
    CHECK(rc == SG_OK);
    const Expect e = model(w, cap);
    CHECK(error == e.error);
    CHECK(count == e.recs.size());
    if (count != e.recs.size()) return;
    for (size_t i = 0; i < count; ++i) {
        CHECK(recs[i].offset == e.recs[i].offset && recs[i].frag_len == e.recs[i].frag_len);
        CHECK(recs[i].type == e.recs[i].type && recs[i].ver_major == e.recs[i].ver_major &&
              recs[i].ver_minor == e.recs[i].ver_minor);
        CHECK(recs[i].offset + recs[i].frag_len <= w.size());
    }
}

static void put_record(std::vector<uint8_t>& w, uint8_t type, uint32_t len) {
    w.push_back(type);
    w.push_back(3);
    w.push_back(3);
    w.push_back((uint8_t)(len >> 8));
    w.push_back((uint8_t)len);
    for (uint32_t i = 0; i < len; ++i) w.push_back((uint8_t)rnd());
}

static void parser_corpus() {
    // valid streams and every truncation of one (an incomplete record is no error)
    std::vector<uint8_t> w;
    const uint32_t lens[] = {16, 17, 31, 32, 100, 16384 + 16, 16400, 1000, 16, 18432 - 2048};
    for (uint32_t i = 0; i < 10; ++i) put_record(w, (uint8_t)(20 + i % 4), lens[i]);
    check_parse(w);
    for (size_t cut = 0; cut <= w.size(); cut += (cut < 64 || w.size() - cut < 64) ? 1 : 97)
        check_parse(std::vector<uint8_t>(w.begin(), w.begin() + (long)cut));
    for (size_t m = 0; m <= 11; ++m) check_parse(w, m);  // max_records caps the parse
    // every content-type byte in the first and in a later record
    for (int t = 0; t < 256; ++t) {
        std::vector<uint8_t> a;
        put_record(a, (uint8_t)t, 16);
        check_parse(a);
        std::vector<uint8_t> b;
        put_record(b, 23, 40);
        put_record(b, (uint8_t)t, 20);
        check_parse(b);
    }
    // every length class at its edges: < 16 (short), 16..16400, 16401..18432
    // (decrypted > 2^14), > 18432 (overflow), 0xffff; complete and header-only
    const uint32_t edge[] = {0, 1, 15, 16, 17, 16399, 16400, 16401, 16402, 18431, 18432, 18433, 18434, 30000, 65535};
    for (uint32_t len : edge) {
        std::vector<uint8_t> a;
        put_record(a, 23, 64);
        if (len <= 20000) {
            put_record(a, 23, len);
        } else {
            a.insert(a.end(), {23, 3, 3, (uint8_t)(len >> 8), (uint8_t)len});
        }
        check_parse(a);
        a.resize(64 + 5 + 5);  // the second header only
        check_parse(a);
    }
    // deterministic random corpus: short garbage, mostly-valid streams with one
    // corrupted header byte, and random lengths
    for (int it = 0; it < 20000; ++it) {
        std::vector<uint8_t> a;
        const int kind = (int)(rnd() % 3);
        if (kind == 0) {
            const size_t n = rnd() % 48;
            for (size_t i = 0; i < n; ++i) a.push_back((uint8_t)rnd());
        } else {
            const int nrec = 1 + (int)(rnd() % 5);
            std::vector<size_t> hdr;
            for (int r = 0; r < nrec; ++r) {
                hdr.push_back(a.size());
                put_record(a, (uint8_t)(20 + rnd() % 4), (uint32_t)(rnd() % (kind == 1 ? 300 : 18500)));
            }
            if (kind == 1) a[hdr[rnd() % hdr.size()] + rnd() % 5] ^= (uint8_t)(1u << (rnd() % 8));
            a.resize(a.size() - (rnd() % 2 ? rnd() % (a.size() + 1) : 0));
        }
        check_parse(a, (size_t)(rnd() % 8));
        check_parse(a);
    }
    // argument errors
    size_t count = 0;
    int32_t error = 0;
    sg_wire_record r;
    CHECK(sg_parse_records(nullptr, 5, 1, &r, &count, &error) == SG_E_ARG);
    CHECK(sg_parse_records(nullptr, 0, 0, nullptr, &count, &error) == SG_OK && count == 0 && error == SG_OK);
    const uint8_t one[5] = {23, 3, 3, 0, 16};
    CHECK(sg_parse_records(one, 5, 1, nullptr, &count, &error) == SG_E_ARG);
    CHECK(sg_parse_records(one, 5, 1, &r, nullptr, &error) == SG_E_ARG);
    CHECK(sg_parse_records(one, 5, 1, &r, &count, nullptr) == SG_E_ARG);
}

// ---- the key schedule --------------------------------------------------------
static std::string hex(const uint8_t* p, size_t n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) {
        s += d[p[i] >> 4];
        s += d[p[i] & 15];
    }
    return s;
}

static void keysched() {
    uint8_t h[32];
    sg_sha256(nullptr, 0, h);  // FIPS 180-4 / sha2.rs:123-141
    CHECK(hex(h, 32) == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");
    sg_sha256(reinterpret_cast<const uint8_t*>("abc"), 3, h);
    CHECK(hex(h, 32) == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");
    const char* m448 = "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq";
    sg_sha256(reinterpret_cast<const uint8_t*>(m448), std::strlen(m448), h);
    CHECK(hex(h, 32) == "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1");
    std::vector<uint8_t> mil(1000000, 'a');
    sg_sha256(mil.data(), mil.size(), h);
    CHECK(hex(h, 32) == "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0");
    // RFC 4231 cases 1 and 2 (prf.rs:97-133)
    uint8_t k1[20];
    std::memset(k1, 0x0b, 20);
    CHECK(sg_hmac_sha256(k1, 20, reinterpret_cast<const uint8_t*>("Hi There"), 8, h) == SG_OK);
    CHECK(hex(h, 32) == "b0344c61d8db38535ca8afceaf0bf12b881dc200c9833da726e9376c2e32cff7");
    const char* d2 = "what do ya want for nothing?";
    CHECK(sg_hmac_sha256(reinterpret_cast<const uint8_t*>("Jefe"), 4, reinterpret_cast<const uint8_t*>(d2),
                         std::strlen(d2), h) == SG_OK);
    CHECK(hex(h, 32) == "5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843");
    uint8_t big[65] = {};
    CHECK(sg_hmac_sha256(big, 65, big, 1, h) == SG_E_ARG);  // prf.rs:11-14 unimplemented!()
    // PRF: any split of get_bytes gives the same stream (prf.rs:135-162)
    const uint8_t secret[48] = {1, 2, 3}, seed[77] = {9, 8, 7};
    uint8_t whole[300], parts[300];
    sg_prf* a = sg_prf_new(secret, 48, seed, 77);
    CHECK(a && sg_prf_get_bytes(a, whole, 300) == SG_OK);
    sg_prf_free(a);
    for (int trial = 0; trial < 50; ++trial) {
        sg_prf* b = sg_prf_new(secret, 48, seed, 77);
        size_t pos = 0;
        while (pos < 300) {
            size_t n = 1 + rnd() % 70;
            if (n > 300 - pos) n = 300 - pos;
            CHECK(sg_prf_get_bytes(b, parts + pos, n) == SG_OK);
            pos += n;
        }
        sg_prf_free(b);
        CHECK(std::memcmp(whole, parts, 300) == 0);
    }
    CHECK(sg_prf_new(big, 65, seed, 1) == nullptr);
    // key block for many connections on threads == one at a time
    const uint32_t count = 64;
    std::vector<uint8_t> pm(count * 48), cr(count * 32), sr(count * 32);
    for (auto& x : pm) x = (uint8_t)rnd();
    for (auto& x : cr) x = (uint8_t)rnd();
    for (auto& x : sr) x = (uint8_t)rnd();
    std::vector<uint8_t> ms1(count * 48), c1(count * 32), s1(count * 32), ms4(count * 48), c4(count * 32), s4(count * 32);
    CHECK(sg_derive_keys(count, pm.data(), 48, 48, cr.data(), sr.data(), ms1.data(), c1.data(), s1.data(), 1) == SG_OK);
    CHECK(sg_derive_keys(count, pm.data(), 48, 48, cr.data(), sr.data(), ms4.data(), c4.data(), s4.data(), 4) == SG_OK);
    CHECK(ms1 == ms4 && c1 == c4 && s1 == s4);
    uint8_t vd[12], vd2[12];
    CHECK(sg_finished_verify_data(ms1.data(), 0, h, vd) == SG_OK);
    CHECK(sg_finished_verify_data(ms1.data(), 1, h, vd2) == SG_OK);
    CHECK(std::memcmp(vd, vd2, 12) != 0);
    CHECK(sg_derive_keys(1, pm.data(), 65, 65, cr.data(), sr.data(), nullptr, c1.data(), s1.data(), 1) == SG_E_ARG);
}

int main() {
    parser_corpus();
    keysched();
    if (g_fail) {
        std::fprintf(stderr, "%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("host sanitizer checks passed\n");
    return 0;
}
