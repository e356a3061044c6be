// C++ host-side mirror tests (include/suruga/cipher.hpp, tls.hpp).
//
//   ./test_host cpu   record-layer tests of the reference (src/test.rs:41-100,
//                     src/tls.rs:382-476) with the null cipher, and the framing
//                     through the CPU restatement (oracle/, test infrastructure)
//   ./test_host gpu   the GPU Aead behind the same traits, checked against the
//                     oracle: single records, tamper / short, batched writer and
//                     stream reader, trait-object reader
//
// Driven by tests/test_cpp_host.py.  Exit status = number of failed checks.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/suruga/cipher.hpp"
#include "../../include/suruga/prf.hpp"
#include "../../include/suruga/tls.hpp"
#include "../../oracle/suruga_oracle.h"

using namespace suruga;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                                      \
    do {                                                                                 \
        if (cond) {                                                                      \
            ++g_pass;                                                                    \
        } else {                                                                         \
            ++g_fail;                                                                    \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                                \
    } while (0)

template <class E, class F>
static bool throws(F&& f, std::function<bool(const E&)> pred = nullptr) {
    try {
        f();
    } catch (const E& e) {
        return pred ? pred(e) : true;
    } catch (...) {
        return false;
    }
    return false;
}
static std::function<bool(const TlsError&)> kind_is(TlsErrorKind k) {
    return [k](const TlsError& e) { return e.kind == k; };
}

// ---- test ciphers ---------------------------------------------------------
struct NullEncryptor : Encryptor {  // test.rs:13-20
    Bytes encrypt(Slice, Slice plain, Slice) override { return Bytes(plain.data, plain.data + plain.size); }
};
struct NullDecryptor : Decryptor {  // test.rs:22-27
    Bytes decrypt(Slice, Slice enc, Slice) override { return Bytes(enc.data, enc.data + enc.size); }
    size_t mac_len() const override { return 0; }
};
// The reference algorithm (CPU restatement) behind the traits.
struct OracleEncryptor : Encryptor {
    Bytes key;
    explicit OracleEncryptor(Bytes k) : key(std::move(k)) {}
    Bytes encrypt(Slice nonce, Slice plain, Slice ad) override {
        Bytes out(plain.size + 16);
        so_seal(key.data(), nonce.data, plain.data, plain.size, ad.data, ad.size, out.data());
        return out;
    }
};
struct OracleDecryptor : Decryptor {
    Bytes key;
    explicit OracleDecryptor(Bytes k) : key(std::move(k)) {}
    Bytes decrypt(Slice nonce, Slice enc, Slice ad) override {
        if (enc.size < 16) throw TlsError(TlsErrorKind::BadRecordMac, "message too short");
        Bytes out(enc.size - 16);
        if (so_open(key.data(), nonce.data, enc.data, enc.size, ad.data, ad.size, out.data()) != 0)
            throw TlsError(TlsErrorKind::BadRecordMac, "wrong mac");
        return out;
    }
    size_t mac_len() const override { return 16; }
};

static Bytes key_seq(uint8_t first) {
    Bytes k(32);
    for (int i = 0; i < 32; ++i) k[i] = static_cast<uint8_t>(first + i);
    return k;
}
static Bytes fill(uint64_t seed, uint64_t j, size_t n) {
    Bytes b(n);
    so_fill_record(seed, j, b.data(), n);
    return b;
}
static std::string hex(const uint8_t* p, size_t n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) s += d[p[i] >> 4], s += d[p[i] & 15];
    return s;
}
static const char* kSurveyVector = "59f90370eca7e79052201d20ee020f66fbc2d9037460b094b3443d3ec89ef135";

// ---- CPU: the reference's own record tests ---------------------------------
static void cpu_tests() {
    {  // HostBuffer (tls.hpp): page-aligned; an empty one is valid and stays unregistered
        HostBuffer a(100, false), e(0, true);
        CHECK(a.data() && (reinterpret_cast<uintptr_t>(a.data()) & 4095u) == 0 && a.size() == 100 && !a.registered());
        CHECK(e.data() && e.size() == 0 && !e.registered());
    }
    {  // test.rs:41-63 test_change_cipher_spec_message
        VecWriter out;
        TlsWriter w(out);
        w.set_encryptor(std::make_unique<NullEncryptor>());
        w.write_change_cipher_spec();
        CHECK(out.buf.size() == 6 && out.buf[5] == 1);
        SliceReader in(out.buf);
        TlsReader r(in);
        r.set_decryptor(std::make_unique<NullDecryptor>());
        CHECK(r.read_message().kind == Message::ChangeCipherSpec);
    }
    {  // test.rs:65-100 test_application_message
        Bytes app(RECORD_MAX_LEN + 200, 1);
        VecWriter out;
        TlsWriter w(out);
        w.set_encryptor(std::make_unique<NullEncryptor>());
        w.write_application_data(app);
        SliceReader in(out.buf);
        TlsReader r(in);
        r.set_decryptor(std::make_unique<NullDecryptor>());
        Message m1 = r.read_message(), m2 = r.read_message();
        CHECK(m1.kind == Message::ApplicationData && m1.payload == Bytes(RECORD_MAX_LEN, 1));
        CHECK(m2.kind == Message::ApplicationData && m2.payload == Bytes(200, 1));
    }
    {  // tls.rs:411-425 test_reader
        SliceReader in(Bytes{0x14, 0x03, 0x03, 0x00, 0x01, 0x01});
        TlsReader r(in);
        Record rec = r.read_record();
        CHECK(rec.content_type == ContentType::ChangeCipherSpecTy && rec.ver_major == 3 && rec.ver_minor == 3 &&
              rec.fragment == Bytes{1});
        CHECK(throws<TlsError>([&] { r.read_record(); }, kind_is(TlsErrorKind::IoFailure)));
    }
    {  // tls.rs:427-436 test_reader_unknown (0x18 is not a ContentType)
        SliceReader in(Bytes{0x18, 0x03, 0x03, 0x00, 0x03, 0x01, 0x00, 0x20});
        TlsReader r(in);
        CHECK(throws<TlsError>([&] { r.read_record(); }, kind_is(TlsErrorKind::UnexpectedMessage)));
    }
    {  // tls.rs:438-449 test_reader_too_long
        const size_t n = RECORD_MAX_LEN + 1;
        Bytes b{0x17, 0x03, 0x03, static_cast<uint8_t>(n >> 8), static_cast<uint8_t>(n)};
        b.resize(5 + n, 0xff);
        SliceReader in(b);
        TlsReader r(in);
        CHECK(throws<TlsError>([&] { r.read_record(); }, kind_is(TlsErrorKind::RecordOverflow)));
    }
    {  // tls.rs:451-461 test_reader_zero_length
        for (uint8_t ct : {20, 21, 22}) {
            SliceReader in(Bytes{ct, 0x03, 0x03, 0x00, 0x00});
            TlsReader r(in);
            CHECK(throws<TlsError>([&] { r.read_message(); }, kind_is(TlsErrorKind::UnexpectedMessage)));
        }
    }
    {  // tls.rs:463-475 test_writer_too_long (panics)
        struct Big : Encryptor {
            Bytes encrypt(Slice, Slice, Slice) override { return Bytes(ENC_RECORD_MAX_LEN + 1); }
        };
        VecWriter out;
        TlsWriter w(out);
        w.set_encryptor(std::make_unique<Big>());
        CHECK(throws<std::logic_error>([&] { w.write_record(Record(ContentType::ApplicationDataTy, 3, 3, Bytes{1})); }));
    }
    {  // alerts: known / unknown (alert.rs:5-44, tls.rs:313-329)
        VecWriter out;
        TlsWriter w(out);
        w.write_alert(2, 20);
        w.write_alert(2, 99);
        SliceReader in(out.buf);
        TlsReader r(in);
        Message m = r.read_message();
        CHECK(m.kind == Message::Alert && m.alert_level == 2 && m.alert_description == 20);
        CHECK(throws<TlsError>([&] { r.read_message(); }, kind_is(TlsErrorKind::UnexpectedMessage)));
    }
    {  // framing through the reference algorithm: the survey's sample vector
        VecWriter out;
        TlsWriter w(out);
        w.set_encryptor(std::make_unique<OracleEncryptor>(key_seq(0)));
        w.write_application_data(Bytes(16, 'A'));
        CHECK(out.buf.size() == 37 && out.buf[0] == 23 && out.buf[3] == 0 && out.buf[4] == 32);
        CHECK(hex(out.buf.data() + 5, 32) == kSurveyVector);
        SliceReader in(out.buf);
        TlsReader r(in);
        r.set_decryptor(std::make_unique<OracleDecryptor>(key_seq(0)));
        CHECK(r.read_application_data() == Bytes(16, 'A'));
    }
    {  // prf.rs:137-166 test_get_bytes and prf.rs:98-132 (RFC 4231 case 2)
        Prf p1{Slice(), Slice()};
        Bytes r1;
        for (int i = 0; i < 100; ++i) {
            Bytes b = p1.get_bytes(1);
            r1.insert(r1.end(), b.begin(), b.end());
        }
        Prf p3{Slice(), Slice()};
        Bytes r3 = p3.get_bytes(33);
        Bytes b2 = p3.get_bytes(33);
        Bytes b3 = p3.get_bytes(34);
        r3.insert(r3.end(), b2.begin(), b2.end());
        r3.insert(r3.end(), b3.begin(), b3.end());
        Prf p2{Slice(), Slice()};
        CHECK(r1 == p2.get_bytes(100) && r1 == r3);
        const std::string jefe = "Jefe", msg = "what do ya want for nothing?";
        auto h = hmac_sha256(Slice(reinterpret_cast<const uint8_t*>(jefe.data()), jefe.size()),
                             Slice(reinterpret_cast<const uint8_t*>(msg.data()), msg.size()));
        CHECK(hex(h.data(), 32) == "5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843");
        auto e = sha256(Slice());
        CHECK(hex(e.data(), 32) == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");
        uint8_t cr[32], sr[32];
        for (int i = 0; i < 32; ++i) cr[i] = (uint8_t)i, sr[i] = (uint8_t)(100 + i);
        Bytes pm(32, 7);
        ConnectionKeys k = derive_keys(pm, cr, sr);
        Bytes seed(13 + 64);
        std::memcpy(seed.data(), "master secret", 13);
        std::memcpy(seed.data() + 13, cr, 32);
        std::memcpy(seed.data() + 45, sr, 32);
        CHECK(k.master_secret == Prf(pm, seed).get_bytes(48));
        std::memcpy(seed.data(), "key expansion", 13);
        std::memcpy(seed.data() + 13, sr, 32);
        std::memcpy(seed.data() + 45, cr, 32);
        Prf kb(k.master_secret, seed);
        CHECK(k.client_write_key == kb.get_bytes(32) && k.server_write_key == kb.get_bytes(32));
    }
    {  // cipher suite registration (mod.rs:108-114) and Aead constants (chacha20_poly1305.rs:102-119)
        auto aead = new_aead(TLS_ECDHE_RSA_WITH_CHACHA20_POLY1305_SHA256);
        CHECK(aead->key_size() == 32 && aead->fixed_iv_len() == 0 && aead->mac_len() == 16);
        CHECK(throws<std::invalid_argument>([] { new_aead(CipherSuite{"x", {0xc0, 0x2f}}); }));
    }
}

// ---- GPU ---------------------------------------------------------------------
static void gpu_tests() {
    ChaCha20Poly1305 aead(0);
    const Bytes key = key_seq(0);
    {  // the survey vector through Encryptor::encrypt, and back
        auto enc = aead.new_encryptor(key);
        const uint8_t nonce[8] = {0};
        uint8_t ad[13];
        so_tls_ad(0, 23, 3, 3, 16, ad);
        Bytes ct = enc->encrypt(Slice(nonce, 8), Bytes(16, 'A'), Slice(ad, 13));
        CHECK(hex(ct.data(), ct.size()) == kSurveyVector);
        auto dec = aead.new_decryptor(key);
        CHECK(dec->decrypt(Slice(nonce, 8), ct, Slice(ad, 13)) == Bytes(16, 'A'));
        ct[3] ^= 0x10;
        CHECK(throws<TlsError>([&] { dec->decrypt(Slice(nonce, 8), ct, Slice(ad, 13)); },
                               [](const TlsError& e) { return e.kind == TlsErrorKind::BadRecordMac && e.desc == "wrong mac"; }));
        CHECK(throws<TlsError>([&] { dec->decrypt(Slice(nonce, 8), Slice(ct.data(), 15), Slice(ad, 13)); },
                               [](const TlsError& e) { return e.desc == "message too short"; }));
        CHECK(throws<std::invalid_argument>([&] { enc->encrypt(Slice(nonce, 7), Bytes(1), Slice(ad, 13)); }));
        CHECK(throws<std::invalid_argument>([&] { aead.new_encryptor(Bytes(31)); }));
    }
    {  // random lengths / ad lengths against the oracle
        auto enc = aead.new_encryptor(key_seq(7));
        auto dec = aead.new_decryptor(key_seq(7));
        const size_t lens[] = {0, 1, 15, 16, 17, 63, 64, 65, 1000, 1024, 1025, 4097, 16383, 16384};
        uint64_t j = 0;
        for (size_t n : lens) {
            for (size_t adlen : {0, 5, 13, 32}) {
                Bytes pt = fill(0xC0FFEE, j, n), ad = fill(0xADAD, j, adlen), nonce = fill(0x4E4F, j, 8);
                ++j;
                Bytes ref(n + 16);
                so_seal(key_seq(7).data(), nonce.data(), pt.data(), n, ad.data(), adlen, ref.data());
                Bytes got = enc->encrypt(nonce, pt, ad);
                CHECK(got == ref);
                CHECK(dec->decrypt(nonce, got, ad) == pt);
            }
        }
    }
    {  // batched writer (one sg_write_records per write) -> reference reader
        VecWriter out;
        TlsWriter w(out);
        w.set_encryptor(aead.new_encryptor(key));
        Bytes data = fill(0x53555255, 1, 5 * RECORD_MAX_LEN + 1234);
        w.write_change_cipher_spec();
        w.write_application_data(data);
        w.write_application_data(Bytes{'t', 'a', 'i', 'l'});
        CHECK(w.write_count == 8);
        SliceReader in(out.buf);
        TlsReader r(in);
        r.set_decryptor(std::make_unique<OracleDecryptor>(key));
        CHECK(r.read_message().kind == Message::ChangeCipherSpec);
        Bytes got;
        for (int i = 0; i < 6; ++i) {
            Bytes p = r.read_application_data();
            got.insert(got.end(), p.begin(), p.end());
        }
        CHECK(got == data);
        CHECK(r.read_application_data() == (Bytes{'t', 'a', 'i', 'l'}));
    }
    {  // reference writer -> stream reader (uneven slices) and -> trait-object reader
        VecWriter out;
        TlsWriter w(out);
        w.set_encryptor(std::make_unique<OracleEncryptor>(key_seq(1)));
        std::vector<Bytes> pieces;
        for (size_t n : {size_t(1), size_t(100), RECORD_MAX_LEN, size_t(3000), size_t(17)}) {
            pieces.push_back(fill(9, pieces.size(), n));
            w.write_application_data(pieces.back());
        }
        ChaCha20Poly1305Decryptor dec(key_seq(1), 0);
        RecordStreamReader rd(dec);
        Bytes plain;
        std::vector<std::pair<ContentType, uint32_t>> recs;
        for (size_t i = 0; i < out.buf.size(); i += 7777) {
            rd.feed(out.buf.data() + i, std::min<size_t>(7777, out.buf.size() - i));
            auto got = rd.drain(plain);
            recs.insert(recs.end(), got.begin(), got.end());
        }
        Bytes want;
        for (auto& p : pieces) want.insert(want.end(), p.begin(), p.end());
        CHECK(plain == want && recs.size() == 5 && rd.read_count == 5 && rd.buffered() == 0);
        SliceReader in(out.buf);
        TlsReader r(in);
        r.set_decryptor(aead.new_decryptor(key_seq(1)));
        for (auto& p : pieces) CHECK(r.read_application_data() == p);
    }
    {  // stream reader errors: tampered record 2, unknown type
        VecWriter out;
        TlsWriter w(out);
        w.set_encryptor(std::make_unique<OracleEncryptor>(Bytes(32, 0)));
        for (int j = 0; j < 4; ++j) w.write_application_data(Bytes(500, static_cast<uint8_t>(j)));
        Bytes wire = out.buf;
        const size_t rec = 5 + 516;
        wire[2 * rec + 10] ^= 0x40;
        ChaCha20Poly1305Decryptor dec(Bytes(32, 0), 0);
        RecordStreamReader rd(dec);
        rd.feed(wire.data(), wire.size());
        Bytes plain;
        CHECK(throws<TlsError>([&] { rd.drain(plain); }, kind_is(TlsErrorKind::BadRecordMac)));
        CHECK(rd.read_count == 2 && plain.size() == 1000 && rd.buffered() == 2 * rec);
        RecordStreamReader rd2(dec);
        Bytes bad(out.buf.begin(), out.buf.begin() + rec);
        for (uint8_t b : {0x18, 3, 3, 0, 3, 1, 2, 3}) bad.push_back(b);
        rd2.feed(bad.data(), bad.size());
        Bytes p2;
        CHECK(throws<TlsError>([&] { rd2.drain(p2); }, kind_is(TlsErrorKind::UnexpectedMessage)));
        CHECK(rd2.read_count == 1);
    }
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    try {
        if (mode == "cpu") cpu_tests();
        else if (mode == "gpu") gpu_tests();
        else {
            std::fprintf(stderr, "usage: %s cpu|gpu\n", argv[0]);
            return 2;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "uncaught exception: %s\n", e.what());
        ++g_fail;
    }
    std::printf("%s: %d passed, %d failed\n", mode.c_str(), g_pass, g_fail);
    return g_fail ? 1 : 0;
}
