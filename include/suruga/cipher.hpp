// suruga/cipher.hpp -- C++ host-side mirror of suruga's cipher plugin
// interface (klutzy/suruga src/cipher/mod.rs:14-32, tls_result.rs) with the
// MI355X ChaCha20-Poly1305 behind it.  Header-only over the C ABI in
// ../suruga_gpu.h; link libsuruga_gpu.so.
//
//   trait Aead / Encryptor / Decryptor      mod.rs:14-32   -> suruga::Aead / Encryptor / Decryptor
//   struct ChaCha20Poly1305 (+Encryptor/Decryptor) chacha20_poly1305.rs:44-135
//                                           -> suruga::ChaCha20Poly1305 (GPU)
//   TlsError / TlsErrorKind                 tls_result.rs:5-64 -> suruga::TlsError
//
// Ownership mirrors the reference: the key is moved into the encryptor
// (chacha20_poly1305.rs:121-125), inputs are borrowed, outputs are fresh owned
// buffers.  Panics of the reference (bad key / nonce length, chacha20.rs:26-27)
// are std::invalid_argument here; open failures are TlsError{BadRecordMac}.
#ifndef SURUGA_CIPHER_HPP
#define SURUGA_CIPHER_HPP

#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../suruga_gpu.h"

namespace suruga {

using Bytes = std::vector<uint8_t>;

// Borrowed byte slice (&[u8]).
struct Slice {
    const uint8_t* data = nullptr;
    size_t size = 0;
    Slice() = default;
    Slice(const uint8_t* p, size_t n) : data(p), size(n) {}
    Slice(const Bytes& v) : data(v.data()), size(v.size()) {}  // NOLINT: implicit like &Vec<u8> -> &[u8]
};

// tls_result.rs:5-20
enum class TlsErrorKind {
    UnexpectedMessage,
    BadRecordMac,
    RecordOverflow,
    IllegalParameter,
    DecodeError,
    DecryptError,
    InternalError,
    IoFailure,
    AlertReceived,
};

inline const char* kind_name(TlsErrorKind k) {
    switch (k) {
        case TlsErrorKind::UnexpectedMessage: return "UnexpectedMessage";
        case TlsErrorKind::BadRecordMac: return "BadRecordMac";
        case TlsErrorKind::RecordOverflow: return "RecordOverflow";
        case TlsErrorKind::IllegalParameter: return "IllegalParameter";
        case TlsErrorKind::DecodeError: return "DecodeError";
        case TlsErrorKind::DecryptError: return "DecryptError";
        case TlsErrorKind::InternalError: return "InternalError";
        case TlsErrorKind::IoFailure: return "IoFailure";
        case TlsErrorKind::AlertReceived: return "AlertReceived";
    }
    return "?";
}

// tls_result.rs:22-35 (TlsError { kind, desc })
class TlsError : public std::runtime_error {
public:
    TlsError(TlsErrorKind kind, std::string desc)
        : std::runtime_error(std::string(kind_name(kind)) + ": " + desc), kind(kind), desc(std::move(desc)) {}
    TlsErrorKind kind;
    std::string desc;
};

// Runtime failure of the GPU library (HIP error, no device): not a TLS error.
class GpuError : public std::runtime_error {
public:
    GpuError(int code, const std::string& what) : std::runtime_error(what), code(code) {}
    int code;
};

inline void check_sg(int rc) {
    if (rc < 0) {
        if (rc == SG_E_ARG) throw std::invalid_argument(sg_last_error());
        throw GpuError(rc, sg_last_error());
    }
}

// mod.rs:22-24
class Encryptor {
public:
    virtual ~Encryptor() = default;
    virtual Bytes encrypt(Slice nonce, Slice plain, Slice ad) = 0;
};

// mod.rs:28-32
class Decryptor {
public:
    virtual ~Decryptor() = default;
    virtual Bytes decrypt(Slice nonce, Slice encrypted, Slice ad) = 0;  // throws TlsError
    virtual size_t mac_len() const = 0;
};

// mod.rs:14-20
class Aead {
public:
    virtual ~Aead() = default;
    virtual size_t key_size() const = 0;
    virtual size_t fixed_iv_len() const = 0;
    virtual size_t mac_len() const = 0;
    virtual std::unique_ptr<Encryptor> new_encryptor(Bytes key) const = 0;
    virtual std::unique_ptr<Decryptor> new_decryptor(Bytes key) const = 0;
};

namespace detail {
// One sg_ctx per direction (the reference boxes one key per direction).
class Ctx {
public:
    Ctx(const Bytes& key, int device) {
        if (key.size() != SG_KEY_LEN) throw std::invalid_argument("ChaCha20: key must be 32 bytes");  // chacha20.rs:26
        c_ = sg_ctx_new(key.data(), device);
        if (!c_) throw GpuError(SG_E_NODEV, sg_last_error());
    }
    ~Ctx() { sg_ctx_free(c_); }
    Ctx(const Ctx&) = delete;
    Ctx& operator=(const Ctx&) = delete;
    sg_ctx* get() const { return c_; }

private:
    sg_ctx* c_ = nullptr;
};

inline void check_nonce(Slice nonce) {
    if (nonce.size != SG_NONCE_LEN) throw std::invalid_argument("ChaCha20: nonce must be 8 bytes");  // chacha20.rs:27
}
}  // namespace detail

// chacha20_poly1305.rs:44-59
class ChaCha20Poly1305Encryptor : public Encryptor {
public:
    ChaCha20Poly1305Encryptor(Bytes key, int device) : ctx_(key, device) {}
    Bytes encrypt(Slice nonce, Slice plain, Slice ad) override {
        detail::check_nonce(nonce);
        Bytes out(plain.size + SG_MAC_LEN);
        check_sg(sg_seal(ctx_.get(), nonce.data, nonce.size, plain.data, plain.size, ad.data, ad.size, out.data()));
        return out;
    }
    sg_ctx* handle() const { return ctx_.get(); }  // batched record layer (tls.hpp)

private:
    detail::Ctx ctx_;
};

// chacha20_poly1305.rs:61-100
class ChaCha20Poly1305Decryptor : public Decryptor {
public:
    ChaCha20Poly1305Decryptor(Bytes key, int device) : ctx_(key, device) {}
    Bytes decrypt(Slice nonce, Slice encrypted, Slice ad) override {
        detail::check_nonce(nonce);
        if (encrypted.size < SG_MAC_LEN)  // :68-70
            throw TlsError(TlsErrorKind::BadRecordMac, "message too short");
        Bytes out(encrypted.size - SG_MAC_LEN);
        const int rc = sg_open(ctx_.get(), nonce.data, nonce.size, encrypted.data, encrypted.size, ad.data, ad.size,
                               out.data());
        if (rc == SG_E_SHORT) throw TlsError(TlsErrorKind::BadRecordMac, "message too short");
        if (rc == SG_E_BAD_MAC) throw TlsError(TlsErrorKind::BadRecordMac, "wrong mac");  // :89-90
        check_sg(rc);
        return out;
    }
    size_t mac_len() const override { return SG_MAC_LEN; }  // :96-99
    sg_ctx* handle() const { return ctx_.get(); }

private:
    detail::Ctx ctx_;
};

// chacha20_poly1305.rs:102-135; `device` is the HIP ordinal the contexts use.
class ChaCha20Poly1305 : public Aead {
public:
    explicit ChaCha20Poly1305(int device = 0) : device_(device) {}
    size_t key_size() const override { return sg_key_size(); }
    size_t fixed_iv_len() const override { return sg_fixed_iv_len(); }
    size_t mac_len() const override { return sg_mac_len(); }
    std::unique_ptr<Encryptor> new_encryptor(Bytes key) const override {
        return std::make_unique<ChaCha20Poly1305Encryptor>(std::move(key), device_);
    }
    std::unique_ptr<Decryptor> new_decryptor(Bytes key) const override {
        return std::make_unique<ChaCha20Poly1305Decryptor>(std::move(key), device_);
    }

private:
    int device_;
};

// cipher/mod.rs:100-114 cipher_suite!: the one suite served by this boundary.
struct CipherSuite {
    const char* name;
    uint8_t id[2];
};
inline constexpr CipherSuite TLS_ECDHE_RSA_WITH_CHACHA20_POLY1305_SHA256{
    "TLS_ECDHE_RSA_WITH_CHACHA20_POLY1305_SHA256", {0xcc, 0x13}};

// CipherSuite::new_aead (mod.rs:53-60)
inline std::unique_ptr<Aead> new_aead(const CipherSuite& s, int device = 0) {
    if (s.id[0] == 0xcc && s.id[1] == 0x13) return std::make_unique<ChaCha20Poly1305>(device);
    throw std::invalid_argument(std::string("unsupported cipher suite ") + s.name);
}

}  // namespace suruga

#endif  // SURUGA_CIPHER_HPP
