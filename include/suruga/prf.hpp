// suruga/prf.hpp -- C++ mirror of suruga's TLS 1.2 PRF and the client key
// schedule (src/cipher/prf.rs, src/client.rs:130-225) over the C ABI.
#ifndef SURUGA_PRF_HPP
#define SURUGA_PRF_HPP

#include <array>
#include <memory>

#include "cipher.hpp"

namespace suruga {

inline std::array<uint8_t, 32> sha256(Slice msg) {  // crypto/sha2.rs:18
    std::array<uint8_t, 32> out;
    sg_sha256(msg.data, msg.size, out.data());
    return out;
}

inline std::array<uint8_t, 32> hmac_sha256(Slice key, Slice msg) {  // prf.rs:8-29
    std::array<uint8_t, 32> out;
    check_sg(sg_hmac_sha256(key.data, key.size, msg.data, msg.size, out.data()));
    return out;
}

// prf.rs:31-89
class Prf {
public:
    Prf(Slice secret, Slice seed) : h_(sg_prf_new(secret.data, secret.size, seed.data, seed.size), &sg_prf_free) {
        if (!h_) throw std::invalid_argument(sg_last_error());
    }
    Bytes get_bytes(size_t n) {
        Bytes out(n);
        check_sg(sg_prf_get_bytes(h_.get(), out.data(), n));
        return out;
    }

private:
    std::unique_ptr<sg_prf, void (*)(sg_prf*)> h_;
};

// client.rs:130-163: one connection's AEAD keys.
struct ConnectionKeys {
    Bytes master_secret, client_write_key, server_write_key;
};
inline ConnectionKeys derive_keys(Slice pre_master, const uint8_t client_random[32], const uint8_t server_random[32]) {
    ConnectionKeys k{Bytes(48), Bytes(32), Bytes(32)};
    check_sg(sg_derive_keys(1, pre_master.data, pre_master.size, pre_master.size, client_random, server_random,
                            k.master_secret.data(), k.client_write_key.data(), k.server_write_key.data(), 1));
    return k;
}

}  // namespace suruga

#endif  // SURUGA_PRF_HPP
