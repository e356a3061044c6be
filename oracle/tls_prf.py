"""CPU restatement of suruga's TLS 1.2 key schedule -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this (the checker of suruga_amd's sg_keysched.cpp); no
product path uses it.  Follows, line by line:

* hmac_sha256      src/cipher/prf.rs:8-29   (ipad 0x36 / opad 0x5c over a 64-byte
                                              block; keys > 64 bytes: unimplemented!)
* Prf              src/cipher/prf.rs:31-89  (A(1) = HMAC(secret, seed);
                                              next_block = HMAC(secret, A || seed),
                                              A <- HMAC(secret, A); get_bytes keeps the
                                              unused tail of a block in `buf`)
* derive_keys      src/client.rs:130-163    (master secret, key expansion order)
* verify_data      src/client.rs:184-192, 213-221

SHA-256 itself is Python's hashlib (OpenSSL), pinned to the reference by the
sha2.rs:123-141 answers in tests/test_keysched.py.  Parity pinned by the
reference's own vectors (prf.rs:95-167, sha2.rs:123-141) -- see tests.
"""
from __future__ import annotations

import hashlib


def sha256(msg: bytes) -> bytes:
    return hashlib.sha256(msg).digest()


def hmac_sha256(key: bytes, msg: bytes) -> bytes:  # prf.rs:8-29
    B = 64
    if len(key) > B:
        raise NotImplementedError("prf.rs:11-14 unimplemented!()")
    i_msg = bytearray([0x36] * B)
    o_msg = bytearray([0x5C] * B)
    for i, k in enumerate(key):
        i_msg[i] ^= k
        o_msg[i] ^= k
    h_i = sha256(bytes(i_msg) + msg)
    return sha256(bytes(o_msg) + h_i)


class Prf:  # prf.rs:31-89
    def __init__(self, secret: bytes, seed: bytes):
        self.secret, self.seed = bytes(secret), bytes(seed)
        self.a = hmac_sha256(self.secret, self.seed)
        self.buf = b""

    def next_block(self) -> bytes:
        nxt = hmac_sha256(self.secret, self.a + self.seed)
        self.a = hmac_sha256(self.secret, self.a)
        return nxt

    def get_bytes(self, size: int) -> bytes:
        buflen = len(self.buf)
        if buflen > 0:
            if buflen <= size:
                ret, self.buf = self.buf, b""
            else:
                ret, self.buf = self.buf[:size], self.buf[size:]
        else:
            ret = b""
        while len(ret) < size:
            block = self.next_block()
            slice_len = size - len(ret)
            if slice_len > 32:
                ret += block
            else:
                ret += block[:slice_len]
                self.buf = block[slice_len:]
                break
        return ret


def derive_keys(pre_master: bytes, client_random: bytes, server_random: bytes):
    """client.rs:130-163 -> (master_secret, client write key, server write key)."""
    master = Prf(pre_master, b"master secret" + client_random + server_random).get_bytes(48)
    prf = Prf(master, b"key expansion" + server_random + client_random)
    write_key = prf.get_bytes(32)
    read_key = prf.get_bytes(32)
    return master, write_key, read_key


def verify_data(master: bytes, server: bool, handshake_hash: bytes) -> bytes:  # client.rs:184-192, 213-221
    label = b"server finished" if server else b"client finished"
    return Prf(master, label + handshake_hash).get_bytes(12)
