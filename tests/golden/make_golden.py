#!/usr/bin/env python3
"""Generate the committed parity fixtures under tests/golden/.

Run in the build container only (needs /root/reference for the KAT
extraction and OpenSSL libcrypto for the cross-check); the GPU box only reads
the JSON this writes.  The fixtures are DATA: inputs and expected outputs.

1. reference_kats.json -- the known-answer vectors held by the reference's own
   unit tests, extracted (bytes only) from
     src/crypto/chacha20.rs:169-228  test_chacha20 (5 keystreams)
     src/crypto/poly1305.rs:406-458  test_poly1305_examples (4 MACs)
   The key/nonce set-up of test_chacha20 (:173-210) is procedural; it is
   restated below.

2. aead_vectors.json -- AEAD-level vectors (the reference has none, SURVEY.md
   8c): seal outputs of suruga's draft-agl-04 construction
   (chacha20_poly1305.rs:19-94 with tls.rs:103-112 nonce/AD) computed by an
   independent pure-Python restatement (big-integer Poly1305, the textbook
   definition) and cross-checked, primitive by primitive, against OpenSSL
   3.0 libcrypto: EVP_chacha20 with IV = le32(counter) || 0^4 || nonce8
   reproduces suruga's state layout (counter in word 12, word 13 = 0,
   chacha20.rs:41-46) and EVP_MAC "POLY1305" with key r || s matches
   poly1305::authenticate.  OpenSSL's own EVP_chacha20_poly1305 is the RFC 7539
   construction and is NOT used.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes as C
import ctypes.util
import hashlib
import json
import os
import random
import re
import struct
from pathlib import Path

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("SURUGA_REFERENCE", "/root/reference"))
FILL_SEED = 0x53555255  # "SURU"
P1305 = (1 << 130) - 5

# ---------------------------------------------------------------------------
# independent restatement (pure Python)
# ---------------------------------------------------------------------------
M32 = 0xFFFFFFFF


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & M32


def chacha_block(key: bytes, nonce: bytes, counter: int) -> bytes:
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    s += list(struct.unpack("<8I", key))
    s += [counter & M32, 0]
    s += list(struct.unpack("<2I", nonce))
    x = s[:]

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return struct.pack("<16I", *[(x[i] + s[i]) & M32 for i in range(16)])


def chacha_xor(key: bytes, nonce: bytes, counter: int, data: bytes) -> bytes:
    out = bytearray()
    for off in range(0, len(data), 64):
        ks = chacha_block(key, nonce, counter)
        counter = (counter + 1) & M32  # word 12 only, no carry (chacha20.rs:114-121)
        chunk = data[off:off + 64]
        out += bytes(a ^ b for a, b in zip(chunk, ks))
    return bytes(out)


def poly1305(msg: bytes, key32: bytes) -> bytes:
    r = int.from_bytes(key32[:16], "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    s = int.from_bytes(key32[16:32], "little")
    h = 0
    for off in range(0, len(msg), 16):
        blk = msg[off:off + 16]
        h = ((h + int.from_bytes(blk + b"\x01", "little")) * r) % P1305
    return ((h + s) % (1 << 128)).to_bytes(16, "little")


def mac_input(ad: bytes, ct: bytes) -> bytes:
    # chacha20_poly1305.rs:24-30: ad || le64(|ad|) || ct || le64(|ct|)
    return ad + struct.pack("<Q", len(ad)) + ct + struct.pack("<Q", len(ct))


def seal(key: bytes, nonce: bytes, pt: bytes, ad: bytes) -> bytes:
    pk = chacha_block(key, nonce, 0)
    ct = chacha_xor(key, nonce, 1, pt)
    return ct + poly1305(mac_input(ad, ct), pk[:32])


def tls_nonce(seq: int) -> bytes:
    return struct.pack(">Q", seq)  # u64_be_array (util.rs:43-45, tls.rs:103)


def tls_ad(seq: int, n: int, ctype: int = 23, ver=(3, 3)) -> bytes:
    return struct.pack(">Q", seq) + bytes([ctype, ver[0], ver[1]]) + struct.pack(">H", n)


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def fill_record(seed: int, j: int, n: int) -> bytes:
    out = bytearray()
    for w in range((n + 7) // 8):
        out += struct.pack("<Q", splitmix64(seed ^ ((j << 32) & 0xFFFFFFFFFFFFFFFF) ^ w))
    return bytes(out[:n])


# ---------------------------------------------------------------------------
# OpenSSL cross-check (primitives only)
# ---------------------------------------------------------------------------
class OpenSSL:
    def __init__(self):
        path = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = C.CDLL(path)
        L.EVP_CIPHER_CTX_new.restype = C.c_void_p
        L.EVP_chacha20.restype = C.c_void_p
        L.EVP_EncryptInit_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_char_p]
        L.EVP_EncryptUpdate.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int), C.c_char_p, C.c_int]
        L.EVP_CIPHER_CTX_free.argtypes = [C.c_void_p]
        L.EVP_MAC_fetch.restype = C.c_void_p
        L.EVP_MAC_fetch.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
        L.EVP_MAC_CTX_new.restype = C.c_void_p
        L.EVP_MAC_CTX_new.argtypes = [C.c_void_p]
        L.EVP_MAC_init.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p]
        L.EVP_MAC_update.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        L.EVP_MAC_final.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_size_t), C.c_size_t]
        L.EVP_MAC_CTX_free.argtypes = [C.c_void_p]
        self.L = L
        self.mac = L.EVP_MAC_fetch(None, b"POLY1305", None)
        assert self.mac, "OpenSSL POLY1305 unavailable"

    def chacha20(self, key, nonce, counter, data):
        L = self.L
        ctx = L.EVP_CIPHER_CTX_new()
        iv = struct.pack("<I", counter) + b"\x00" * 4 + nonce
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_chacha20(), None, key, iv) == 1
        out = C.create_string_buffer(len(data) + 64)
        ol = C.c_int(0)
        if data:
            assert L.EVP_EncryptUpdate(ctx, out, C.byref(ol), data, len(data)) == 1
        L.EVP_CIPHER_CTX_free(ctx)
        return out.raw[:ol.value]

    def poly1305(self, msg, key32):
        L = self.L
        ctx = L.EVP_MAC_CTX_new(self.mac)
        assert L.EVP_MAC_init(ctx, key32, 32, None) == 1
        if msg:
            assert L.EVP_MAC_update(ctx, msg, len(msg)) == 1
        out = C.create_string_buffer(16)
        ol = C.c_size_t(0)
        assert L.EVP_MAC_final(ctx, out, C.byref(ol), 16) == 1
        L.EVP_MAC_CTX_free(ctx)
        return out.raw[:16]

    def seal(self, key, nonce, pt, ad):
        pk = self.chacha20(key, nonce, 0, b"\x00" * 32)
        ct = self.chacha20(key, nonce, 1, pt)
        return ct + self.poly1305(mac_input(ad, ct), pk)


# ---------------------------------------------------------------------------
# KAT extraction from the reference's unit tests (bytes only)
# ---------------------------------------------------------------------------
def _bytes_literals(src: str):
    """b"\\x.." literals (with line continuations) in source order."""
    out = []
    for m in re.finditer(r'b"((?:\\x[0-9a-fA-F]{2}|\\\n\s*)*)"', src):
        body = re.sub(r"\\\n\s*", "", m.group(1))
        out.append(bytes(int(h, 16) for h in re.findall(r"\\x([0-9a-fA-F]{2})", body)))
    return out


def chacha_kats():
    path = REF / "src/crypto/chacha20.rs"
    src = path.read_text()
    streams = _bytes_literals(src[src.index("fn test_chacha20"):])
    assert len(streams) == 5, len(streams)
    # key/nonce set-up of test_chacha20 (chacha20.rs:173-210)
    k0, n0 = bytes(32), bytes(8)
    k1 = bytes(31) + b"\x01"
    n7 = bytes(7) + b"\x01"
    n0_1 = b"\x01" + bytes(7)
    kseq, nseq = bytes(range(32)), bytes(range(8))
    setups = [(k0, n0, "chacha20.rs:175-179"), (k1, n0, "chacha20.rs:181-186"),
              (k0, n7, "chacha20.rs:188-194"), (k0, n0_1, "chacha20.rs:196-203"),
              (kseq, nseq, "chacha20.rs:205-227")]
    return [{"key": k.hex(), "nonce": n.hex(), "keystream": ks.hex(), "source": srcref}
            for (k, n, srcref), ks in zip(setups, streams)]


def poly_kats():
    path = REF / "src/crypto/poly1305.rs"
    src = path.read_text()
    body = src[src.index("fn test_poly1305_examples"):]
    body = body[:body.index("for &(msg")]
    tuples = re.findall(r"\(\s*&\[(.*?)\]\s*,\s*\[(.*?)\]\s*,\s*\[(.*?)\]\s*,\s*\[(.*?)\]\s*\)", body, re.S)
    assert len(tuples) == 4, len(tuples)

    def arr(s):
        return bytes(int(h, 16) for h in re.findall(r"0x([0-9a-fA-F]{2})", s))

    return [{"msg": arr(a).hex(), "r": arr(b).hex(), "s": arr(c).hex(), "tag": arr(d).hex(),
             "source": "poly1305.rs:409-452"} for a, b, c, d in tuples]


def int1305_coeffs():
    """COEFFS table of poly1305.rs:321-340 (limb values, restated)."""
    m26, m25 = (1 << 26) - 1, (1 << 25) - 1
    return [[0, 0, 0, 0, 0], [1, 0, 0, 0, 0], [1, 1, 1, 1, 1], [m26, m26, m26, m26, m25],
            [0, 1, 2, 3, 4], [5, 6, 7, 8, 9], [1 << 23, 3 << 20, 0, 5 << 21, 0], [1 << 20] * 5,
            [1 << 24] * 5, [m25] * 5, [0x3fffffb - 1, 0x3ffffff, 0x3ffffff, 0x3ffffff, 0x3ffffff]]


# ---------------------------------------------------------------------------
def main():
    ossl = OpenSSL()
    kats = {"chacha20": chacha_kats(), "poly1305": poly_kats(), "int1305_coeffs": int1305_coeffs(),
            "int1305_coeffs_source": "poly1305.rs:321-340"}
    for v in kats["chacha20"]:
        key, nonce, ks = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["keystream"])
        assert chacha_xor(key, nonce, 0, bytes(len(ks))) == ks
        assert ossl.chacha20(key, nonce, 0, bytes(len(ks))) == ks
    for v in kats["poly1305"]:
        key32 = bytes.fromhex(v["r"]) + bytes.fromhex(v["s"])
        assert poly1305(bytes.fromhex(v["msg"]), key32).hex() == v["tag"]
        assert ossl.poly1305(bytes.fromhex(v["msg"]), key32).hex() == v["tag"]

    vectors = []
    key = bytes(range(32))

    def add(name, key, nonce, pt, ad, tls=None, full=True, gen=None):
        out = seal(key, nonce, pt, ad)
        assert out == ossl.seal(key, nonce, pt, ad), name
        v = {"name": name, "key": key.hex(), "nonce": nonce.hex(), "ad": ad.hex(), "n": len(pt)}
        if tls is not None:
            v["tls_seq"] = tls
        if gen is not None:
            v["pt_gen"] = gen
        else:
            v["pt"] = pt.hex()
        if full:
            v["ct_tag"] = out.hex()
        v["tag"] = out[-16:].hex()
        v["ct_sha256"] = hashlib.sha256(out[:-16]).hexdigest()
        vectors.append(v)

    # survey sample: key 00..1f, seq 0, type 23, ver 3.3, pt "A"*16
    pt = b"A" * 16
    add("survey_sample", key, tls_nonce(0), pt, tls_ad(0, 16), tls=0)
    assert vectors[-1]["ct_tag"] == "59f90370eca7e79052201d20ee020f66fbc2d9037460b094b3443d3ec89ef135"

    lengths = [0, 1, 15, 16, 17, 63, 64, 65, 255, 256, 1023, 1024, 4095, 16383, 16384]
    seqs = [0, 1, 0xFFFFFFFF, 0x100000000, 0xFFFFFFFFFFFFFFFF]
    for n in lengths:
        seq = 0
        pt = fill_record(FILL_SEED, seq, n)
        add(f"tls_len{n}", key, tls_nonce(seq), pt, tls_ad(seq, n), tls=seq, full=n <= 1024,
            gen=None if n <= 1024 else {"seed": FILL_SEED, "j": seq})
    for seq in seqs[1:]:
        for n in (1, 64, 1024, 16384):
            pt = fill_record(FILL_SEED, seq & 0xFFFFFFFF, n)
            add(f"tls_seq{seq:#x}_len{n}", key, tls_nonce(seq), pt, tls_ad(seq, n), tls=seq,
                full=n <= 1024, gen=None if n <= 1024 else {"seed": FILL_SEED, "j": seq & 0xFFFFFFFF})
    rng = random.Random(0x5EED)
    for adlen in (0, 5, 13, 32, 255):
        for n in (0, 17, 100, 1000):
            k = bytes(rng.randrange(256) for _ in range(32))
            nonce = bytes(rng.randrange(256) for _ in range(8))
            ad = bytes(rng.randrange(256) for _ in range(adlen))
            pt = bytes(rng.randrange(256) for _ in range(n))
            add(f"explicit_ad{adlen}_len{n}", k, nonce, pt, ad)
    # reference test key variants at TLS framing
    for i, (k, tag) in enumerate([(bytes(32), "zero_key"), (bytes(31) + b"\x01", "key31")]):
        pt = fill_record(FILL_SEED, 7, 300)
        add(f"tls_{tag}_len300", k, tls_nonce(7), pt, tls_ad(7, 300), tls=7)

    # tamper cases (open must return BadRecordMac): indices into ct_tag
    tampers = [
        {"vector": "tls_len1024", "flip": 0, "expect": "BadRecordMac/wrong mac"},
        {"vector": "tls_len1024", "flip": 1023, "expect": "BadRecordMac/wrong mac"},
        {"vector": "tls_len1024", "flip": 1024 + 15, "expect": "BadRecordMac/wrong mac"},
        {"vector": "tls_len0", "flip": 0, "expect": "BadRecordMac/wrong mac"},
        {"vector": "explicit_ad13_len17", "flip": 5, "expect": "BadRecordMac/wrong mac"},
    ]
    short = [{"len": L, "expect": "BadRecordMac/message too short"} for L in (0, 1, 15)]

    (HERE / "reference_kats.json").write_text(json.dumps(kats, indent=1) + "\n")
    doc = {
        "construction": "draft-agl-tls-chacha20poly1305-04 as in klutzy/suruga "
                        "src/cipher/chacha20_poly1305.rs (NOT RFC 7539)",
        "generator": "tests/golden/make_golden.py (pure-Python restatement, cross-checked "
                     "against OpenSSL libcrypto EVP_chacha20 + EVP_MAC POLY1305)",
        "pt_gen_rule": "byte i of record j = byte (i mod 8) of splitmix64(seed ^ (j << 32) ^ (i / 8))",
        "vectors": vectors, "tamper": tampers, "short": short,
    }
    (HERE / "aead_vectors.json").write_text(json.dumps(doc, indent=1) + "\n")
    print(f"wrote {len(kats['chacha20'])} + {len(kats['poly1305'])} KATs, {len(vectors)} AEAD vectors")


if __name__ == "__main__":
    main()
