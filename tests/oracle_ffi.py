"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of suruga's algorithm (oracle/suruga_oracle.c)
used as the parity checker.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg load it.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

SO_OK, SO_BAD_MAC, SO_SHORT = 0, 1, 2


class Int1305(C.Structure):
    _fields_ = [("v", C.c_uint32 * 5)]

    @classmethod
    def of(cls, limbs):
        x = cls()
        for i, v in enumerate(limbs):
            x.v[i] = v
        return x

    def limbs(self):
        return list(self.v)


class Oracle:
    def __init__(self, path: Path | None = None):
        if path is None and os.environ.get("SURUGA_ORACLE_LIB"):
            # another build of the same restatement (tests/test_sanitizers.py: -DSO_DEBUG, ASan/UBSan)
            path = Path(os.environ["SURUGA_ORACLE_LIB"])
        if path is None:
            from suruga_amd._build import build_oracle

            path = build_oracle()
        L = C.CDLL(str(path))
        u8p = C.c_char_p
        L.so_int1305_add.restype = Int1305
        L.so_int1305_add.argtypes = [Int1305, Int1305]
        L.so_int1305_mult.restype = Int1305
        L.so_int1305_mult.argtypes = [Int1305, Int1305]
        L.so_int1305_normalize.restype = Int1305
        L.so_int1305_normalize.argtypes = [Int1305]
        L.so_int1305_from_bytes.restype = Int1305
        L.so_int1305_from_bytes.argtypes = [u8p]
        L.so_poly1305_authenticate.argtypes = [u8p, C.c_size_t, u8p, u8p, C.c_void_p]
        L.so_chacha20_new.argtypes = [C.c_void_p, u8p, C.c_size_t, u8p, C.c_size_t]
        L.so_chacha20_new.restype = C.c_int
        L.so_chacha20_encrypt.argtypes = [C.c_void_p, u8p, C.c_size_t, C.c_void_p]
        L.so_seal.argtypes = [u8p, u8p, u8p, C.c_size_t, u8p, C.c_size_t, C.c_void_p]
        L.so_open.argtypes = [u8p, u8p, u8p, C.c_size_t, u8p, C.c_size_t, C.c_void_p]
        L.so_open.restype = C.c_int
        L.so_tls_ad.argtypes = [C.c_uint64, C.c_uint8, C.c_uint8, C.c_uint8, C.c_uint16, C.c_void_p]
        L.so_fill_record.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]
        L.so_splitmix64.restype = C.c_uint64
        L.so_splitmix64.argtypes = [C.c_uint64]
        L.so_seal_batch_tls.argtypes = [u8p, C.c_uint64, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                        C.c_int]
        L.so_open_batch_tls.argtypes = [u8p, C.c_uint64, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                        C.c_void_p, C.c_int]
        L.so_open_batch_tls.restype = C.c_size_t
        L.so_tag_fold_tls.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_size_t, C.c_size_t, C.c_int,
                                      C.c_void_p]
        L.so_tag_fold_mixed.argtypes = [C.c_void_p] * 6 + [C.c_size_t, C.c_int, C.c_void_p]
        L.so_batch_mixed.restype = C.c_size_t
        L.so_batch_mixed.argtypes = [C.c_int] + [C.c_void_p] * 9 + [C.c_size_t, C.c_int]
        self.L = L

    # --- primitives
    def keystream(self, key: bytes, nonce: bytes, n: int) -> bytes:
        st = (C.c_uint32 * 16)()
        if self.L.so_chacha20_new(st, key, len(key), nonce, len(nonce)) != 0:
            raise ValueError("bad key/nonce length")
        out = C.create_string_buffer(max(n, 1))
        self.L.so_chacha20_encrypt(st, bytes(n), n, out)
        return out.raw[:n]

    def poly1305(self, msg: bytes, r: bytes, s: bytes) -> bytes:
        out = C.create_string_buffer(16)
        self.L.so_poly1305_authenticate(msg, len(msg), r, s, out)
        return out.raw

    def add(self, a, b):
        return self.L.so_int1305_add(Int1305.of(a), Int1305.of(b)).limbs()

    def mult(self, a, b):
        return self.L.so_int1305_mult(Int1305.of(a), Int1305.of(b)).limbs()

    def normalize(self, a):
        return self.L.so_int1305_normalize(Int1305.of(a)).limbs()

    # --- AEAD
    def seal(self, key: bytes, nonce: bytes, pt: bytes, ad: bytes) -> bytes:
        out = C.create_string_buffer(len(pt) + 16)
        self.L.so_seal(key, nonce, pt, len(pt), ad, len(ad), out)
        return out.raw

    def open(self, key: bytes, nonce: bytes, data: bytes, ad: bytes):
        out = C.create_string_buffer(max(len(data), 1))
        rc = self.L.so_open(key, nonce, data, len(data), ad, len(ad), out)
        return rc, out.raw[:max(len(data) - 16, 0)]

    def tls_ad(self, seq: int, n: int, ctype: int = 23, major: int = 3, minor: int = 3) -> bytes:
        out = C.create_string_buffer(13)
        self.L.so_tls_ad(seq, ctype, major, minor, n, out)
        return out.raw

    def fill_record(self, seed: int, j: int, n: int) -> bytes:
        out = C.create_string_buffer(max(n, 1))
        self.L.so_fill_record(seed, j, out, n)
        return out.raw[:n]

    def seal_batch_tls(self, key: bytes, seq0: int, pt: bytes, n: int, count: int, threads: int = 1) -> bytes:
        out = C.create_string_buffer((n + 16) * count)
        self.L.so_seal_batch_tls(key, seq0, pt, n, count, out, threads)
        return out.raw

    def open_batch_tls(self, key: bytes, seq0: int, ct: bytes, n: int, count: int, threads: int = 1):
        out = C.create_string_buffer(max(n * count, 1))
        st = C.create_string_buffer(max(count, 1))
        bad = self.L.so_open_batch_tls(key, seq0, ct, n, count, out, st, threads)
        return bad, out.raw[:n * count], st.raw[:count]

    def tag_fold_mixed(self, keys: bytes, key_index, seq, lens, in_off, pt, threads: int = 1) -> bytes:
        """XOR of the tags of a mixed TLS batch (numpy uint32/uint64 arrays, pt a
        uint8 numpy array): record i = pt[in_off[i]:+lens[i]], key key_index[i],
        sequence number seq[i]."""
        import numpy as np

        arrs = [np.ascontiguousarray(a) for a in (key_index.astype(np.uint32), seq.astype(np.uint64),
                                                  lens.astype(np.uint32), in_off.astype(np.uint64))]
        kb = C.create_string_buffer(bytes(keys), len(keys))
        out = C.create_string_buffer(16)
        self.L.so_tag_fold_mixed(kb, *[a.ctypes.data_as(C.c_void_p) for a in arrs],
                                 np.ascontiguousarray(pt).ctypes.data_as(C.c_void_p), len(lens), threads, out)
        return out.raw

    def tag_fold_tls(self, key: bytes, seq0: int, seed: int, j0: int, n: int, count: int, threads: int = 1) -> bytes:
        """XOR of the tags of count sealed fill-rule records (never materialised)."""
        out = C.create_string_buffer(16)
        self.L.so_tag_fold_tls(key, seq0, seed, j0, n, count, threads, out)
        return out.raw


_oracle = None


def oracle() -> Oracle:
    global _oracle
    if _oracle is None:
        _oracle = Oracle()
    return _oracle


class OsslLine:
    """oracle/ossl_aead.c: suruga's AEAD composed from OpenSSL primitives -- the
    optimised-CPU comparison line of bench.py (not a parity reference)."""

    def __init__(self):
        from suruga_amd._build import build_ossl

        path = build_ossl()
        if path is None or not path.exists():
            raise OSError("libossl_aead.so unavailable (no libcrypto headers)")
        self.L = C.CDLL(str(path))
        self.L.ossl_batch_tls.restype = C.c_size_t
        self.L.ossl_batch_tls.argtypes = [C.c_int, C.c_char_p, C.c_uint64, C.c_void_p, C.c_size_t, C.c_size_t,
                                          C.c_void_p, C.c_int]
        self.L.ossl_batch_mixed.restype = C.c_size_t
        self.L.ossl_batch_mixed.argtypes = [C.c_int] + [C.c_void_p] * 8 + [C.c_size_t, C.c_int]

    def seal_batch_tls(self, key, seq0, pt, n, count, threads=1) -> bytes:
        out = C.create_string_buffer((n + 16) * count)
        rc = self.L.ossl_batch_tls(0, key, seq0, C.cast(C.c_char_p(pt), C.c_void_p), n, count, out, threads)
        if rc == C.c_size_t(-1).value:
            raise OSError("POLY1305 not available in libcrypto")
        return out.raw

    def open_batch_tls(self, key, seq0, ct, n, count, threads=1):
        out = C.create_string_buffer(max(n * count, 1))
        bad = self.L.ossl_batch_tls(1, key, seq0, C.cast(C.c_char_p(ct), C.c_void_p), n, count, out, threads)
        return bad, out.raw[:n * count]
