"""TLS 1.2 key schedule (suruga src/cipher/prf.rs, src/client.rs:130-225) over
the C ABI: ``hmac_sha256``, ``Prf`` and the per-connection key derivation that
fills the key tables of the batch calls.  Host code (sg_keysched.cpp); no GPU
needed, no Python fallback."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


def sha256(msg: bytes) -> bytes:  # crypto/sha2.rs:18
    out = (C.c_uint8 * 32)()
    N.load().sg_sha256(msg, len(msg), out)
    return bytes(out)


def hmac_sha256(key: bytes, msg: bytes) -> bytes:  # prf.rs:8-29
    out = (C.c_uint8 * 32)()
    N.check(N.load().sg_hmac_sha256(key, len(key), msg, len(msg), out))
    return bytes(out)


class Prf:
    """prf.rs:31-89: ``Prf(secret, seed).get_bytes(n)`` continues one P_SHA256 stream."""

    def __init__(self, secret: bytes, seed: bytes):
        lib = N.load()
        self._h = lib.sg_prf_new(secret, len(secret), seed, len(seed))
        if not self._h:
            raise ValueError(N.last_error())

    def get_bytes(self, size: int) -> bytes:
        out = (C.c_uint8 * max(size, 1))()
        N.check(N.load().sg_prf_get_bytes(self._h, out, size))
        return bytes(out)[:size]

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            N.load().sg_prf_free(h)


def derive_keys(pre_master, client_random, server_random, threads: int = 8, with_master: bool = False):
    """client.rs:130-163 for many connections.

    pre_master: uint8 [count, pm_len]; randoms: uint8 [count, 32].  Returns
    (client_write_keys, server_write_keys[, master_secrets]) as uint8 arrays
    [count, 32] (and [count, 48]) -- the client encrypts with the first and
    decrypts with the second; a server the other way round."""
    pm = np.ascontiguousarray(pre_master, dtype=np.uint8)
    cr = np.ascontiguousarray(client_random, dtype=np.uint8)
    sr = np.ascontiguousarray(server_random, dtype=np.uint8)
    count = pm.shape[0]
    if cr.shape != (count, 32) or sr.shape != (count, 32):
        raise ValueError("randoms must be [count, 32]")
    cw = np.empty((count, 32), dtype=np.uint8)
    sw = np.empty((count, 32), dtype=np.uint8)
    ms = np.empty((count, 48), dtype=np.uint8) if with_master else None
    p = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None  # noqa: E731
    N.check(N.load().sg_derive_keys(count, p(pm), pm.shape[1], pm.shape[1], p(cr), p(sr), p(ms), p(cw), p(sw),
                                    threads))
    return (cw, sw, ms) if with_master else (cw, sw)


def verify_data(master_secret: bytes, server: bool, handshake_hash: bytes) -> bytes:  # client.rs:184-221
    out = (C.c_uint8 * 12)()
    N.check(N.load().sg_finished_verify_data(master_secret, int(server), handshake_hash, out))
    return bytes(out)
