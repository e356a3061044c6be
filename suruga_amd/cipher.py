"""Host-side mirror of suruga's cipher plugin interface (src/cipher/mod.rs).

Same names, argument meaning and error behaviour as the reference traits, so
the parity tests read like the reference's own tests:

* ``Aead`` (mod.rs:14-20): ``key_size``, ``fixed_iv_len``, ``mac_len``,
  ``new_encryptor(key)``, ``new_decryptor(key)``.
* ``Encryptor.encrypt(nonce, plain, ad) -> bytes`` (mod.rs:22-24): seal,
  returns ``ct || tag``; infallible except for the reference's panics
  (wrong key / nonce length, chacha20.rs:26-27), raised here as ValueError.
* ``Decryptor.decrypt(nonce, encrypted, ad) -> bytes`` (mod.rs:28-32): open,
  raises ``TlsError(TlsErrorKind.BadRecordMac, ...)`` exactly where the
  reference returns ``Err`` (chacha20_poly1305.rs:68-70, 89-90).
* ``ChaCha20Poly1305`` (chacha20_poly1305.rs:102-135): the only suite,
  ``TLS_ECDHE_RSA_WITH_CHACHA20_POLY1305_SHA256`` (0xcc, 0x13, mod.rs:108-114),
  backed by the gfx950 kernels through the C ABI.
"""
from __future__ import annotations

import abc
import ctypes as C
import enum

from . import _native as N


class TlsErrorKind(enum.Enum):
    """src/tls_result.rs:5-20"""

    UnexpectedMessage = 0
    BadRecordMac = 1
    RecordOverflow = 2
    IllegalParameter = 3
    DecodeError = 4
    DecryptError = 5
    InternalError = 6
    IoFailure = 7
    AlertReceived = 8


class TlsError(Exception):
    """src/tls_result.rs:22-35 (``TlsError { kind, desc }``)."""

    def __init__(self, kind: TlsErrorKind, desc: str):
        super().__init__(f"{kind.name}: {desc}")
        self.kind = kind
        self.desc = desc


class Encryptor(abc.ABC):
    @abc.abstractmethod
    def encrypt(self, nonce: bytes, plain: bytes, ad: bytes) -> bytes: ...


class Decryptor(abc.ABC):
    @abc.abstractmethod
    def decrypt(self, nonce: bytes, encrypted: bytes, ad: bytes) -> bytes: ...

    @abc.abstractmethod
    def mac_len(self) -> int: ...


class Aead(abc.ABC):
    @abc.abstractmethod
    def key_size(self) -> int: ...

    @abc.abstractmethod
    def fixed_iv_len(self) -> int: ...

    @abc.abstractmethod
    def mac_len(self) -> int: ...

    @abc.abstractmethod
    def new_encryptor(self, key: bytes) -> Encryptor: ...

    @abc.abstractmethod
    def new_decryptor(self, key: bytes) -> Decryptor: ...


class _GpuCtx:
    """Owns one ``sg_ctx`` (one direction, key moved in: chacha20_poly1305.rs:121-134)."""

    def __init__(self, key: bytes, device: int):
        key = bytes(key)
        if len(key) != N.SG_KEY_LEN:
            # ChaCha20::new panics on a wrong key length (chacha20.rs:26)
            raise ValueError(f"key must be {N.SG_KEY_LEN} bytes, got {len(key)}")
        self._lib = N.load()
        ptr = self._lib.sg_ctx_new(key, device)
        if not ptr:
            raise N.NativeError(N.SG_E_HIP, N.last_error())
        self._ptr = ptr

    def close(self) -> None:
        if getattr(self, "_ptr", None):
            self._lib.sg_ctx_free(self._ptr)
            self._ptr = None

    def __del__(self):  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass


def _check_nonce(nonce: bytes) -> bytes:
    nonce = bytes(nonce)
    if len(nonce) != N.SG_NONCE_LEN:
        # ChaCha20::new panics on a wrong nonce length (chacha20.rs:27)
        raise ValueError(f"nonce must be {N.SG_NONCE_LEN} bytes, got {len(nonce)}")
    return nonce


class ChaCha20Poly1305Encryptor(_GpuCtx, Encryptor):
    """chacha20_poly1305.rs:44-59"""

    def encrypt(self, nonce: bytes, plain: bytes, ad: bytes) -> bytes:
        nonce, plain, ad = _check_nonce(nonce), bytes(plain), bytes(ad)
        out = (C.c_uint8 * (len(plain) + N.SG_MAC_LEN))()
        N.check(self._lib.sg_seal(self._ptr, nonce, len(nonce), plain, len(plain), ad, len(ad), out))
        return bytes(out)


class ChaCha20Poly1305Decryptor(_GpuCtx, Decryptor):
    """chacha20_poly1305.rs:61-100"""

    def decrypt(self, nonce: bytes, encrypted: bytes, ad: bytes) -> bytes:
        nonce, encrypted, ad = _check_nonce(nonce), bytes(encrypted), bytes(ad)
        n = max(len(encrypted) - N.SG_MAC_LEN, 0)
        out = (C.c_uint8 * max(n, 1))()
        rc = N.check(self._lib.sg_open(self._ptr, nonce, len(nonce), encrypted, len(encrypted), ad,
                                       len(ad), out))
        if rc == N.SG_E_SHORT:
            raise TlsError(TlsErrorKind.BadRecordMac, "message too short")
        if rc == N.SG_E_BAD_MAC:
            raise TlsError(TlsErrorKind.BadRecordMac, "wrong mac")
        return bytes(out)[:n]

    def mac_len(self) -> int:
        return N.SG_MAC_LEN


class ChaCha20Poly1305(Aead):
    """chacha20_poly1305.rs:102-135 -- GPU-backed drop-in."""

    def __init__(self, device: int = 0):
        self.device = device

    def key_size(self) -> int:
        return int(N.load().sg_key_size())

    def fixed_iv_len(self) -> int:
        return int(N.load().sg_fixed_iv_len())

    def mac_len(self) -> int:
        return int(N.load().sg_mac_len())

    def new_encryptor(self, key: bytes) -> ChaCha20Poly1305Encryptor:
        return ChaCha20Poly1305Encryptor(key, self.device)

    def new_decryptor(self, key: bytes) -> ChaCha20Poly1305Decryptor:
        return ChaCha20Poly1305Decryptor(key, self.device)


class CipherSuite(enum.Enum):
    """mod.rs:39-114: code point -> Aead factory.  One suite (0xcc, 0x13)."""

    TLS_ECDHE_RSA_WITH_CHACHA20_POLY1305_SHA256 = (0xCC, 0x13)
    UnknownCipherSuite = None

    def new_aead(self, device: int = 0) -> Aead:
        if self is CipherSuite.UnknownCipherSuite:
            raise AssertionError("unreachable")  # mod.rs:58
        return ChaCha20Poly1305(device)
