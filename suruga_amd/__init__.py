"""suruga_amd -- MI355X-native (gfx950) drop-in for suruga's record-layer
ChaCha20-Poly1305 AEAD (klutzy/suruga src/crypto + src/cipher).

Layout:
  include/suruga_gpu.h       C ABI (the drop-in boundary; at the repo root)
  suruga_amd/csrc/           gfx950 HIP kernels + C-ABI implementation
  suruga_amd/cipher.py       mirror of suruga's Aead/Encryptor/Decryptor traits
  suruga_amd/batch.py        device-resident batch seal/open (record-layer batching)
  suruga_amd/_native.py      ctypes binding of libsuruga_gpu.so

The HIP library is the only compute path; importing the cipher classes works
without a GPU, calling them needs one (and fails loudly otherwise).
"""
from . import _native
from .cipher import (Aead, ChaCha20Poly1305, ChaCha20Poly1305Decryptor, ChaCha20Poly1305Encryptor,
                     CipherSuite, Decryptor, Encryptor, TlsError, TlsErrorKind)

__all__ = [
    "Aead", "ChaCha20Poly1305", "ChaCha20Poly1305Decryptor", "ChaCha20Poly1305Encryptor",
    "CipherSuite", "Decryptor", "Encryptor", "TlsError", "TlsErrorKind", "load_native",
]


def load_native():
    """Load libsuruga_gpu.so (raises ImportError when it has not been built)."""
    return _native.load()
