"""CPU check of the decomposition behind the lock-step kernel's MFMA Poly1305
(`mfma_mac` and the LS keying constant in suruga_amd/csrc/sg_kernels.hip,
DESIGN.md §4.5).

The model follows the kernel step for step: the PL = 64 slot grid
(`mac_geom`), slot 32 s + q in row q, the signed base-256 digits of
P_s = r^(32 (2k - 1 - s) + 1) (bytes of V + 0x80..80, each minus 0x80), the
i8 operands (stream byte with the top bit flipped), the 2^24 accumulator
seed, the exact row assembly X_q = sum_c S[q][c] 2^(8c), the row weights
W_q = r^(31 - q) and the constant term

    ctot = K G(N) + 2^128 G(B) + [rem < 16] (2^(8 rem) - 2^128) r - J (1 + G(31)),
    G(N) = G(32) sum_{t < 2k} r^(32 t).

The result must equal suruga's Poly1305 (poly1305.rs:195-315, through the
oracle) on the AEAD MAC stream ad || le64(|ad|) || ct || le64(|ct|)
(chacha20_poly1305.rs:19-42) for lengths the lock-step kernel takes.  The
bounds the kernel relies on (every seeded product entry a positive 25-bit
integer) are asserted too.
"""
import struct

import numpy as np
import pytest

P = (1 << 130) - 5
K_BIAS = sum(128 << (8 * a) for a in range(16))
J_SEED = sum((1 << 24) << (8 * c) for c in range(32))
C80 = sum(0x80 << (8 * a) for a in range(17))


def mac_geom(adlen: int, n: int, pl: int = 64):
    """sg_kernels.hip mac_geom: stream length, blocks, blocks per lane (odd), virtual blocks."""
    L = adlen + 16 + n
    B = (L + 15) // 16
    k = ((B + pl - 1) // pl) | 1
    return L, B, k, pl * k - B


def geo(r: int, m: int) -> int:
    """G(m) = sum_{e=1..m} r^e mod p."""
    return sum(pow(r, e, P) for e in range(1, m + 1)) % P


def signed_digits(v: int) -> list[int]:
    u = v + C80
    d = [((u >> (8 * a)) & 0xFF) ^ 0x80 for a in range(17)]
    return [x - 256 if x >= 128 else x for x in d]


def mfma_model_tag(stream: bytes, adlen: int, n: int, r: int, s: int) -> bytes:
    L, B, k, z = mac_geom(adlen, n)
    assert L == len(stream)
    rows = 2 * k
    rem = L - 16 * (B - 1)
    blocks = np.zeros((64 * k, 16), dtype=np.int64)  # virtual slots stay zero
    padded = stream + bytes(16 * B - L)
    blocks[z:] = np.frombuffer(padded, dtype=np.uint8).reshape(B, 16)
    a_op = (blocks ^ 0x80).astype(np.int64)
    a_op[a_op >= 128] -= 256  # i8 view of the flipped byte = byte - 128
    a_op = a_op.reshape(rows, 32, 16).transpose(1, 0, 2)  # [q][s][a]: slot 32 s + q
    digits = np.array([signed_digits(pow(r, 32 * (rows - 1 - s) + 1, P)) for s in range(rows)], dtype=np.int64)
    for j in range(rows):
        assert sum(int(x) << (8 * a) for a, x in enumerate(digits[j])) == pow(r, 32 * (rows - 1 - j) + 1, P)
    S = np.full((32, 32), 1 << 24, dtype=np.int64)
    for a in range(16):  # Toeplitz B: column c holds digit c - a
        tb = np.zeros((rows, 32), dtype=np.int64)
        tb[:, a:a + 17] = digits[:, :min(17, 32 - a)]
        S += a_op[:, :, a] @ tb
    assert S.min() > 0 and S.max() < (1 << 25)
    h = 0
    for q in range(32):
        x = sum(int(S[q, c]) << (8 * c) for c in range(32))
        h += x * pow(r, 31 - q, P)
    r32 = pow(r, 32, P)
    g31 = geo(r, 31)
    gn = (g31 + r32) * (1 + geo(r32, rows - 1)) % P
    assert gn == geo(r, 64 * k)
    ctot = K_BIAS * gn + (1 << 128) * geo(r, B) - J_SEED * (1 + g31)
    if rem < 16:
        ctot += ((1 << (8 * rem)) - (1 << 128)) * r
    h = (h + ctot) % P
    return ((h + s) % (1 << 128)).to_bytes(16, "little")


@pytest.mark.parametrize("adlen,n", [(13, 16384), (13, 8193), (13, 12345), (0, 10000), (7, 16383), (255, 16000)])
def test_mfma_decomposition_matches_reference_poly1305(oracle, adlen, n):
    rng = np.random.default_rng(n * 31 + adlen)
    ad = rng.bytes(adlen)
    ct = rng.bytes(n)
    stream = ad + struct.pack("<Q", adlen) + ct + struct.pack("<Q", n)  # chacha20_poly1305.rs:24-30
    rk = bytearray(rng.bytes(16))
    sk = rng.bytes(16)
    want = oracle.poly1305(stream, bytes(rk), sk)  # the oracle clamps r (poly1305.rs:197-203)
    r = int.from_bytes(rk, "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    got = mfma_model_tag(stream, adlen, n, r, int.from_bytes(sk, "little"))
    assert got == want
