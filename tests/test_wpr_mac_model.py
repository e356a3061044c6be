"""CPU check of the decomposition behind the wave-per-record kernel's Poly1305
(sg_wpr_kernel and sg_wpr_keying_kernel in suruga_amd/csrc/sg_wpr.hip,
DESIGN.md §4.5).

The model follows the kernel step for step on a full 16 KiB record:

* ciphertext chunk m = 256 j + 128 h + 4 q + i (iteration j, lane 32 h + q,
  chunk i of the lane's 64-byte block) is the i8 B operand (byte - 128) of
  MFMA step (j, i), column q;
* the T operand row c holds the signed base-256 digits of
  V = r^(128 k + 5 - i + delta) for bytes a' < 16 - sigma and of
  P = r^(128 k + 4 - i + delta) otherwise (k = (1 - h) + 2 (3 - j)), read as
  two 16-byte windows of the 48-byte digit lines the kernel builds in LDS
  (V window at 48 iv + 47 - c, P window at 48 iv - 17 - c, iv = 5 k + 4 - i);
* the 32 x 32 accumulator is seeded with 2^24 and must stay a positive 25-bit
  integer;
* lane (hh, q) assembles X = sum_r D[c_r][q] 2^(8 c_r - 32 hh),
  c_r = (r & 3) + 8 (r >> 2) + 4 hh, and multiplies it by
  W = hi[hh][a] lo[b] = 2^(32 hh) R^(8 a + b), R = r^4, 31 - q = 8 a + b;
* the keying kernel's constant term ctot = prefix (ad || le64(|ad|), Horner)
  + suffix (le64(n)) + pads (2^128 per full block, 2^(8 rem) on the last)
  + i8 bias (128 r^delta G(1024) (A1 r + A2)) - seed (2^24 J sum_q W_q),
  with G(1024) = (r + r^2 + r^3 + r^4) (sum_a R^(8a)) (sum_b R^b) sum_k T^k.

The result must equal suruga's Poly1305 (poly1305.rs:195-315, through the
oracle) over the AEAD MAC stream ad || le64(|ad|) || ct || le64(|ct|)
(chacha20_poly1305.rs:19-42) for every AD length class the kernel takes.
"""
import struct

import numpy as np
import pytest

P = (1 << 130) - 5
C80 = sum(0x80 << (8 * a) for a in range(17))
N = 16384


def signed_digits(v: int) -> list[int]:
    """The kernel's digit lines: bytes of v + 0x80..80, each minus 0x80."""
    u = v + C80
    d = [((u >> (8 * a)) & 0xFF) ^ 0x80 for a in range(17)]
    return [x - 256 if x >= 128 else x for x in d]


def geo(r: int, m: int) -> int:
    return sum(pow(r, e, P) for e in range(1, m + 1)) % P


def keying(ad: bytes, r: int):
    """sg_wpr_keying_kernel: the tables and the constant term of one record."""
    adlen = len(ad)
    o = adlen + 8
    sig, beta = o & 15, o >> 4
    L = adlen + 16 + N
    B = (L + 15) // 16
    rem = L - 16 * (B - 1)
    delta = B - beta - 1 - 1024
    assert delta in (0, 1)
    rd = [pow(r, 1 + delta + u, P) for u in range(5)]
    tk = [pow(r, 128 * k, P) for k in range(8)]
    R = pow(r, 4, P)
    lo = [pow(R, b, P) for b in range(8)]
    hi = [[pow(R, 8 * a, P) * (1 << (32 * h)) % P for a in range(4)] for h in range(2)]
    sw = sum(lo) * sum(hi[0]) % P
    g = sum(pow(r, e, P) for e in range(1, 5)) * sw * sum(tk) % P
    assert g == geo(r, 1024)
    gb = (g + pow(r, 1024, P) * geo(r, B - 1024)) % P
    pads = (1 << 128) * gb + ((1 << (8 * rem)) + P - (1 << 128)) * r
    a1 = sum(0x80 << (8 * k) for k in range(sig, 16))
    a2 = sum(0x80 << (8 * k) for k in range(sig))
    bias = g * (a1 * r + a2) * pow(r, delta, P)
    cj = (P - ((1 << 24) * sum(1 << (8 * c) for c in range(32))) % P) % P
    seed = cj * sw
    pre = ad + struct.pack("<Q", adlen)
    hp = 0
    for b in range(beta + 1):
        hp = (hp * r + int.from_bytes(pre[16 * b:16 * b + 16], "little")) % P
    prefix = hp * pow(r, 1024, P) * rd[0]
    x = N << (8 * sig)
    suffix = (x % (1 << 128)) * rd[0] + (x >> 128) * pow(r, delta, P)
    ctot = (pads + bias + seed + prefix + suffix) % P
    return dict(sig=sig, rd=rd, tk=tk, lo=lo, hi=hi, ctot=ctot)


def wpr_tag(ad: bytes, ct: bytes, r: int, s: int) -> bytes:
    assert len(ct) == N
    kt = keying(ad, r)
    sig = kt["sig"]
    lines = np.zeros(40 * 48 + 16, dtype=np.int64)
    for line in range(40):
        k, u = divmod(line, 5)
        d = signed_digits(kt["rd"][u] * kt["tk"][k] % P)
        for i in range(17):  # digit i at byte 47 - sigma - i of the line
            lines[48 * line + 47 - sig - i] = d[i]
    chunks = np.frombuffer(ct, dtype=np.uint8).astype(np.int64).reshape(1024, 16) - 128
    D = np.full((32, 32), 1 << 24, dtype=np.int64)  # [c][q]
    for j in range(4):
        for i in range(4):
            for h in range(2):
                k = (1 - h) + 2 * (3 - j)
                iv = 5 * k + 4 - i
                T = np.zeros((32, 16), dtype=np.int64)
                for c in range(32):
                    vw = lines[48 * iv + 47 - c:48 * iv + 47 - c + 16]
                    pw = lines[48 * iv - 17 - c:48 * iv - 17 - c + 16]
                    T[c] = np.concatenate([vw[:16 - sig], pw[16 - sig:]])
                m = 256 * j + 128 * h + 4 * np.arange(32) + i
                D += T @ chunks[m].T
    assert D.min() > 0 and D.max() < (1 << 25)
    h = 0
    for q in range(32):
        a, b = divmod(31 - q, 8)
        for hh in range(2):
            x = sum(int(D[(r_ & 3) + 8 * (r_ >> 2) + 4 * hh, q]) << (8 * (r_ & 3) + 64 * (r_ >> 2)) for r_ in range(16))
            h += kt["hi"][hh][a] * kt["lo"][b] * x
    h = (h + kt["ctot"]) % P
    return ((h + s) % (1 << 128)).to_bytes(16, "little")


@pytest.mark.parametrize("adlen", [13, 0, 1, 7, 8, 24, 100, 255])
def test_wpr_decomposition_matches_reference_poly1305(oracle, adlen):
    rng = np.random.default_rng(1000 + adlen)
    ad = rng.bytes(adlen)
    ct = rng.bytes(N)
    stream = ad + struct.pack("<Q", adlen) + ct + struct.pack("<Q", N)  # chacha20_poly1305.rs:24-30
    rk, sk = rng.bytes(16), rng.bytes(16)
    want = oracle.poly1305(stream, rk, sk)  # the oracle clamps r (poly1305.rs:197-203)
    r = int.from_bytes(rk, "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    assert wpr_tag(ad, ct, r, int.from_bytes(sk, "little")) == want


@pytest.mark.parametrize("fill", [0x00, 0xFF])
def test_wpr_accumulator_bounds_extreme_bytes(oracle, fill):
    """All-zero and all-0xff ciphertext: the seeded accumulator stays in (0, 2^25)."""
    ad = bytes(13)
    ct = bytes([fill]) * N
    rk, sk = bytes([0xFF] * 16), bytes(16)
    stream = ad + struct.pack("<Q", 13) + ct + struct.pack("<Q", N)
    r = int.from_bytes(rk, "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    assert wpr_tag(ad, ct, r, 0) == oracle.poly1305(stream, rk, sk)
