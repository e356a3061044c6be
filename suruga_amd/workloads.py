"""Synthetic workloads of BASELINE.json / SURVEY.md 8(d).

C1: N records x 16 KiB, one key (0x00..0x1f), seq = seq0 + i.
C2: N records of 64*k bytes, k in 1..256 drawn from Zipf(s=1.1) over k
    (seed 0x5A49 "ZI"; P(64 B) = 0.21, mean 2155 B); 256 connection keys,
    record i belongs to connection i mod 256 with its own seq = i / 256.
    Packed layout: plaintext and ct||tag back to back (every offset 16-aligned
    since lengths are multiples of 64).

Only metadata is built on the host (numpy); record bytes are generated on the
device by sg_fill_records.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

FILL_SEED = 0x53555255  # "SURU"
ZIPF_SEED = 0x5A49      # "ZI"
KEY_SEED = 0x4B455953   # "KEYS"
MASK64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
    return x ^ (x >> 31)


def connection_key(j: int) -> bytes:
    """key_j = le64(splitmix64(KEY_SEED ^ (j << 8) ^ w)) for w = 0..3."""
    return b"".join(splitmix64(KEY_SEED ^ (j << 8) ^ w).to_bytes(8, "little") for w in range(4))


def zipf_lengths(count: int, seed: int = ZIPF_SEED, s: float = 1.1, kmax: int = 256) -> np.ndarray:
    k = np.arange(1, kmax + 1, dtype=np.float64)
    p = k ** -s
    p /= p.sum()
    rng = np.random.default_rng(seed)
    return (64 * (rng.choice(kmax, size=count, p=p) + 1)).astype(np.uint32)


@dataclass
class Layout:
    count: int
    lens: np.ndarray          # uint32 plaintext lengths
    in_off: np.ndarray        # uint64 plaintext offsets
    out_off: np.ndarray       # uint64 ct||tag offsets
    key_index: np.ndarray     # uint32
    seq: np.ndarray           # uint64
    keys: bytes               # num_keys * 32
    pt_bytes: int
    ct_bytes: int

    @property
    def payload(self) -> int:
        return int(self.lens.astype(np.uint64).sum())


def c2_layout(count: int, num_keys: int = 256, ct_align: int = 16, pt_align: int = 64) -> Layout:
    """ct_align / pt_align: the sealed records (ct || tag) / plaintext records
    start on multiples of that many bytes (16 / 64: back to back)."""
    lens = zipf_lengths(count)
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    slot = (lens.astype(np.uint64) + 16 + (ct_align - 1)) // ct_align * ct_align
    pslot = (lens.astype(np.uint64) + (pt_align - 1)) // pt_align * pt_align
    if count > 1:
        in_off[1:] = np.cumsum(pslot[:-1], dtype=np.uint64)
        out_off[1:] = np.cumsum(slot[:-1], dtype=np.uint64)
    idx = np.arange(count, dtype=np.uint64)
    key_index = (idx % num_keys).astype(np.uint32)
    seq = (idx // num_keys).astype(np.uint64)
    keys = b"".join(connection_key(j) for j in range(num_keys))
    return Layout(count, lens, in_off, out_off, key_index, seq, keys, int(pslot.sum()), int(slot.sum()))
