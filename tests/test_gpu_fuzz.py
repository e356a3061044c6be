"""Randomised batch parity (GPU): mixed batches drawn at random -- lengths
over every route of the device bucketing (packed 64 B-4 KiB records, the
wave-per-record buckets, the size classes, ragged and edge lengths), 16-byte
aligned or odd offsets, TLS mode (random sequence numbers, content type and
version, tls.rs:103-112) or explicit nonces and AD of a random length 0-255
(chacha20_poly1305.rs:19-42), eight keys -- sealed on the GPU and compared
byte for byte with the oracle, then opened with random tampering of the
ciphertext, the tag or (explicit mode) the AD and a few truncated records:
statuses equal the reference's Ok / Err(BadRecordMac) ("wrong mac" 1, "too
short" 2, chacha20_poly1305.rs:65-94), every other record's plaintext equals
the input, and failed records' output is zero-filled unless
SG_BATCH_KEEP_FAILED is set.
"""
from __future__ import annotations

import struct

import numpy as np
import pytest

from test_gpu_parity import dev_bytes, host, torch_mod

pytestmark = pytest.mark.gpu

EDGES = [0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 129, 4032, 4095, 4096, 4097, 4160, 8192, 12352, 16320, 16383, 16384]


def _lengths(rng, count, explicit):
    kind = rng.random(count)
    lens = np.where(kind < 0.45, 64 * rng.integers(1, 257, size=count),   # packed and bucket routes
                    rng.integers(0, 16385, size=count))                    # ragged: size classes
    edges = rng.choice(EDGES, size=count)
    lens = np.where(kind > 0.9, edges, lens)
    if explicit:  # explicit mode takes records up to SG_MAX_RECORD_LEN
        big = rng.random(count) < 0.02
        lens[big] = rng.integers(16385, 32769, size=int(big.sum()))
    return lens.astype(np.uint32)


@pytest.mark.parametrize("seed", list(range(11, 27)))
def test_random_mixed_batches(gpu, oracle, seed):
    torch = torch_mod()
    from suruga_amd import batch as B

    rng = np.random.default_rng(0xF022 + seed)
    count = int(rng.integers(700, 1500))
    explicit = seed % 2 == 0
    aligned = seed % 4 < 2
    lens = _lengths(rng, count, explicit)
    pad = 16 if aligned else 1
    skew_i, skew_o = (0, 0) if aligned else (3, 7)
    step_i = (lens.astype(np.uint64) + pad - 1) // pad * pad + skew_i
    step_o = (lens.astype(np.uint64) + 16 + pad - 1) // pad * pad + skew_o
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    in_off[1:] = np.cumsum(step_i[:-1])
    out_off[1:] = np.cumsum(step_o[:-1])
    pt_bytes, ct_bytes = int(in_off[-1] + step_i[-1]), int(out_off[-1] + step_o[-1])
    pt_h = rng.bytes(pt_bytes)
    keys_h = rng.bytes(8 * 32)
    kidx = rng.integers(0, 8, size=count).astype(np.uint32)
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    keys = dev_bytes(keys_h).view(8, 32)
    if explicit:
        adlen = int(rng.integers(0, 256))
        stride = max(adlen, 1)
        nonces_h = rng.bytes(8 * count)
        ads_h = bytearray(rng.bytes(stride * count))
        mode = dict(tls=False, nonces=dev_bytes(nonces_h), ads=dev_bytes(bytes(ads_h)), ad_len=adlen, ad_stride=stride)

        def nonce_ad(i, n, ads=ads_h):
            return nonces_h[8 * i:8 * i + 8], bytes(ads[i * stride:i * stride + adlen])
    else:
        seqs = rng.integers(0, 2**63, size=count, dtype=np.uint64)
        seqs[:2] = [2**32 - 1, 2**64 - 1]
        ctype, minor = int(rng.choice([20, 21, 22, 23])), int(rng.integers(0, 4))
        mode = dict(seq=dev(seqs), content_type=ctype, version=(3, minor))

        def nonce_ad(i, n, ads=None):
            s = int(seqs[i])
            return struct.pack(">Q", s), oracle.tls_ad(s, n, ctype, 3, minor)
    common = dict(count=count, keys=keys, key_index=dev(kidx), **mode)

    ct = torch.zeros(ct_bytes, dtype=torch.uint8, device="cuda")
    B.seal(B.Batch(inp=dev_bytes(pt_h), out=ct, lens=dev(lens), max_len=int(lens.max()), in_off=dev(in_off),
                   out_off=dev(out_off), **common))
    torch.cuda.synchronize()
    ct_h = bytearray(host(ct))
    for i in range(count):
        k = keys_h[32 * int(kidx[i]):32 * int(kidx[i]) + 32]
        n, o, q = int(lens[i]), int(in_off[i]), int(out_off[i])
        nonce, ad = nonce_ad(i, n)
        assert bytes(ct_h[q:q + n + 16]) == oracle.seal(k, nonce, pt_h[o:o + n], ad), (seed, i, n)

    # open: tamper ~3 % of the records (ciphertext, tag or, explicit, AD), truncate a few
    exp_st = bytearray(count)
    olens = (lens + 16).astype(np.uint32)
    for i in rng.choice(count, size=max(3, count // 33), replace=False):
        i, n = int(i), int(lens[i])
        where = int(rng.integers(0, 3 if explicit and adlen else 2))
        if where == 0 and n:
            ct_h[int(out_off[i]) + int(rng.integers(0, n))] ^= 1 << int(rng.integers(0, 8))
        elif where == 2:
            ads_h[i * stride + int(rng.integers(0, adlen))] ^= 0x20
        else:
            ct_h[int(out_off[i]) + n + int(rng.integers(0, 16))] ^= 0x80
        exp_st[i] = 1
    for i in rng.choice(count, size=3, replace=False):
        i = int(i)
        olens[i] = int(rng.integers(0, 16))
        exp_st[i] = 2
    if explicit:
        common["ads"] = dev_bytes(bytes(ads_h))
    keep = bool(seed % 3 == 0)
    back = torch.full((pt_bytes,), 0xEE, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    B.open_(B.Batch(inp=dev_bytes(bytes(ct_h)), out=back, lens=dev(olens), max_len=int(olens.max()),
                    in_off=dev(out_off), out_off=dev(in_off), status=st, keep_failed=keep, **common))
    torch.cuda.synchronize()
    assert host(st) == bytes(exp_st), seed
    back_h = host(back)
    for i in range(count):
        o, n = int(in_off[i]), int(lens[i])
        if exp_st[i] == 0:
            assert back_h[o:o + n] == pt_h[o:o + n], (seed, i, n)
        elif exp_st[i] == 1 and not keep:
            assert back_h[o:o + n] == bytes(n), (seed, i, n)  # nothing of a failed record is released


@pytest.mark.parametrize("lockstep,packed", [(0, 0), (0, 1), (1, 0)])
@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_random_mixed_batches_every_kernel_form(gpu, oracle, seed, lockstep, packed):
    """The same random batches with the wave-per-record kernel and / or the
    packed kernel switched off (sg_set_lockstep / sg_set_packed): every record
    then runs on another route (size classes), bit-exact all the same."""
    from suruga_amd import _native

    lib = _native.load()
    prev_l, prev_p = lib.sg_set_lockstep(lockstep), lib.sg_set_packed(packed)
    try:
        test_random_mixed_batches(gpu, oracle, seed)
    finally:
        lib.sg_set_lockstep(prev_l)
        lib.sg_set_packed(prev_p)
