"""Key schedule: sg_keysched.cpp against the reference's
own vectors (crypto/sha2.rs:123-141, cipher/prf.rs:95-167), Python's stdlib
hmac/hashlib and the oracle restatement (oracle/tls_prf.py); then derived key
tables driving the GPU batch path (GPU)."""
from __future__ import annotations

import hashlib
import hmac
import os
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
import tls_prf as ORC  # noqa: E402  (test infrastructure)

from suruga_amd import keysched as K  # noqa: E402
from suruga_amd import _native as N  # noqa: E402

# crypto/sha2.rs:124-135
SHA256_ANSWERS = [
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
]
# cipher/prf.rs:98-132 (RFC 4231 cases 1-4)
HMAC_VALUES = [
    ("0b" * 20, b"Hi There".hex(), "b0344c61d8db38535ca8afceaf0bf12b881dc200c9833da726e9376c2e32cff7"),
    ("4a656665", b"what do ya want for nothing?".hex(),
     "5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843"),
    ("aa" * 20, "dd" * 50, "773ea91e36800e46854db8ebd09181a72959098b3ef8c122d9635514ced565fe"),
    (bytes(range(1, 26)).hex(), "cd" * 50, "82558a389a443c0ea4cc819899f2083a85f0faa3e578f8077a2e3ff46729665b"),
]


@pytest.mark.parametrize("msg,want", SHA256_ANSWERS)
def test_sha256_reference_answers(msg, want):
    assert K.sha256(msg).hex() == want
    assert ORC.sha256(msg).hex() == want


def test_sha256_lengths_vs_hashlib():
    rng = np.random.default_rng(1)
    for n in list(range(0, 130)) + [1000, 4097]:
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert K.sha256(m) == hashlib.sha256(m).digest()


@pytest.mark.parametrize("key,msg,want", HMAC_VALUES)
def test_hmac_reference_vectors(key, msg, want):
    k, m = bytes.fromhex(key), bytes.fromhex(msg)
    assert K.hmac_sha256(k, m).hex() == want
    assert ORC.hmac_sha256(k, m).hex() == want


def test_hmac_vs_stdlib_and_long_key():
    rng = np.random.default_rng(2)
    for kl in (0, 1, 32, 48, 63, 64):
        for ml in (0, 1, 77, 200):
            k = rng.integers(0, 256, kl, dtype=np.uint8).tobytes()
            m = rng.integers(0, 256, ml, dtype=np.uint8).tobytes()
            assert K.hmac_sha256(k, m) == hmac.new(k, m, hashlib.sha256).digest()
    with pytest.raises(N.NativeError):  # prf.rs:11-14 unimplemented!() for keys > 64 B
        K.hmac_sha256(bytes(65), b"x")


def test_prf_get_bytes_reference():  # prf.rs:137-166 test_get_bytes
    p1 = K.Prf(b"", b"")
    ret1 = b"".join(p1.get_bytes(1) for _ in range(100))
    ret2 = K.Prf(b"", b"").get_bytes(100)
    p3 = K.Prf(b"", b"")
    ret3 = p3.get_bytes(33) + p3.get_bytes(33) + p3.get_bytes(100 - 66)
    assert ret1 == ret2 == ret3
    assert ret1 == ORC.Prf(b"", b"").get_bytes(100)


def test_prf_vs_oracle_split_patterns():
    rng = np.random.default_rng(3)
    for _ in range(20):
        secret = rng.integers(0, 256, int(rng.integers(0, 65)), dtype=np.uint8).tobytes()
        seed = rng.integers(0, 256, int(rng.integers(0, 100)), dtype=np.uint8).tobytes()
        sizes = [int(x) for x in rng.integers(0, 70, 6)]
        a, b = K.Prf(secret, seed), ORC.Prf(secret, seed)
        assert [a.get_bytes(s) for s in sizes] == [b.get_bytes(s) for s in sizes]


def test_derive_keys_vs_oracle():
    rng = np.random.default_rng(4)
    count = 300
    pm = rng.integers(0, 256, (count, 32), dtype=np.uint8)   # ECDHE P-256 shared x (kex.rs)
    cr = rng.integers(0, 256, (count, 32), dtype=np.uint8)
    sr = rng.integers(0, 256, (count, 32), dtype=np.uint8)
    cw, sw, ms = K.derive_keys(pm, cr, sr, threads=4, with_master=True)
    for i in (0, 1, 150, 299):
        m, w, r = ORC.derive_keys(pm[i].tobytes(), cr[i].tobytes(), sr[i].tobytes())
        assert ms[i].tobytes() == m and cw[i].tobytes() == w and sw[i].tobytes() == r
    cw1, sw1 = K.derive_keys(pm, cr, sr, threads=1)
    assert np.array_equal(cw, cw1) and np.array_equal(sw, sw1)


def test_finished_verify_data_vs_oracle():
    ms, hh = os.urandom(48), hashlib.sha256(b"handshake messages").digest()
    for server in (False, True):
        assert K.verify_data(ms, server, hh) == ORC.verify_data(ms, server, hh)


@pytest.mark.gpu
def test_derived_key_table_drives_batch_seal(gpu, oracle):
    """Key tables from the schedule -> TLS-mode batch seal on the GPU -> the
    peer (server) opens with the same keys through the oracle."""
    import torch

    from suruga_amd import batch as B

    rng = np.random.default_rng(5)
    conns, per = 16, 8
    pm = rng.integers(0, 256, (conns, 32), dtype=np.uint8)
    cr = rng.integers(0, 256, (conns, 32), dtype=np.uint8)
    sr = rng.integers(0, 256, (conns, 32), dtype=np.uint8)
    cw, _ = K.derive_keys(pm, cr, sr)
    n, count = 700, conns * per
    dev = torch.device("cuda", 0)
    pts = [oracle.fill_record(11, i, n) for i in range(count)]
    pt = torch.tensor(np.frombuffer(b"".join(pts), dtype=np.uint8), device=dev)
    ct = torch.empty(count * (n + 16), dtype=torch.uint8, device=dev)
    kidx = torch.tensor([i % conns for i in range(count)], dtype=torch.int32, device=dev)
    seq = torch.tensor([i // conns for i in range(count)], dtype=torch.int64, device=dev)
    keys = torch.tensor(cw, device=dev)
    b = B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=n + 16,
                key_index=kidx, seq=seq)
    B.seal(b)
    torch.cuda.synchronize()
    got = ct.cpu().numpy().tobytes()
    for i in range(count):
        nonce = (i // conns).to_bytes(8, "big")
        ad = oracle.tls_ad(i // conns, n)
        rc, back = oracle.open(cw[i % conns].tobytes(), nonce, got[i * (n + 16):(i + 1) * (n + 16)], ad)
        assert rc == 0 and back == pts[i]
