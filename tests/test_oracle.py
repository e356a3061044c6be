"""CPU tests: the oracle (C restatement of suruga's algorithm) against the
reference's own known-answer tests and the generated AEAD fixtures.

Mirrors the reference's unit tests:
  chacha20.rs:162-228          check_keystream / test_chacha20
  poly1305.rs:354-404          test_add / test_normalize / test_mult (Int1305 algebra)
  poly1305.rs:406-458          test_poly1305_examples
  chacha20_poly1305.rs         (no reference test) -> aead_vectors.json
"""
from __future__ import annotations

import hashlib
import struct

import pytest

from conftest import vector_pt

P = (1 << 130) - 5


def value(limbs):
    return sum(v << (26 * i) for i, v in enumerate(limbs))


# ---- chacha20.rs:162-228 ----------------------------------------------------
def test_chacha20_keystream_kats(oracle, kats):
    assert len(kats["chacha20"]) == 5
    for v in kats["chacha20"]:
        ks = bytes.fromhex(v["keystream"])
        assert oracle.keystream(bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), len(ks)) == ks, v["source"]


def test_chacha20_rejects_bad_lengths(oracle):
    # ChaCha20::new asserts key.len() == 32 and nonce.len() == 8 (chacha20.rs:26-27)
    with pytest.raises(ValueError):
        oracle.keystream(bytes(31), bytes(8), 1)
    with pytest.raises(ValueError):
        oracle.keystream(bytes(32), bytes(12), 1)


def test_chacha20_stream_continues_across_calls(oracle, kats):
    # encrypt() never resets the counter; the 256-byte KAT spans 4 blocks
    v = kats["chacha20"][4]
    ks = bytes.fromhex(v["keystream"])
    assert len(ks) == 256
    assert oracle.keystream(bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), 100) == ks[:100]


# ---- poly1305.rs:321-404 (Int1305 algebra) ----------------------------------
def test_int1305_add_associative(oracle, kats):
    coeffs = kats["int1305_coeffs"]
    for a in coeffs:
        for b in coeffs:
            for c in coeffs:
                abc = oracle.add(oracle.add(a, b), c)
                bca = oracle.add(oracle.add(b, c), a)
                acb = oracle.add(oracle.add(a, c), b)
                assert oracle.normalize(abc) == oracle.normalize(bca) == oracle.normalize(acb)


def test_int1305_normalize(oracle, kats):
    p = [0x3fffffb, 0x3ffffff, 0x3ffffff, 0x3ffffff, 0x3ffffff]
    assert oracle.normalize(p) == [0] * 5
    large, small = [0, 10, 5, 10, 1 << 26], [5, 10, 5, 10, 0]
    assert oracle.normalize(large) == small
    assert oracle.normalize(small) == small
    for a in kats["int1305_coeffs"]:
        assert oracle.normalize(oracle.normalize(a)) == oracle.normalize(a)
        assert value(oracle.normalize(a)) == value(a) % P


def test_int1305_mult_associative_and_exact(oracle, kats):
    coeffs = kats["int1305_coeffs"]
    for a in coeffs:
        for b in coeffs:
            ab = oracle.mult(a, b)
            assert value(ab) % P == (value(a) * value(b)) % P
            for c in coeffs:
                abc = oracle.normalize(oracle.mult(ab, c))
                bca = oracle.normalize(oracle.mult(oracle.mult(b, c), a))
                acb = oracle.normalize(oracle.mult(oracle.mult(a, c), b))
                assert abc == bca == acb


# ---- poly1305.rs:406-458 ----------------------------------------------------
def test_poly1305_examples(oracle, kats):
    assert len(kats["poly1305"]) == 4
    for v in kats["poly1305"]:
        tag = oracle.poly1305(bytes.fromhex(v["msg"]), bytes.fromhex(v["r"]), bytes.fromhex(v["s"]))
        assert tag.hex() == v["tag"]


# ---- AEAD (chacha20_poly1305.rs) fixtures ------------------------------------
def test_aead_vectors_seal(oracle, aead_vectors):
    for v in aead_vectors["vectors"]:
        key, nonce, ad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["ad"])
        pt = vector_pt(v, oracle)
        out = oracle.seal(key, nonce, pt, ad)
        if "ct_tag" in v:
            assert out.hex() == v["ct_tag"], v["name"]
        assert out[-16:].hex() == v["tag"], v["name"]
        assert hashlib.sha256(out[:-16]).hexdigest() == v["ct_sha256"], v["name"]


def test_aead_vectors_open_roundtrip(oracle, aead_vectors):
    for v in aead_vectors["vectors"]:
        key, nonce, ad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["ad"])
        pt = vector_pt(v, oracle)
        rc, back = oracle.open(key, nonce, oracle.seal(key, nonce, pt, ad), ad)
        assert rc == 0 and back == pt, v["name"]


def test_tls_nonce_and_ad_rules(oracle, aead_vectors):
    # tls.rs:103-112: nonce = be64(seq), ad = be64(seq) || 23 || 3 || 3 || be16(n)
    for v in aead_vectors["vectors"]:
        if "tls_seq" not in v:
            continue
        seq, n = v["tls_seq"], v["n"]
        assert bytes.fromhex(v["nonce"]) == struct.pack(">Q", seq)
        assert bytes.fromhex(v["ad"]) == oracle.tls_ad(seq, n)


def test_open_tamper_is_bad_record_mac(oracle, aead_vectors):
    by_name = {v["name"]: v for v in aead_vectors["vectors"]}
    for t in aead_vectors["tamper"]:
        v = by_name[t["vector"]]
        key, nonce, ad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["ad"])
        data = bytearray(oracle.seal(key, nonce, vector_pt(v, oracle), ad))
        data[t["flip"]] ^= 0x01
        rc, _ = oracle.open(key, nonce, bytes(data), ad)
        assert rc == 1  # BadRecordMac "wrong mac" (chacha20_poly1305.rs:89-90)
        # wrong AD or nonce must also fail
        rc, _ = oracle.open(key, nonce, oracle.seal(key, nonce, b"x", ad), ad + b"!")
        assert rc == 1


def test_open_short_is_bad_record_mac(oracle, aead_vectors):
    for s in aead_vectors["short"]:
        rc, _ = oracle.open(bytes(32), bytes(8), bytes(s["len"]), b"")
        assert rc == 2  # "message too short" (chacha20_poly1305.rs:68-70)


def test_batch_driver_matches_single(oracle):
    key = bytes(range(32))
    n, count = 100, 37
    pt = b"".join(oracle.fill_record(0x53555255, j, n) for j in range(count))
    ct1 = oracle.seal_batch_tls(key, 5, pt, n, count, threads=1)
    ct4 = oracle.seal_batch_tls(key, 5, pt, n, count, threads=4)
    assert ct1 == ct4
    for j in (0, 17, 36):
        seq = 5 + j
        single = oracle.seal(key, struct.pack(">Q", seq), pt[j * n:(j + 1) * n], oracle.tls_ad(seq, n))
        assert ct1[j * (n + 16):(j + 1) * (n + 16)] == single
    bad, back, st = oracle.open_batch_tls(key, 5, ct1, n, count, threads=3)
    assert bad == 0 and back == pt and st == bytes(count)


def test_fill_record_rule(oracle):
    # byte i of record j = byte (i mod 8) of splitmix64(seed ^ (j << 32) ^ (i / 8))
    seed, j = 0x53555255, 3
    buf = oracle.fill_record(seed, j, 20)
    for i in range(20):
        w = oracle.L.so_splitmix64(seed ^ (j << 32) ^ (i // 8))
        assert buf[i] == (w >> (8 * (i % 8))) & 0xFF


def test_openssl_comparison_line_matches_oracle(oracle):
    """bench.py's optimised-CPU line must compute suruga's AEAD, not RFC 7539."""
    from oracle_ffi import OsslLine

    try:
        ossl = OsslLine()
    except OSError as e:
        pytest.skip(str(e))
    key = bytes(range(32))
    for n, count in ((0, 3), (1, 5), (64, 4), (1000, 7), (16384, 3)):
        pt = b"".join(oracle.fill_record(7, j, n) for j in range(count))
        ct = ossl.seal_batch_tls(key, 0xFFFFFFFE, pt, n, count, threads=2)
        assert ct == oracle.seal_batch_tls(key, 0xFFFFFFFE, pt, n, count)
        bad, back = ossl.open_batch_tls(key, 0xFFFFFFFE, ct, n, count, threads=2)
        assert bad == 0 and back == pt
        if count:
            t = bytearray(ct)
            t[-1] ^= 1
            assert ossl.open_batch_tls(key, 0xFFFFFFFE, bytes(t), n, count)[0] == 1


def test_tag_fold_mixed_equals_per_record_seals(oracle):
    """The full-size C2 checker of bench.py (so_tag_fold_mixed) folds exactly
    the tags the per-record seal gives (TLS nonce/AD, per-connection keys)."""
    import struct

    import numpy as np

    from suruga_amd import workloads as W

    lay = W.c2_layout(300)
    pt = np.frombuffer(np.random.default_rng(2).bytes(lay.pt_bytes), dtype=np.uint8)
    seqs = lay.seq + np.uint64(7)
    fold = oracle.tag_fold_mixed(lay.keys, lay.key_index, seqs, lay.lens, lay.in_off, pt, threads=4)
    acc = bytearray(16)
    for i in range(lay.count):
        k = lay.keys[32 * int(lay.key_index[i]):32 * int(lay.key_index[i]) + 32]
        s, n, o = int(seqs[i]), int(lay.lens[i]), int(lay.in_off[i])
        tag = oracle.seal(k, struct.pack(">Q", s), pt[o:o + n].tobytes(), oracle.tls_ad(s, n))[-16:]
        acc = bytearray(a ^ b for a, b in zip(acc, tag))
    assert fold == bytes(acc)


def test_mixed_batch_drivers_match_per_record_seals(oracle):
    """The C2 CPU baselines (so_batch_mixed, ossl_batch_mixed) seal every record
    of a Zipf layout exactly as the per-record seal does and open it back;
    a tampered record fails alone."""
    import ctypes as C
    import struct

    import numpy as np

    from oracle_ffi import OsslLine
    from suruga_amd import workloads as W

    lay = W.c2_layout(200)
    pt = np.frombuffer(np.random.default_rng(5).bytes(lay.pt_bytes), dtype=np.uint8).copy()
    seqs = (lay.seq + np.uint64(3)).astype(np.uint64)
    kb = np.frombuffer(bytes(lay.keys), dtype=np.uint8).copy()
    ki, lens = lay.key_index.astype(np.uint32), lay.lens.astype(np.uint32)
    olens = (lens + 16).astype(np.uint32)
    io, oo = lay.in_off.astype(np.uint64), lay.out_off.astype(np.uint64)
    P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    lines = [("oracle", lambda *a: oracle.L.so_batch_mixed(*a))]
    try:
        S = OsslLine().L
        lines.append(("ossl", lambda op, *a: S.ossl_batch_mixed(op, *a[:8], *a[9:])))
    except OSError:
        pass
    for name, run in lines:
        ct = np.zeros(lay.ct_bytes, dtype=np.uint8)
        back = np.zeros(lay.pt_bytes, dtype=np.uint8)
        st = np.full(lay.count, 9, dtype=np.uint8)
        assert run(0, P(kb), P(ki), P(seqs), P(lens), P(io), P(oo), P(pt), P(ct), None, lay.count, 3) == 0
        for i in (0, 1, lay.count // 2, lay.count - 1):
            k = bytes(lay.keys[32 * int(ki[i]):32 * int(ki[i]) + 32])
            s, n, a, q = int(seqs[i]), int(lens[i]), int(io[i]), int(oo[i])
            exp = oracle.seal(k, struct.pack(">Q", s), pt[a:a + n].tobytes(), oracle.tls_ad(s, n))
            assert ct[q:q + n + 16].tobytes() == exp, name
        ct[int(oo[7]) + int(lens[7])] ^= 1  # record 7's tag
        bad = run(1, P(kb), P(ki), P(seqs), P(olens), P(oo), P(io), P(ct), P(back), P(st), lay.count, 3)
        assert bad == 1, name
        if name == "oracle":
            assert st[7] == 1 and int(st.sum()) == 1
        ok = np.ones(lay.pt_bytes, dtype=bool)
        ok[int(io[7]):int(io[7]) + int(lens[7])] = False
        assert np.array_equal(back[ok], pt[ok]), name
