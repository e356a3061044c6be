"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle and
the committed fixtures.  Bit-exact on every byte of ciphertext, tag and
plaintext; open status equal to the reference's Ok/Err(BadRecordMac).

Configs (BASELINE.json): C0 = 1K x 1 KiB (full check), C1 = 1M x 16 KiB
(checked here on a 4096-record subset byte for byte, and at 65536 records by
round trip + XOR-fold of every tag against the multi-threaded oracle),
C2 = Zipf sizes with 256 keys (checked on a sample), plus ragged lengths,
misaligned offsets, explicit nonces/AD of every length class, tampering.
"""
from __future__ import annotations

import hashlib
import os
import struct

import numpy as np
import pytest

from conftest import vector_pt

pytestmark = pytest.mark.gpu

SEED = 0x53555255
KEY = bytes(range(32))


def torch_mod():
    import torch

    return torch


def dev_bytes(b: bytes):
    torch = torch_mod()
    t = torch.frombuffer(bytearray(b) if b else bytearray(1), dtype=torch.uint8)
    return t[:len(b)].to("cuda") if b else torch.zeros(1, dtype=torch.uint8, device="cuda")


def host(t) -> bytes:
    return bytes(t.cpu().numpy().tobytes())


# ---------------------------------------------------------------------------
# single-record Encryptor / Decryptor (the trait-object path, tls.rs:114, 268)
# ---------------------------------------------------------------------------
def test_single_record_vectors(gpu, oracle, aead_vectors):
    from suruga_amd import ChaCha20Poly1305, TlsError, TlsErrorKind

    aead = ChaCha20Poly1305()
    for v in aead_vectors["vectors"]:
        key, nonce, ad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["ad"])
        pt = vector_pt(v, oracle)
        enc, dec = aead.new_encryptor(key), aead.new_decryptor(key)
        out = enc.encrypt(nonce, pt, ad)
        if "ct_tag" in v:
            assert out.hex() == v["ct_tag"], v["name"]
        assert out[-16:].hex() == v["tag"], v["name"]
        assert hashlib.sha256(out[:-16]).hexdigest() == v["ct_sha256"], v["name"]
        assert dec.decrypt(nonce, out, ad) == pt, v["name"]
        assert dec.mac_len() == 16
        bad = bytearray(out)
        bad[-1] ^= 0x80
        with pytest.raises(TlsError) as e:
            dec.decrypt(nonce, bytes(bad), ad)
        assert e.value.kind is TlsErrorKind.BadRecordMac and e.value.desc == "wrong mac"


def test_single_record_tamper_and_short(gpu, oracle, aead_vectors):
    from suruga_amd import ChaCha20Poly1305, TlsError, TlsErrorKind

    by_name = {v["name"]: v for v in aead_vectors["vectors"]}
    aead = ChaCha20Poly1305()
    for t in aead_vectors["tamper"]:
        v = by_name[t["vector"]]
        key, nonce, ad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["ad"])
        data = bytearray(aead.new_encryptor(key).encrypt(nonce, vector_pt(v, oracle), ad))
        data[t["flip"]] ^= 0x01
        with pytest.raises(TlsError) as e:
            aead.new_decryptor(key).decrypt(nonce, bytes(data), ad)
        assert e.value.kind is TlsErrorKind.BadRecordMac
    dec = aead.new_decryptor(KEY)
    for s in aead_vectors["short"]:
        with pytest.raises(TlsError) as e:
            dec.decrypt(bytes(8), bytes(s["len"]), b"")
        assert e.value.kind is TlsErrorKind.BadRecordMac and e.value.desc == "message too short"
    # exactly 16 bytes = empty plaintext + tag: valid when produced by seal
    out = aead.new_encryptor(KEY).encrypt(bytes(8), b"", b"")
    assert len(out) == 16 and dec.decrypt(bytes(8), out, b"") == b""


def test_single_record_random_lengths(gpu, oracle):
    from suruga_amd import ChaCha20Poly1305

    rng = np.random.default_rng(7)
    aead = ChaCha20Poly1305()
    for _ in range(60):
        n = int(rng.integers(0, 18433))
        adlen = int(rng.integers(0, 256))
        key = rng.bytes(32)
        nonce, ad, pt = rng.bytes(8), rng.bytes(adlen), rng.bytes(n)
        out = aead.new_encryptor(key).encrypt(nonce, pt, ad)
        assert out == oracle.seal(key, nonce, pt, ad), (n, adlen)
        assert aead.new_decryptor(key).decrypt(nonce, out, ad) == pt


# ---------------------------------------------------------------------------
# batch, TLS mode
# ---------------------------------------------------------------------------
def tls_batch(count, n, *, seq0=0, key=KEY, j0=0):
    """Device plaintext (fill rule), sealed + opened through the batch ABI."""
    torch = torch_mod()
    from suruga_amd import batch as B

    keys = dev_bytes(key).view(1, 32)
    pt = torch.empty(count * n if n else 1, dtype=torch.uint8, device="cuda")
    if n:
        B.fill_records(pt, n, n, count, SEED, j0)
    ct = torch.empty(count * (n + 16), dtype=torch.uint8, device="cuda")
    B.seal(B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n,
                   out_stride=n + 16, seq0=seq0))
    back = torch.empty(count * n if n else 1, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    B.open_(B.Batch(count=count, keys=keys, inp=ct, out=back, uniform_len=n + 16, in_stride=n + 16,
                    out_stride=n, seq0=seq0, status=st))
    torch.cuda.synchronize()
    return pt, ct, back, st


def test_c0_1k_x_1kib_bit_exact(gpu, oracle):
    count, n = 1024, 1024
    pt, ct, back, st = tls_batch(count, n)
    pt_h = host(pt)
    assert pt_h == b"".join(oracle.fill_record(SEED, j, n) for j in range(count))
    assert host(ct) == oracle.seal_batch_tls(KEY, 0, pt_h, n, count, threads=8)
    assert host(back) == pt_h
    assert host(st) == bytes(count)


def test_c1_subset_4096_x_16kib_bit_exact(gpu, oracle):
    count, n = 4096, 16384
    pt, ct, back, st = tls_batch(count, n, seq0=1000)
    pt_h = host(pt)
    assert host(ct) == oracle.seal_batch_tls(KEY, 1000, pt_h, n, count, threads=16)
    assert host(back) == pt_h and host(st) == bytes(count)


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 63, 64, 65, 100, 127, 128, 129, 255, 256, 257, 511, 512, 513,
                               1000, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097, 5000, 8192, 8193, 16383,
                               16384, 18432])
def test_batch_lengths(gpu, oracle, n):
    count = 33
    pt, ct, back, st = tls_batch(count, n, seq0=0xFFFFFFF0)
    pt_h = host(pt)[:count * n]
    assert host(ct) == oracle.seal_batch_tls(KEY, 0xFFFFFFF0, pt_h, n, count, threads=4)
    assert host(back)[:count * n] == pt_h and host(st) == bytes(count)


def test_batch_seq_edges(gpu, oracle):
    torch = torch_mod()
    from suruga_amd import batch as B

    seqs = [0, 1, 0xFFFFFFFF, 0x100000000, 0xFFFFFFFFFFFFFFFF, 0x0123456789ABCDEF]
    n, count = 300, len(seqs)
    pt_h = b"".join(oracle.fill_record(SEED, j, n) for j in range(count))
    keys = dev_bytes(KEY).view(1, 32)
    seq_t = torch.tensor(np.array(seqs, dtype=np.uint64).view(np.int64), device="cuda")
    pt = dev_bytes(pt_h)
    ct = torch.empty(count * (n + 16), dtype=torch.uint8, device="cuda")
    B.seal(B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=n + 16,
                   seq=seq_t))
    torch.cuda.synchronize()
    got = host(ct)
    for j, s in enumerate(seqs):
        exp = oracle.seal(KEY, struct.pack(">Q", s), pt_h[j * n:(j + 1) * n], oracle.tls_ad(s, n))
        assert got[j * (n + 16):(j + 1) * (n + 16)] == exp, hex(s)


def test_batch_ragged_offsets_keys_and_tamper(gpu, oracle):
    """C2-shaped: ragged lengths (incl. 0 and non-multiples of 16), 256-entry key
    table, per-record key_index/seq, packed unaligned offsets; then open with one
    tampered record and one truncated record."""
    torch = torch_mod()
    from suruga_amd import batch as B

    rng = np.random.default_rng(11)
    count = 700
    lens = rng.integers(0, 4097, size=count).astype(np.uint32)
    lens[:8] = [0, 1, 15, 16, 17, 63, 64, 65]
    keys_h = rng.bytes(256 * 32)
    kidx = (np.arange(count) % 256).astype(np.uint32)
    seqs = (np.arange(count) // 256).astype(np.uint64)
    gap = rng.integers(0, 7, size=count)  # unaligned packing
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    pos_i = pos_o = 0
    for i in range(count):
        pos_i += int(gap[i]); in_off[i] = pos_i; pos_i += int(lens[i])
        pos_o += int(gap[i]); out_off[i] = pos_o; pos_o += int(lens[i]) + 16
    pt_h = rng.bytes(pos_i + 16)
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    keys = dev_bytes(keys_h).view(256, 32)
    pt = dev_bytes(pt_h)
    ct = torch.zeros(pos_o + 16, dtype=torch.uint8, device="cuda")
    common = dict(count=count, keys=keys, key_index=dev(kidx), seq=dev(seqs), max_len=int(lens.max()) + 16)
    B.seal(B.Batch(inp=pt, out=ct, lens=dev(lens), in_off=dev(in_off), out_off=dev(out_off), **common))
    torch.cuda.synchronize()
    ct_h = bytearray(host(ct))
    for i in range(count):
        k = keys_h[32 * kidx[i]:32 * kidx[i] + 32]
        s, n = int(seqs[i]), int(lens[i])
        exp = oracle.seal(k, struct.pack(">Q", s), pt_h[in_off[i]:in_off[i] + n], oracle.tls_ad(s, n))
        assert bytes(ct_h[out_off[i]:out_off[i] + n + 16]) == exp, i
    # open: tamper record 5, truncate record 9 to 10 bytes
    ct_h[int(out_off[5])] ^= 1
    olens = (lens + 16).astype(np.uint32)
    olens[9] = 10
    back = torch.full((pos_i + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    B.open_(B.Batch(inp=dev_bytes(bytes(ct_h)), out=back, lens=dev(olens), in_off=dev(out_off),
                    out_off=dev(in_off), status=st, **common))
    torch.cuda.synchronize()
    st_h = host(st)
    exp_st = bytearray(count)
    exp_st[5], exp_st[9] = 1, 2
    assert st_h == bytes(exp_st)
    back_h = host(back)
    # a record that fails its tag releases no plaintext (chacha20_poly1305.rs:89-93): zero-filled
    assert back_h[in_off[5]:in_off[5] + lens[5]] == bytes(int(lens[5]))
    for i in range(count):
        if i in (5, 9):
            continue
        assert back_h[in_off[i]:in_off[i] + lens[i]] == pt_h[in_off[i]:in_off[i] + lens[i]], i


@pytest.mark.parametrize("n", [5, 100, 200, 400, 777, 3000])
def test_batch_explicit_mode(gpu, oracle, n):
    """Explicit nonce/AD of every length class; small n puts 2..8 MAC lanes on
    a record, so the zero gap before the MAC stream spans several lanes' bytes."""
    torch = torch_mod()
    from suruga_amd import batch as B

    rng = np.random.default_rng(3 + n)
    for adlen in (0, 1, 5, 13, 17, 32, 255):
        count = 40
        nonces_h, ads_h, pt_h = rng.bytes(8 * count), rng.bytes(max(adlen, 1) * count), rng.bytes(n * count)
        keys = dev_bytes(KEY).view(1, 32)
        ct = torch.empty(count * (n + 16), dtype=torch.uint8, device="cuda")
        B.seal(B.Batch(count=count, keys=keys, inp=dev_bytes(pt_h), out=ct, uniform_len=n, in_stride=n,
                       out_stride=n + 16, tls=False, nonces=dev_bytes(nonces_h), ads=dev_bytes(ads_h),
                       ad_len=adlen, ad_stride=max(adlen, 1)))
        torch.cuda.synchronize()
        got = host(ct)
        for j in range(count):
            ad = ads_h[j * max(adlen, 1):j * max(adlen, 1) + adlen]
            exp = oracle.seal(KEY, nonces_h[8 * j:8 * j + 8], pt_h[j * n:(j + 1) * n], ad)
            assert got[j * (n + 16):(j + 1) * (n + 16)] == exp, (adlen, j)


def test_c1_scale_roundtrip_and_tag_fold(gpu, oracle):
    """65536 x 16 KiB (1 GiB): every record round-trips on device, and the
    XOR-fold of all 65536 tags equals the multi-threaded oracle's."""
    torch = torch_mod()
    from suruga_amd import batch as B

    count, n = 65536, 16384
    pt, ct, back, st = tls_batch(count, n, seq0=7)
    mism = torch.zeros(1, dtype=torch.int64, device="cuda")
    B.compare_records(pt, n, back, n, n, count, mism)
    torch.cuda.synchronize()
    assert int(mism.item()) == 0 and int(st.sum().item()) == 0
    tags = ct.view(count, n + 16)[:, n:].cpu().numpy()
    fold = np.bitwise_xor.reduce(tags, axis=0).tobytes()
    ct_ref = oracle.seal_batch_tls(KEY, 7, host(pt), n, count, threads=min(16, os.cpu_count() or 1))
    ref_tags = np.frombuffer(ct_ref, dtype=np.uint8).reshape(count, n + 16)[:, n:]
    assert fold == np.bitwise_xor.reduce(ref_tags, axis=0).tobytes()
    # and a strided sample of whole records byte for byte
    ct_h = ct.view(count, n + 16)
    ref = np.frombuffer(ct_ref, dtype=np.uint8).reshape(count, n + 16)
    for i in list(range(0, count, 4099)) + [count // 2, count - 1]:
        assert np.array_equal(ct_h[i].cpu().numpy(), ref[i]), i


def test_c2_zipf_sample_bit_exact(gpu, oracle):
    """C2 shape: Zipf 64 B-16 KiB, 256 connection keys, seq = i / 256; mixed
    sizes go through device bucketing into all eight size classes."""
    torch = torch_mod()
    from suruga_amd import batch as B
    from suruga_amd import workloads as W

    count = 3000
    lay = W.c2_layout(count)
    classes = {0 if int(x) <= 128 else min(7, ((int(x) - 1) >> 7).bit_length()) for x in lay.lens}
    assert classes == set(range(8))  # include/suruga_gpu.h size classes: n <= 128 << c
    rng = np.random.default_rng(5)
    pt_h = rng.bytes(lay.pt_bytes)
    t64 = lambda a: torch.from_numpy(a.view(np.int64)).to("cuda")
    t32 = lambda a: torch.from_numpy(a.view(np.int32)).to("cuda")
    keys = dev_bytes(lay.keys).view(-1, 32)
    ct = torch.zeros(lay.ct_bytes, dtype=torch.uint8, device="cuda")
    maxl = int(lay.lens.max())
    common = dict(count=count, keys=keys, key_index=t32(lay.key_index), seq=t64(lay.seq))
    B.seal(B.Batch(inp=dev_bytes(pt_h), out=ct, lens=t32(lay.lens), max_len=maxl, in_off=t64(lay.in_off),
                   out_off=t64(lay.out_off), **common))
    torch.cuda.synchronize()
    ct_h = host(ct)
    for i in range(count):
        k = lay.keys[32 * lay.key_index[i]:32 * lay.key_index[i] + 32]
        s, n, o, q = int(lay.seq[i]), int(lay.lens[i]), int(lay.in_off[i]), int(lay.out_off[i])
        exp = oracle.seal(k, struct.pack(">Q", s), pt_h[o:o + n], oracle.tls_ad(s, n))
        assert ct_h[q:q + n + 16] == exp, (i, n)
    back = torch.zeros(lay.pt_bytes, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    B.open_(B.Batch(inp=ct, out=back, lens=t32(lay.lens + 16), max_len=maxl + 16, in_off=t64(lay.out_off),
                    out_off=t64(lay.in_off), status=st, **common))
    torch.cuda.synchronize()
    assert host(st) == bytes(count) and host(back) == pt_h


def test_mixed_batch_graph_capture(gpu, oracle):
    """A mixed-size batch captured into a HIP graph (the library then uses
    persistent class grids instead of reading the class populations back) and
    replayed: same bytes as the oracle."""
    torch = torch_mod()
    from suruga_amd import batch as B
    from suruga_amd import workloads as W

    count = 1500
    lay = W.c2_layout(count)
    rng = np.random.default_rng(17)
    pt_h = rng.bytes(lay.pt_bytes)
    t64 = lambda a: torch.from_numpy(a.view(np.int64)).to("cuda")
    t32 = lambda a: torch.from_numpy(a.view(np.int32)).to("cuda")
    keys = dev_bytes(lay.keys).view(-1, 32)
    pt = dev_bytes(pt_h)
    ct = torch.zeros(lay.ct_bytes, dtype=torch.uint8, device="cuda")
    ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device="cuda")
    lens, in_off, out_off = t32(lay.lens), t64(lay.in_off), t64(lay.out_off)
    kidx, seq = t32(lay.key_index), t64(lay.seq)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b = B.Batch(count=count, keys=keys, inp=pt, out=ct, lens=lens, max_len=int(lay.lens.max()), in_off=in_off,
                    out_off=out_off, key_index=kidx, seq=seq, workspace=ws, stream=torch.cuda.current_stream())
        B.seal(b)
    ct.zero_()
    g.replay()
    torch.cuda.synchronize()
    ct_h = host(ct)
    for i in range(0, count, 7):
        k = lay.keys[32 * lay.key_index[i]:32 * lay.key_index[i] + 32]
        s, n, o, q = int(lay.seq[i]), int(lay.lens[i]), int(lay.in_off[i]), int(lay.out_off[i])
        exp = oracle.seal(k, struct.pack(">Q", s), pt_h[o:o + n], oracle.tls_ad(s, n))
        assert ct_h[q:q + n + 16] == exp, (i, n)


def test_full_record_batch_graph_capture(gpu, oracle):
    """The C1 path (keying pre-pass + wave-per-record kernel) of a seal and an
    open captured into one HIP graph and replayed twice, the second time on new
    plaintext and with the sequence numbers moved on (both read from device
    memory): every record round-trips, and the sealed records equal the
    oracle's, byte for byte on every tag and on a strided sample."""
    torch = torch_mod()
    from suruga_amd import batch as B

    count, n = 2051, 16384
    keys = dev_bytes(KEY).view(1, 32)
    pt = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    ct = torch.zeros(count * (n + 16), dtype=torch.uint8, device="cuda")
    back = torch.zeros(count * n, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device="cuda")
    seq = torch.arange(count, dtype=torch.int64, device="cuda")
    B.fill_records(pt, n, n, count, SEED, 0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        B.seal(B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=n + 16,
                       seq=seq, workspace=ws, stream=cur))
        B.open_(B.Batch(count=count, keys=keys, inp=ct, out=back, uniform_len=n + 16, in_stride=n + 16,
                        out_stride=n, seq=seq, status=st, workspace=ws, stream=cur))
    for rnd, (j0, s0) in enumerate([(0, 0), (7 * count, 2**32 - 5)]):
        B.fill_records(pt, n, n, count, SEED, j0)
        seq.copy_(torch.arange(count, dtype=torch.int64, device="cuda") + s0)
        ct.zero_()
        back.zero_()
        st.fill_(0xFF)
        g.replay()
        torch.cuda.synchronize()
        assert host(st) == bytes(count) and bool(torch.equal(back, pt)), rnd
        ref = np.frombuffer(oracle.seal_batch_tls(KEY, s0, host(pt), n, count, threads=min(16, os.cpu_count() or 1)),
                            dtype=np.uint8).reshape(count, n + 16)
        got = ct.view(count, n + 16)
        assert np.array_equal(got[:, n:].cpu().numpy(), ref[:, n:]), rnd
        for i in list(range(0, count, 257)) + [count - 1]:
            assert np.array_equal(got[i].cpu().numpy(), ref[i]), (rnd, i)


@pytest.mark.parametrize("adlen", [13, 0, 3, 29])
def test_length_sweep_every_mac_geometry(gpu, oracle, adlen):
    """Every payload length 0..2200 and every 37th length up to 2^14 + 2048 in
    one mixed batch (all eight size classes, device bucketing), against the
    oracle byte for byte, then opened.  For TLS AD the sweep takes 252
    distinct (MAC lanes, leading virtual blocks) pairs, every odd blocks-per-lane
    k = 1..19, the partially virtual lane at many offsets and final MAC blocks
    of every length 1..16 (poly1305.rs:213-228).
    adlen 13 is TLS mode (nonce and AD built on device, tls.rs:103-112); the
    others pass explicit per-record nonces and AD."""
    torch = torch_mod()
    from suruga_amd import batch as B

    lens = np.concatenate([np.arange(0, 2201), np.arange(2201, 16384 + 2049, 37)]).astype(np.uint32)
    count = len(lens)
    rng = np.random.default_rng(1000 + adlen)
    # records 16-byte aligned (vector path) except every 5th, packed at an odd offset
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    pi = po = 0
    for i in range(count):
        pi += 3 if i % 5 == 4 else (-pi) % 16
        po += 3 if i % 5 == 4 else (-po) % 16
        in_off[i], out_off[i] = pi, po
        pi += int(lens[i])
        po += int(lens[i]) + 16
    pt_h = rng.bytes(pi + 16)
    nonces_h = rng.bytes(8 * count)
    ads_h = rng.bytes(max(adlen, 1) * count)
    seqs = np.arange(count, dtype=np.uint64) * 7919
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    keys = dev_bytes(KEY).view(1, 32)
    if adlen == 13:
        mode = dict(seq=dev(seqs))
    else:
        mode = dict(tls=False, nonces=dev_bytes(nonces_h), ads=dev_bytes(ads_h), ad_len=adlen,
                    ad_stride=max(adlen, 1))
    ct = torch.zeros(po + 16, dtype=torch.uint8, device="cuda")
    common = dict(count=count, keys=keys, max_len=int(lens.max()) + 16, **mode)
    B.seal(B.Batch(inp=dev_bytes(pt_h), out=ct, lens=dev(lens), in_off=dev(in_off), out_off=dev(out_off),
                   **common))
    torch.cuda.synchronize()
    ct_h = host(ct)
    for i in range(count):
        n = int(lens[i])
        if adlen == 13:
            s = int(seqs[i])
            nonce, ad = struct.pack(">Q", s), oracle.tls_ad(s, n)
        else:
            nonce, ad = nonces_h[8 * i:8 * i + 8], ads_h[i * max(adlen, 1):i * max(adlen, 1) + adlen]
        exp = oracle.seal(KEY, nonce, pt_h[in_off[i]:in_off[i] + n], ad)
        assert ct_h[out_off[i]:out_off[i] + n + 16] == exp, (adlen, n)
    back = torch.zeros(pi + 16, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    B.open_(B.Batch(inp=ct, out=back, lens=dev((lens + 16).astype(np.uint32)), in_off=dev(out_off),
                    out_off=dev(in_off), status=st, **common))
    torch.cuda.synchronize()
    assert host(st) == bytes(count)
    back_h = host(back)
    for i in range(count):
        assert back_h[in_off[i]:in_off[i] + lens[i]] == pt_h[in_off[i]:in_off[i] + lens[i]], (adlen, int(lens[i]))


# ---------------------------------------------------------------------------
# wave-per-record kernel (uniform batches of full 16 KiB records, sg_wpr.hip)
# ---------------------------------------------------------------------------
@pytest.fixture(params=[1, 0], ids=["wpr", "sizeclass"])
def kernel_form(request, gpu):
    from suruga_amd import _native as N

    lib = N.load()
    prev = lib.sg_set_lockstep(request.param)
    assert lib.sg_set_lockstep(-1) == request.param
    yield request.param
    lib.sg_set_lockstep(prev)


@pytest.mark.parametrize("adlen", [13, 0, 1, 7, 8, 24, 100, 255])
def test_full_record_kernel_geometries(gpu, oracle, kernel_form, adlen):
    """Full 16 KiB records (the wave-per-record kernel's batches) for TLS and
    explicit AD of every stream phase (|ad| + 8 mod 16 = 5, 8, 9, 15, 0, 12,
    12, 7: MAC chunks split 11/5, 8/8, ... between blocks; delta 0 and 1),
    record counts that leave 1..7 inactive waves in the last workgroup, strides
    with padding, per-record key_index and seq arrays, then open with a tampered
    tag byte, a tampered ciphertext byte and a tampered AD; both kernel forms
    against the oracle byte for byte."""
    torch = torch_mod()
    from suruga_amd import batch as B

    n = 16384
    rng = np.random.default_rng(77 + adlen)
    keys_h = rng.bytes(4 * 32)
    keys = dev_bytes(keys_h).view(4, 32)
    for count, pad in ((1, 0), (5, 16), (8, 0), (9, 48), (23, 0)):
        si, so = n + pad, n + 16 + pad
        pt_h = rng.bytes(si * count)
        nonces_h = rng.bytes(8 * count)
        ads_h = rng.bytes(max(adlen, 1) * count)
        kidx = (np.arange(count) * 3 % 4).astype(np.uint32)
        seqs = (np.arange(count, dtype=np.uint64) * 0x100000001 + 0xFFFFFFF0)
        dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
        if adlen == 13:
            mode = dict(seq=dev(seqs))
        else:
            mode = dict(tls=False, nonces=dev_bytes(nonces_h), ads=dev_bytes(ads_h), ad_len=adlen,
                        ad_stride=max(adlen, 1))
        mode["key_index"] = dev(kidx)
        ct = torch.zeros(so * count, dtype=torch.uint8, device="cuda")
        B.seal(B.Batch(count=count, keys=keys, inp=dev_bytes(pt_h), out=ct, uniform_len=n, in_stride=si,
                       out_stride=so, **mode))
        torch.cuda.synchronize()
        ct_h = bytearray(host(ct))
        for i in range(count):
            k = keys_h[32 * kidx[i]:32 * kidx[i] + 32]
            if adlen == 13:
                s = int(seqs[i])
                nonce, ad = struct.pack(">Q", s), oracle.tls_ad(s, n)
            else:
                nonce, ad = nonces_h[8 * i:8 * i + 8], ads_h[i * max(adlen, 1):i * max(adlen, 1) + adlen]
            exp = oracle.seal(k, nonce, pt_h[i * si:i * si + n], ad)
            assert bytes(ct_h[i * so:i * so + n + 16]) == exp, (kernel_form, adlen, count, i)
        exp_st = bytearray(count)
        ct_h[(count - 1) * so + n + 5] ^= 0x40  # last record: a tag byte
        exp_st[count - 1] = 1
        if count > 2:
            ct_h[1 * so + 4097] ^= 0x01  # record 1: a ciphertext byte of chunk 1
            exp_st[1] = 1
        ads_in = bytearray(ads_h)
        if count > 3 and adlen not in (0, 13):
            ads_in[3 * max(adlen, 1)] ^= 0x10  # record 3: its AD (explicit mode)
            exp_st[3] = 1
        if adlen != 13:
            mode["ads"] = dev_bytes(bytes(ads_in))
        back = torch.zeros(si * count, dtype=torch.uint8, device="cuda")
        st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
        keep = count % 2 == 1  # odd counts: keep the failed records' decryption, even: zero-filled
        B.open_(B.Batch(count=count, keys=keys, inp=dev_bytes(bytes(ct_h)), out=back, uniform_len=n + 16,
                        in_stride=so, out_stride=si, status=st, keep_failed=keep, **mode))
        torch.cuda.synchronize()
        assert host(st) == bytes(exp_st), (kernel_form, adlen, count)
        back_h = host(back)
        for i in range(count):  # decrypted unconditionally (chacha20_poly1305.rs:80-82)
            exp_pt = bytearray(pt_h[i * si:i * si + n])
            if i == 1 and count > 2:
                exp_pt[4097] ^= 0x01
            if exp_st[i] and not keep:  # no plaintext with the Err (:89-93)
                exp_pt = bytearray(n)
            assert back_h[i * si:i * si + n] == bytes(exp_pt), (kernel_form, adlen, count, i)


def test_full_record_kernel_persistent_groups(gpu, oracle, kernel_form):
    """More record groups than resident workgroups (each workgroup walks several
    groups and prefetches the next record's first chunk and keying table), with
    a partial last group: 8195 x 16 KiB, compared byte for byte with the oracle
    on a strided sample plus an XOR-fold of every tag, and opened on device."""
    torch = torch_mod()
    from suruga_amd import batch as B

    count, n = 8195, 16384
    pt, ct, back, st = tls_batch(count, n, seq0=0xFFFFFF00)
    mism = torch.zeros(1, dtype=torch.int64, device="cuda")
    B.compare_records(pt, n, back, n, n, count, mism)
    torch.cuda.synchronize()
    assert int(mism.item()) == 0 and host(st) == bytes(count)
    pt_h = host(pt)
    ct_ref = oracle.seal_batch_tls(KEY, 0xFFFFFF00, pt_h, n, count, threads=min(16, os.cpu_count() or 1))
    ref = np.frombuffer(ct_ref, dtype=np.uint8).reshape(count, n + 16)
    got = ct.view(count, n + 16)
    tags = got[:, n:].cpu().numpy()
    assert np.bitwise_xor.reduce(tags, axis=0).tobytes() == np.bitwise_xor.reduce(ref[:, n:], axis=0).tobytes()
    assert np.array_equal(tags, ref[:, n:])
    for i in list(range(0, count, 511)) + [count - 3, count - 2, count - 1]:
        assert np.array_equal(got[i].cpu().numpy(), ref[i]), i


def test_single_record_limits(gpu, oracle):
    """AD of 255 bytes and a 32768-byte record are accepted
    and bit-exact; 256 bytes of AD and 32769-byte records are SG_E_ARG."""
    import ctypes as C

    from suruga_amd import ChaCha20Poly1305
    from suruga_amd import _native as N

    lib = N.load()
    aead = ChaCha20Poly1305()
    enc, dec = aead.new_encryptor(KEY), aead.new_decryptor(KEY)
    nonce = bytes(range(8))
    ad, pt = bytes(range(255)), oracle.fill_record(SEED, 3, 32768)
    ct = enc.encrypt(nonce, pt, ad)
    assert ct == oracle.seal(KEY, nonce, pt, ad)
    assert dec.decrypt(nonce, ct, ad) == pt
    out = (C.c_uint8 * (32769 + 16))()
    assert lib.sg_seal(enc._ptr, nonce, 8, pt, 100, bytes(256), 256, out) == N.SG_E_ARG
    big = bytes(32769)
    assert lib.sg_seal(enc._ptr, nonce, 8, big, len(big), ad, 13, out) == N.SG_E_ARG
    assert lib.sg_open(dec._ptr, nonce, 8, big + bytes(16), len(big) + 16, ad, 13, out) == N.SG_E_ARG


def _mixed_wpr_layout(count, rng, aligned=True):
    """Lengths that fill every wave-per-record bucket (4 KiB < n <= 16 KiB,
    multiples of 64: J = 2, 3, 4 chunks, their edges) and the size classes
    around them (n <= 4096, n not a multiple of 64); records packed at 16-byte
    (or, aligned=False, odd) offsets."""
    edges = [4096, 4160, 8192, 8256, 12288, 12352, 16320, 16384, 5000, 4097, 16383, 64, 0, 1, 2049]
    lens = np.where(rng.random(count) < 0.75, 64 * rng.integers(65, 257, size=count),
                    rng.integers(0, 16385, size=count)).astype(np.uint32)
    lens[:len(edges)] = edges
    pad = 16 if aligned else 1
    step_i = ((lens.astype(np.uint64) + pad - 1) // pad) * pad + (0 if aligned else 3)
    step_o = ((lens.astype(np.uint64) + 16 + pad - 1) // pad) * pad + (0 if aligned else 5)
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    in_off[1:] = np.cumsum(step_i[:-1])
    out_off[1:] = np.cumsum(step_o[:-1])
    return lens, in_off, out_off, int(in_off[-1] + step_i[-1]), int(out_off[-1] + step_o[-1])


@pytest.mark.parametrize("count", [600, 24000])
def test_mixed_batch_wave_per_record_buckets(gpu, oracle, count):
    """Mixed TLS batches whose 4-16 KiB records (multiples of 64 bytes, 16-byte
    aligned) run on the wave-per-record kernel, right-aligned in its 16 KiB
    frame (sg_wpr.hip), in three chunk-count buckets; the rest on the size
    classes.  24000 records put ~6000 in each bucket, more than the two
    statically assigned groups per workgroup, so the device group counter and
    the descriptor prefetch run too.  Every byte against the oracle; open with
    tampering in the first (partial) chunk, the last chunk and the tag of
    bucket records, and a truncated record."""
    torch = torch_mod()
    from suruga_amd import batch as B

    rng = np.random.default_rng(29 + count)
    lens, in_off, out_off, pt_bytes, ct_bytes = _mixed_wpr_layout(count, rng)
    buckets = {(int(n) + 4095) // 4096 for n in lens if 4096 < n <= 16384 and n % 64 == 0}
    assert buckets == {2, 3, 4}
    keys_h = rng.bytes(256 * 32)
    kidx = rng.integers(0, 256, size=count).astype(np.uint32)
    seqs = rng.integers(0, 2**63, size=count, dtype=np.uint64)
    seqs[:3] = [0, 2**32 - 1, 2**64 - 1]
    pt_h = rng.bytes(pt_bytes)
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    keys = dev_bytes(keys_h).view(256, 32)
    d_lens, d_olens, d_in, d_out = dev(lens), dev((lens + 16).astype(np.uint32)), dev(in_off), dev(out_off)
    common = dict(count=count, keys=keys, key_index=dev(kidx), seq=dev(seqs))
    ct = torch.zeros(ct_bytes, dtype=torch.uint8, device="cuda")
    B.seal(B.Batch(inp=dev_bytes(pt_h), out=ct, lens=d_lens, max_len=int(lens.max()), in_off=d_in, out_off=d_out,
                   **common))
    torch.cuda.synchronize()
    ct_h = bytearray(host(ct))
    for i in range(count):
        k = keys_h[32 * int(kidx[i]):32 * int(kidx[i]) + 32]
        s, n, o, q = int(seqs[i]), int(lens[i]), int(in_off[i]), int(out_off[i])
        exp = oracle.seal(k, struct.pack(">Q", s), pt_h[o:o + n], oracle.tls_ad(s, n))
        assert bytes(ct_h[q:q + n + 16]) == exp, (i, n)
    # open: tamper bucket records (J = 2, 3, 4) at their first byte, their last
    # ciphertext byte, their tag; truncate one record
    bucket_recs = [i for i in range(count) if 4096 < lens[i] <= 16384 and lens[i] % 64 == 0]
    tamper = {bucket_recs[0]: 0, bucket_recs[1]: int(lens[bucket_recs[1]]) - 1, bucket_recs[2]: int(lens[bucket_recs[2]]) + 7}
    for i, at in tamper.items():
        ct_h[int(out_off[i]) + at] ^= 0x40
    olens = (lens + 16).astype(np.uint32)
    short = bucket_recs[3]
    olens[short] = 15
    back = torch.zeros(pt_bytes, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    d_olens = dev(olens)
    B.open_(B.Batch(inp=dev_bytes(bytes(ct_h)), out=back, lens=d_olens, max_len=int(olens.max()), in_off=d_out,
                    out_off=d_in, status=st, keep_failed=True, **common))
    torch.cuda.synchronize()
    exp_st = bytearray(count)
    for i in tamper:
        exp_st[i] = 1
    exp_st[short] = 2
    assert host(st) == bytes(exp_st)
    back_h = host(back)
    for i in range(count):
        if exp_st[i]:
            continue
        o, n = int(in_off[i]), int(lens[i])
        assert back_h[o:o + n] == pt_h[o:o + n], (i, n)
    # the reference decrypts a tampered record anyway (chacha20_poly1305.rs:80-82):
    # the plaintext under the flipped byte differs from the input in that byte only
    i = bucket_recs[0]
    o = int(in_off[i])
    assert back_h[o] == pt_h[o] ^ 0x40 and back_h[o + 1:o + int(lens[i])] == pt_h[o + 1:o + int(lens[i])]


def test_mixed_batch_unaligned_records_skip_buckets(gpu, oracle):
    """The same lengths at odd offsets: no record is 16-byte aligned, so every
    one runs on the size classes (byte-granular where needed); bit-exact."""
    torch = torch_mod()
    from suruga_amd import batch as B

    rng = np.random.default_rng(31)
    count = 300
    lens, in_off, out_off, pt_bytes, ct_bytes = _mixed_wpr_layout(count, rng, aligned=False)
    pt_h = rng.bytes(pt_bytes)
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    keys = dev_bytes(KEY).view(1, 32)
    ct = torch.zeros(ct_bytes, dtype=torch.uint8, device="cuda")
    d_lens, d_in, d_out = dev(lens), dev(in_off), dev(out_off)
    B.seal(B.Batch(count=count, keys=keys, inp=dev_bytes(pt_h), out=ct, lens=d_lens, max_len=int(lens.max()),
                   in_off=d_in, out_off=d_out, seq0=5))
    torch.cuda.synchronize()
    ct_h = host(ct)
    for i in range(count):
        n, o, q = int(lens[i]), int(in_off[i]), int(out_off[i])
        exp = oracle.seal(KEY, struct.pack(">Q", 5 + i), pt_h[o:o + n], oracle.tls_ad(5 + i, n))
        assert ct_h[q:q + n + 16] == exp, (i, n)


@pytest.fixture(params=[1, 0], ids=["packed", "classes"])
def small_form(request, gpu):
    from suruga_amd import _native

    lib = _native.load()
    prev = lib.sg_set_packed(request.param)
    assert lib.sg_set_packed(-1) == request.param
    yield request.param
    lib.sg_set_packed(prev)


@pytest.mark.parametrize("count,buckets", [(777, True), (9000, True), (2500, False)])
def test_mixed_batch_packed_small_records(gpu, oracle, small_form, count, buckets):
    """Mixed TLS batches whose 64 B-4 KiB records (multiples of 64 bytes,
    16-byte aligned) run on the packed kernel (sg_pack.hip: 128-record runs
    from a device counter on a persistent grid, blocks end to end over the
    lanes, keyed in the kernel), beside records of other lengths (size classes)
    and 4-16 KiB ones (wave-per-record buckets; none with buckets=False, so
    that only the packed launch and the classes run beside the keying
    stream); and the same batch on the size classes (small_form 0).  Every
    block count 1..64 occurs, runs of sixty-four 4 KiB records fill a run's 64
    chunks, and the count is not a multiple of the run size.  Every byte
    against the oracle; open with tampering in the first byte, the last
    ciphertext byte and the tag of packed records, and a truncated record."""
    torch = torch_mod()
    from suruga_amd import batch as B

    # the smaller batch with another record header (AD bytes 8-10, tls.rs:105-112)
    ctype, minor = (22, 1) if count < 1000 else (23, 3)
    rng = np.random.default_rng(41 + count)
    lens = (64 * rng.integers(1, 65, size=count)).astype(np.uint32)
    lens[100:300] = 4096                       # whole runs of 64 x 64 blocks
    lens[300:364] = 64 * (np.arange(64) + 1)   # every block count
    odd = rng.random(count) < 0.1
    lens[odd] = rng.integers(0, 4200 if buckets else 4096, size=int(odd.sum())).astype(np.uint32)  # size classes
    big = rng.random(count) < (0.03 if buckets else 0.0)
    lens[big] = (64 * rng.integers(65, 257, size=int(big.sum()))).astype(np.uint32)  # buckets
    step_i = (lens.astype(np.uint64) + 15) // 16 * 16
    step_o = (lens.astype(np.uint64) + 16 + 15) // 16 * 16
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    in_off[1:] = np.cumsum(step_i[:-1])
    out_off[1:] = np.cumsum(step_o[:-1])
    pt_bytes, ct_bytes = int(in_off[-1] + step_i[-1]), int(out_off[-1] + step_o[-1])
    packed = [i for i in range(count) if 64 <= lens[i] <= 4096 and lens[i] % 64 == 0]
    assert len(packed) > count // 2
    keys_h = rng.bytes(256 * 32)
    kidx = rng.integers(0, 256, size=count).astype(np.uint32)
    seqs = rng.integers(0, 2**63, size=count, dtype=np.uint64)
    seqs[:3] = [0, 2**32 - 1, 2**64 - 1]
    pt_h = rng.bytes(pt_bytes)
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    keys = dev_bytes(keys_h).view(256, 32)
    common = dict(count=count, keys=keys, key_index=dev(kidx), seq=dev(seqs), content_type=ctype, version=(3, minor))
    ct = torch.zeros(ct_bytes, dtype=torch.uint8, device="cuda")
    B.seal(B.Batch(inp=dev_bytes(pt_h), out=ct, lens=dev(lens), max_len=int(lens.max()), in_off=dev(in_off),
                   out_off=dev(out_off), **common))
    torch.cuda.synchronize()
    ct_h = bytearray(host(ct))
    for i in range(count):
        k = keys_h[32 * int(kidx[i]):32 * int(kidx[i]) + 32]
        s, n, o, q = int(seqs[i]), int(lens[i]), int(in_off[i]), int(out_off[i])
        exp = oracle.seal(k, struct.pack(">Q", s), pt_h[o:o + n], oracle.tls_ad(s, n, ctype, 3, minor))
        assert bytes(ct_h[q:q + n + 16]) == exp, (i, n)
    tamper = {packed[0]: 0, packed[1]: int(lens[packed[1]]) - 1, packed[2]: int(lens[packed[2]]) + 9}
    for i, at in tamper.items():
        ct_h[int(out_off[i]) + at] ^= 0x08
    olens = (lens + 16).astype(np.uint32)
    short = packed[3]
    olens[short] = 15
    back = torch.zeros(pt_bytes, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    B.open_(B.Batch(inp=dev_bytes(bytes(ct_h)), out=back, lens=dev(olens), max_len=int(olens.max()),
                    in_off=dev(out_off), out_off=dev(in_off), status=st, keep_failed=True, **common))
    torch.cuda.synchronize()
    exp_st = bytearray(count)
    for i in tamper:
        exp_st[i] = 1
    exp_st[short] = 2
    assert host(st) == bytes(exp_st)
    back_h = host(back)
    for i in range(count):
        if exp_st[i]:
            continue
        o, n = int(in_off[i]), int(lens[i])
        assert back_h[o:o + n] == pt_h[o:o + n], (i, n)
    i = packed[0]  # decrypted anyway (chacha20_poly1305.rs:80-82)
    o = int(in_off[i])
    assert back_h[o] == pt_h[o] ^ 0x08 and back_h[o + 1:o + int(lens[i])] == pt_h[o + 1:o + int(lens[i])]


@pytest.mark.parametrize("keep", [False, True])
def test_open_failure_output_contract(gpu, oracle, keep):
    """sg_open_batch on uniform 16 KiB records (the wave-per-record kernel) and on
    1 KiB records (size classes): a record with a flipped tag byte has status 1
    and, by default, a zero-filled output (the reference returns only Err,
    chacha20_poly1305.rs:89-93); with SG_BATCH_KEEP_FAILED its output is the
    always-computed decryption (:80-82).  The other records are intact."""
    torch = torch_mod()
    from suruga_amd import batch as B

    for n, count in ((16384, 24), (1024, 50)):
        pt = torch.empty(count * n, dtype=torch.uint8, device="cuda")
        B.fill_records(pt, n, n, count, 0x5EED, j0=0)
        keys = dev_bytes(KEY).view(1, 32)
        ct = torch.empty(count * (n + 16), dtype=torch.uint8, device="cuda")
        B.seal(B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=n + 16))
        bad = (3, count - 1)
        for i in bad:
            ct[i * (n + 16) + n + 5] ^= 1
        back = torch.full((count * n,), 0xEE, dtype=torch.uint8, device="cuda")
        st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
        B.open_(B.Batch(count=count, keys=keys, inp=ct, out=back, uniform_len=n + 16, in_stride=n + 16, out_stride=n,
                        status=st, keep_failed=keep))
        torch.cuda.synchronize()
        exp_st = bytearray(count)
        for i in bad:
            exp_st[i] = 1
        assert host(st) == bytes(exp_st)
        back_h, pt_h = host(back), host(pt)
        for i in range(count):
            got = back_h[i * n:(i + 1) * n]
            if i in bad:
                assert got == (pt_h[i * n:(i + 1) * n] if keep else bytes(n)), (n, i)
            else:
                assert got == pt_h[i * n:(i + 1) * n], (n, i)


def test_overlong_record_on_null_stream(gpu, oracle):
    """A record longer than max_len on the NULL stream: the call returns SG_E_ARG
    only after the device work is done, the record's status is 3 (skipped, its
    output untouched) and every other record is opened correctly."""
    torch = torch_mod()
    from suruga_amd import _native as N
    from suruga_amd import batch as B

    count, n = 40, 512
    lens = np.full(count, n, dtype=np.uint32)
    lens[7] = 2000
    in_off = np.arange(count, dtype=np.uint64) * 4096
    out_off = np.arange(count, dtype=np.uint64) * 4096
    pt_h = np.random.default_rng(9).bytes(count * 4096)
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    keys = dev_bytes(KEY).view(1, 32)
    ct = torch.zeros(count * 4096, dtype=torch.uint8, device="cuda")
    B.seal(B.Batch(count=count, keys=keys, inp=dev_bytes(pt_h), out=ct, lens=dev(lens), max_len=2000,
                   in_off=dev(in_off), out_off=dev(out_off), seq0=11))
    torch.cuda.synchronize()
    back = torch.full((count * 4096,), 0xEE, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    ob = B.Batch(count=count, keys=keys, inp=ct, out=back, lens=dev(lens + 16), max_len=n + 16, in_off=dev(out_off),
                 out_off=dev(in_off), seq0=11, status=st, stream=0).to_c()
    import ctypes as C

    rc = N.load().sg_open_batch(C.byref(ob))
    assert rc == N.SG_E_ARG and "max_len" in N.last_error()
    # no synchronize here: the NULL-stream call has already finished
    st_h = bytes(st.cpu().numpy())
    exp = bytearray(count)
    exp[7] = 3
    assert st_h == bytes(exp)
    back_h = host(back)
    for i in range(count):
        o = int(in_off[i])
        if i == 7:
            assert back_h[o:o + 2000] == b"\xee" * 2000
        else:
            assert back_h[o:o + n] == pt_h[o:o + n], i


@pytest.mark.parametrize("shape", ["uniform16k", "mixed"])
def test_key_index_out_of_range_stays_in_table(gpu, oracle, shape):
    """key_index[i] >= num_keys (a caller bug): the kernels clamp it to
    num_keys - 1 instead of reading past the key table (suruga_gpu.h), on the
    wave-per-record path (uniform 16 KiB records) and on every path of a mixed
    batch; every record is sealed with the key it was given or the clamped one,
    and opens again."""
    torch = torch_mod()
    from suruga_amd import batch as B

    rng = np.random.default_rng(71)
    count, nk = 600, 4
    lens = (np.full(count, 16384) if shape == "uniform16k" else
            np.where(rng.random(count) < 0.5, 64 * rng.integers(1, 257, size=count),
                     rng.integers(0, 16385, size=count))).astype(np.uint32)
    step_i = (lens.astype(np.uint64) + 15) // 16 * 16
    step_o = (lens.astype(np.uint64) + 16 + 15) // 16 * 16
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    in_off[1:] = np.cumsum(step_i[:-1])
    out_off[1:] = np.cumsum(step_o[:-1])
    pt_bytes, ct_bytes = int(in_off[-1] + step_i[-1]), int(out_off[-1] + step_o[-1])
    kidx = rng.integers(0, nk, size=count).astype(np.uint32)
    kidx[::7] = nk
    kidx[3::11] = 0xFFFFFFFF
    keys_h = rng.bytes(nk * 32)
    pt_h = rng.bytes(pt_bytes)
    dev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda")
    common = dict(count=count, keys=dev_bytes(keys_h).view(nk, 32), key_index=dev(kidx), seq0=9)
    ct = torch.zeros(ct_bytes, dtype=torch.uint8, device="cuda")
    if shape == "uniform16k":
        B.seal(B.Batch(inp=dev_bytes(pt_h), out=ct, uniform_len=16384, in_stride=16384, out_stride=16400, **common))
    else:
        B.seal(B.Batch(inp=dev_bytes(pt_h), out=ct, lens=dev(lens), max_len=int(lens.max()), in_off=dev(in_off),
                       out_off=dev(out_off), **common))
    torch.cuda.synchronize()
    ct_h = host(ct)
    for i in range(count):
        k = min(int(kidx[i]), nk - 1)
        s, n, o, q = 9 + i, int(lens[i]), int(in_off[i]), int(out_off[i])
        exp = oracle.seal(keys_h[32 * k:32 * k + 32], struct.pack(">Q", s), pt_h[o:o + n], oracle.tls_ad(s, n))
        assert ct_h[q:q + n + 16] == exp, (i, n, int(kidx[i]))
    back = torch.zeros(pt_bytes, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    if shape == "uniform16k":
        B.open_(B.Batch(inp=ct, out=back, uniform_len=16400, in_stride=16400, out_stride=16384, status=st, **common))
    else:
        B.open_(B.Batch(inp=ct, out=back, lens=dev((lens + 16).astype(np.uint32)), max_len=int(lens.max()) + 16,
                        in_off=dev(out_off), out_off=dev(in_off), status=st, **common))
    torch.cuda.synchronize()
    assert host(st) == bytes(count)
    back_h = host(back)
    for i in range(count):
        o, n = int(in_off[i]), int(lens[i])
        assert back_h[o:o + n] == pt_h[o:o + n], (i, n)
