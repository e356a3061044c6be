"""Seal and open from two threads at once (the reference's reader and writer
run on independent threads: client.rs:19-21,269; Encryptor: Send,
cipher/mod.rs:18-19).

1. Record path: one thread writes 128 MiB through sg_write_records on its
   context while another reads a pre-sealed 128 MiB wire through
   sg_read_records on a second context.  Both results are bit-exact (the
   concurrent wire equals the serial one, the read-back equals the input).
   The two at once are not slower than one after the other, with pageable
   buffers (the staged path: both share the copy pool) and with registered
   ones (zero-copy: both share the host link), within a margin for the
   boxes' spread (round 5 saw 19.3 ms concurrent against 17.1 serial on one
   box and 12.3 against 15.9 on another; round 6, profiles/r06d: 1.26-1.34x
   faster pageable, 1.06-1.09x registered).  Neither call holds a lock the
   other needs across its waits: a small read started while a large write is
   in flight finishes long before the write.
2. Device batches: seal on one HIP stream and open on another, enqueued from
   two threads, each checked against the oracle.
"""
from __future__ import annotations

import ctypes as C
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEY = bytes(range(32))
REC = 1 << 14


def _lib():
    from suruga_amd import _native as N

    return N, N.load()


def _write(N, lib, ctx, data, wire, call=16 << 20):
    wl = C.c_size_t(0)
    seq, pos, wpos = 0, 0, 0
    while pos < data.size:
        n = min(call, data.size - pos)
        seq += N.check(lib.sg_write_records(ctx, seq, 23, 3, 3, C.c_void_p(data.ctypes.data + pos), n,
                                            C.c_void_p(wire.ctypes.data + wpos), wire.size - wpos, C.byref(wl)))
        pos += n
        wpos += wl.value
    return wpos


def _read(N, lib, ctx, wire, wlen, back, call=16 << 20):
    res = N.SgReadResult()
    seq, pos, opos = 0, 0, 0
    while pos < wlen:
        n = min(call + (call >> 10) + 64, wlen - pos)
        N.check(lib.sg_read_records(ctx, seq, C.c_void_p(wire.ctypes.data + pos), n,
                                    C.c_void_p(back.ctypes.data + opos), back.size - opos, None, None, 1 << 20,
                                    C.byref(res)))
        assert res.error == N.SG_OK
        seq += res.records
        pos += res.consumed
        opos += res.out_len
    return opos


def test_record_path_write_and_read_overlap(gpu):
    from suruga_amd import ChaCha20Poly1305

    N, lib = _lib()
    total = 128 << 20
    data = np.random.default_rng(7).integers(0, 256, size=total, dtype=np.uint8)
    aead = ChaCha20Poly1305()
    enc, dec = aead.new_encryptor(KEY), aead.new_decryptor(KEY)
    wire0 = np.empty(lib.sg_wire_bound(total), dtype=np.uint8)
    wire1 = np.empty_like(wire0)
    back = np.empty(total, dtype=np.uint8)
    wlen = _write(N, lib, enc._ptr, data, wire0)  # the wire the reader consumes; also warms both contexts
    assert _read(N, lib, dec._ptr, wire0, wlen, back) == total
    assert np.array_equal(back, data)

    def serial():
        t0 = time.perf_counter()
        _write(N, lib, enc._ptr, data, wire1)
        _read(N, lib, dec._ptr, wire0, wlen, back)
        return time.perf_counter() - t0

    def concurrent():
        errs = []

        def run(fn):
            try:
                fn()
            except Exception as e:  # reported below
                errs.append(repr(e))

        ta = threading.Thread(target=run, args=(lambda: _write(N, lib, enc._ptr, data, wire1),))
        tb = threading.Thread(target=run, args=(lambda: _read(N, lib, dec._ptr, wire0, wlen, back),))
        t0 = time.perf_counter()
        ta.start()
        tb.start()
        ta.join()
        tb.join()
        assert not errs, errs
        return time.perf_counter() - t0

    def serial_vs_concurrent(tag):
        ts = min(serial() for _ in range(2))
        back[:] = 0
        wire1[:] = 0
        tc = min(concurrent() for _ in range(2))
        assert np.array_equal(wire1[:wlen], wire0[:wlen]), f"{tag}: concurrent seal differs from the serial one"
        assert np.array_equal(back, data), f"{tag}: concurrent open differs from the input"
        print(f"{tag}: serial {ts * 1e3:.1f} ms, concurrent {tc * 1e3:.1f} ms")
        # no regression: the reader and the writer at once take no longer than
        # one after the other (15 % margin for the spread between boxes)
        assert tc <= 1.15 * ts, f"{tag}: concurrent {tc * 1e3:.1f} ms vs serial {ts * 1e3:.1f} ms"

    serial_vs_concurrent("pageable")
    regs = (data, wire0, wire1, back)
    for a in regs:
        N.check(lib.sg_host_register(a.ctypes.data, a.nbytes))
    try:
        serial_vs_concurrent("registered")
    finally:
        for a in regs:
            N.check(lib.sg_host_unregister(a.ctypes.data))

    # a 2 MiB read started 5 ms into a 256 MiB write on the other context ends
    # long before the write: no lock is held across the write's waits
    big = np.tile(data, 2)
    wbig = np.empty(lib.sg_wire_bound(big.size), dtype=np.uint8)
    small_wlen = (2 << 20) // REC * (5 + REC + 16)
    small_back = np.empty(2 << 20, dtype=np.uint8)
    stamps = {}

    def big_write():
        stamps["a0"] = time.perf_counter()
        _write(N, lib, enc._ptr, big, wbig)
        stamps["a1"] = time.perf_counter()

    def small_read():
        stamps["b0"] = time.perf_counter()
        assert _read(N, lib, dec._ptr, wire0, small_wlen, small_back) == small_back.size
        stamps["b1"] = time.perf_counter()

    for _ in range(2):
        ta = threading.Thread(target=big_write)
        ta.start()
        time.sleep(0.005)
        small_read()
        ta.join()
        a, b = stamps["a1"] - stamps["a0"], stamps["b1"] - stamps["b0"]
        print(f"256 MiB write {a * 1e3:.1f} ms, 2 MiB read inside it {b * 1e3:.1f} ms")
        assert np.array_equal(small_back, data[:small_back.size])
        assert stamps["b1"] < stamps["a1"] and b < 0.5 * a, (a, b)


def test_device_batches_on_two_streams(gpu, oracle):
    import torch

    from suruga_amd import batch as B

    N, lib = _lib()
    n, count = REC, 2048
    dev = torch.device("cuda", 0)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    keys = torch.tensor(list(KEY), dtype=torch.uint8, device=dev).view(1, 32)
    pt = torch.empty(count * n, dtype=torch.uint8, device=dev)
    B.fill_records(pt, n, n, count, 11, j0=0)
    ct_ref = oracle.seal_batch_tls(KEY, 0, pt.cpu().numpy().tobytes(), n, count, threads=16)
    ct_in = torch.frombuffer(bytearray(ct_ref), dtype=torch.uint8).to(dev)
    ct = torch.empty(count * (n + 16), dtype=torch.uint8, device=dev)
    back = torch.empty(count * n, dtype=torch.uint8, device=dev)
    status = torch.full((count,), 9, dtype=torch.uint8, device=dev)
    wsa = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
    wsb = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    seal = B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=n + 16, seq0=0,
                   workspace=wsa, stream=sa).to_c()
    opn = B.Batch(count=count, keys=keys, inp=ct_in, out=back, uniform_len=n + 16, in_stride=n + 16, out_stride=n,
                  seq0=0, status=status, workspace=wsb, stream=sb).to_c()
    errs = []

    def run(fn, c):
        try:
            for _ in range(4):
                N.check(fn(C.byref(c)))
        except Exception as e:  # reported below
            errs.append(repr(e))

    ta = threading.Thread(target=run, args=(lib.sg_seal_batch, seal))
    tb = threading.Thread(target=run, args=(lib.sg_open_batch, opn))
    ta.start()
    tb.start()
    ta.join()
    tb.join()
    torch.cuda.synchronize()
    assert not errs, errs
    assert bytes(ct.cpu().numpy().tobytes()) == ct_ref
    assert int((status != 0).sum().item()) == 0
    assert torch.equal(back, pt)


def _mixed_layout(rng, count):
    """A mixed TLS batch: packed 64 B-4 KiB records, 4-16 KiB bucket records
    and ragged size-class records, 16-byte aligned slots."""
    lens = (64 * rng.integers(1, 65, size=count)).astype(np.uint32)
    big = rng.random(count) < 0.06
    lens[big] = (64 * rng.integers(65, 257, size=int(big.sum()))).astype(np.uint32)
    odd = rng.random(count) < 0.08
    lens[odd] = rng.integers(0, 5000, size=int(odd.sum())).astype(np.uint32)
    step_i = (lens.astype(np.uint64) + 15) // 16 * 16
    step_o = (lens.astype(np.uint64) + 16 + 15) // 16 * 16
    in_off = np.zeros(count, dtype=np.uint64)
    out_off = np.zeros(count, dtype=np.uint64)
    in_off[1:] = np.cumsum(step_i[:-1])
    out_off[1:] = np.cumsum(step_o[:-1])
    return lens, in_off, out_off, int(in_off[-1] + step_i[-1]), int(out_off[-1] + step_o[-1])


def test_mixed_batches_on_two_streams(gpu, oracle):
    """mixed batches fork onto pooled side streams; two
    threads run mixed TLS batches (packed, bucket and size-class records) on
    two caller streams of different priority, many times over, so that the side
    streams one call returns to the pool are asked for by the other call while
    its kernels may still be queued.  A side stream is reused only once idle,
    so the batches stay independent; every byte against the oracle."""
    import struct

    import torch

    from suruga_amd import batch as B

    N, lib = _lib()
    rng = np.random.default_rng(5)
    dev = torch.device("cuda", 0)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev, priority=min(lo, hi))
    tdev = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to(dev)  # noqa: E731
    jobs = []
    for j, st in enumerate((sa, sb)):
        count = 1500 + 300 * j
        lens, in_off, out_off, pt_bytes, ct_bytes = _mixed_layout(rng, count)
        keys_h = rng.bytes(16 * 32)
        kidx = rng.integers(0, 16, size=count).astype(np.uint32)
        seqs = rng.integers(0, 2**40, size=count, dtype=np.uint64)
        pt_h = rng.bytes(pt_bytes)
        exp = bytearray(ct_bytes)
        for i in range(count):
            k = keys_h[32 * int(kidx[i]):32 * int(kidx[i]) + 32]
            s, n, o, q = int(seqs[i]), int(lens[i]), int(in_off[i]), int(out_off[i])
            exp[q:q + n + 16] = oracle.seal(k, struct.pack(">Q", s), pt_h[o:o + n], oracle.tls_ad(s, n))
        keys = torch.frombuffer(bytearray(keys_h), dtype=torch.uint8).to(dev).view(16, 32)
        ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
        common = dict(count=count, keys=keys, key_index=tdev(kidx), seq=tdev(seqs), workspace=ws, stream=st)
        if j == 0:  # thread A seals
            out = torch.zeros(ct_bytes, dtype=torch.uint8, device=dev)
            b = B.Batch(inp=torch.frombuffer(bytearray(pt_h), dtype=torch.uint8).to(dev), out=out, lens=tdev(lens),
                        max_len=int(lens.max()), in_off=tdev(in_off), out_off=tdev(out_off), **common)
            jobs.append((lib.sg_seal_batch, b, out, bytes(exp), None, None))
        else:       # thread B opens
            out = torch.zeros(pt_bytes, dtype=torch.uint8, device=dev)
            status = torch.full((count,), 0xFF, dtype=torch.uint8, device=dev)
            olens = (lens + 16).astype(np.uint32)
            b = B.Batch(inp=torch.frombuffer(bytearray(exp), dtype=torch.uint8).to(dev), out=out, lens=tdev(olens),
                        max_len=int(olens.max()), in_off=tdev(out_off), out_off=tdev(in_off), status=status, **common)
            want = bytearray(pt_bytes)
            for i in range(count):
                o, n = int(in_off[i]), int(lens[i])
                want[o:o + n] = pt_h[o:o + n]
            jobs.append((lib.sg_open_batch, b, out, bytes(want), status, (lens, in_off)))
    torch.cuda.synchronize()
    cs = [job[1].to_c() for job in jobs]
    errs = []

    def run(fn, c):
        try:
            for _ in range(12):
                N.check(fn(C.byref(c)))
        except Exception as e:  # reported below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(job[0], c)) for job, c in zip(jobs, cs)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    fn, b, out, want, status, meta = jobs[0]
    got = out.cpu().numpy().tobytes()
    assert got == want, "seal thread's batch differs from the oracle"
    fn, b, out, want, status, (lens, in_off) = jobs[1]
    assert int((status != 0).sum().item()) == 0
    got = out.cpu().numpy().tobytes()
    for i in range(len(lens)):
        o, n = int(in_off[i]), int(lens[i])
        assert got[o:o + n] == want[o:o + n], i
