"""Seal and open from two threads at once (the reference's reader and writer
run on independent threads: client.rs:19-21,269; Encryptor: Send,
cipher/mod.rs:18-19).

1. Record path: one thread writes 128 MiB through sg_write_records on its
   context while another reads a pre-sealed 128 MiB wire through
   sg_read_records on a second context.  Both results are bit-exact (the
   concurrent wire equals the serial one, the read-back equals the input), and
   the concurrent wall time is below the serial sum: neither call holds a lock
   the other needs across its waits, and each context has its own streams.
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

    ts = min(serial() for _ in range(2))
    back[:] = 0
    wire1[:] = 0
    tc = min(concurrent() for _ in range(2))
    assert np.array_equal(wire1[:wlen], wire0[:wlen]), "concurrent seal differs from the serial one"
    assert np.array_equal(back, data), "concurrent open differs from the input"
    print(f"serial {ts * 1e3:.1f} ms, concurrent {tc * 1e3:.1f} ms")
    assert tc < 0.95 * ts, (ts, tc)


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
