"""Randomised record-layer parity (GPU): sg_write_records / sg_read_records
(tls.rs:126-147, 217-281) over streams of random length -- empty, shorter
than a record, ragged tails, exact multiples of 2^14 and several pipeline
chunks -- from pageable or sg_host_register'ed buffers.  Every wire record is
compared with the oracle's TLS sealing (header, ciphertext, tag), the read
returns the stream, the per-record types and lengths; then one random fault
per stream: a flipped ciphertext or tag byte (BadRecordMac after the records
before it), an unknown content type (UnexpectedMessage, tls.rs:218-225), or
an incomplete last record (not an error: the complete ones are delivered and
consumed, the partial one is left in the buffer).  Nothing of an undelivered
record reaches `out`.
"""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REC = 1 << 14
WREC = 5 + REC + 16


@pytest.mark.parametrize("seed", list(range(16)))
def test_random_record_streams(gpu, oracle, seed):
    from suruga_amd import ChaCha20Poly1305
    from suruga_amd import _native as N

    lib = N.load()
    rng = np.random.default_rng(0x5EC0 + seed)
    total = int(rng.choice([0, int(rng.integers(1, REC)), REC * int(rng.integers(1, 5)),
                            int(rng.integers(REC, 300 * REC)), 600 * REC + int(rng.integers(1, REC))]))
    registered = seed % 2 == 1
    key = rng.bytes(32)
    seq0 = int(rng.integers(0, 2**62))
    enc, dec = ChaCha20Poly1305().new_encryptor(key), ChaCha20Poly1305().new_decryptor(key)
    data = np.frombuffer(rng.bytes(total), dtype=np.uint8).copy() if total else np.zeros(1, dtype=np.uint8)
    cap = max(int(lib.sg_wire_bound(total)), 1)
    wire = np.zeros(cap, dtype=np.uint8)
    out = np.full(max(total, 1), 0xEE, dtype=np.uint8)
    nrec_max = total // REC + 2
    types = np.zeros(nrec_max, dtype=np.uint8)
    flens = np.zeros(nrec_max, dtype=np.uint32)
    bufs = (data, wire, out) if registered and total else ()
    for a in bufs:
        N.check(lib.sg_host_register(a.ctypes.data, a.nbytes))
    try:
        wl = C.c_size_t(0)
        nrec = N.check(lib.sg_write_records(enc._ptr, seq0, 23, 3, 3, data.ctypes.data, total, wire.ctypes.data, cap,
                                            C.byref(wl)))
        wlen = wl.value
        assert nrec == -(-total // REC)
        assert wlen == total + nrec * 21
        for r in range(nrec):
            n = min(REC, total - r * REC)
            hdr = bytes([23, 3, 3]) + struct.pack(">H", n + 16)
            exp = hdr + oracle.seal(key, struct.pack(">Q", seq0 + r), data[r * REC:r * REC + n].tobytes(),
                                    oracle.tls_ad(seq0 + r, n))
            assert wire[r * WREC:r * WREC + 5 + n + 16].tobytes() == exp, (seed, r)

        res = N.SgReadResult()

        def read(wlen_):
            out[:] = 0xEE
            N.check(lib.sg_read_records(dec._ptr, seq0, wire.ctypes.data, wlen_, out.ctypes.data, out.size,
                                        types.ctypes.data, flens.ctypes.data, nrec_max, C.byref(res)))
            return res.records, res.consumed, res.out_len, res.error

        assert read(wlen) == (nrec, wlen, total, N.SG_OK)
        assert np.array_equal(out[:total], data[:total])
        assert (types[:nrec] == 23).all()
        assert [int(x) for x in flens[:nrec]] == [min(REC, total - r * REC) for r in range(nrec)]
        if nrec == 0:
            return

        # one fault
        fault = int(rng.integers(0, 3))
        r = int(rng.integers(0, nrec))
        n = min(REC, total - r * REC)
        if fault == 0:  # a ciphertext or tag byte
            at = r * WREC + 5 + int(rng.integers(0, n + 16))
            wire[at] ^= 0x04
            got = read(wlen)
            assert got[0] == r and got[3] == N.SG_E_BAD_MAC and got[2] == r * REC, (seed, got)
            wire[at] ^= 0x04
        elif fault == 1:  # an unknown content type in record r's header
            wire[r * WREC] = 99
            got = read(wlen)
            assert got[0] == r and got[3] == N.SG_E_UNEXPECTED_MESSAGE and got[2] == r * REC, (seed, got)
            wire[r * WREC] = 23
        else:  # the stream cut inside its last record: the complete ones are delivered
            cut = (nrec - 1) * WREC + int(rng.integers(0, 5 + min(REC, total - (nrec - 1) * REC) + 16))
            got = read(cut)
            assert got == (nrec - 1, (nrec - 1) * WREC, (nrec - 1) * REC, N.SG_OK), (seed, got)
            r = nrec - 1
        assert np.array_equal(out[:r * REC], data[:r * REC])
        rest = out[r * REC:total]
        # nothing of the undelivered records: cleared (zero-copy) or never written (staged)
        assert np.isin(rest, (0, 0xEE)).all(), seed
    finally:
        for a in bufs:
            N.check(lib.sg_host_unregister(a.ctypes.data))
