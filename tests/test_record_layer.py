"""Record layer (src/tls.rs, src/test.rs): the reference's own record tests
with the null cipher (CPU), and the batched GPU write/read paths checked
against the oracle-backed per-record path (GPU)."""
from __future__ import annotations

import io
import struct

import pytest

from suruga_amd.cipher import Decryptor, Encryptor, TlsError, TlsErrorKind
from suruga_amd.tls import (ENC_RECORD_MAX_LEN, RECORD_MAX_LEN, ContentType, Record, RecordStreamReader,
                            TlsReader, TlsWriter)


class NullEncryptor(Encryptor):  # src/test.rs:13-20
    def encrypt(self, nonce, plain, ad):
        return bytes(plain)


class NullDecryptor(Decryptor):  # src/test.rs:22-27
    def decrypt(self, nonce, encrypted, ad):
        return bytes(encrypted)

    def mac_len(self):
        return 0


class OracleEncryptor(Encryptor):
    """The CPU restatement behind the Encryptor trait (test infrastructure)."""

    def __init__(self, oracle, key):
        self.o, self.key = oracle, key

    def encrypt(self, nonce, plain, ad):
        return self.o.seal(self.key, nonce, plain, ad)


class OracleDecryptor(Decryptor):
    def __init__(self, oracle, key):
        self.o, self.key = oracle, key

    def decrypt(self, nonce, encrypted, ad):
        rc, pt = self.o.open(self.key, nonce, encrypted, ad)
        if rc == 2:
            raise TlsError(TlsErrorKind.BadRecordMac, "message too short")
        if rc != 0:
            raise TlsError(TlsErrorKind.BadRecordMac, "wrong mac")
        return pt

    def mac_len(self):
        return 16


def null_tls(reader, writer):  # src/test.rs:29-39
    r, w = TlsReader(reader), TlsWriter(writer)
    r.set_decryptor(NullDecryptor())
    w.set_encryptor(NullEncryptor())
    return r, w


# ---- src/test.rs ------------------------------------------------------------
def test_change_cipher_spec_message():
    out = io.BytesIO()
    _, w = null_tls(io.BytesIO(), out)
    w.write_change_cipher_spec()
    data = out.getvalue()
    assert len(data) == 1 + 2 + 2 + 1 and data[5] == 1
    r, _ = null_tls(io.BytesIO(data), io.BytesIO())
    assert r.read_message() == ("ChangeCipherSpec", None)


def test_application_message():
    app = b"\x01" * (RECORD_MAX_LEN + 200)
    out = io.BytesIO()
    _, w = null_tls(io.BytesIO(), out)
    w.write_application_data(app)
    r, _ = null_tls(io.BytesIO(out.getvalue()), io.BytesIO())
    assert r.read_message() == ("ApplicationData", b"\x01" * RECORD_MAX_LEN)
    assert r.read_message() == ("ApplicationData", b"\x01" * 200)


# ---- src/tls.rs:382-476 ----------------------------------------------------------
def test_reader():
    r = TlsReader(io.BytesIO(bytes([0x14, 0x03, 0x03, 0x00, 0x01, 0x01])))
    rec = r.read_record()
    assert (rec.content_type, rec.ver_major, rec.ver_minor, rec.fragment) == \
        (ContentType.ChangeCipherSpecTy, 3, 3, b"\x01")
    with pytest.raises(TlsError) as e:
        r.read_record()
    assert e.value.kind is TlsErrorKind.IoFailure


def test_reader_unknown():
    r = TlsReader(io.BytesIO(bytes([0x18, 0x03, 0x03, 0x00, 0x03, 0x01, 0x00, 0x20])))
    with pytest.raises(TlsError) as e:
        r.read_record()
    assert e.value.kind is TlsErrorKind.UnexpectedMessage


def test_reader_too_long():
    n = RECORD_MAX_LEN + 1
    r = TlsReader(io.BytesIO(bytes([0x17, 0x03, 0x03, n >> 8, n & 0xFF]) + b"\xff" * n))
    with pytest.raises(TlsError) as e:
        r.read_record()
    assert e.value.kind is TlsErrorKind.RecordOverflow


def test_reader_zero_length():
    for ct in (20, 21, 22):
        r = TlsReader(io.BytesIO(bytes([ct, 0x03, 0x03, 0x00, 0x00])))
        with pytest.raises(TlsError) as e:
            r.read_message()
        assert e.value.kind is TlsErrorKind.UnexpectedMessage


def test_alert_messages():
    out = io.BytesIO()
    w = TlsWriter(out)
    w.write_alert(2, 20)   # fatal bad_record_mac
    w.write_alert(2, 99)   # not an AlertDescription (alert.rs:13-44)
    r = TlsReader(io.BytesIO(out.getvalue()))
    assert r.read_message() == ("Alert", (2, 20))
    with pytest.raises(TlsError) as e:
        r.read_message()
    assert e.value.kind is TlsErrorKind.UnexpectedMessage


def test_writer_too_long():
    class Enc(Encryptor):
        def encrypt(self, nonce, fragment, ad):
            return bytes(ENC_RECORD_MAX_LEN + 1)

    w = TlsWriter(io.BytesIO())
    w.set_encryptor(Enc())
    with pytest.raises(AssertionError):
        w.write_record(Record(ContentType.ApplicationDataTy, 3, 3, b"\x01"))


def test_record_framing_with_oracle_cipher(oracle):
    """write_record framing + AD/nonce rules through the reference algorithm."""
    key = bytes(range(32))
    out = io.BytesIO()
    w = TlsWriter(out)
    w.set_encryptor(OracleEncryptor(oracle, key))
    w.write_application_data(b"A" * 16)
    wire = out.getvalue()
    assert wire[:5] == bytes([23, 3, 3, 0, 32])
    # the survey's sample vector: seq 0, type 23, ver 3.3
    assert wire[5:].hex() == "59f90370eca7e79052201d20ee020f66fbc2d9037460b094b3443d3ec89ef135"
    r = TlsReader(io.BytesIO(wire))
    r.set_decryptor(OracleDecryptor(oracle, key))
    assert r.read_application_data() == b"A" * 16


# ---- GPU: batched record layer -------------------------------------------------
@pytest.mark.gpu
def test_gpu_batched_writer_matches_reference_reader(gpu, oracle):
    from suruga_amd import ChaCha20Poly1305

    key = bytes(range(32))
    data = oracle.fill_record(0x53555255, 1, 5 * RECORD_MAX_LEN + 1234)
    out = io.BytesIO()
    w = TlsWriter(out)
    w.set_encryptor(ChaCha20Poly1305().new_encryptor(key))
    w.write_change_cipher_spec()          # 1 record (seq 0), batched path
    w.write_application_data(data)        # 6 records (seq 1..6)
    w.write_application_data(b"tail")     # seq 7
    assert w.write_count == 8
    r = TlsReader(io.BytesIO(out.getvalue()))
    r.set_decryptor(OracleDecryptor(oracle, key))
    assert r.read_message() == ("ChangeCipherSpec", None)
    got = b"".join(r.read_application_data() for _ in range(6))
    assert got == data and r.read_application_data() == b"tail"


@pytest.mark.gpu
def test_gpu_stream_reader_matches_reference_writer(gpu, oracle):
    from suruga_amd import ChaCha20Poly1305

    key = bytes(range(1, 33))
    out = io.BytesIO()
    w = TlsWriter(out)
    w.set_encryptor(OracleEncryptor(oracle, key))
    pieces = [oracle.fill_record(7, j, n) for j, n in enumerate([0, 1, 100, RECORD_MAX_LEN, 3000, 17])]
    for p in pieces:
        w.write_application_data(p)  # write of 0 bytes emits no record
    wire = out.getvalue()
    rd = RecordStreamReader(None, ChaCha20Poly1305().new_decryptor(key))
    # feed in uneven slices: partial records stay buffered
    got = []
    for i in range(0, len(wire), 7777):
        rd.feed(wire[i:i + 7777])
        got += rd.drain()
    assert [p for _, p in got] == [p for p in pieces if p]
    assert all(t is ContentType.ApplicationDataTy for t, _ in got)
    assert rd.read_count == 5 and not rd.buf


@pytest.mark.gpu
def test_gpu_stream_reader_errors(gpu, oracle):
    from suruga_amd import ChaCha20Poly1305

    key = bytes(32)
    out = io.BytesIO()
    w = TlsWriter(out)
    w.set_encryptor(OracleEncryptor(oracle, key))
    for j in range(4):
        w.write_application_data(bytes([j]) * 500)
    wire = bytearray(out.getvalue())
    rec = 5 + 516
    wire[2 * rec + 10] ^= 0x40  # corrupt record 2
    rd = RecordStreamReader(None, ChaCha20Poly1305().new_decryptor(key))
    rd.feed(bytes(wire))
    with pytest.raises(TlsError) as e:
        rd.drain()
    assert e.value.kind is TlsErrorKind.BadRecordMac
    assert rd.read_count == 2 and len(rd.buf) == 2 * rec  # records 0, 1 delivered
    # unknown content type after a good record
    rd2 = RecordStreamReader(None, ChaCha20Poly1305().new_decryptor(key))
    rd2.feed(bytes(out.getvalue()[:rec]) + bytes([0x18, 3, 3, 0, 3, 1, 2, 3]))
    with pytest.raises(TlsError) as e:
        rd2.drain()
    assert e.value.kind is TlsErrorKind.UnexpectedMessage and rd2.read_count == 1
    # oversize header
    rd3 = RecordStreamReader(None, ChaCha20Poly1305().new_decryptor(key))
    n = ENC_RECORD_MAX_LEN + 1
    rd3.feed(bytes([23, 3, 3, n >> 8, n & 0xFF]))
    with pytest.raises(TlsError) as e:
        rd3.drain()
    assert e.value.kind is TlsErrorKind.RecordOverflow


@pytest.mark.gpu
def test_gpu_per_record_reader(gpu, oracle):
    """The trait-object path: TlsReader.read_record -> Decryptor.decrypt on the GPU."""
    from suruga_amd import ChaCha20Poly1305

    key = bytes(range(32))
    out = io.BytesIO()
    w = TlsWriter(out)
    w.set_encryptor(OracleEncryptor(oracle, key))
    w.write_application_data(b"x" * 40000)
    r = TlsReader(io.BytesIO(out.getvalue()))
    r.set_decryptor(ChaCha20Poly1305().new_decryptor(key))
    assert b"".join(r.read_application_data() for _ in range(3)) == b"x" * 40000
    tampered = bytearray(out.getvalue())
    tampered[-1] ^= 1
    r = TlsReader(io.BytesIO(bytes(tampered)))
    r.set_decryptor(ChaCha20Poly1305().new_decryptor(key))
    r.read_record(), r.read_record()
    with pytest.raises(TlsError) as e:
        r.read_record()
    assert e.value.kind is TlsErrorKind.BadRecordMac
    assert struct.pack(">Q", r.read_count) == bytes(7) + b"\x02"


def test_parse_records_header_checks_cpu():
    """sg_parse_records (host only, no GPU call): the header checks of
    sg_read_records in TlsReader::read_record's order (tls.rs:218-238,
    258-262, 269-272) on the reference's own reader cases, called through the
    C ABI on the CPU.  (The same parser runs under ASan/UBSan over a corpus in
    tests/test_sanitizers.py.)"""
    import ctypes as C

    from suruga_amd import _native as N

    lib = N.load()

    def parse(wire: bytes, max_records: int = 64):
        recs = (N.SgWireRecord * max_records)()
        count, err = C.c_size_t(0), C.c_int32(0)
        buf = (C.c_uint8 * max(len(wire), 1)).from_buffer_copy(wire or b"\0")
        N.check(lib.sg_parse_records(buf, len(wire), max_records, recs, C.byref(count), C.byref(err)))
        return [(r.offset, r.frag_len, r.type, r.ver_major, r.ver_minor) for r in recs[:count.value]], err.value

    def rec(t, n, fill=0xAB):
        return bytes([t, 3, 3, n >> 8, n & 0xFF]) + bytes([fill]) * n

    two = rec(23, 16) + rec(22, 300)
    assert parse(two) == ([(5, 16, 23, 3, 3), (26, 300, 22, 3, 3)], N.SG_OK)
    assert parse(two, 1) == ([(5, 16, 23, 3, 3)], N.SG_OK)             # max_records
    assert parse(two[:-1]) == ([(5, 16, 23, 3, 3)], N.SG_OK)           # incomplete: wait for bytes
    assert parse(rec(23, 16) + bytes([0x18, 3, 3, 0, 3, 1, 0, 0x20])) == \
        ([(5, 16, 23, 3, 3)], N.SG_E_UNEXPECTED_MESSAGE)               # tls.rs test_reader_unknown
    big = ENC_RECORD_MAX_LEN + 1
    assert parse(bytes([0x17, 3, 3, big >> 8, big & 0xFF]))[1] == N.SG_E_RECORD_OVERFLOW  # header alone suffices
    assert parse(rec(23, 15))[1] == N.SG_E_SHORT                        # < mac_len (tls.rs:258-262)
    assert parse(rec(23, RECORD_MAX_LEN + 17))[1] == N.SG_E_RECORD_OVERFLOW  # decrypted > 2^14 (:269-272)
    assert parse(rec(23, RECORD_MAX_LEN + 16)) == ([(5, RECORD_MAX_LEN + 16, 23, 3, 3)], N.SG_OK)
    assert parse(b"") == ([], N.SG_OK)


@pytest.mark.gpu
def test_gpu_zero_copy_record_path(gpu, oracle):
    """sg_host_register'ed caller buffers: sg_write_records
    DMAs the plaintext straight from `data` and the sealed fragments straight
    into their wire slots, sg_read_records the fragments straight from the wire
    and the plaintext straight into `out`.  The wire equals the staged path's
    (and the oracle's) byte for byte, the read-back equals the input; with a
    corrupted record the records before it are delivered and `out` holds
    nothing of it or of any record after it."""
    import ctypes as C

    import numpy as np

    from suruga_amd import ChaCha20Poly1305
    from suruga_amd import _native as N

    lib = N.load()
    key = bytes(range(7, 39))
    total = 600 * RECORD_MAX_LEN + 4321  # three chunks of 256 records and a ragged tail
    data = np.frombuffer(oracle.fill_record(0x5A, 3, total), dtype=np.uint8).copy()
    enc, dec = ChaCha20Poly1305().new_encryptor(key), ChaCha20Poly1305().new_decryptor(key)
    cap = lib.sg_wire_bound(total)
    staged = np.zeros(cap, dtype=np.uint8)
    wl = C.c_size_t(0)
    nrec = N.check(lib.sg_write_records(enc._ptr, 5, 23, 3, 3, data.ctypes.data, total, staged.ctypes.data, cap,
                                        C.byref(wl)))
    wlen = wl.value
    wire = np.zeros(cap, dtype=np.uint8)
    out = np.full(total, 0xEE, dtype=np.uint8)
    for a in (data, wire, out):
        N.check(lib.sg_host_register(a.ctypes.data, a.nbytes))
    try:
        wl2 = C.c_size_t(0)
        assert N.check(lib.sg_write_records(enc._ptr, 5, 23, 3, 3, data.ctypes.data, total, wire.ctypes.data, cap,
                                            C.byref(wl2))) == nrec
        assert wl2.value == wlen and np.array_equal(wire[:wlen], staged[:wlen])
        # spot-check against the oracle: first, a middle and the last record
        rec = 5 + RECORD_MAX_LEN + 16
        for r in (0, 300, nrec - 1):
            n = min(RECORD_MAX_LEN, total - r * RECORD_MAX_LEN)
            pt = data[r * RECORD_MAX_LEN:r * RECORD_MAX_LEN + n].tobytes()
            exp = oracle.seal(key, struct.pack(">Q", 5 + r), pt, oracle.tls_ad(5 + r, n))
            assert wire[r * rec + 5:r * rec + 5 + n + 16].tobytes() == exp, r
        res = N.SgReadResult()
        N.check(lib.sg_read_records(dec._ptr, 5, wire.ctypes.data, wlen, out.ctypes.data, total, None, None, 1 << 20,
                                    C.byref(res)))
        assert (res.records, res.consumed, res.out_len, res.error) == (nrec, wlen, total, N.SG_OK)
        assert np.array_equal(out, data)
        # a corrupted record in the second chunk: records before it delivered, nothing after
        bad = 300
        wire[bad * rec + 5 + 1000] ^= 0x10
        out[:] = 0xEE
        N.check(lib.sg_read_records(dec._ptr, 5, wire.ctypes.data, wlen, out.ctypes.data, total, None, None, 1 << 20,
                                    C.byref(res)))
        assert (res.records, res.out_len, res.error) == (bad, bad * RECORD_MAX_LEN, N.SG_E_BAD_MAC)
        assert np.array_equal(out[:bad * RECORD_MAX_LEN], data[:bad * RECORD_MAX_LEN])
        leaked = [r for r in range(bad, nrec)
                  if r * RECORD_MAX_LEN < total and
                  np.array_equal(out[r * RECORD_MAX_LEN:min(total, (r + 1) * RECORD_MAX_LEN)],
                                 data[r * RECORD_MAX_LEN:min(total, (r + 1) * RECORD_MAX_LEN)])]
        assert leaked == [], f"plaintext of undelivered records {leaked[:5]} in out"
    finally:
        for a in (data, wire, out):
            N.check(lib.sg_host_unregister(a.ctypes.data))


@pytest.mark.gpu
def test_gpu_zero_copy_odd_length_records(gpu, oracle):
    """Registered-buffer read of 600 equal records of an odd plaintext length
    (1001 B: the open batch writes the plaintext back to back at a packed,
    unaligned 1001-byte stride, i.e. the byte-granular output and scrub paths,
    advisor r5).  `out` equals the staged path's and the input; with a
    corrupted record in the first chunk and, separately, one in the second,
    the records before it are delivered and no byte of `out` from it on holds
    plaintext: cleared by a zero-copy chunk, untouched by a staged one
    (tls.rs:268: nothing of a failed record or of any record after it).  (The
    direct pipeline stages chunks of records other than full 16 KiB ones;
    SG_RECORD_SDMA=1 takes them zero-copy.)"""
    import ctypes as C

    import numpy as np

    from suruga_amd import ChaCha20Poly1305
    from suruga_amd import _native as N

    lib = N.load()
    key = bytes(range(11, 43))
    n, count, seq0 = 1001, 600, 9
    data = np.frombuffer(oracle.fill_record(0x3C, 5, n * count), dtype=np.uint8).copy()
    pitch = 5 + n + 16
    wire = np.zeros(pitch * count, dtype=np.uint8)
    for r in range(count):
        ct = oracle.seal(key, struct.pack(">Q", seq0 + r), data[r * n:(r + 1) * n].tobytes(), oracle.tls_ad(seq0 + r, n))
        wire[r * pitch:(r + 1) * pitch] = np.frombuffer(bytes([23, 3, 3]) + struct.pack(">H", n + 16) + ct,
                                                       dtype=np.uint8)
    dec = ChaCha20Poly1305().new_decryptor(key)
    res = N.SgReadResult()

    def read(w, out):
        N.check(lib.sg_read_records(dec._ptr, seq0, w.ctypes.data, w.size, out.ctypes.data, out.size, None, None,
                                    1 << 20, C.byref(res)))
        return res.records, res.out_len, res.error

    staged = np.full(n * count, 0xEE, dtype=np.uint8)
    assert read(wire.copy(), staged) == (count, n * count, N.SG_OK)
    assert np.array_equal(staged, data)
    out = np.full(n * count, 0xEE, dtype=np.uint8)
    for a in (wire, out):
        N.check(lib.sg_host_register(a.ctypes.data, a.nbytes))
    try:
        assert read(wire, out) == (count, n * count, N.SG_OK)
        assert np.array_equal(out, staged)
        for bad, pos in ((100, 7), (300, n - 1)):  # first chunk; second chunk, the last byte
            w = wire[bad * pitch + 5 + pos]
            wire[bad * pitch + 5 + pos] ^= 0x01
            out[:] = 0xEE
            assert read(wire, out) == (bad, bad * n, N.SG_E_BAD_MAC)
            assert np.array_equal(out[:bad * n], data[:bad * n])
            # nothing of the failed record or of any record after it: cleared
            # (a zero-copy chunk) or never written (a staged one)
            rest = out[bad * n:]
            assert np.isin(rest, (0, 0xEE)).all(), f"bytes of undelivered records left in out (bad record {bad})"
            wire[bad * pitch + 5 + pos] = w
    finally:
        for a in (wire, out):
            N.check(lib.sg_host_unregister(a.ctypes.data))


@pytest.mark.gpu
def test_gpu_zero_copy_edges(gpu, oracle):
    """Registered-buffer edges: a write shorter than one record, and a read
    whose second chunk mixes content types (equal, back-to-back fragments: the
    wire image is still copied in whole and taken apart in HBM, but nonce and
    AD go explicit, tls.rs:250-265).  Both equal the staged path byte for
    byte; the types come back per record."""
    import ctypes as C

    import numpy as np

    from suruga_amd import ChaCha20Poly1305
    from suruga_amd import _native as N

    lib = N.load()
    key = bytes(range(3, 35))
    enc, dec = ChaCha20Poly1305().new_encryptor(key), ChaCha20Poly1305().new_decryptor(key)

    # (a) 100 bytes: one short record, zero-copy against staged
    small = np.frombuffer(oracle.fill_record(0x11, 1, 100), dtype=np.uint8).copy()
    cap = lib.sg_wire_bound(100)
    staged, wire = np.zeros(cap, dtype=np.uint8), np.zeros(cap, dtype=np.uint8)
    wl = C.c_size_t(0)
    assert N.check(lib.sg_write_records(enc._ptr, 9, 23, 3, 3, small.ctypes.data, 100, staged.ctypes.data, cap,
                                        C.byref(wl))) == 1
    for a in (small, wire):
        N.check(lib.sg_host_register(a.ctypes.data, a.nbytes))
    try:
        wl2 = C.c_size_t(0)
        assert N.check(lib.sg_write_records(enc._ptr, 9, 23, 3, 3, small.ctypes.data, 100, wire.ctypes.data, cap,
                                            C.byref(wl2))) == 1
        assert wl2.value == wl.value == 5 + 100 + 16 and np.array_equal(wire, staged)
        assert wire[5:121].tobytes() == oracle.seal(key, struct.pack(">Q", 9), small.tobytes(), oracle.tls_ad(9, 100))
    finally:
        for a in (small, wire):
            N.check(lib.sg_host_unregister(a.ctypes.data))

    # (b) 300 application-data records then 10 handshake records, one stream
    n1, n2 = 300, 10
    d1 = np.frombuffer(oracle.fill_record(0x21, 2, n1 * RECORD_MAX_LEN), dtype=np.uint8).copy()
    d2 = np.frombuffer(oracle.fill_record(0x22, 3, n2 * RECORD_MAX_LEN), dtype=np.uint8).copy()
    c1, c2 = lib.sg_wire_bound(d1.size), lib.sg_wire_bound(d2.size)
    w1, w2 = np.zeros(c1, dtype=np.uint8), np.zeros(c2, dtype=np.uint8)
    l1, l2 = C.c_size_t(0), C.c_size_t(0)
    N.check(lib.sg_write_records(enc._ptr, 0, 23, 3, 3, d1.ctypes.data, d1.size, w1.ctypes.data, c1, C.byref(l1)))
    N.check(lib.sg_write_records(enc._ptr, n1, 22, 3, 3, d2.ctypes.data, d2.size, w2.ctypes.data, c2, C.byref(l2)))
    stream = np.concatenate([w1[:l1.value], w2[:l2.value]])
    expect = np.concatenate([d1, d2])
    results = {}
    for registered in (False, True):
        out = np.full(expect.size, 0xEE, dtype=np.uint8)
        types = np.zeros(n1 + n2, dtype=np.uint8)
        if registered:
            for a in (stream, out):
                N.check(lib.sg_host_register(a.ctypes.data, a.nbytes))
        try:
            res = N.SgReadResult()
            N.check(lib.sg_read_records(dec._ptr, 0, stream.ctypes.data, stream.size, out.ctypes.data, out.size,
                                        types.ctypes.data, None, 1 << 20, C.byref(res)))
        finally:
            if registered:
                for a in (stream, out):
                    N.check(lib.sg_host_unregister(a.ctypes.data))
        assert (res.records, res.consumed, res.out_len, res.error) == (n1 + n2, stream.size, expect.size, N.SG_OK)
        assert np.array_equal(out, expect), registered
        assert (types[:n1] == 23).all() and (types[n1:] == 22).all()
        results[registered] = out
    assert np.array_equal(results[False], results[True])


def test_frame_record_index_math():
    """sg_frame_kernel finds the wire record of destination byte b as
    r = (b * rdiv) >> 40, rdiv = ceil(2^40 / pitch) (sg_kernels.hip), for
    images below 2^24 bytes (launch_frame's guard).  Exact for every pitch a
    wire record can have (5-byte header + 16..2^14+16 byte fragment, and any
    pitch below 2^16): the error term b (rdiv pitch - 2^40) / 2^40 stays below
    1 / pitch; and brute force over every b for the record layer's pitch."""
    import numpy as np

    limit = 1 << 24
    for pitch in range(21, 1 << 16):
        rdiv = -(-(1 << 40) // pitch)
        assert (limit - 1) * (rdiv * pitch - (1 << 40)) < (1 << 40), pitch
    pitch = 5 + RECORD_MAX_LEN + 16
    rdiv = np.uint64(-(-(1 << 40) // pitch))
    b = np.arange(limit, dtype=np.uint64)
    assert np.array_equal((b * rdiv) >> np.uint64(40), b // np.uint64(pitch))
