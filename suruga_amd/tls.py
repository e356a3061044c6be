"""Record layer mirror of suruga's src/tls.rs (TlsWriter / TlsReader), with the
batched GPU path.

The classes keep the reference's names, framing and errors:

* ``TlsWriter.write_record`` (tls.rs:99-135): seq = be64(write_count), AD =
  seq || type || major || minor || be16(len), header type|major|minor|be16,
  oversize encrypted fragment -> panic (here AssertionError).
* ``TlsWriter.write_data`` (tls.rs:137-147): 2^14-byte fragments.  With the GPU
  encryptor the whole call is ONE ``sg_write_records`` (records sealed in
  batches with pinned double-buffered staging); with any other Encryptor
  (e.g. the null cipher of src/test.rs) it is the reference's per-record loop.
* ``TlsReader.read_record`` (tls.rs:217-281): unknown type ->
  UnexpectedMessage, length > 2^14+2048 -> RecordOverflow, short ->
  BadRecordMac, then ``Decryptor.decrypt``.  ``read_message`` (tls.rs:294-348)
  for ChangeCipherSpec / Alert / ApplicationData records (handshake messages
  are returned unparsed: the handshake is out of scope).
* ``RecordStreamReader``: the batched read path over a byte stream, one
  ``sg_read_records`` per receive buffer.
"""
from __future__ import annotations

import ctypes as C
import enum
import struct
from dataclasses import dataclass

from . import _native as N
from .cipher import ChaCha20Poly1305Decryptor, ChaCha20Poly1305Encryptor, TlsError, TlsErrorKind

TLS_VERSION = (3, 3)                       # tls.rs:17
RECORD_MAX_LEN = 1 << 14                   # tls.rs:32
ENC_RECORD_MAX_LEN = (1 << 14) + 2048      # tls.rs:35


# alert.rs:5-44: the AlertLevel / AlertDescription values FromPrimitive accepts
ALERT_LEVELS = frozenset({1, 2})
ALERT_DESCRIPTIONS = frozenset({0, 10, 20, 21, 22, 30, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 60, 70, 71,
                                80, 90, 100, 110})


class ContentType(enum.IntEnum):
    """tls.rs:19-29"""

    ChangeCipherSpecTy = 20
    AlertTy = 21
    HandshakeTy = 22
    ApplicationDataTy = 23


@dataclass
class Record:
    """tls.rs:38-61 (``Record::new`` panics when the fragment exceeds 2^14)."""

    content_type: ContentType
    ver_major: int
    ver_minor: int
    fragment: bytes

    def __post_init__(self):
        if len(self.fragment) > RECORD_MAX_LEN:
            raise AssertionError(f"record too long: {len(self.fragment)} > 2^14")


_ERR_KIND = {
    N.SG_E_BAD_MAC: (TlsErrorKind.BadRecordMac, "wrong mac"),
    N.SG_E_SHORT: (TlsErrorKind.BadRecordMac, "encrypted message too short"),
    N.SG_E_UNEXPECTED_MESSAGE: (TlsErrorKind.UnexpectedMessage, "unexpected ContentType"),
    N.SG_E_RECORD_OVERFLOW: (TlsErrorKind.RecordOverflow, "TLSEncryptedText too long"),
}


def _sink(writer):
    for name in ("sendall", "write"):
        f = getattr(writer, name, None)
        if f is not None:
            return f
    raise TypeError("writer needs write() or sendall()")


class TlsWriter:
    """tls.rs:63-171"""

    def __init__(self, writer):
        self.writer = writer
        self._write = _sink(writer)
        self.encryptor = None
        self.write_count = 0

    def set_encryptor(self, encryptor) -> None:  # tls.rs:91-97
        assert self.encryptor is None
        self.encryptor = encryptor
        self.write_count = 0

    def write_record(self, record: Record) -> None:  # tls.rs:99-135
        if self.encryptor is None:
            fragment = record.fragment
        else:
            seq = struct.pack(">Q", self.write_count)
            ad = seq + bytes([record.content_type, record.ver_major, record.ver_minor]) + \
                struct.pack(">H", len(record.fragment))
            fragment = self.encryptor.encrypt(seq, record.fragment, ad)
        if len(fragment) > ENC_RECORD_MAX_LEN:
            raise AssertionError(f"record too long: {len(fragment)} > 2^14 + 2048")
        self._write(bytes([record.content_type, record.ver_major, record.ver_minor]) +
                    struct.pack(">H", len(fragment)) + fragment)
        self.write_count += 1

    def write_data(self, ty: ContentType, data: bytes) -> None:  # tls.rs:137-147
        major, minor = TLS_VERSION
        if isinstance(self.encryptor, ChaCha20Poly1305Encryptor) and len(data) > 0:
            wire = (C.c_uint8 * N.load().sg_wire_bound(len(data)))()
            wl = C.c_size_t(0)
            src = (C.c_uint8 * len(data)).from_buffer_copy(data) if not isinstance(data, bytearray) else \
                (C.c_uint8 * len(data)).from_buffer(data)
            nrec = N.check(N.load().sg_write_records(self.encryptor._ptr, self.write_count, int(ty), major, minor,
                                                     src, len(data), wire, len(wire), C.byref(wl)))
            self._write(bytes(memoryview(wire)[:wl.value]))
            self.write_count += nrec
            return
        for off in range(0, len(data), RECORD_MAX_LEN):
            self.write_record(Record(ty, major, minor, bytes(data[off:off + RECORD_MAX_LEN])))

    def write_alert(self, level: int, description: int) -> None:  # tls.rs:154-158
        self.write_data(ContentType.AlertTy, bytes([level, description]))

    def write_change_cipher_spec(self) -> None:  # tls.rs:161-163
        self.write_data(ContentType.ChangeCipherSpecTy, b"\x01")

    def write_application_data(self, data: bytes) -> None:  # tls.rs:165-170
        if self.encryptor is None:
            raise AssertionError("attempted to write ApplicationData before handshake")
        self.write_data(ContentType.ApplicationDataTy, data)


class _Source:
    """read_exact over a file-like or socket (util.rs:97-102 ReadExt)."""

    def __init__(self, reader):
        self.reader = reader
        self.buf = bytearray()

    def _more(self, n: int) -> bytes:
        f = getattr(self.reader, "recv", None) or self.reader.read
        return f(n)

    def read_exact(self, n: int) -> bytes:
        while len(self.buf) < n:
            chunk = self._more(max(n - len(self.buf), 1 << 16))
            if not chunk:
                raise TlsError(TlsErrorKind.IoFailure, "io error: unexpected EOF")
            self.buf += chunk
        out = bytes(self.buf[:n])
        del self.buf[:n]
        return out


class TlsReader:
    """tls.rs:173-380"""

    def __init__(self, reader):
        self.src = _Source(reader)
        self.decryptor = None
        self.read_count = 0

    def set_decryptor(self, decryptor) -> None:  # tls.rs:206-212
        assert self.decryptor is None
        self.decryptor = decryptor
        self.read_count = 0

    def read_record(self) -> Record:  # tls.rs:217-281
        ty = self.src.read_exact(1)[0]
        try:
            content_type = ContentType(ty)
        except ValueError:
            raise TlsError(TlsErrorKind.UnexpectedMessage, f"unexpected ContentType: {ty}") from None
        major, minor = self.src.read_exact(1)[0], self.src.read_exact(1)[0]
        length = struct.unpack(">H", self.src.read_exact(2))[0]
        if length > ENC_RECORD_MAX_LEN:
            raise TlsError(TlsErrorKind.RecordOverflow, f"TLSEncryptedText too long: {length}")
        fragment = self.src.read_exact(length)
        if self.decryptor is None:
            if len(fragment) > RECORD_MAX_LEN:
                raise TlsError(TlsErrorKind.RecordOverflow, f"decrypted record too long: {len(fragment)}")
            record = Record(content_type, major, minor, fragment)
        else:
            seq = struct.pack(">Q", self.read_count)
            mac_len = self.decryptor.mac_len()
            if len(fragment) < mac_len:
                raise TlsError(TlsErrorKind.BadRecordMac, f"encrypted message too short: {len(fragment)}")
            ad = seq + bytes([ty, major, minor]) + struct.pack(">H", len(fragment) - mac_len)
            data = self.decryptor.decrypt(seq, fragment, ad)
            if len(data) > RECORD_MAX_LEN:
                raise AssertionError(f"decrypted record too long: {len(data)}")  # tls.rs:269-272 panics
            record = Record(content_type, major, minor, data)
        self.read_count += 1
        return record

    def read_message(self):  # tls.rs:294-348 (handshake messages returned unparsed)
        while True:
            record = self.read_record()
            ct = record.content_type
            if ct is ContentType.ChangeCipherSpecTy:
                if record.fragment != b"\x01":
                    raise TlsError(TlsErrorKind.UnexpectedMessage, "invalid ChangeCipherSpec arrived")
                return ("ChangeCipherSpec", None)
            if ct is ContentType.AlertTy:
                if len(record.fragment) == 0:
                    raise TlsError(TlsErrorKind.UnexpectedMessage, "zero-length Alert record arrived")
                if len(record.fragment) < 2:
                    raise TlsError(TlsErrorKind.UnexpectedMessage, "awkward Alert record arrived")
                if record.fragment[0] not in ALERT_LEVELS or record.fragment[1] not in ALERT_DESCRIPTIONS:
                    raise TlsError(TlsErrorKind.UnexpectedMessage, f"unknown alert: {list(record.fragment)}")
                return ("Alert", (record.fragment[0], record.fragment[1]))
            if ct is ContentType.HandshakeTy:
                if len(record.fragment) == 0:
                    raise TlsError(TlsErrorKind.UnexpectedMessage, "zero-length Handshake arrived")
                return ("Handshake", record.fragment)
            return ("ApplicationData", record.fragment)

    def read_application_data(self) -> bytes:  # tls.rs:350-364
        if self.decryptor is None:
            raise AssertionError("ApplicationData called before handshake")
        kind, payload = self.read_message()
        if kind != "ApplicationData":
            raise NotImplementedError(kind)  # the reference: unimplemented!()
        return payload


class RecordStreamReader:
    """Batched TlsReader over a byte stream: every complete record in the
    receive buffer is opened by one ``sg_read_records`` call."""

    def __init__(self, reader, decryptor: ChaCha20Poly1305Decryptor, max_records: int = 1 << 16):
        self.reader = reader
        self.dec = decryptor
        self.read_count = 0
        self.buf = bytearray()
        self.max_records = max_records
        self.types = (C.c_uint8 * max_records)()
        self.lens = (C.c_uint32 * max_records)()

    def feed(self, data: bytes) -> None:
        self.buf += data

    def drain(self):
        """Open every complete buffered record -> list of (content_type, plaintext)."""
        if not self.buf:
            return []
        lib = N.load()
        src = (C.c_uint8 * len(self.buf)).from_buffer(self.buf)
        out = (C.c_uint8 * max(len(self.buf), 1))()
        res = N.SgReadResult()
        N.check(lib.sg_read_records(self.dec._ptr, self.read_count, src, len(self.buf), out, len(out),
                                    self.types, self.lens, self.max_records, C.byref(res)))
        del src
        msgs, pos = [], 0
        for i in range(res.records):
            n = self.lens[i]
            msgs.append((ContentType(self.types[i]), bytes(memoryview(out)[pos:pos + n])))
            pos += n
        del self.buf[:res.consumed]
        self.read_count += res.records
        if res.error != N.SG_OK:
            kind, desc = _ERR_KIND.get(res.error, (TlsErrorKind.InternalError, f"status {res.error}"))
            raise TlsError(kind, desc)
        return msgs
