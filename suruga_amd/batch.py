"""Device-resident batch seal/open (``sg_seal_batch`` / ``sg_open_batch``).

This is the batched form of the record layer's hot loop: ``TlsWriter``'s
``write_data`` chunk loop (tls.rs:137-147 -> write_record tls.rs:99-135) and
``TlsReader::read_record`` (tls.rs:217-281).  In TLS mode the nonce
(``u64_be_array(seq)``, tls.rs:103) and the 13-byte additional data
(tls.rs:105-112 / 250-265) are built on the device from the sequence number,
so a call carries only record bytes, lengths and keys.

Tensors are torch tensors on the GPU (PyTorch is used here only for device
memory and streams); all arithmetic runs in the gfx950 kernels.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

from . import _native as N

APPLICATION_DATA = 23  # ContentType::ApplicationDataTy (tls.rs:26)
TLS_VERSION = (3, 3)   # tls.rs:17


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return int(t.data_ptr())


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        import torch

        return int(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


@dataclass
class Batch:
    """Arguments of one ``sg_*_batch`` call (see include/suruga_gpu.h)."""

    count: int
    keys: object                      # uint8 [num_keys, 32], device
    inp: object                       # uint8 device buffer
    out: object                       # uint8 device buffer
    uniform_len: int = 0
    lens: object = None               # uint32 [count] device, or None
    max_len: int = 0
    in_stride: int = 0
    out_stride: int = 0
    in_off: object = None             # uint64 [count] device, or None
    out_off: object = None
    key_index: object = None          # uint32 [count] device, or None
    tls: bool = True
    seq0: int = 0
    seq: object = None                # uint64 [count] device, or None
    content_type: int = APPLICATION_DATA
    version: tuple = TLS_VERSION
    nonces: object = None             # explicit mode: uint8 [count, 8]
    ads: object = None                # explicit mode: uint8 [count, ad_stride]
    ad_len: int = 0
    ad_stride: int = 0
    status: object = None             # uint8 [count] device (open)
    workspace: object = None          # uint8 [>= workspace_size(count)] device, or None
    stream: object = None             # torch.cuda.Stream / raw handle (0: the NULL stream) / None = current stream
    keep_failed: bool = False         # open: keep the unauthenticated plaintext of BAD_MAC records

    def to_c(self) -> N.SgBatch:
        b = N.SgBatch()
        b.count = self.count
        b.flags = (N.SG_BATCH_TLS if self.tls else 0) | (N.SG_BATCH_KEEP_FAILED if self.keep_failed else 0)
        b.keys = _ptr(self.keys)
        b.num_keys = int(self.keys.shape[0]) if hasattr(self.keys, "shape") and self.keys.dim() == 2 else max(
            1, int(self.keys.numel()) // 32)
        b.key_index = _ptr(self.key_index)
        b.seq = _ptr(self.seq)
        b.seq0 = self.seq0 & 0xFFFFFFFFFFFFFFFF
        b.content_type = self.content_type
        b.ver_major, b.ver_minor = self.version
        b.nonces = _ptr(self.nonces)
        b.ads = _ptr(self.ads)
        b.ad_len = self.ad_len
        b.ad_stride = self.ad_stride
        b.in_ = _ptr(self.inp)
        b.in_off = _ptr(self.in_off)
        b.in_stride = self.in_stride
        b.out = _ptr(self.out)
        b.out_off = _ptr(self.out_off)
        b.out_stride = self.out_stride
        b.len = _ptr(self.lens)
        b.uniform_len = self.uniform_len
        b.max_len = self.max_len
        b.status = _ptr(self.status)
        b.stream = _stream_handle(self.stream)
        b.workspace = _ptr(self.workspace)
        b.workspace_size = int(self.workspace.numel()) if self.workspace is not None else 0
        return b


def workspace_size(count: int) -> int:
    return int(N.load().sg_workspace_size(count))


def seal(batch: Batch) -> None:
    """Seal every record: out_i = ct_i || tag_i (chacha20_poly1305.rs:48-59)."""
    cb = batch.to_c()
    N.check(N.load().sg_seal_batch(C.byref(cb)))


def open_(batch: Batch) -> None:
    """Open every record; per-record status lands in ``batch.status``
    (0 ok, 1 BadRecordMac "wrong mac", 2 BadRecordMac "message too short")."""
    if batch.status is None:
        raise ValueError("open needs a status tensor")
    cb = batch.to_c()
    N.check(N.load().sg_open_batch(C.byref(cb)))


def fill_records(buf, stride: int, length: int, count: int, seed: int, j0: int = 0, stream=None) -> None:
    """Synthetic records generated on the device (splitmix64 rule)."""
    N.check(N.load().sg_fill_records(_ptr(buf), stride, length, count, seed & (2**64 - 1), j0,
                                     _stream_handle(stream)))


def compare_records(a, stride_a: int, b, stride_b: int, length: int, count: int, mismatches,
                    stream=None) -> None:
    N.check(N.load().sg_compare_records(_ptr(a), stride_a, _ptr(b), stride_b, length, count,
                                        _ptr(mismatches), _stream_handle(stream)))


def set_timing(enable: bool) -> None:
    N.check(N.load().sg_set_timing(1 if enable else 0))


def timing_read() -> dict:
    d = [C.c_double() for _ in range(3)]
    u = [C.c_uint32() for _ in range(3)]
    N.check(N.load().sg_timing_read(C.byref(d[0]), C.byref(d[1]), C.byref(d[2]), C.byref(u[0]),
                                    C.byref(u[1]), C.byref(u[2])))
    return {"seal_ms": d[0].value, "open_ms": d[1].value, "keying_ms": d[2].value,
            "n_seal": u[0].value, "n_open": u[1].value, "n_keying": u[2].value}
