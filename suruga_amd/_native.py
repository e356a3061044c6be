"""ctypes binding of the C ABI in ``include/suruga_gpu.h``.

The shared library is the only compute path: if it is missing or cannot be
loaded this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

from ._build import LIB

SG_OK = 0
SG_E_BAD_MAC = 1
SG_E_SHORT = 2
SG_E_ARG = -1
SG_E_HIP = -2
SG_E_NODEV = -3

SG_BATCH_TLS = 0x1
SG_BATCH_KEEP_FAILED = 0x2
SG_KEY_LEN = 32
SG_NONCE_LEN = 8
SG_MAC_LEN = 16
SG_MAX_AD_LEN = 255
SG_MAX_RECORD_LEN = 32768

# Every symbol include/suruga_gpu.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "sg_key_size", "sg_fixed_iv_len", "sg_mac_len", "sg_abi_version",
    "sg_ctx_new", "sg_ctx_free", "sg_seal", "sg_open",
    "sg_workspace_size", "sg_seal_batch", "sg_open_batch",
    "sg_fill_records", "sg_compare_records",
    "sg_last_error", "sg_build_info", "sg_source_hash", "sg_set_timing", "sg_timing_read", "sg_set_lockstep", "sg_set_packed",
    "sg_wire_bound", "sg_write_records", "sg_read_records", "sg_parse_records", "sg_record_timing",
    "sg_host_register", "sg_host_unregister",
    "sg_sha256", "sg_hmac_sha256", "sg_prf_new", "sg_prf_get_bytes", "sg_prf_free",
    "sg_derive_keys", "sg_finished_verify_data",
]


class SgBatch(C.Structure):
    """Mirror of ``struct sg_batch``."""

    _fields_ = [
        ("count", C.c_uint32),
        ("flags", C.c_uint32),
        ("keys", C.c_void_p),
        ("num_keys", C.c_uint32),
        ("key_index", C.c_void_p),
        ("seq", C.c_void_p),
        ("seq0", C.c_uint64),
        ("content_type", C.c_uint8),
        ("ver_major", C.c_uint8),
        ("ver_minor", C.c_uint8),
        ("_pad0", C.c_uint8),
        ("nonces", C.c_void_p),
        ("ads", C.c_void_p),
        ("ad_len", C.c_uint32),
        ("ad_stride", C.c_uint32),
        ("in_", C.c_void_p),
        ("in_off", C.c_void_p),
        ("in_stride", C.c_uint64),
        ("out", C.c_void_p),
        ("out_off", C.c_void_p),
        ("out_stride", C.c_uint64),
        ("len", C.c_void_p),
        ("uniform_len", C.c_uint32),
        ("max_len", C.c_uint32),
        ("status", C.c_void_p),
        ("stream", C.c_void_p),
        ("workspace", C.c_void_p),
        ("workspace_size", C.c_size_t),
    ]


class SgReadResult(C.Structure):
    """Mirror of ``struct sg_read_result``."""

    _fields_ = [("records", C.c_uint64), ("consumed", C.c_uint64), ("out_len", C.c_uint64),
                ("error", C.c_int32), ("_pad", C.c_uint32)]


class SgWireRecord(C.Structure):
    """Mirror of ``struct sg_wire_record``."""

    _fields_ = [("offset", C.c_uint64), ("frag_len", C.c_uint32), ("type", C.c_uint8), ("ver_major", C.c_uint8),
                ("ver_minor", C.c_uint8), ("_pad", C.c_uint8)]


SG_E_UNEXPECTED_MESSAGE = 3
SG_E_RECORD_OVERFLOW = 4
SG_RECORD_MAX_LEN = 16384
SG_ENC_RECORD_MAX_LEN = 16384 + 2048
SG_HEADER_LEN = 5


class NativeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"suruga_gpu error {code}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()


def provenance_error(got: str, want: str, allow_variant: bool):
    """None when a library embedding source marker `got` may run in a tree
    whose sources hash to `want`, else the reason.  Experiment variants
    (tools/build_variant.py, _build.build_library(defines=...)) embed
    "<tree hash>+var:<name>:<edit hash>" and run only on explicit request
    (SURUGA_ALLOW_VARIANT=1, as tools/ab_libs.sh sets).  allow_variant ==
    "foreign" (SURUGA_ALLOW_VARIANT=foreign) also admits a variant built from an
    earlier tree -- the A/B of a change against the build before it
    (tools/build_variant.py with no edits) -- and nothing unmarked."""
    if got == want:
        return None
    if allow_variant == "foreign" and "+var:" in got:
        return None
    if got.startswith(want + "+var:"):
        if allow_variant:
            return None
        return (f"is an experiment variant ({got}) of this tree: set SURUGA_ALLOW_VARIANT=1 to time it; "
                "the product runs only the tree's own build")
    return (f"was built from other sources (embedded hash {got}, tree {want}): "
            "rebuild with `python -m suruga_amd._build`")


def _declare(lib: C.CDLL) -> None:
    u8p = C.POINTER(C.c_uint8)
    lib.sg_key_size.restype = C.c_size_t
    lib.sg_fixed_iv_len.restype = C.c_size_t
    lib.sg_mac_len.restype = C.c_size_t
    lib.sg_abi_version.restype = C.c_int
    lib.sg_ctx_new.restype = C.c_void_p
    lib.sg_ctx_new.argtypes = [C.c_char_p, C.c_int]
    lib.sg_ctx_free.restype = None
    lib.sg_ctx_free.argtypes = [C.c_void_p]
    for f in (lib.sg_seal, lib.sg_open):
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                      C.c_char_p, C.c_size_t, u8p]
    lib.sg_workspace_size.restype = C.c_size_t
    lib.sg_workspace_size.argtypes = [C.c_uint32]
    for f in (lib.sg_seal_batch, lib.sg_open_batch):
        f.restype = C.c_int
        f.argtypes = [C.POINTER(SgBatch)]
    lib.sg_fill_records.restype = C.c_int
    lib.sg_fill_records.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64,
                                    C.c_uint64, C.c_void_p]
    lib.sg_compare_records.restype = C.c_int
    lib.sg_compare_records.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint32,
                                       C.c_uint32, C.c_void_p, C.c_void_p]
    lib.sg_last_error.restype = C.c_char_p
    lib.sg_build_info.restype = C.c_char_p
    lib.sg_source_hash.restype = C.c_char_p
    lib.sg_set_timing.restype = C.c_int
    lib.sg_set_timing.argtypes = [C.c_int]
    lib.sg_set_lockstep.restype = C.c_int
    lib.sg_set_lockstep.argtypes = [C.c_int]
    lib.sg_set_packed.restype = C.c_int
    lib.sg_set_packed.argtypes = [C.c_int]
    lib.sg_timing_read.restype = C.c_int
    d = C.POINTER(C.c_double)
    u = C.POINTER(C.c_uint32)
    lib.sg_timing_read.argtypes = [d, d, d, u, u, u]
    lib.sg_wire_bound.restype = C.c_size_t
    lib.sg_wire_bound.argtypes = [C.c_size_t]
    lib.sg_write_records.restype = C.c_int64
    lib.sg_write_records.argtypes = [C.c_void_p, C.c_uint64, C.c_uint8, C.c_uint8, C.c_uint8, C.c_void_p,
                                     C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.sg_read_records.restype = C.c_int
    lib.sg_read_records.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                    C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(SgReadResult)]
    lib.sg_host_register.restype = C.c_int
    lib.sg_host_register.argtypes = [C.c_void_p, C.c_size_t]
    lib.sg_host_unregister.restype = C.c_int
    lib.sg_host_unregister.argtypes = [C.c_void_p]
    lib.sg_parse_records.restype = C.c_int
    lib.sg_parse_records.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.POINTER(SgWireRecord),
                                     C.POINTER(C.c_size_t), C.POINTER(C.c_int32)]
    lib.sg_record_timing.restype = C.c_int
    lib.sg_record_timing.argtypes = [d, d, d, d]
    vp = C.c_void_p
    lib.sg_sha256.restype = None
    lib.sg_sha256.argtypes = [vp, C.c_size_t, vp]
    lib.sg_hmac_sha256.restype = C.c_int
    lib.sg_hmac_sha256.argtypes = [vp, C.c_size_t, vp, C.c_size_t, vp]
    lib.sg_prf_new.restype = vp
    lib.sg_prf_new.argtypes = [vp, C.c_size_t, vp, C.c_size_t]
    lib.sg_prf_get_bytes.restype = C.c_int
    lib.sg_prf_get_bytes.argtypes = [vp, vp, C.c_size_t]
    lib.sg_prf_free.restype = None
    lib.sg_prf_free.argtypes = [vp]
    lib.sg_derive_keys.restype = C.c_int
    lib.sg_derive_keys.argtypes = [C.c_uint32, vp, C.c_size_t, C.c_size_t, vp, vp, vp, vp, vp, C.c_int]
    lib.sg_finished_verify_data.restype = C.c_int
    lib.sg_finished_verify_data.argtypes = [vp, C.c_int, vp, vp]


def load(path: Path | None = None) -> C.CDLL:
    """Load (once) and return the native library.  Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is None:
            # SURUGA_GPU_LIB: load another build of the same library (A/B kernel
            # experiments, tools/ab_bench.sh); still the HIP library, never a fallback
            p = Path(path or os.environ.get("SURUGA_GPU_LIB") or LIB)
            if not p.exists():
                raise ImportError(
                    f"{p} is missing: build it with `python -m suruga_amd._build` "
                    "(hipcc --offload-arch=gfx950); there is no CPU fallback")
            lib = C.CDLL(str(p))
            _declare(lib)
            # provenance: the library must have been built from this tree's
            # sources (a stale prebuilt .so whose file time happens to be newer
            # would otherwise run silently)
            from ._build import source_hash

            got, want = lib.sg_source_hash().decode(), source_hash()
            av = os.environ.get("SURUGA_ALLOW_VARIANT")
            err = provenance_error(got, want, "foreign" if av == "foreign" else av == "1")
            if err:
                raise ImportError(f"{p} {err}")
            global _lib_path
            _lib_path = str(p.resolve())
            _lib = lib
        return _lib


_lib_path = None


def loaded_info() -> dict:
    """Which library this process runs and the source hash it carries (bench provenance)."""
    lib = load()
    return {"path": _lib_path, "source_hash": lib.sg_source_hash().decode()}


def last_error() -> str:
    return load().sg_last_error().decode(errors="replace")


def check(code: int) -> int:
    """Raise NativeError for negative (argument / runtime) codes."""
    if code < 0:
        raise NativeError(code, last_error())
    return code
