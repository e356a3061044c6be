"""CPU tests of the drop-in boundary: the C-ABI library builds for gfx950,
loads, exports every symbol include/suruga_gpu.h declares, reports the
reference's Aead constants, and rejects bad arguments before touching a GPU.
No compute calls are made here (there is no GPU in the build container)."""
from __future__ import annotations

import ctypes as C
from pathlib import Path
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = ROOT / "include" / "suruga_gpu.h"


def declared_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sg_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from suruga_amd import _build, _native

    _build.build_library()
    return _native.load()


def test_library_is_gfx950_code_object(lib):
    from suruga_amd._build import LIB

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={LIB}"], capture_output=True, text=True)
    if out.returncode == 0 and out.stdout.strip():
        assert "gfx950" in out.stdout
    else:  # fall back to scanning the fat binary for the target id
        assert b"gfx950" in LIB.read_bytes()


def test_exports_every_declared_symbol(lib):
    from suruga_amd._native import EXPORTS

    syms = declared_symbols()
    assert len(syms) >= 15
    assert sorted(EXPORTS) == syms
    for s in syms:
        assert hasattr(lib, s), f"{s} not exported"


def test_aead_constants(lib):
    # chacha20_poly1305.rs:15-17, 104-119
    assert lib.sg_key_size() == 32
    assert lib.sg_fixed_iv_len() == 0
    assert lib.sg_mac_len() == 16
    assert lib.sg_abi_version() == 1
    assert b"gfx950" in lib.sg_build_info()


def test_batch_argument_errors_without_gpu(lib):
    from suruga_amd._native import SG_E_ARG, SgBatch

    assert lib.sg_seal_batch(None) == SG_E_ARG
    b = SgBatch()
    b.count = 4  # keys/in/out missing
    assert lib.sg_seal_batch(C.byref(b)) == SG_E_ARG
    assert b"non-NULL" in lib.sg_last_error()
    b.keys, b.in_, b.out, b.num_keys = 0x1000, 0x2000, 0x3000, 1
    b.flags = 1
    b.uniform_len = 40000  # > SG_MAX_RECORD_LEN
    b.in_stride = b.out_stride = 40016
    assert lib.sg_seal_batch(C.byref(b)) == SG_E_ARG
    assert b"SG_MAX_RECORD_LEN" in lib.sg_last_error()
    b.uniform_len = 64
    assert lib.sg_open_batch(C.byref(b)) == SG_E_ARG  # open needs a status array
    b.count = 0
    assert lib.sg_seal_batch(C.byref(b)) == 0  # empty batch is a no-op


def test_explicit_mode_limits_are_sg_e_arg_without_gpu(lib):
    """explicit-mode AD above SG_MAX_AD_LEN (255) and records
    above SG_MAX_RECORD_LEN (32 KiB) are SG_E_ARG, where the reference's
    Encryptor::encrypt (cipher/mod.rs:22-24) accepts any length.  The checks
    run before any device work, so they are pinned here on the CPU."""
    from suruga_amd._native import SG_E_ARG, SgBatch

    b = SgBatch()
    b.count, b.num_keys, b.flags = 4, 1, 0  # explicit mode
    b.keys, b.in_, b.out, b.nonces, b.ads = 0x1000, 0x2000, 0x3000, 0x4000, 0x5000
    b.uniform_len, b.in_stride, b.out_stride = 64, 64, 80
    b.ad_len = 256
    assert lib.sg_seal_batch(C.byref(b)) == SG_E_ARG
    assert b"SG_MAX_AD_LEN" in lib.sg_last_error()
    b.ad_len = 255
    b.uniform_len, b.in_stride, b.out_stride = 32769, 32769, 32785
    assert lib.sg_seal_batch(C.byref(b)) == SG_E_ARG
    assert b"SG_MAX_RECORD_LEN" in lib.sg_last_error()
    b.status = 0x6000
    b.uniform_len = 32769 + 16  # open: the ciphertext carries the tag
    assert lib.sg_open_batch(C.byref(b)) == SG_E_ARG
    assert b"SG_MAX_RECORD_LEN" in lib.sg_last_error()


def test_single_record_argument_errors_without_gpu(lib):
    from suruga_amd._native import SG_E_ARG

    out = (C.c_uint8 * 64)()
    assert lib.sg_seal(None, bytes(8), 8, b"", 0, b"", 0, out) == SG_E_ARG
    assert lib.sg_ctx_new(None, 0) is None


def test_python_mirror_constants_without_gpu():
    from suruga_amd import ChaCha20Poly1305, CipherSuite

    aead = CipherSuite.TLS_ECDHE_RSA_WITH_CHACHA20_POLY1305_SHA256.new_aead()
    assert isinstance(aead, ChaCha20Poly1305)
    assert (aead.key_size(), aead.fixed_iv_len(), aead.mac_len()) == (32, 0, 16)
    with pytest.raises(ValueError):
        aead.new_encryptor(bytes(31))  # ChaCha20::new panics (chacha20.rs:26)


def test_no_cpu_fallback_in_product():
    """The product library must not link the oracle or carry a CPU path."""
    from suruga_amd._build import HIP_SOURCES

    for src in HIP_SOURCES:
        text = src.read_text()
        assert "oracle" not in text.lower()
    for py in (ROOT / "suruga_amd").glob("*.py"):
        text = py.read_text()
        assert "import oracle" not in text and "oracle_ffi" not in text, py


def test_product_sources_carry_no_wrong_output_switches():
    """The timing-experiment switches of round 1 that skipped the MAC or the
    rounds (tags wrong) are not in the product sources, and _build refuses
    them (SG_LS_NO*, SG_LS_COMPILED, SG_EXP_*, SG_MAC_GLOBAL_A)."""
    from suruga_amd import _build

    for src in _build.HIP_DEPS:
        text = src.read_text()
        for tok in ("SG_LS_NOMAC", "SG_LS_NOROUNDS", "SG_LS_COMPILED", "SG_EXP_", "SG_MAC_GLOBAL_A", "SG_MACX"):
            assert tok not in text, (src.name, tok)
    with pytest.raises(ValueError):
        _build.build_library(out=ROOT / "build_variant_never_written.so", defines=["-DSG_LS_NOMAC=1"])
    with pytest.raises(ValueError):
        _build.build_library(defines=["-DSG_SALU_PRE=0"])  # product lib: no switches at all


def test_missing_library_fails_loudly(tmp_path):
    """A missing HIP library is an ImportError naming the build step, never a
    silent CPU path (the loader is the product's only way to the kernels)."""
    code = ("import sys; from pathlib import Path; from suruga_amd import _native as N\n"
            "try:\n    N.load(Path(sys.argv[1]))\nexcept ImportError as e:\n"
            "    print('IMPORTERROR', e); raise SystemExit(0)\nraise SystemExit(1)\n")
    p = subprocess.run([__import__("sys").executable, "-c", code, str(tmp_path / "absent.so")], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "IMPORTERROR" in p.stdout and "no CPU fallback" in p.stdout, p.stdout + p.stderr


def test_record_header_parser_without_gpu(lib):
    """sg_read_records checks headers (tls.rs:218-238) before any device work:
    with no complete valid record in the buffer it returns the header error
    without touching the context, so an opaque dummy handle suffices here."""
    from suruga_amd._native import SG_E_RECORD_OVERFLOW, SG_E_SHORT, SG_E_UNEXPECTED_MESSAGE, SgReadResult

    dummy = C.create_string_buffer(64)  # never dereferenced on these paths
    res = SgReadResult()

    def parse(wire: bytes):
        buf = C.create_string_buffer(wire, len(wire))
        out = C.create_string_buffer(max(len(wire), 1))
        assert lib.sg_read_records(C.cast(dummy, C.c_void_p), 0, buf, len(wire), out, len(out), None, None, 16,
                                   C.byref(res)) == 0
        return res.error, res.records, res.consumed

    assert parse(bytes([0x18, 3, 3, 0, 3, 1, 2, 3])) == (SG_E_UNEXPECTED_MESSAGE, 0, 0)  # tls.rs:427-436
    n = 16384 + 2048 + 1
    assert parse(bytes([23, 3, 3, n >> 8, n & 0xFF])) == (SG_E_RECORD_OVERFLOW, 0, 0)   # tls.rs:232-234
    assert parse(bytes([23, 3, 3, 0, 15]) + bytes(15)) == (SG_E_SHORT, 0, 0)             # < mac_len
    n = 16384 + 17
    assert parse(bytes([23, 3, 3, n >> 8, n & 0xFF]) + bytes(n)) == (SG_E_RECORD_OVERFLOW, 0, 0)
    assert parse(bytes([23, 3, 3, 0, 40]) + bytes(10)) == (0, 0, 0)   # incomplete: wait for more bytes
    assert parse(bytes([23, 3])) == (0, 0, 0)
    assert lib.sg_wire_bound(0) == 0
    assert lib.sg_wire_bound(1) == 1 + 21
    assert lib.sg_wire_bound(16384) == 16384 + 21
    assert lib.sg_wire_bound(16385) == 16385 + 42


def test_library_carries_the_tree_source_hash(lib):
    """Provenance: the library embeds the hash of the sources it
    was built from, and it equals the hash of this tree's sources."""
    from suruga_amd import _build

    want = _build.source_hash()
    assert lib.sg_source_hash().decode() == want
    assert _build.embedded_hash(_build.LIB) == want
    assert f"sg-src:{want}".encode() in lib.sg_build_info()


def test_stale_library_is_refused(tmp_path, lib):
    """A library built from other sources (here: the product library with its
    embedded hash rewritten) is refused by the loader, not run."""
    from suruga_amd import _build

    data = _build.LIB.read_bytes()
    want = _build.source_hash()
    other = ("0123456789abcdef" if want != "0123456789abcdef" else "fedcba9876543210").encode()
    stale = tmp_path / "libsuruga_gpu_stale.so"
    stale.write_bytes(data.replace(b"sg-src:" + want.encode(), b"sg-src:" + other))
    code = ("import sys; from pathlib import Path; from suruga_amd import _native as N\n"
            "try:\n    N.load(Path(sys.argv[1]))\nexcept ImportError as e:\n"
            "    print('IMPORTERROR', e); raise SystemExit(0)\nraise SystemExit(1)\n")
    p = subprocess.run([__import__("sys").executable, "-c", code, str(stale)], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0 and "IMPORTERROR" in p.stdout and "other sources" in p.stdout, p.stdout + p.stderr


def test_unknown_batch_flags_are_rejected(lib):
    from suruga_amd._native import SG_BATCH_KEEP_FAILED, SG_BATCH_TLS, SG_E_ARG, SgBatch

    b = SgBatch()
    b.count, b.num_keys = 4, 1
    b.keys, b.in_, b.out, b.status = 0x1000, 0x2000, 0x3000, 0x4000
    b.uniform_len, b.in_stride, b.out_stride = 64, 64, 80
    b.flags = SG_BATCH_TLS | 0x4
    assert lib.sg_open_batch(C.byref(b)) == SG_E_ARG and b"unknown flags" in lib.sg_last_error()
    assert SG_BATCH_KEEP_FAILED == 0x2


def test_no_kernel_uses_scratch(tmp_path, lib):
    """The wave-per-record and packed kernels count their own vector-memory
    operations (exact s_waitcnt vmcnt, sg_wpr.hip); a compiler spill to scratch
    would add vector-memory operations they do not count.  Every kernel of the
    library must have a zero private segment (no VGPR spills to memory)."""
    import shutil

    from suruga_amd._build import LIB

    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not (Path(objdump).exists() and Path(readelf).exists()):
        pytest.skip("ROCm llvm tools absent")
    local = tmp_path / "lib.so"
    shutil.copy(LIB, local)
    subprocess.run([objdump, "--offloading", str(local)], cwd=tmp_path, capture_output=True, timeout=120)
    cos = sorted(tmp_path.glob("lib.so.*gfx950"))
    assert cos, "no gfx950 code object in the library"
    seen = 0
    for co in cos:
        notes = subprocess.run([readelf, "--notes", str(co)], capture_output=True, text=True, timeout=120).stdout
        names = re.findall(r"\.name:\s+(\S+)", notes)
        sizes = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)]
        assert len(names) == len(sizes)
        for nm, sz in zip(names, sizes):
            assert sz == 0, f"{nm} uses {sz} bytes of scratch"
        seen += len(names)
    assert seen >= 20


def test_variant_marker_needs_explicit_opt_in():
    """experiment variants embed "<tree hash>+var:<name>:<edit hash>";
    the loader refuses them unless SURUGA_ALLOW_VARIANT=1, and refuses any other
    hash outright."""
    from suruga_amd._native import provenance_error

    want = "0123456789abcdef"
    assert provenance_error(want, want, False) is None
    var = want + "+var:pk_nomac:1a2b3c4d"
    assert "SURUGA_ALLOW_VARIANT" in provenance_error(var, want, False)
    assert provenance_error(var, want, True) is None
    assert "other sources" in provenance_error("fedcba9876543210", want, True)
    assert "other sources" in provenance_error("fedcba9876543210+var:x:00", want, True)
