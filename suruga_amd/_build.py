"""Build recipes for the in-tree native artefacts.

* ``suruga_amd/libsuruga_gpu.so`` -- the product: gfx950 HIP kernels + C ABI
  (``include/suruga_gpu.h``), compiled with ``hipcc --offload-arch=gfx950``.
* ``oracle/liboracle.so`` -- the CPU parity checker (test infrastructure only),
  compiled with ``gcc`` from ``oracle/suruga_oracle.c``.

Both are built in-tree so that they travel to the GPU box with the repo
snapshot.  The reference (Rust, klutzy/suruga) cannot be compiled here: there
is no rustc/cargo in the image, so there is no
``oracle/_ref`` build.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "suruga_amd"
CSRC = PKG / "csrc"
LIB = PKG / "libsuruga_gpu.so"
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "liboracle.so"

HIP_SOURCES = [CSRC / "sg_kernels.hip", CSRC / "sg_wpr.hip", CSRC / "sg_pack.hip", CSRC / "sg_capi.cpp", CSRC / "sg_record.cpp",
               CSRC / "sg_keysched.cpp", CSRC / "sg_wire.cpp"]
HIP_DEPS = HIP_SOURCES + [CSRC / "sg_internal.h", CSRC / "sg_device.h", CSRC / "sg_host.h", CSRC / "sg_err.h",
                          CSRC / "sg_wire.h", CSRC / "sg_chacha_grp.inc",
                          ROOT / "include" / "suruga_gpu.h"]
ORACLE_SOURCES = [ORACLE_DIR / "suruga_oracle.c"]
ORACLE_DEPS = ORACLE_SOURCES + [ORACLE_DIR / "suruga_oracle.h", ORACLE_DIR / "so_pool.h"]


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def source_hash() -> str:
    """SHA-256 (first 16 hex digits) of every source and header the HIP library
    is built from (HIP_DEPS, in order, with their names).  The build embeds it
    (sg_build_info / sg_source_hash), _native.load() refuses a library whose
    embedded hash differs from the tree's, and build_library() rebuilds on a
    mismatch whatever the file times say."""
    import hashlib

    h = hashlib.sha256()
    for d in HIP_DEPS:
        h.update(d.name.encode() + b"\0" + d.read_bytes() + b"\0")
    return h.hexdigest()[:16]


def embedded_hash(lib: Path):
    """The source hash a built library carries (None: none / unreadable)."""
    import re

    try:
        m = re.search(rb"sg-src:([0-9a-f]{16}(?:\+var:[A-Za-z0-9_.:-]+)?)", lib.read_bytes())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _run(cmd) -> None:
    proc = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{proc.stdout}\n{proc.stderr}")


def hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = Path(rocm) / "bin" / "hipcc"
    return str(cand) if cand.exists() else "hipcc"


# Switches of earlier timing experiments that produced wrong tags.  They are
# gone from the product sources (tests/test_abi.py checks), and a build of the
# product library refuses them outright.
FORBIDDEN_DEFINE_PREFIXES = ("-DSG_LS_NO", "-DSG_LS_COMPILED", "-DSG_EXP_", "-DSG_MAC_GLOBAL_A", "-DSG_MACX")


def build_library(force: bool = False, out: Path | None = None, defines=()) -> Path:
    """Compile the gfx950 HIP library (seconds).  ``out``/``defines`` build an
    experiment variant (e.g. ``-DSG_WPR_PROFILE=1``) next to the product library;
    the product library itself is only ever built without defines."""
    target = Path(out) if out else LIB
    bad = [d for d in defines if str(d).startswith(FORBIDDEN_DEFINE_PREFIXES)]
    if bad:
        raise ValueError(f"wrong-output experiment switches are not buildable: {bad}")
    if defines and target.resolve() == LIB.resolve():
        raise ValueError("the product library is built without -D switches; pass out= for a variant")
    src = source_hash()
    marker = src
    if defines:  # a -D variant never carries the product's identity (see _native.load)
        import hashlib

        marker = f"{src}+var:defs:{hashlib.sha256(repr(tuple(defines)).encode()).hexdigest()[:8]}"
    if force or defines or _stale(target, HIP_DEPS) or embedded_hash(target) != src:
        import tempfile
        from concurrent.futures import ThreadPoolExecutor

        tmp = target.with_suffix(f".so.tmp{os.getpid()}")  # concurrent builders never share a temp file
        # no wave-aggregating rewrite of atomics: sg_wpr_kernel's group-counter
        # fetch must not wait for its return right away (sg_wpr.hip)
        flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-mllvm",
                 "-amdgpu-atomic-optimizer-strategy=None", "-Wall", "-Wno-unused-result", *defines,
                 f'-DSG_SOURCE_HASH="{marker}"']
        # one translation unit per compiler process (the kernels take most of a
        # minute each), then one link
        with tempfile.TemporaryDirectory(prefix="sg_build_") as td:
            objs = [Path(td) / f"{p.stem}.o" for p in HIP_SOURCES]
            jobs = int(os.environ.get("MAX_JOBS", "0") or 0) or min(len(HIP_SOURCES), os.cpu_count() or 1)
            with ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
                list(ex.map(lambda po: _run([hipcc(), *flags, "-c", "-o", str(po[1]), str(po[0])]),
                            zip(HIP_SOURCES, objs)))
            _run([hipcc(), "--offload-arch=gfx950", "-fPIC", "-shared", "-o", str(tmp), *map(str, objs)])
        os.replace(tmp, target)
    return target


def build_oracle(force: bool = False) -> Path:
    """Compile the CPU restatement used as the parity checker."""
    if force or _stale(ORACLE_LIB, ORACLE_DEPS):
        tmp = ORACLE_LIB.with_suffix(f".so.tmp{os.getpid()}")
        _run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-fPIC", "-shared", "-pthread",
              "-o", str(tmp), *map(str, ORACLE_SOURCES)])
        os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


CPP_TEST_SRC = ROOT / "tests" / "cpp" / "test_host.cpp"
CPP_TEST_BIN = ROOT / "tests" / "cpp" / "test_host"
CPP_TEST_DEPS = [CPP_TEST_SRC, ROOT / "include" / "suruga" / "cipher.hpp", ROOT / "include" / "suruga" / "tls.hpp",
                 ROOT / "include" / "suruga" / "prf.hpp",
                 ROOT / "include" / "suruga_gpu.h", ORACLE_DIR / "suruga_oracle.h"]


def build_cpp_tests(force: bool = False) -> Path:
    """The C++ host-mirror test program (include/suruga/*.hpp), linked against
    both in-tree libraries."""
    lib, orc = build_library(), build_oracle()
    if force or _stale(CPP_TEST_BIN, CPP_TEST_DEPS + [lib, orc]):
        tmp = CPP_TEST_BIN.with_suffix(f".tmp{os.getpid()}")
        _run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-o", str(tmp), str(CPP_TEST_SRC),
              f"-L{lib.parent}", f"-L{orc.parent}", "-lsuruga_gpu", "-loracle",
              "-Wl,-rpath,$ORIGIN/../../suruga_amd:$ORIGIN/../../oracle"])
        os.replace(tmp, CPP_TEST_BIN)
    return CPP_TEST_BIN


OSSL_SRC = ORACLE_DIR / "ossl_aead.c"
OSSL_LIB = ORACLE_DIR / "libossl_aead.so"


def build_ossl(force: bool = False):
    """The OpenSSL-composed CPU comparison line (bench only).  Optional: None
    when libcrypto headers are absent."""
    if not Path("/usr/include/openssl/evp.h").exists():
        return OSSL_LIB if OSSL_LIB.exists() else None
    if force or _stale(OSSL_LIB, [OSSL_SRC, ORACLE_DIR / "so_pool.h"]):
        tmp = OSSL_LIB.with_suffix(f".so.tmp{os.getpid()}")
        _run(["gcc", "-O2", "-std=c11", "-Wall", "-fPIC", "-shared", "-pthread", "-o", str(tmp), str(OSSL_SRC),
              "-lcrypto"])
        os.replace(tmp, OSSL_LIB)
    return OSSL_LIB


LOOPBACK_SRC = ROOT / "tools" / "loopback_cpp.cpp"
LOOPBACK_BIN = ROOT / "tools" / "loopback_cpp"


def build_loopback_cpp(force: bool = False) -> Path:
    """tools/loopback_cpp: C4 over a loopback socket in C++ (include/suruga over
    the C ABI), linked against the in-tree library (a measuring tool, not the
    product)."""
    lib = build_library()
    deps = [LOOPBACK_SRC, ROOT / "include" / "suruga" / "cipher.hpp", ROOT / "include" / "suruga" / "tls.hpp",
            ROOT / "include" / "suruga_gpu.h", lib]
    if force or _stale(LOOPBACK_BIN, deps):
        tmp = LOOPBACK_BIN.with_suffix(f".tmp{os.getpid()}")
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-pthread", "-o", str(tmp), str(LOOPBACK_SRC),
              f"-L{lib.parent}", "-lsuruga_gpu", "-Wl,-rpath,$ORIGIN/../suruga_amd"])
        os.replace(tmp, LOOPBACK_BIN)
    return LOOPBACK_BIN


def build_all(force: bool = False) -> None:
    build_library(force)
    build_oracle(force)
    build_ossl(force)
    build_cpp_tests(force)
    build_loopback_cpp(force)


if __name__ == "__main__":
    import sys

    build_all(force="--force" in sys.argv)
    print(LIB)
    print(ORACLE_LIB)
