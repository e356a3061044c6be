"""The CPU side under AddressSanitizer / UndefinedBehaviorSanitizer (SURVEY.md
section 5: "keep the same limb-bound invariants as debug asserts in the CPU
restatement; run it under ASan/UBSan in this container").

1. The oracle (oracle/suruga_oracle.c) built with -DSO_DEBUG -- the reference's
   Int1305 debug_assert!s (poly1305.rs:87-125 limb and carry bounds of `mult`,
   :155-159 of `from_bytes`) become live asserts -- and -fsanitize=address,
   undefined, then tests/test_oracle.py (the reference's ChaCha20 and Poly1305
   KATs, the COEFFS algebra, the 54 AEAD vectors, the batch drivers) runs
   against that build in a Python whose first library is libasan.
2. The asserts are live in that build: an Int1305 product of out-of-range
   limbs aborts.
3. The library's host-only sources -- the record header parser that takes a
   peer's bytes (sg_wire.cpp, tls.rs:217-238) and the key schedule
   (sg_keysched.cpp) -- built with g++ -fsanitize=address,undefined into
   tests/cpp/test_host_san.cpp's corpus run.

CPU only: no GPU, no HIP runtime (neither host source includes a HIP header).
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
SAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


def _libasan() -> str:
    p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not p or not Path(p).exists():
        pytest.skip("gcc's libasan.so is not installed")
    return p


@pytest.fixture(scope="module")
def san_oracle(tmp_path_factory):
    out = tmp_path_factory.mktemp("san") / "liboracle_san.so"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-fPIC", "-shared", "-pthread", "-DSO_DEBUG", *SAN,
           "-o", str(out), str(ROOT / "oracle" / "suruga_oracle.c")]
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    return out


def _san_env(lib: Path) -> dict:
    env = dict(os.environ, **SAN_ENV)
    env["LD_PRELOAD"] = _libasan()
    env["SURUGA_ORACLE_LIB"] = str(lib)
    return env


def test_oracle_kats_under_asan_ubsan_with_debug_asserts(san_oracle):
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        str(ROOT / "tests" / "test_oracle.py")],
                       capture_output=True, text=True, timeout=900, cwd=ROOT, env=_san_env(san_oracle))
    tail = (p.stdout + p.stderr)[-4000:]
    assert p.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error" not in tail, tail
    assert " passed" in p.stdout


def test_debug_asserts_are_live(san_oracle):
    """The same build aborts on an Int1305 product of out-of-range limbs (the
    bound debug_assert!(carry <= 25 * ((1 << 26) - 1)) of poly1305.rs:87-93)."""
    code = ("import sys; sys.path.insert(0, 'tests'); from oracle_ffi import Oracle, Int1305; "
            "o = Oracle(); big = Int1305.of([0xffffffff] * 5); o.L.so_int1305_mult(big, big); print('no abort')")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                       env=_san_env(san_oracle))
    assert p.returncode != 0 and "no abort" not in p.stdout, p.stdout + p.stderr[-2000:]
    assert "Assertion" in p.stderr or "assert" in p.stderr.lower(), p.stderr[-2000:]


def test_host_sources_under_asan_ubsan(tmp_path):
    exe = tmp_path / "test_host_san"
    csrc = ROOT / "suruga_amd" / "csrc"
    cmd = ["g++", "-std=c++17", "-Wall", "-Wextra", "-pthread", *SAN, "-o", str(exe),
           str(ROOT / "tests" / "cpp" / "test_host_san.cpp"), str(csrc / "sg_wire.cpp"), str(csrc / "sg_keysched.cpp")]
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-4000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=dict(os.environ, **SAN_ENV))
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "host sanitizer checks passed" in r.stdout
