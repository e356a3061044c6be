"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = Path(__file__).resolve().parent / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
if str(Path(__file__).resolve().parent) not in sys.path:
    sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")


@pytest.fixture(scope="session")
def oracle():
    from oracle_ffi import oracle as get

    return get()


@pytest.fixture(scope="session")
def kats():
    return json.loads((GOLDEN / "reference_kats.json").read_text())


@pytest.fixture(scope="session")
def aead_vectors():
    return json.loads((GOLDEN / "aead_vectors.json").read_text())


@pytest.fixture(scope="session")
def gpu():
    """The HIP library on a real gfx950 device; fails (never skips) without one,
    so a GPU run can not pass on a silent fallback."""
    import torch

    from suruga_amd import _build, _native

    _build.build_library()
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    lib = _native.load()
    return lib


def vector_pt(v, oracle):
    if "pt" in v:
        return bytes.fromhex(v["pt"])
    g = v["pt_gen"]
    return oracle.fill_record(g["seed"], g["j"], v["n"])
