"""The C++ host-side mirror (include/suruga/cipher.hpp, tls.hpp): the
reference's record tests in C++ (CPU) and the GPU Aead behind the C++ traits
checked against the oracle (GPU).  tests/cpp/test_host.cpp holds the checks."""
from __future__ import annotations

import subprocess

import pytest

from suruga_amd import _build


@pytest.fixture(scope="module")
def test_bin():
    return _build.build_cpp_tests()


def _run(binary, mode):
    proc = subprocess.run([str(binary), mode], capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert "0 failed" in proc.stdout


def test_cpp_record_layer_cpu(test_bin):
    _run(test_bin, "cpu")


@pytest.mark.gpu
def test_cpp_gpu_aead_and_record_layer(gpu, test_bin):
    _run(test_bin, "gpu")
