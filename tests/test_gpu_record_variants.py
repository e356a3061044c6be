"""The record layer's pipeline switches, each bit-exact (GPU).

sg_record.cpp reads its pipeline switches once per process from the
environment, so every form runs the record-layer GPU tests
(tests/test_record_layer.py: staged and zero-copy writes against the oracle,
reads with corrupted records, odd lengths, mixed content types) and the
per-direction + duplex record-path check in a child process of its own:

* SG_RECORD_SDMA=1: staged calls through the copy-engine pipeline instead of
  the direct one;
* SG_RECORD_SDMA=1 SG_RECORD_DEVICE_WAITS=1: round 5's device-waited form;
* SG_RECORD_KD2H=1: zero-copy output by kernel stores instead of an SDMA D2H;
* SG_COPY_STREAMS=0 SG_RECORD_SLOTS=2: per-slot streams, the shallowest
  pipeline;
* SG_ZERO_COPY=0: registered buffers through the staged path;
* SG_DIRECT_PRIO=0: the direct pipeline's kernel streams at default priority.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent

VARIANTS = {
    "sdma": {"SG_RECORD_SDMA": "1"},
    "device_waits": {"SG_RECORD_SDMA": "1", "SG_RECORD_DEVICE_WAITS": "1"},
    "kd2h": {"SG_RECORD_KD2H": "1"},
    "slot_streams": {"SG_COPY_STREAMS": "0", "SG_RECORD_SLOTS": "2"},
    "no_zero_copy": {"SG_ZERO_COPY": "0"},
    "direct_default_prio": {"SG_DIRECT_PRIO": "0"},
}


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_record_pipeline_variant_bit_exact(gpu, name):
    env = dict(os.environ, **VARIANTS[name])
    args = [sys.executable, "-u", "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
            "tests/test_record_layer.py", "tests/test_gpu_loopback.py::test_record_path_both_directions_bit_exact"]
    p = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    tail = (p.stdout + p.stderr)[-3000:]
    assert p.returncode == 0, tail
    assert " passed" in p.stdout and "skipped" not in p.stdout.splitlines()[-1], tail
