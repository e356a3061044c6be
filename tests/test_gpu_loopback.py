"""C4 on the GPU: an application stream through sg_write_records, a loopback
TCP connection and sg_read_records (tools/tls_loopback.py, the TlsWriter /
TlsReader data path of tls.rs:126-147 and :238-281 with the handshake
bypassed as in src/test.rs:29-39).  Every wire byte the writer sent is
compared with the oracle's TLS sealing of the same records (header, ct, tag:
chacha20_poly1305.rs:48-59, tls.rs:103-112), and every byte the reader
delivered with the stream that went in, at 64 MiB and at C4's full 1 GiB.
Also the copy-inclusive record path per direction and duplex
(tools/record_path_bench.py) at a reduced size.
"""
from __future__ import annotations

import struct
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

KEY_C2S = bytes(range(32))
REC = 1 << 14


@pytest.mark.parametrize("total", [64 << 20, 1 << 30], ids=["64MiB", "1GiB"])
def test_loopback_wire_equals_oracle(gpu, oracle, total):
    """64 MiB, and C4's full 1 GiB stream (BASELINE.json configs[4]): every
    wire record against the oracle, every delivered byte against the input."""
    import tls_loopback as TL

    wchunk = 16 << 20
    res = TL.run(total, wchunk, 0, capture=True)
    assert res["correct"], {k: v for k, v in res.items() if k != "wire"}
    assert res["reader"]["bytes"] == total and res["reader"]["mismatched_bytes"] == 0
    wire = res["wire"]
    nrec = total // REC
    assert res["writer"]["records"] == nrec and len(wire) == nrec * (5 + REC + 16)
    stream = np.tile(TL.stream_pattern(wchunk), total // wchunk)
    expect = oracle.seal_batch_tls(KEY_C2S, 0, stream.tobytes(), REC, nrec, threads=16)
    w = np.frombuffer(wire, dtype=np.uint8).reshape(nrec, 5 + REC + 16)
    hdr = bytes([23, 3, 3]) + struct.pack(">H", REC + 16)
    assert (w[:, :5] == np.frombuffer(hdr, dtype=np.uint8)).all()
    body = np.frombuffer(expect, dtype=np.uint8).reshape(nrec, REC + 16)
    bad = np.nonzero((w[:, 5:] != body).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} records differ from the oracle, first {bad[:8]}"


def test_record_path_both_directions_bit_exact(gpu):
    import record_path_bench as RP

    for registered in (False, True):
        r = RP.one(32 << 20, 8 << 20, 0, registered)
        assert r["correct"], r
        assert r["records"] == (32 << 20) // REC
        # a writer and a reader on two contexts at once: both outputs bit-exact
        assert r["duplex"]["correct"] and not r["duplex"]["errors"], r["duplex"]


@pytest.mark.parametrize("total", [64 << 20, 1 << 30], ids=["64MiB", "1GiB"])
@pytest.mark.parametrize("registered", [False, True])
def test_cpp_loopback_every_byte(gpu, registered, total):
    """tools/loopback_cpp (C4 in C++ over include/suruga, no Python on the data
    path): 64 MiB and C4's full 1 GiB over a loopback socket, staged and
    zero-copy (registered buffers); the harness compares every delivered byte
    with the stream."""
    import json
    import subprocess

    from suruga_amd import _build

    exe = _build.build_loopback_cpp()
    args = [str(exe), "--bytes", str(total), "--chunk", str(8 << 20), "--block", str(8 << 20)]
    p = subprocess.run(args + (["--registered"] if registered else []), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    j = json.loads(p.stdout.strip().splitlines()[-1])
    assert j["correct"] and j["registered"] is registered
    assert j["reader"]["bytes"] == total and j["reader"]["mismatched_bytes"] == 0
    assert j["writer"]["records"] == total // REC == j["reader"]["records"]
