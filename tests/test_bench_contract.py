"""bench.py's output contract and its multi-rank path.  CPU: argument parsing
only.  GPU: a small N=1 run and an N=2 run launched the way the driver launches
it (torch.distributed.run, 127.0.0.1), both ranks on the one card of the test
box with the gloo process group (RCCL needs one device per rank)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(out: str):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_help():
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--help"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "--gpus" in p.stdout and "--strong" in p.stdout


@pytest.mark.gpu
def test_bench_single_gpu_small(gpu):
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--records", "4096", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _last_json(p.stdout)
    assert KEYS <= set(j) and j["n_gpus"] == 1 and j["correct"] and j["value"] > 0
    assert set(j["roofline"]) >= {"bound", "achieved", "peak", "unit", "frac", "traffic"}


@pytest.mark.gpu
@pytest.mark.parametrize("strong", [False, True])
def test_bench_two_ranks_one_card(gpu, strong):
    env = dict(os.environ, SG_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"), "--gpus", "2",
           "--records", "4096", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"] + (["--strong"] if strong else [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _last_json(p.stdout)
    assert j["n_gpus"] == 2 and j["correct"] and j["scaling"] == ("strong" if strong else "weak")
    if strong:
        assert j["records_per_s"] * j["ms_per_step"] / 1e3 == pytest.approx(4096, rel=1e-3)
    else:
        assert j["records_per_s"] * j["ms_per_step"] / 1e3 == pytest.approx(8192, rel=1e-3)
    # root scatter -> per-rank seal -> root gather, timed apart and verified (north star: RCCL over xGMI
    # only to scatter inputs / gather outputs; gloo through host memory in this one-card rehearsal)
    sg = j["scatter_gather"]
    assert sg["verified"] and sg["records_per_rank"] == (2048 if strong else 4096)
    assert sg["scatter_ms"] > 0 and sg["gather_ms"] > 0


def test_bench_rejects_gpus_world_size_mismatch():
    """A launcher's WORLD_SIZE that differs from --gpus is an error, not a
    silently smaller run (CPU: fails before any GPU call)."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=3" in (p.stderr + p.stdout)


@pytest.mark.gpu
def test_bench_gpus_two_launches_its_own_ranks(gpu):
    """`bench.py --gpus 2` with no launcher starts both ranks itself (the form the
    driver uses), both on the test box's one card with the gloo group."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["SG_DIST_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--records", "4096", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline"], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _last_json(p.stdout)
    assert j["n_gpus"] == 2 and j["correct"] and j["scaling"] == "weak"
    assert j["records_per_s"] * j["ms_per_step"] / 1e3 == pytest.approx(8192, rel=1e-3)
    assert j["scatter_gather"]["verified"]
