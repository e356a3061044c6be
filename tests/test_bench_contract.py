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
                        "--no-cpu-baseline", "--record-path-bytes", str(24 << 20)], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _last_json(p.stdout)
    assert KEYS <= set(j) and j["n_gpus"] == 1 and j["correct"] and j["value"] > 0
    # the copy-inclusive record path: pageable and registered
    # buffers, each one direction at a time and duplex, every byte verified and a
    # sample of the wire against the oracle
    rp = j["record_path"]
    assert rp["correct"] and rp["bytes"] == 24 << 20
    for mode in ("pageable", "registered"):
        r = rp[mode]
        assert r["correct"] and r["wire_sample_ok"] and r["duplex"]["correct"] and r["registered"] == (mode == "registered")
        assert r["write_gibs"] > 0 and r["read_gibs"] > 0 and r["duplex"]["gibs"] > 0
        assert set(r["write_split"]) == {"h2d_ms_per_gib", "kernel_ms_per_gib", "d2h_ms_per_gib", "host_ms_per_gib"}
    assert set(j["roofline"]) >= {"bound", "achieved", "peak", "unit", "frac", "traffic"}
    # the C2 sub-record (BASELINE configs[2]) under the same protocol, checked against the oracle
    c2 = j["c2"]
    assert c2["correct"] and c2["bitexact_fold"] and c2["bitexact_sample"] and c2["value"] > 0
    assert c2["steps"] == 60 and set(c2["roofline"]) >= {"achieved", "frac", "traffic"}
    assert c2["config"]["record_bytes"] == "zipf" and c2["config"]["records_per_gpu"] == 4096
    # energy per record over the energy window (board power x event-timed launch time / records)
    e = j["energy"]
    if "unavailable" not in e:
        assert j["energy_per_record_uj"] == e["energy_per_record_uj"] > 0
        assert e["board_power_w"] > 0 and e["seal_uj_per_record"] > 0 and e["open_uj_per_record"] > 0


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


def _verdict_worker(rank, world, port, q):
    """Each rank seals its records with the oracle (standing in for the GPU),
    checks the XOR-fold of its tags against the oracle's fold as bench.py does;
    rank 1 corrupts one tag first.  bench.rank_verdict ANDs the ranks."""
    import torch.distributed as dist

    sys.path.insert(0, str(ROOT))
    import bench
    from oracle_ffi import oracle as get_oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o, n, key = get_oracle(), 256, bytes(range(32))
        tags = []
        for i in range(rank * 4, rank * 4 + 4):
            ct = o.seal(key, i.to_bytes(8, "big"), o.fill_record(0x53555255, i, n), o.tls_ad(i, n))
            tags.append(bytearray(ct[n:]))
        if rank == 1:
            tags[2][5] ^= 0x01  # one corrupted tag on rank 1
        fold = bytes(a ^ b ^ c ^ d for a, b, c, d in zip(*tags))
        exact = {"bitexact_fold": fold == o.tag_fold_tls(key, rank * 4, 0x53555255, rank * 4, n, 4, 1),
                 "bitexact_sample": True}
        mine = {"rank": rank, "local_rank": rank, "device": 0, "roundtrip_ok": True, **exact}
        correct, ranks, flags = bench.rank_verdict(dist, mine)
        line = bench.correctness_fields(correct, ranks, flags, exact) if rank == 0 else None
        q.put((rank, line, bench.exit_code(correct)))
    finally:
        dist.destroy_process_group()


def test_bench_correct_is_and_over_ranks_gloo():
    """a corrupted tag on rank 1 makes rank 0's line say
    "correct": false (and that rank's flag false), and every rank exits 3."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_verdict_worker, args=(2, _port(), q), nprocs=2, join=True, start_method="spawn")
    res = {r: (line, rc) for r, line, rc in (q.get(timeout=60) for _ in range(2))}
    line, rc0 = res[0]
    assert line["correct"] is False and line["bitexact_fold"] is False
    assert [r["bitexact_fold"] for r in line["ranks"]] == [True, False]
    assert rc0 == 3 and res[1][1] == 3


@pytest.mark.gpu
def test_bench_failing_rank_fails_the_line(gpu):
    """The real bench path: two gloo ranks on the test box's card, rank 1's
    bit-exactness check forced to fail (SG_BENCH_CORRUPT_RANK=1): rank 0 prints
    "correct": false and the run exits non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(SG_DIST_BACKEND="gloo", SG_BENCH_CORRUPT_RANK="1")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--records", "4096", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--sg-records", "0"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, env=env)
    assert p.returncode != 0
    j = _last_json(p.stdout)
    assert j["correct"] is False and j["bitexact_fold"] is False
    assert [r["rank"] for r in j["ranks"]] == [0, 1] and j["ranks"][0]["bitexact_fold"] is True


@pytest.mark.gpu
def test_bench_local_rank_maps_to_visible_device(gpu):
    """LOCAL_RANK=1 on a one-GPU box runs on device 1 mod 1 = 0, and the line
    names the device each rank used."""
    import torch

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    env["LOCAL_RANK"] = "1"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--records", "4096", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--record-path-bytes", "0"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _last_json(p.stdout)
    nd = torch.cuda.device_count()
    assert j["correct"] and j["ranks"][0]["local_rank"] == 1 and j["ranks"][0]["device"] == 1 % nd


@pytest.mark.gpu
def test_bench_c2_two_ranks_scatter_gather(gpu):
    """--workload c2 at N=2 (gloo, one card): the byte-balanced scatter ->
    per-rank mixed seal -> gather round trip is timed and verified."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["SG_DIST_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--workload", "c2", "--records", "8192",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--sg-records", "1024"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _last_json(p.stdout)
    sg = j["scatter_gather"]
    assert j["correct"] and sg["verified"] and sg["split"] == "byte_balanced_ranges" and sg["records"] == 2048
    assert sg["ranges"][0][0] == 0 and sg["ranges"][-1][1] == 2048


@pytest.mark.gpu
def test_bench_two_real_devices(gpu):
    """with two or more GPUs visible, `bench.py --gpus 2`
    runs its ranks on two different cards (distinct PCI addresses) over RCCL
    and the line is correct.  Skipped on a one-GPU box."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                                                            "SG_DIST_BACKEND")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--records", "4096", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--c2-steps", "0", "--energy-seconds", "0"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    j = _last_json(p.stdout)
    assert j["n_gpus"] == 2 and j["correct"]
    assert [r["device"] for r in j["ranks"]] == [0, 1]
    assert len({r["pci_bus"] for r in j["ranks"]}) == 2


def test_energy_fields():
    """energy_per_record_uj = mean board power of the window's second half x
    the dominant launch's event time / records; reported as unavailable without
    a power reading."""
    sys.path.insert(0, str(ROOT))
    import bench

    tm = {"seal_ms": 7.2, "open_ms": 7.3, "keying_ms": 0.13, "n_seal": 100}
    mon = {"board_power_w": {"mean": 1400.0}, "sclk_mhz": {"mean": 1850.0}, "window_s": 2.0}
    e = bench.energy_fields(mon, tm, 1 << 20, "open")
    assert e["energy_per_record_uj"] == pytest.approx(1400.0 * 7.3e-3 / (1 << 20) * 1e6, rel=1e-3)
    assert e["seal_uj_per_record"] == pytest.approx(1400.0 * 7.2e-3 / (1 << 20) * 1e6, rel=1e-3)
    assert "unavailable" in bench.energy_fields({"board_power_w": None}, tm, 1 << 20, "open")


def test_issue_roofline_model():
    """valu_roofline: the ARX stream at 2 / 4 clocks per
    add-xor / rotate, the other VALU split by the census's full-rate share,
    priced at the sampled clock; C2 prices each kernel's PMC VALU with its
    census mix; missing inputs are reported, not guessed."""
    sys.path.insert(0, str(ROOT))
    import bench

    name = "void sg::(anonymous namespace)::sg_wpr_kernel<false, true, 4u, false>(sg::KParams, sg::WprList)"
    isa = {"model": "m", "kernels": {name: {"arx_full": 2448, "arx_rot": 1228, "other_valu": 672, "other_full": 336,
                                            "valu": 4348, "clk_per_valu": 2.72, "clk_per_valu_whole": 2.72}}}
    tj = {"seal_valu_per_record": 4320.0}
    r = bench.issue_roofline("seal", "c1", 1 << 20, 256, 7.25, tj, isa, 1750.0)
    clk = 2 * 2448 + 4 * 1228 + (4320 - 3676) * (2 * 0.5 + 4 * 0.5)
    assert r["issue_clk_per_record"] == pytest.approx(clk, abs=0.1)
    assert r["issue_bound_ms"] == pytest.approx(clk * 1024 / 1750e3, rel=1e-3)
    assert r["frac"] == pytest.approx(r["issue_bound_ms"] / 7.25, rel=1e-3)
    tj2 = {"seal_valu_by_kernel": {name: 1.0e9}}
    r2 = bench.issue_roofline("seal", "c2", 1 << 20, 256, 1.3, tj2, isa, 2200.0)
    assert r2["issue_bound_ms"] == pytest.approx(1.0e9 * 2.72 / 1024 / 2200e3, rel=1e-3)
    assert "unavailable" in bench.issue_roofline("seal", "c1", 1 << 20, 256, 7.25, tj, None, 1750.0)
    assert "unavailable" in bench.issue_roofline("seal", "c1", 1 << 20, 256, 7.25, tj, isa, None)
