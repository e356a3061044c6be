"""Multi-rank path on CPU with gloo, world_size 2 and 4: each rank
seals its own contiguous record range (sequence numbers lo..hi-1, no data-path
collective), the union over ranks equals the single-process result, and the
benchmark's timing protocol (barrier + MAX over ranks, suruga_amd.shard.timed)
agrees on every rank.  The per-rank compute here is the oracle on CPU; the GPU
path is the same record range handed to sg_seal_batch (bench.py)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from suruga_amd import shard
from suruga_amd.workloads import zipf_lengths

KEY = bytes(range(32))
TOTAL, N = 37, 300


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fold(oracle, lo, hi):
    acc = bytearray(16)
    for i in range(lo, hi):
        pt = oracle.fill_record(0x53555255, i, N)
        ct = oracle.seal(KEY, i.to_bytes(8, "big"), pt, oracle.tls_ad(i, N))
        for k in range(16):
            acc[k] ^= ct[N + k]
    return bytes(acc)


def _worker(rank, world, port, expect_fold):
    import torch

    from oracle_ffi import oracle as get_oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard.record_range(TOTAL, rank, world)
        o = get_oracle()
        mine = {}
        elapsed = shard.timed(dist, lambda: mine.__setitem__("fold", _fold(o, lo, hi)), 1)
        folds = [torch.zeros(16, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(folds, torch.tensor(list(mine["fold"]), dtype=torch.uint8))
        total = bytearray(16)
        for f in folds:
            for k in range(16):
                total[k] ^= int(f[k])
        assert bytes(total) == expect_fold
        ranges = [None] * world
        dist.all_gather_object(ranges, (lo, hi))
        assert ranges[0][0] == 0 and ranges[-1][1] == TOTAL
        assert all(ranges[r][1] == ranges[r + 1][0] for r in range(world - 1))
        times = [None] * world
        dist.all_gather_object(times, elapsed)
        assert len(set(times)) == 1  # every rank reports the same MAX
        assert shard.max_over_ranks(dist, float(rank)) == world - 1
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_shard_records_gloo(oracle, world):
    expect = _fold(oracle, 0, TOTAL)
    mp.spawn(_worker, args=(world, _free_port(), expect), nprocs=world, join=True)


def test_record_range_partitions():
    for total in (0, 1, 7, 1 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard.record_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1
            assert all(rs[r][1] == rs[r + 1][0] for r in range(world - 1))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_byte_balanced_ranges_c2(world):
    lens = zipf_lengths(1 << 14)
    rs = shard.byte_balanced_ranges(lens, world)
    assert rs[0][0] == 0 and rs[-1][1] == len(lens)
    total = int(np.sum(lens))
    for lo, hi in rs:
        assert abs(int(np.sum(lens[lo:hi])) - total / world) <= 16384


def _sg_worker(rank, world, port):
    """Root rank 0 scatters every rank's plaintext records, each rank seals its
    slice (oracle on CPU here, sg_seal_batch in bench.py), rank 0 gathers the
    sealed records: the bytes that come back equal a single-process seal."""
    import torch

    from oracle_ffi import oracle as get_oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = get_oracle()
        per = 3
        rec = lambda i: o.fill_record(0x53555255, i, N)  # noqa: E731
        as_t = lambda b: torch.tensor(list(b), dtype=torch.uint8)  # noqa: E731
        chunks = [as_t(b"".join(rec(r * per + j) for j in range(per))) for r in range(world)] if rank == 0 else None
        mine = torch.empty(per * N, dtype=torch.uint8)
        shard.timed_collective(dist, lambda: shard.scatter_records(dist, 0, mine, chunks), reps=2)
        assert bytes(mine.numpy()) == b"".join(rec(rank * per + j) for j in range(per))
        sealed = b""
        for j in range(per):
            i = rank * per + j
            sealed += o.seal(KEY, i.to_bytes(8, "big"), bytes(mine.numpy())[j * N:(j + 1) * N], o.tls_ad(i, N))
        back = [torch.empty(per * (N + 16), dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
        shard.gather_records(dist, 0, as_t(sealed), back)
        if rank == 0:
            got = b"".join(bytes(t.numpy()) for t in back)
            exp = b"".join(o.seal(KEY, i.to_bytes(8, "big"), rec(i), o.tls_ad(i, N)) for i in range(world * per))
            assert got == exp
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_scatter_seal_gather_gloo(world):
    mp.spawn(_sg_worker, args=(world, _free_port()), nprocs=world, join=True)
