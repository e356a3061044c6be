"""Multi-rank path on the GPU (tls.rs:132,278: the only
cross-record state is the sequence number, known up front).

1. World 2 (gloo group, both ranks on the test box's one card): each rank
   seals its own contiguous record range with sg_seal_batch (seq = lo + i), no
   data-path collective; the XOR of the per-rank tag folds equals the oracle's
   fold over the whole range.
2. World 1 with the nccl (RCCL) backend: scatter_records / gather_records of
   device tensors round-trip, so an RCCL process group has been created and
   used before an 8-GPU node runs bench.py.
"""
from __future__ import annotations

import os
import socket

import pytest

pytestmark = pytest.mark.gpu

KEY = bytes(range(32))
SEED = 0x53555255
N, TOTAL = 16384, 8192


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fold_worker(rank, world, port, q):
    import ctypes as C

    import numpy as np
    import torch
    import torch.distributed as dist

    from suruga_amd import batch as B
    from suruga_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        lo, hi = shard.record_range(TOTAL, rank, world)
        count = hi - lo
        keys = torch.tensor(list(KEY), dtype=torch.uint8, device=dev).view(1, 32)
        pt = torch.empty(count * N, dtype=torch.uint8, device=dev)
        ct = torch.empty(count * (N + 16), dtype=torch.uint8, device=dev)
        ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
        B.fill_records(pt, N, N, count, SEED, j0=lo)
        b = B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=N, in_stride=N, out_stride=N + 16, seq0=lo,
                    workspace=ws, stream=torch.cuda.current_stream(dev)).to_c()
        lib = B.N.load()
        B.N.check(lib.sg_seal_batch(C.byref(b)))
        torch.cuda.synchronize()
        tags = ct.view(count, N + 16)[:, N:].cpu().numpy()
        fold = np.bitwise_xor.reduce(tags, axis=0)
        folds = [torch.zeros(16, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(folds, torch.from_numpy(fold.copy()))
        total = np.zeros(16, dtype=np.uint8)
        for f in folds:
            total ^= f.numpy()
        if rank == 0:
            q.put(bytes(total))
    finally:
        dist.destroy_process_group()


def test_two_ranks_hip_tag_fold(gpu, oracle):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_fold_worker, args=(2, _free_port(), q), nprocs=2, join=True, start_method="spawn")
    got = q.get()
    expect = oracle.tag_fold_tls(KEY, 0, SEED, 0, N, TOTAL, threads=16)
    assert got == expect


def _nccl_worker(rank, world, port):
    import torch
    import torch.distributed as dist

    from suruga_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        g = torch.Generator(device="cpu").manual_seed(5)
        src = torch.randint(0, 256, (world * 4096,), dtype=torch.uint8, generator=g).to(dev)
        chunks = list(src.chunk(world))
        mine = torch.empty(4096, dtype=torch.uint8, device=dev)
        shard.scatter_records(dist, 0, mine, chunks)
        torch.cuda.synchronize()
        assert torch.equal(mine, chunks[rank])
        back = [torch.empty(4096, dtype=torch.uint8, device=dev) for _ in range(world)]
        shard.gather_records(dist, 0, mine, back)
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(back), src)
        assert shard.max_over_ranks(dist, 3.5, device=dev) == 3.5
    finally:
        dist.destroy_process_group()


def test_world1_nccl_scatter_gather(gpu):
    import torch.multiprocessing as mp

    mp.start_processes(_nccl_worker, args=(1, _free_port()), nprocs=1, join=True, start_method="spawn")
