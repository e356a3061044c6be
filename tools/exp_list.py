#!/usr/bin/env python3
"""Experiment: direct vs list-driven (bucketed) launches on identical records.

Times sg_seal_batch for N records of n bytes (a) with uniform_len (direct
launch of the record's size class) and (b) with a lens[] array (classify +
list kernel), to separate the list kernel's scheduling cost from the
per-byte cost of the size class.  Prints one JSON line per case."""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from suruga_amd import batch as B  # noqa: E402


def run(count, n, use_lens, reps=5):
    dev = torch.device("cuda", 0)
    keys = torch.arange(32, dtype=torch.uint8, device=dev).view(1, 32)
    pt = torch.empty(count * n, dtype=torch.uint8, device=dev)
    ct = torch.empty(count * (n + 16), dtype=torch.uint8, device=dev)
    B.fill_records(pt, n, n, count, 1)
    ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
    kw = dict(count=count, keys=keys, inp=pt, out=ct, in_stride=n, out_stride=n + 16, workspace=ws)
    if use_lens:
        lens = torch.full((count,), n, dtype=torch.int32, device=dev)
        b = B.Batch(lens=lens, max_len=n, **kw)
    else:
        b = B.Batch(uniform_len=n, **kw)
    c = b.to_c()
    lib = B.N.load()
    for _ in range(2):
        B.N.check(lib.sg_seal_batch(C.byref(c)))
    torch.cuda.synchronize()
    B.set_timing(True)
    for _ in range(reps):
        B.N.check(lib.sg_seal_batch(C.byref(c)))
    tm = B.timing_read()
    B.set_timing(False)
    ms = tm["seal_ms"]
    print(json.dumps({"count": count, "n": n, "path": "list" if use_lens else "direct", "seal_ms": round(ms, 4),
                      "GBps_payload": round(count * n / ms / 1e6, 1)}), flush=True)
    del pt, ct, ws
    torch.cuda.empty_cache()


if __name__ == "__main__":
    for count, n in [(1 << 20, 16384), (1 << 20, 12288), (1 << 19, 8192), (1 << 19, 6144), (1 << 20, 4096),
                     (1 << 20, 2048), (1 << 20, 1024), (1 << 21, 512), (1 << 21, 256), (1 << 21, 128), (1 << 21, 64)]:
        for use_lens in (False, True):
            run(count, n, use_lens)
