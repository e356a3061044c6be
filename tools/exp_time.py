#!/usr/bin/env python3
"""Time seal/open of C1-shaped batches for the library named by
SURUGA_GPU_LIB (experiment builds, see sg_kernels.hip SG_EXP) or the product.
Prints one JSON line: per-launch device ms from HIP events on the launch stream."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from suruga_amd import batch as B  # noqa: E402


def main(count=1 << 20, n=16384, reps=5):
    dev = torch.device("cuda", 0)
    keys = torch.arange(32, dtype=torch.uint8, device=dev).view(1, 32)
    pt = torch.empty(count * n, dtype=torch.uint8, device=dev)
    ct = torch.empty(count * (n + 16), dtype=torch.uint8, device=dev)
    back = torch.empty(count * n, dtype=torch.uint8, device=dev)
    st = torch.empty(count, dtype=torch.uint8, device=dev)
    ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
    B.fill_records(pt, n, n, count, 1)
    s = B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=n + 16, workspace=ws).to_c()
    o = B.Batch(count=count, keys=keys, inp=ct, out=back, uniform_len=n + 16, in_stride=n + 16, out_stride=n,
                status=st, workspace=ws).to_c()
    lib = B.N.load()
    for _ in range(2):
        B.N.check(lib.sg_seal_batch(C.byref(s)))
        B.N.check(lib.sg_open_batch(C.byref(o)))
    torch.cuda.synchronize()
    B.set_timing(True)
    for _ in range(reps):
        B.N.check(lib.sg_seal_batch(C.byref(s)))
        B.N.check(lib.sg_open_batch(C.byref(o)))
    tm = B.timing_read()
    B.set_timing(False)
    print(json.dumps({"lib": os.environ.get("SURUGA_GPU_LIB", "product"), "build": lib.sg_build_info().decode()[-60:],
                      "count": count, "n": n, "seal_ms": round(tm["seal_ms"], 4), "open_ms": round(tm["open_ms"], 4),
                      "keying_ms": round(tm["keying_ms"], 4)}), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
