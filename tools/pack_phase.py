#!/usr/bin/env python3
"""Where does a C2 launch of sg_pack_kernel spend its time?

Seals the C2 workload (Zipf 64 B-16 KiB, 256 keys) through an experiment build
compiled with -DSG_PACK_PROFILE=1 (same output; waves 0 and 7 of each
workgroup stamp s_memtime at the phase boundaries) and prints the average
phase lengths in clock ticks.  Build the variant on the CPU first:

    python -c "from pathlib import Path; from suruga_amd import _build; \\
_build.build_library(out=Path('tools/exp/lib_pack_prof.so'), defines=['-DSG_PACK_PROFILE=1'])"
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("SURUGA_GPU_LIB", str(ROOT / "tools" / "exp" / "lib_pack_prof.so"))


def main():
    import torch
    from suruga_amd import batch as B
    from suruga_amd import workloads as W
    from suruga_amd import _native as N

    lib = N.load()
    count = 1 << 20
    lay = W.c2_layout(count)
    t64 = lambda a: torch.from_numpy(a.view(np.int64)).to("cuda")
    t32 = lambda a: torch.from_numpy(a.view(np.int32)).to("cuda")
    pt = torch.empty(lay.pt_bytes, dtype=torch.uint8, device="cuda")
    ct = torch.empty(lay.ct_bytes, dtype=torch.uint8, device="cuda")
    keys = torch.frombuffer(bytearray(lay.keys), dtype=torch.uint8).to("cuda").view(-1, 32)
    b = B.Batch(count=count, keys=keys, inp=pt, out=ct, lens=t32(lay.lens), max_len=int(lay.lens.max()),
                in_off=t64(lay.in_off), out_off=t64(lay.out_off), key_index=t32(lay.key_index), seq=t64(lay.seq))
    for _ in range(3):
        B.seal(b)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (8192 * 16))()
    n = lib.sg_pack_profile_read(buf, len(buf))
    assert n > 0, n
    cols = n // 8192  # 12 stamps, 16 with the round sums of tools/archive/variants/pk_prof2.py
    a = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(8192, cols).astype(np.int64)
    a = a[a[:, 0] != 0]
    d = lambda i, j: float(np.mean(a[:, j] - a[:, i]))
    print(f"workgroups {len(a)}  (s_memtime ticks)")
    print(f"  setup: zero + loads                  {d(0, 8):9.0f}")
    print(f"  setup: block 0                       {d(8, 9):9.0f}")
    print(f"  setup: slot + tables                 {d(9, 10):9.0f}")
    print(f"  setup: constant term + scan          {d(10, 1):9.0f}")
    print(f"  setup (wave 0: zero, scan, keying)   {d(0, 1):9.0f}")
    print(f"  setup syncs + base scan              {d(1, 2):9.0f}")
    print(f"  rounds wave 0                        {d(2, 3):9.0f}")
    print(f"  rounds wave 7                        {d(6, 7):9.0f}")
    print(f"  wait for the last wave               {d(3, 4):9.0f}")
    print(f"  finish                               {d(4, 5):9.0f}")
    print(f"  whole workgroup                      {d(0, 5):9.0f}")
    if cols >= 16:
        nr = float(np.mean(a[:, 15]))
        print(f"  wave 0's rounds with a chunk         {nr:9.2f}")
        for j, what in ((12, "before the asm (loads, lookup)"), (13, "ChaCha20 asm (with barriers)"),
                        (14, "after (FF, XOR, stores, MAC)")):
            print(f"    per round: {what:31s} {float(np.mean(a[:, j])) / nr:9.0f}")


if __name__ == "__main__":
    main()
