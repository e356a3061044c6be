"""Experiment: C2 seal/open kernel time against the alignment of the record
slots (the bench packs ct||tag byte-tight, so ciphertext records start at
16-byte multiples while plaintext records start at 64-byte multiples).

Usage (GPU box): python tools/c2_layout_probe.py [--records N]
Prints one JSON line per alignment: seal/open ms (HIP events on the launch
stream, mean of 10) and whether every record round-trips.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--aligns", default="16,64,128")
    args = ap.parse_args()
    import torch

    from suruga_amd import batch as B
    from suruga_amd import workloads as W

    dev = torch.device("cuda", 0)
    count = args.records
    lay = W.c2_layout(count)
    t64 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
    t32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)  # noqa: E731
    keys = torch.tensor(list(lay.keys), dtype=torch.uint8, device=dev).view(-1, 32)
    ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
    status = torch.empty(count, dtype=torch.uint8, device=dev)
    lens = lay.lens.astype(np.uint64)
    for al in [int(a) for a in args.aligns.split(",")]:
        slot = (lens + 16 + al - 1) // al * al
        out_off = np.zeros(count, dtype=np.uint64)
        out_off[1:] = np.cumsum(slot[:-1], dtype=np.uint64)
        ct_bytes = int(out_off[-1] + slot[-1])
        pt = torch.empty(lay.pt_bytes, dtype=torch.uint8, device=dev)
        ct = torch.empty(ct_bytes, dtype=torch.uint8, device=dev)
        back = torch.empty(lay.pt_bytes, dtype=torch.uint8, device=dev)
        B.fill_records(pt, 0, lay.pt_bytes, 1, 0x53555255)
        maxl = int(lay.lens.max())
        # device metadata held in variables: the C structs carry raw pointers
        d_lens, d_olens, d_in, d_out = t32(lay.lens), t32(lay.lens + 16), t64(lay.in_off), t64(out_off)
        d_kidx, d_seq = t32(lay.key_index), t64(lay.seq)
        sb = B.Batch(count=count, keys=keys, inp=pt, out=ct, lens=d_lens, max_len=maxl, in_off=d_in, out_off=d_out,
                     key_index=d_kidx, seq=d_seq, workspace=ws).to_c()
        ob = B.Batch(count=count, keys=keys, inp=ct, out=back, lens=d_olens, max_len=maxl + 16, in_off=d_out,
                     out_off=d_in, key_index=d_kidx, seq=d_seq, status=status, workspace=ws).to_c()
        import ctypes as C

        lib = B.N.load()
        for _ in range(3):
            B.N.check(lib.sg_seal_batch(C.byref(sb)))
            B.N.check(lib.sg_open_batch(C.byref(ob)))
        torch.cuda.synchronize()
        B.set_timing(True)
        for _ in range(10):
            B.N.check(lib.sg_seal_batch(C.byref(sb)))
            B.N.check(lib.sg_open_batch(C.byref(ob)))
        tm = B.timing_read()
        B.set_timing(False)
        torch.cuda.synchronize()
        ok = bool(torch.equal(pt, back)) and int((status != 0).sum().item()) == 0
        print(json.dumps({"ct_align": al, "seal_ms": round(tm["seal_ms"], 4), "open_ms": round(tm["open_ms"], 4),
                          "keying_ms": round(tm["keying_ms"], 4), "roundtrip": ok}), flush=True)
        del pt, ct, back


if __name__ == "__main__":
    main()
