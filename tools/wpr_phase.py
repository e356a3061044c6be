#!/usr/bin/env python3
"""Where does a C1 launch of sg_wpr_kernel spend its time?

Runs the C1 workload (2^20 x 16 KiB TLS records, seal then open) through an
experiment build of the library compiled with -DSG_WPR_PROFILE=1 (same output;
every wave accumulates s_memtime deltas per phase) and prints, per kernel, the
share of each phase in the waves' lifetime.  Build the variant on the CPU first:

    python -c "from pathlib import Path; from suruga_amd import _build; \
_build.build_library(out=Path('tools/libsuruga_gpu_prof.so'), defines=['-DSG_WPR_PROFILE=1'])"

then on the GPU box:  python tools/wpr_phase.py [--json-out gpurun_out/phase.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

PHASES = ["table_wait", "prologue", "chunk_wait", "rounds_mac", "xor_stage_store", "life", "records", "epilogue",
          "realtime", "spare"]
NW, NP = 4096, 10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=str(ROOT / "tools" / "libsuruga_gpu_prof.so"))
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--json-out")
    ap.add_argument("--no-check", action="store_true", help="timing experiments with wrong tags")
    a = ap.parse_args()
    os.environ["SURUGA_GPU_LIB"] = a.lib
    os.environ.setdefault("SURUGA_ALLOW_VARIANT", "1")  # a -D build carries a variant marker (_build)
    import torch

    from suruga_amd import batch as B

    lib = B.N.load()
    if not hasattr(lib, "sg_wpr_profile_read"):  # the product library: just run the launches (for rocprofv3)
        rd = lambda buf, n: NW * NP
        prof = False
    else:
        rd = lib.sg_wpr_profile_read
        rd.argtypes, rd.restype = [C.c_void_p, C.c_size_t], C.c_int
        prof = True
    buf = (C.c_ulonglong * (NW * NP))()
    dev = torch.device("cuda", 0)
    n, count = 16384, a.records
    stream = torch.cuda.current_stream(dev)
    ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
    status = torch.empty(count, dtype=torch.uint8, device=dev)
    key = bytes(range(32))
    keys = torch.tensor(list(key), dtype=torch.uint8, device=dev).view(1, 32)
    pt = torch.empty(count * n, dtype=torch.uint8, device=dev)
    ct = torch.empty(count * (n + 16), dtype=torch.uint8, device=dev)
    back = torch.empty(count * n, dtype=torch.uint8, device=dev)
    B.fill_records(pt, n, n, count, 7, j0=0)
    seal = B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=n + 16, seq0=0,
                   workspace=ws, stream=stream).to_c()
    opn = B.Batch(count=count, keys=keys, inp=ct, out=back, uniform_len=n + 16, in_stride=n + 16, out_stride=n,
                  seq0=0, status=status, workspace=ws, stream=stream).to_c()
    out = {}
    for name, fn, c in (("seal", lib.sg_seal_batch, seal), ("open", lib.sg_open_batch, opn)):
        for _ in range(2):  # warm-up launch, then the measured one
            rd(buf, NW * NP)
            B.N.check(fn(C.byref(c)))
            torch.cuda.synchronize()
        got = rd(buf, NW * NP)
        assert got == NW * NP, got
        if not prof:
            continue
        rows = [buf[w * NP:(w + 1) * NP] for w in range(NW)]
        rows = [r for r in rows if r[5] > 0]
        tot = [sum(r[k] for r in rows) for k in range(NP)]
        life = tot[5]
        res = {"waves": len(rows), "records_per_wave": tot[6] / len(rows),
               "life_cycles_mean": life / len(rows)}
        for k, ph in enumerate(PHASES):
            if ph in ("life", "records", "realtime", "spare"):
                continue
            res[ph] = round(tot[k] / life, 4)
        res["clock_ghz"] = round(tot[5] / tot[8] * 0.1, 3)  # s_memtime ticks per 100 MHz realtime tick
        t0 = min(r[9] for r in rows)
        starts = [(r[9] - t0) / 100.0 for r in rows]  # us
        ends = [(r[9] + r[8] - t0) / 100.0 for r in rows]
        res["wave_start_us"] = {"max": round(max(starts), 1), "mean": round(sum(starts) / len(starts), 1)}
        res["wave_end_us"] = {"min": round(min(ends), 1), "mean": round(sum(ends) / len(ends), 1),
                              "max": round(max(ends), 1)}
        # by XCD (workgroup b runs on XCD b % 8) and by workgroup-of-the-pair (b // 8 parity)
        allrows = [buf[w * NP:(w + 1) * NP] for w in range(NW)]
        by = {}
        for w, r in enumerate(allrows):
            if r[5] == 0:
                continue
            b = w // 8
            e = (r[9] + r[8] - t0) / 100.0
            by.setdefault(("xcd", b % 8), []).append(e)
            by.setdefault(("half", (b // 256)), []).append(e)
        res["end_by_group_us"] = {f"{k[0]}{k[1]}": [round(min(v)), round(sum(v) / len(v)), round(max(v))]
                                  for k, v in sorted(by.items())}
        res["unaccounted"] = round(1 - sum(res[p] for p in PHASES if p in res), 4)
        # per record-group cycles (all waves run the same number of groups)
        res["cycles_per_group"] = {p: round(tot[k] / tot[6]) for k, p in enumerate(PHASES)
                                   if p not in ("life", "records", "realtime", "spare")}
        out[name] = res
    torch.cuda.synchronize()
    print(json.dumps(out, indent=1))
    if not a.no_check:
        assert int((status != 0).sum().item()) == 0
        assert torch.equal(pt, back)
    if a.json_out:
        Path(a.json_out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
