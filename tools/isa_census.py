#!/usr/bin/env python3
"""Static ISA census of every product kernel -> profiles/isa_<source hash>.json.

Compiles the three HIP sources with the product flags and --save-temps (CPU
only, hipcc cross-compiles gfx950), then runs tools/isa_count.py's census on
each kernel: its record loop (the body between the loop header and its
back-edge) for the persistent kernels, otherwise the whole function.  Per
kernel (rocprofv3's demangled name):

  arx_full / arx_rot   VALU inside the generated double-round asm
                       (v_add/v_xor pair at 2 clocks in lock-step, v_alignbit
                       at 4: profiles/r01_valu_issue_probes.md)
  other_valu           every other VALU of the census (static, all paths),
                       split into other_full (full-rate opcodes: add, xor,
                       and, or, mov, right shifts, bitop3) and other_half
  mfma, lds, vmem, salu
  clk_per_valu         the issue model's clocks per VALU instruction of this
                       mix: full-rate opcodes 2 (paired with the SIMD's other
                       lock-step wave, as the FF A/B of profiles/r04_ab shows
                       outside the asm too), every other VALU 4

bench.py prices the PMC-counted dynamic VALU of a launch with clk_per_valu
(valu_roofline), and DESIGN.md §4.2's ISA table is this file's C1 entry.
Usage: python tools/isa_census.py [--keep DIR]
"""
from __future__ import annotations

import json
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import isa_count as ic  # noqa: E402

from suruga_amd import _build  # noqa: E402

FULL = ic.FULL


def demangle(names):
    p = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
    return p.stdout.splitlines()


def census_file(path: Path):
    lines = path.read_text().splitlines()
    names = [l[:-1].split(":")[0] for l in lines if l.startswith("_Z") and l.rstrip().endswith(":") is False
             and ":" in l and "sg_" in l.split(":")[0]]
    names = []
    for l in lines:
        if l.startswith("_Z") and ":" in l:
            nm = l.split(":")[0]
            if "_kernel" in nm and nm not in names:
                names.append(nm)
    out = {}
    for mangled, dem in zip(names, demangle(names)):
        body_all = ic.kernel_lines(str(path), mangled)
        body = ic.loop_body(body_all)
        looped = len(body) != len(body_all)
        arx, other, kinds, _ = ic.census(body)
        af = sum(v for k, v in arx.items() if k in FULL)
        ar = sum(arx.values()) - af
        oth = sum(other.values())
        oth_full = sum(v for k, v in other.items() if k.split("_e32")[0].split("_e64")[0] in FULL)
        tot = af + ar + oth
        out[dem] = {"scope": "record loop" if looped else "whole kernel", "arx_full": af, "arx_rot": ar,
                    "other_valu": oth, "other_full": oth_full, "other_half": oth - oth_full, "valu": tot,
                    "mfma": kinds.get("mfma", 0), "lds": kinds.get("lds", 0),
                    "vmem": kinds.get("vmem", 0), "salu": kinds.get("salu", 0),
                    "clk_per_valu": round((2 * (af + oth_full) + 4 * (ar + oth - oth_full)) / tot, 4) if tot else None,
                    "other_by_op": dict(other.most_common(16))}
        # the whole function's mix (setup and tails included): what bench.py
        # prices a kernel's PMC-counted VALU with (a loop region of a kernel
        # with a complex CFG need not hold all of its per-iteration code)
        warx, woth, _, _ = ic.census(body_all)
        waf = sum(v for k, v in warx.items() if k in FULL)
        war = sum(warx.values()) - waf
        wof = sum(v for k, v in woth.items() if k.split("_e32")[0].split("_e64")[0] in FULL)
        wtot = waf + war + sum(woth.values())
        out[dem]["whole"] = {"arx_full": waf, "arx_rot": war, "other_full": wof,
                             "other_half": sum(woth.values()) - wof, "valu": wtot}
        out[dem]["clk_per_valu_whole"] = round((2 * (waf + wof) + 4 * (wtot - waf - wof)) / wtot, 4) if wtot else None
    return out


def main():
    keep = None
    if "--keep" in sys.argv:
        keep = Path(sys.argv[sys.argv.index("--keep") + 1])
        keep.mkdir(parents=True, exist_ok=True)
    src = _build.source_hash()
    with tempfile.TemporaryDirectory(prefix="sg_isa_") as td:
        wd = keep or Path(td)
        kernels = {}
        for s in (_build.CSRC / "sg_wpr.hip", _build.CSRC / "sg_pack.hip", _build.CSRC / "sg_kernels.hip"):
            flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-mllvm",
                     "-amdgpu-atomic-optimizer-strategy=None", "--save-temps", f'-DSG_SOURCE_HASH="{src}"']
            subprocess.run([_build.hipcc(), *flags, "-c", "-o", str(wd / f"{s.stem}.o"), str(s)], cwd=wd, check=True,
                           capture_output=True)
            kernels.update(census_file(wd / f"{s.stem}-hip-amdgcn-amd-amdhsa-gfx950.s"))
    res = {"source_hash": src, "model": "clocks per wave64 VALU: full-rate opcodes (v_add/v_xor/v_and/v_or/v_mov/"
                                        "right shifts/bitop3) 2, paired in lock-step; rotates and every other VALU 4 "
                                        "(profiles/r01_valu_issue_probes.md)",
           "kernels": kernels}
    dst = ROOT / "profiles" / f"isa_{src}.json"
    dst.write_text(json.dumps(res, indent=1) + "\n")
    print(dst)
    for k, v in kernels.items():
        if "wpr_kernel<false, true, 4u, false>" in k or "wpr_kernel<true, true, 4u, false>" in k:
            print(k, {x: v[x] for x in ("arx_full", "arx_rot", "other_full", "other_half", "mfma", "clk_per_valu")})


if __name__ == "__main__":
    main()
