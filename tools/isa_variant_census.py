#!/usr/bin/env python3
"""Static census of the C1 seal kernel's record loop for the product and for
edited copies (tools/archive/variants/*.py edit files): the difference per variant is
the instruction count of the part it removes, which DESIGN.md §4.2 tables
next to the measured time that part costs (the same variants timed on the GPU,
profiles/r04_ab/).  CPU only.

Usage: python tools/isa_variant_census.py [variant ...]   (default: the wpr timing variants)
"""
from __future__ import annotations

import json
import runpy
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import isa_count as ic  # noqa: E402

from suruga_amd import _build  # noqa: E402

KERNEL = "sg_wpr_kernelILb0ELb1ELj4ELb0E"  # seal, TLS, 16 KiB, uniform


def census(edits):
    with tempfile.TemporaryDirectory(prefix="sg_ivc_") as td:
        tdp = Path(td)
        shutil.copytree(_build.CSRC, tdp / "pkg" / "csrc")
        shutil.copytree(ROOT / "include", tdp / "include")
        for fname, old, new, *mode in edits:
            f = tdp / "pkg" / "csrc" / fname
            txt = f.read_text()
            n = txt.count(old)
            if n != 1 and not (mode == ["all"] and n >= 1):
                raise SystemExit(f"edit matches {n} times in {fname}: {old[:60]!r}")
            f.write_text(txt.replace(old, new))
        subprocess.run([_build.hipcc(), "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-mllvm",
                        "-amdgpu-atomic-optimizer-strategy=None", "--save-temps", f"-I{tdp / 'include'}",
                        '-DSG_SOURCE_HASH="x"', "-c", "-o", "w.o", str(tdp / "pkg" / "csrc" / "sg_wpr.hip")],
                       cwd=tdp, check=True, capture_output=True)
        body = ic.loop_body(ic.kernel_lines(str(tdp / "sg_wpr-hip-amdgcn-amd-amdhsa-gfx950.s"), KERNEL))
        arx, other, kinds, _ = ic.census(body)
        return {"arx": sum(arx.values()), "other": sum(other.values()), "mfma": kinds.get("mfma", 0),
                "lds": kinds.get("lds", 0), "other_by_op": dict(other)}


def main():
    names = sys.argv[1:] or ["wpr_nomac", "wpr_nomfma", "wpr_nopro", "wpr_noepi", "wpr_noff"]
    base = census([])
    out = {"source_hash": _build.source_hash(), "kernel": KERNEL, "product": base, "variants": {}}
    for n in names:
        c = census(runpy.run_path(str(ROOT / "tools" / "variants" / f"{n}.py"))["EDITS"])
        ops = set(base["other_by_op"]) | set(c["other_by_op"])
        out["variants"][n] = {"removes_other_valu": base["other"] - c["other"], "removes_arx": base["arx"] - c["arx"],
                              "removes_mfma": base["mfma"] - c["mfma"], "removes_lds": base["lds"] - c["lds"],
                              "removed_by_op": {o: base["other_by_op"].get(o, 0) - c["other_by_op"].get(o, 0)
                                                for o in sorted(ops)
                                                if base["other_by_op"].get(o, 0) != c["other_by_op"].get(o, 0)}}
        print(n, {k: v for k, v in out["variants"][n].items() if k != "removed_by_op"})
    dst = ROOT / "profiles" / f"isa_parts_{out['source_hash']}.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(dst)


if __name__ == "__main__":
    main()
