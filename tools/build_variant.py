#!/usr/bin/env python3
"""Build an experiment variant of the HIP library from edited copies of the
sources into ablib/<name>.so (same-box A/B with tools/ab_libs.sh).

The product sources are never modified: the csrc/ tree is copied to a
temporary directory, the edits of an edit file are applied there (each edit
must match exactly once), and the copy is compiled with the product flags and
the marker "<tree hash>+var:<name>:<hash of the edits and defines>", so that
a variant never carries the product's identity: _native.load() accepts it
(named by SURUGA_GPU_LIB) only with SURUGA_ALLOW_VARIANT=1, and bench.py
prints the loaded library's path and marker in its line.  Timing-only variants (skipped work, wrong output)
live only in ablib/ and in the edit files under tools/archive/variants/.

Usage: python tools/build_variant.py <name> <edits.py> [-DNAME=V ...]
  edits.py defines EDITS = [(file, old, new[, "all"]), ...]
"""
from __future__ import annotations

import runpy
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from suruga_amd import _build  # noqa: E402


def main() -> None:
    name, edit_file, *defines = sys.argv[1:]
    edits = runpy.run_path(edit_file)["EDITS"] if edit_file != "-" else []
    out = ROOT / "ablib" / f"{name}.so"
    out.parent.mkdir(exist_ok=True)
    with tempfile.TemporaryDirectory(prefix="sg_var_") as td:
        tdp = Path(td)
        shutil.copytree(_build.CSRC, tdp / "pkg" / "csrc")  # ../../include resolves as in the tree
        shutil.copytree(ROOT / "include", tdp / "include")
        for fname, old, new, *mode in edits:  # mode "all": every occurrence (at least one)
            f = tdp / "pkg" / "csrc" / fname
            txt = f.read_text()
            n = txt.count(old)
            if n != 1 and not (mode == ["all"] and n >= 1):
                raise SystemExit(f"edit matches {n} times in {fname}: {old[:60]!r}")
            f.write_text(txt.replace(old, new))
        srcs = [tdp / "pkg" / "csrc" / p.name for p in _build.HIP_SOURCES]
        import hashlib

        eh = hashlib.sha256(repr((edits, defines)).encode()).hexdigest()[:8]
        marker = f"{_build.source_hash()}+var:{name}:{eh}"
        flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-mllvm",
                 "-amdgpu-atomic-optimizer-strategy=None", "-Wall", "-Wno-unused-result", f"-I{tdp / 'include'}",
                 *defines, f'-DSG_SOURCE_HASH="{marker}"']
        objs = [tdp / f"{s.stem}.o" for s in srcs]

        def cc(so):
            s, o = so
            r = subprocess.run([_build.hipcc(), *flags, "-c", "-o", str(o), str(s)], capture_output=True, text=True)
            if r.returncode:
                raise SystemExit(r.stderr[-4000:])

        with ThreadPoolExecutor(max_workers=len(srcs)) as ex:
            list(ex.map(cc, zip(srcs, objs)))
        subprocess.run([_build.hipcc(), "--offload-arch=gfx950", "-fPIC", "-shared", "-o", str(out),
                        *map(str, objs)], check=True)
    print(out)


if __name__ == "__main__":
    main()
