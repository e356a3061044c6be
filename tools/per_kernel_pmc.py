#!/usr/bin/env python3
"""Per-kernel means of every PMC counter of a tools/profile_round.sh run
(gpurun_out/prof_<tag>/pmc_*/.../*counter_collection.csv), one row per kernel
name: the counters tools/pmc_traffic.py sums by direction, split by kernel
(the C2 batch runs the packed kernel, three bucket kernels and their keying
beside each other, so the per-direction sums hide which one spends what).
Usage: python tools/per_kernel_pmc.py <tag> [--json-out F]"""
from __future__ import annotations

import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main(tag: str, out: str | None = None):
    src = ROOT / "gpurun_out" / f"prof_{tag}"
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(src.glob("pmc_*/**/*counter_collection.csv")):
        per = collections.defaultdict(float)  # (dispatch, kernel, counter) -> summed over dims
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row.get("Dispatch_Id"), row.get("Kernel_Name"), row.get("Counter_Name"))
                per[key] += float(row.get("Counter_Value") or 0)
        for (d, k, c), v in per.items():
            acc[k][c].append(v)
    res = {}
    for k, cs in acc.items():
        short = k.replace("void sg::(anonymous namespace)::", "").replace("sg::(anonymous namespace)::", "").split("(")[0]
        res[short] = {c: round(sum(v) / len(v), 1) for c, v in cs.items()}
        res[short]["dispatches"] = max(len(v) for v in cs.values())
    print(json.dumps(res, indent=1))
    if out:
        Path(out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[a.index("--json-out") + 1] if "--json-out" in a else None)
