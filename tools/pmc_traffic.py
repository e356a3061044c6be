#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/.

Reads gpurun_out/prof_<tag>/ and writes
  profiles/<tag>_kernel_stats.csv      rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc_summary.json      per-kernel mean of every PMC counter
  profiles/traffic_<tag>.json          HBM bytes per launch of the seal/open kernels

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3): on gfx950
FETCH_SIZE (KiB) reports half the bytes of a wide (16 B/lane) coalesced read,
so read bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact for 16-B stores.
The sg_compare_kernel in the same run (reads 2 * records * record_bytes with
16-B loads) is reported as the calibration check.
"""
from __future__ import annotations

import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def kind(name: str):
    if "aead_kernel<false>" in name or "seal" in name and "sg_" in name:
        return "seal"
    if "aead_kernel<true>" in name or "open" in name and "sg_" in name:
        return "open"
    for k in ("keying", "compare", "fill"):
        if k in name:
            return k
    return None


def main(tag: str, records: int = 1 << 20, record_bytes: int = 16384):
    src = ROOT / "gpurun_out" / f"prof_{tag}"
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    ks = src / "kt" / "run_kernel_stats.csv"
    if ks.exists():
        shutil.copy(ks, dst / f"{tag}_kernel_stats.csv")
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(src.glob("pmc_*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = kind(r["Kernel_Name"])
            if not k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            acc[k]["dispatch_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    summ = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
    (dst / f"{tag}_pmc_summary.json").write_text(json.dumps(summ, indent=1) + "\n")
    traffic = {"records": records, "record_bytes": record_bytes, "tag": tag,
               "method": "2*1024*FETCH_SIZE + 1024*WRITE_SIZE (gfx950 FETCH_SIZE half-count correction)"}
    for k in ("seal", "open", "compare"):
        if k in summ and "FETCH_SIZE" in summ[k] and "WRITE_SIZE" in summ[k]:
            rd = 2 * 1024 * summ[k]["FETCH_SIZE"]
            wr = 1024 * summ[k]["WRITE_SIZE"]
            traffic[f"{k}_read_bytes"] = rd
            traffic[f"{k}_write_bytes"] = wr
            traffic[f"{k}_bytes_per_launch"] = rd + wr
    if "compare_read_bytes" in traffic:
        traffic["calibration"] = {"compare_expected_read": 2 * records * record_bytes,
                                  "compare_measured_read": traffic["compare_read_bytes"]}
    for k in ("seal", "open"):
        if k in summ and "GRBM_GUI_ACTIVE" in summ[k]:
            traffic[f"{k}_clock_ghz"] = summ[k]["GRBM_GUI_ACTIVE"] / 8 / summ[k]["dispatch_ns"]
        if k in summ and "SQ_INSTS_VALU" in summ[k]:
            traffic[f"{k}_valu_per_record"] = summ[k]["SQ_INSTS_VALU"] / records
    (dst / f"traffic_{tag}.json").write_text(json.dumps(traffic, indent=1) + "\n")
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
