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
import re
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def kind(name: str):
    m = re.search(r"(?:aead(?:_list|_ls)?|wpr|pack)_kernel<(false|true)", name)
    if m:
        return "seal" if m.group(1) == "false" else "open"
    m = re.search(r"(wpr_keying|keying|classify)_kernel<(false|true)", name)
    if m:
        return f"{m.group(1)}_{'seal' if m.group(2) == 'false' else 'open'}"
    for k in ("compare", "fill"):
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
    # steady state: per kernel, the average duration over its dispatches after
    # the first SKIP (the first launches run on a GPU coming out of idle), next
    # to the all-dispatch average of the stats summary
    kt = src / "kt" / "run_kernel_trace.csv"
    if kt.exists():
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(kt)):
            per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        SKIP = 4
        rows = []
        for name, d in per.items():
            if kind(name) is None and "rocclr" in name:
                continue
            steady = d[SKIP:] if len(d) > SKIP else d
            rows.append({"kernel": name, "dispatches": len(d), "avg_ns_all": round(sum(d) / len(d), 1),
                         "steady_dispatches": len(steady), "avg_ns_steady": round(sum(steady) / len(steady), 1),
                         "min_ns": min(d), "max_ns": max(d)})
        rows.sort(key=lambda x: -x["avg_ns_all"] * x["dispatches"])
        with open(dst / f"{tag}_kernel_steady.csv", "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0]) if rows else ["kernel"])
            w.writeheader()
            w.writerows(rows)
    # Per BATCH (one sg_seal_batch / sg_open_batch call) sums: a mixed-size batch
    # launches classify + one list kernel per size class; a batch is counted by
    # its keying dispatch.  For C1 a batch is exactly one aead kernel launch.
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    nbatch = collections.defaultdict(lambda: collections.defaultdict(int))
    # SQ_INSTS_VALU per record kernel (by name) of the seal / open batches, for
    # bench.py's per-kernel issue bound (valu_roofline of mixed batches)
    valu_by = collections.defaultdict(lambda: collections.defaultdict(float))
    valu_file = None
    for f in sorted(src.glob("pmc_*/run_counter_collection.csv")):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = kind(r["Kernel_Name"])
            if not k:
                continue
            if k in ("seal", "open") and r["Counter_Name"] == "SQ_INSTS_VALU":
                valu_by[k][r["Kernel_Name"]] += float(r["Counter_Value"])
                valu_file = f.parent.name
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            nbatch[k][r["Counter_Name"]] += 0
            key = (k, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                acc[k]["dispatch_ns@" + f.parent.name] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                base = k.split("_")[-1] if k.startswith(("keying", "wpr_keying", "classify")) else None
                # a batch has one keying dispatch of each kind it uses: mixed
                # batches run sg_keying_kernel (and maybe sg_wpr_keying_kernel),
                # uniform 16 KiB batches sg_wpr_keying_kernel alone
                if k.startswith("keying"):
                    nbatch[base]["@" + f.parent.name] += 1
                elif k.startswith("wpr_keying"):
                    nbatch[base]["@w" + f.parent.name] += 1
                elif k in ("compare", "fill"):
                    nbatch[k]["@" + f.parent.name] += 1

    def batches(k, counter_file):
        n = nbatch[k].get("@" + counter_file, 0) or nbatch[k].get("@w" + counter_file, 0)
        return n if n else 1

    summ = {}
    for k, d in acc.items():
        out = {}
        for f in sorted(src.glob("pmc_*/run_counter_collection.csv")):
            cols = {r["Counter_Name"] for r in csv.DictReader(open(f)) if kind(r["Kernel_Name"]) == k}
            nb = batches(k, f.parent.name) if k in ("seal", "open", "compare", "fill") else 1
            if k.startswith(("keying", "wpr_keying", "classify")):
                nb = batches(k.split("_")[-1], f.parent.name)
            for c in cols:
                out[c] = d[c] / nb
            if "dispatch_ns@" + f.parent.name in d:
                out.setdefault("dispatch_ns", d["dispatch_ns@" + f.parent.name] / nb)
        summ[k] = out
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
        traffic["calibration"] = {"compare_expected_read": 2 * records * record_bytes if record_bytes != "zipf"
                                  else None,
                                  "compare_measured_read": traffic["compare_read_bytes"]}
    for k in ("seal", "open"):
        if k in summ and "GRBM_GUI_ACTIVE" in summ[k]:
            traffic[f"{k}_clock_ghz"] = summ[k]["GRBM_GUI_ACTIVE"] / 8 / summ[k]["dispatch_ns"]
        if k in summ and "SQ_INSTS_VALU" in summ[k]:
            traffic[f"{k}_valu_per_record"] = summ[k]["SQ_INSTS_VALU"] / records
        if valu_by.get(k) and valu_file:
            nb = batches(k, valu_file)
            traffic[f"{k}_valu_by_kernel"] = {name: v / nb for name, v in valu_by[k].items()}
    # the build string of the library the profiled bench ran (its JSON line in
    # the kernel-trace log), so a summary can never be stamped with a newer build
    log = src / "kt_bench.log"
    for line in (log.read_text(errors="replace").splitlines() if log.exists() else []):
        if line.startswith("{") and '"kernels"' in line:
            try:
                cfgj = json.loads(line)["config"]
                traffic["kernels"] = cfgj["kernels"]
                if "layout" in cfgj:
                    traffic["layout"] = cfgj["layout"]
            except (ValueError, KeyError):
                pass
    (dst / f"traffic_{tag}.json").write_text(json.dumps(traffic, indent=1) + "\n")
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    # pmc_traffic.py <tag> [records] [record_bytes|zipf]
    a = sys.argv[1:]
    rb = a[2] if len(a) > 2 else "16384"
    main(a[0] if a else "r01", int(a[1]) if len(a) > 1 else 1 << 20, rb if rb == "zipf" else int(rb))
