#!/usr/bin/env python3
"""Static instruction census of one kernel in a hipcc --save-temps .s file.

Usage: isa_count.py <file.s> <kernel-substring> [--blocks]

Counts the VALU / SALU / LDS / VMEM / MFMA instructions of the kernel's
record loop (the basic blocks between the loop header -- the target of the
last backward branch -- and that branch), split into

  * ARX: VALU inside the inline-asm double rounds (SG_CHACHA_* macros, i.e.
    every ;;#ASMSTART block that contains v_alignbit_b32) -- the ChaCha20
    stream of chacha20.rs:53-109;
  * other VALU by mnemonic, which is the non-ARX issue DESIGN.md §4.2 tables.

The issue model of profiles/r01_valu_issue_probes.md prices full-rate ops
(add/sub/xor/or/and/not/mov/lshrrev/ashrrev/bitop3) at 2 clocks when paired
and every other VALU at 4.
"""
from __future__ import annotations

import re
import sys
from collections import Counter

FULL = {"v_add_u32", "v_sub_u32", "v_xor_b32", "v_or_b32", "v_and_b32", "v_not_b32", "v_mov_b32",
        "v_lshrrev_b32", "v_ashrrev_i32", "v_bitop3_b32", "v_subrev_u32", "v_mov_b64"}


def kernel_lines(path: str, name: str):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and name in l:
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"kernel {name!r} not found")


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_cbranch", "s_branch", "s_setprio", "s_sleep",
                      "s_endpgm", "s_sched")):
        return "ctl"
    if op.startswith("s_"):
        return "salu"
    return "other"


def census(body, blocks=False):
    in_asm = False
    asm_buf = []
    arx = Counter()
    other = Counter()
    kinds = Counter()
    cur = None
    per_block = {}
    for l in body:
        s = l.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm, asm_buf = True, []
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            is_arx = any(x.startswith("v_alignbit_b32") for x in asm_buf)
            for op in asm_buf:
                k = classify(op)
                kinds[k] += 1
                if k == "valu":
                    (arx if is_arx else other)[op] += 1
            continue
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            per_block.setdefault(cur, Counter())
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        if in_asm:
            asm_buf.append(op)
            continue
        k = classify(op)
        kinds[k] += 1
        if cur:
            per_block[cur][k] += 1
        if k == "valu":
            other[op] += 1
    return arx, other, kinds, per_block


def loop_body(lines):
    """Lines of the kernel's main loop: the smallest loop (a label and a
    backward branch to it) that contains every ChaCha20 double-round asm block
    -- the record loop of the wave-per-record kernel, the chunk-round loop of
    the packed kernel; the whole kernel when no loop holds them all."""
    labels = {}
    arx = []
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
        s = l.strip()
        if s.startswith(";;#ASMSTART"):
            start = i
        elif s.startswith(";;#ASMEND") and start is not None:
            if any(x.strip().startswith("v_alignbit_b32") for x in lines[start:i]):
                arx.append((start, i))
            start = None
    best = None
    for i, l in enumerate(lines):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            lo = labels[m.group(1)]
            if arx and not all(lo <= a and b <= i for a, b in arx):
                continue
            if best is None or i - lo < best[1] - best[0]:
                best = (lo, i)
    if best is None:
        return lines
    return lines[best[0]:best[1] + 1]


def cycles(arx: Counter, other: Counter) -> tuple[float, float]:
    a = sum(2 * v if k in FULL else 4 * v for k, v in arx.items())
    o = sum(4 * v for v in other.values())  # unpaired: every non-ARX VALU at 4
    return a, o


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, name)
    body = loop_body(lines)
    arx, other, kinds, per_block = census(body)
    na, no = sum(arx.values()), sum(other.values())
    ca, co = cycles(arx, other)
    print(f"kernel {name}: loop {len(body)} lines")
    print(f"  VALU {na + no}: ARX {na} ({ca:.0f} clk paired model), other {no} ({co:.0f} clk at 4)")
    print(f"  kinds: {dict(kinds)}")
    print("  ARX ops:", dict(arx.most_common()))
    print("  other VALU:")
    for op, v in other.most_common():
        print(f"    {v:5d} {op}")
    if "--blocks" in sys.argv:
        for b, c in per_block.items():
            if c:
                print(b, dict(c))


if __name__ == "__main__":
    main()
