#!/usr/bin/env python3
"""Board power of a plain device-to-device copy of C1's bytes (round 6, the
floor of the record's data path): 16 GiB copied HBM -> HBM by
torch (its copy kernel), back to back for --seconds, the board power and sclk
sampled by suruga_amd.devmon, the second half of the window priced.  Prints one
JSON line: TB/s (read + write bytes), mean board power, sclk, and the energy per
16 KiB of payload moved (the unit of C1's µJ per record)."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    import torch

    from suruga_amd import devmon

    dev = torch.device("cuda", 0)
    pr = torch.cuda.get_device_properties(dev)
    bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
    n = a.gib << 30
    src = torch.empty(n, dtype=torch.uint8, device=dev)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    src.fill_(7)
    for _ in range(3):
        dst.copy_(src)
    torch.cuda.synchronize()
    mon = devmon.Sampler(bus).start()
    ev = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src)
        e1.record()
        ev.append((time.perf_counter(), e0, e1))
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    mon.stop()
    half = t0 + (t1 - t0) / 2
    late = [(t, e0.elapsed_time(e1)) for t, e0, e1 in ev if t >= half]
    ms = sum(d for _, d in late) / len(late)
    pw = [s["power_w"] for s in mon.samples if "power_w" in s and s["t"] >= half]
    mhz = [s["sclk_mhz"] for s in mon.samples if "sclk_mhz" in s and s["t"] >= half]
    w = sum(pw) / len(pw) if pw else None
    out = {"bytes_moved_per_copy": 2 * n, "copy_ms": round(ms, 4), "tb_per_s": round(2 * n / ms / 1e9, 3),
           "board_power_w": round(w, 1) if w else None, "sclk_mhz": round(sum(mhz) / len(mhz), 1) if mhz else None,
           "uj_per_16kib_payload": round(w * ms * 1e-3 / (n / 16384) * 1e6, 3) if w else None,
           "copies": len(ev), "note": "torch copy kernel, HBM -> HBM; C1's record moves the same 2 x 16 KiB (plus 69 B)"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
