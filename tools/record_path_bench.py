#!/usr/bin/env python3
"""Copy-inclusive rate of the GPU record path, one direction at a time and
both at once (C4's host side, tls.rs:126-130 write / :238-281 read).

Writer: sg_write_records over a host buffer of application data (fragment into
2^14-byte records, pinned staging, H2D, seal, D2H, 5-byte headers) into a host
wire buffer.  Reader: sg_read_records over that wire back into a host buffer.
Both are timed wall-clock around the calls, from and to pageable host memory,
so every copy is inside the number.  The read-back is compared with the input
byte for byte.  Duplex (round 6): a writer and a reader on two contexts and
two threads at once -- the writer seals the stream again into a second wire
buffer while the reader opens the first, as suruga's client runs its reader and
writer independently over a cloned socket (client.rs:19-24, 269-271) -- timed
wall-clock around both; `duplex_gibs` counts the bytes of both directions and
both outputs are checked.  Prints one JSON line (and writes it with --json-out): GiB/s of
application data per direction plus the per-GiB split of H2D, kernel, D2H and
host framing time (sg_record_timing) for SG_COPY_THREADS = each --threads value.

    python tools/record_path_bench.py [--bytes 1073741824] [--call-bytes 67108864]
        [--threads 1,4,8] [--json-out profiles/r02_record_path.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

KEY = bytes(range(32))


def one(total: int, call: int, device: int, registered: bool = False, check_wire=None, data=None,
        repeats: int = 3) -> dict:
    """check_wire(data, wire, wlen) -> bool: an extra check of the timed
    write's wire (bench.py: a sample of records against the oracle).  data:
    the application bytes (uint8 array of `total`; default: random)."""
    import numpy as np

    from suruga_amd import ChaCha20Poly1305
    from suruga_amd import _native as N

    lib = N.load()
    if data is None:
        data = np.frombuffer(np.random.default_rng(0xC4).bytes(total), dtype=np.uint8).copy()
    wire = np.empty(lib.sg_wire_bound(total), dtype=np.uint8)
    wire2 = np.empty_like(wire)
    back = np.empty(total, dtype=np.uint8)
    aead = ChaCha20Poly1305(device)
    enc, dec = aead.new_encryptor(KEY), aead.new_decryptor(KEY)
    if registered:  # the zero-copy path: DMA straight between these buffers and the device
        for a in (data, wire, wire2, back):
            N.check(lib.sg_host_register(a.ctypes.data, a.nbytes))

    def timing(acc):
        v = [C.c_double() for _ in range(4)]
        lib.sg_record_timing(*[C.byref(x) for x in v])
        for k, x in zip(("h2d", "kernel", "d2h", "host"), v):
            acc[k] = acc.get(k, 0.0) + x.value

    def write_all(acc, dst=wire):
        wl = C.c_size_t(0)
        seq, pos, wpos = 0, 0, 0
        while pos < total:
            n = min(call, total - pos)
            seq += N.check(lib.sg_write_records(enc._ptr, seq, 23, 3, 3, C.c_void_p(data.ctypes.data + pos), n,
                                                C.c_void_p(dst.ctypes.data + wpos), dst.size - wpos,
                                                C.byref(wl)))
            if acc is not None:
                timing(acc)
            pos += n
            wpos += wl.value
        return seq, wpos

    def read_all(wlen, acc):
        res = N.SgReadResult()
        seq, pos, opos = 0, 0, 0
        while pos < wlen:
            n = min(call + (call >> 10) + 64, wlen - pos)  # about `call` bytes of records per call
            N.check(lib.sg_read_records(dec._ptr, seq, C.c_void_p(wire.ctypes.data + pos), n,
                                        C.c_void_p(back.ctypes.data + opos), back.size - opos, None, None,
                                        1 << 20, C.byref(res)))
            if res.error != N.SG_OK:
                raise RuntimeError(f"record error {res.error} after {seq + res.records} records")
            if acc is not None:
                timing(acc)
            seq += res.records
            pos += res.consumed
            opos += res.out_len
        return seq, opos

    # each measurement `repeats` times (the host link and the host's memory
    # bandwidth vary by tens of percent between runs of ~30 ms): the median
    # is reported, every run is listed
    import statistics

    write_all(None)  # warm-up: staging allocation, page faults of the buffers
    wacc, racc = {}, {}
    tws, trs = [], []
    for i in range(repeats):
        acc = {}
        t0 = time.perf_counter()
        nrec, wlen = write_all(acc)
        tws.append(time.perf_counter() - t0)
        wacc = acc if tws[-1] == min(tws) else wacc
    tw = statistics.median(tws)
    read_all(wlen, None)
    for i in range(repeats):
        acc = {}
        back[:] = 0
        t0 = time.perf_counter()
        rrec, olen = read_all(wlen, acc)
        trs.append(time.perf_counter() - t0)
        racc = acc if trs[-1] == min(trs) else racc
    tr = statistics.median(trs)
    ok = rrec == nrec and olen == total and bool(np.array_equal(back, data))
    wire_ok = None if check_wire is None else bool(check_wire(data, wire, wlen))
    # duplex: the writer into wire2 and the reader from wire, two threads (ctypes
    # releases the GIL for the calls)
    import threading

    back[:] = 0
    stamps, errs = {}, []

    def timed(name, fn):
        try:
            t0 = time.perf_counter()
            fn()
            stamps[name] = time.perf_counter() - t0
        except Exception as e:  # reported below
            errs.append(repr(e))

    tds, dok = [], True
    for i in range(repeats):
        back[:] = 0
        wire2[:] = 0
        ths = [threading.Thread(target=timed, args=("write", lambda: write_all(None, wire2))),
               threading.Thread(target=timed, args=("read", lambda: read_all(wlen, None)))]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        tds.append(time.perf_counter() - t0)
        dok = dok and not errs and bool(np.array_equal(back, data)) and bool(np.array_equal(wire2[:wlen], wire[:wlen]))
    td = statistics.median(tds)
    if registered:
        for a in (data, wire, wire2, back):
            N.check(lib.sg_host_unregister(a.ctypes.data))
    gib = total / 2**30
    per = lambda acc: {k + "_ms_per_gib": round(v / gib, 2) for k, v in acc.items()}  # noqa: E731
    return {"write_gibs": round(gib / tw, 3), "read_gibs": round(gib / tr, 3), "write_ms": round(tw * 1e3, 1),
            "read_ms": round(tr * 1e3, 1), "repeats": repeats, "write_ms_all": [round(t * 1e3, 1) for t in tws],
            "read_ms_all": [round(t * 1e3, 1) for t in trs], "records": nrec, "correct": ok,
            "split_note": "per GiB, of the fastest run", "write_split": per(wacc),
            "read_split": per(racc), "registered": registered, "wire_sample_ok": wire_ok,
            "duplex": {"gibs": round(2 * gib / td, 3), "ms": round(td * 1e3, 1), "ms_all": [round(t * 1e3, 1) for t in tds],
                       "write_ms": round(stamps.get("write", 0) * 1e3, 1),
                       "read_ms": round(stamps.get("read", 0) * 1e3, 1),
                       "vs_slower_single": round((2 * gib / td) / min(gib / tw, gib / tr), 3),
                       "vs_serial": round((tw + tr) / td, 3), "correct": dok, "errors": errs}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--call-bytes", type=int, default=64 << 20, help="application bytes per write call")
    ap.add_argument("--threads", default="1,4,8", help="SG_COPY_THREADS values (one child process each)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--registered", default="0", help="0, 1 or 0,1: caller buffers registered with sg_host_register "
                    "(the zero-copy path)")
    ap.add_argument("--pin", type=int, default=1, help="1: run on the CPUs of the GPU's NUMA node "
                    "(devmon.pin_to_gpu_node; host buffers and copy threads next to the card's link)")
    ap.add_argument("--json-out")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--watchdog", type=float, default=0, help="dump every thread's stack and exit after this many s")
    a = ap.parse_args()
    if a.watchdog:
        import faulthandler

        faulthandler.dump_traceback_later(a.watchdog, exit=True)
    if a.child:
        pin = None
        if a.pin:
            import torch

            from suruga_amd import devmon

            pr = torch.cuda.get_device_properties(a.device)
            bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
            cpus, how = devmon.pin_to_gpu_node(bus)
            pin = {"cpus": len(cpus) if cpus else None, "how": how}
        r = one(a.bytes, a.call_bytes, a.device, a.registered == "1")
        r["pinned"] = pin
        print(json.dumps(r))
        return
    runs = {}
    for reg in a.registered.split(","):
        for t in [int(x) for x in a.threads.split(",")]:
            env = dict(os.environ, SG_COPY_THREADS=str(t))
            p = subprocess.run([sys.executable, __file__, "--child", "--bytes", str(a.bytes), "--call-bytes",
                                str(a.call_bytes), "--device", str(a.device), "--registered", reg, "--pin",
                                str(a.pin)], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                raise SystemExit(f"threads={t} registered={reg} failed:\n{p.stdout}\n{p.stderr}")
            runs[str(t) + ("+registered" if reg == "1" else "")] = json.loads(p.stdout.strip().splitlines()[-1])
    from suruga_amd import _native as N

    lib = N.load()
    out = {"config": f"C4 host side: {a.bytes} B application data, {a.call_bytes} B per sg_write_records call, "
                     "pageable host buffers (\"+registered\": registered with sg_host_register, the zero-copy path), "
                     "one direction at a time (write_gibs, read_gibs) and both at once on two contexts and threads "
                     "(duplex.gibs: both directions' bytes over the wall time), wall clock around the calls",
           "kernels": lib.sg_build_info().decode(), "library": N.loaded_info(),
           "host_cpus": len(os.sched_getaffinity(0)), "by_copy_threads": runs,
           "correct": all(r["correct"] and r["duplex"]["correct"] for r in runs.values())}
    print(json.dumps(out))
    if a.json_out:
        Path(a.json_out).write_text(json.dumps(out, indent=1) + "\n")
    sys.exit(0 if out["correct"] else 1)


if __name__ == "__main__":
    main()
