#!/usr/bin/env python3
"""C4 of BASELINE.json: an application stream through the GPU record layer
over a loopback TCP connection, host<->device copies included.

Writer thread: TlsWriter-style batched sealing (sg_write_records: fragment into
2^14-byte records, seal on the GPU with pinned double-buffered staging, frame
5-byte headers) and socket.sendall.  Reader thread: recv into a buffer and
sg_read_records (parse headers, open on the GPU, strip framing).  Keys are
fixed (the handshake is bypassed, as in src/test.rs:29-39's null_tls); every
received byte is compared with what was sent.

Prints one JSON line (--json-out also writes it to a file): end-to-end GiB/s
of application data plus the time each side spent in H2D copies, kernels, D2H
copies, host framing and socket I/O, also per GiB.  ``run()`` is the same
stream as a function; tests/test_gpu_loopback.py calls it with
``capture=True`` and checks the captured wire against the oracle.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import socket
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from suruga_amd import ChaCha20Poly1305  # noqa: E402
from suruga_amd import _native as N  # noqa: E402

KEY_C2S = bytes(range(32))


def stream_pattern(wchunk: int):
    """The application stream is this pattern repeated every wchunk bytes."""
    return np.random.default_rng(0xC4).integers(0, 256, size=wchunk, dtype=np.uint8)


def run(total: int = 1 << 30, wchunk: int = 16 << 20, device: int = 0, capture: bool = False) -> dict:
    """One loopback stream; returns the JSON-able result (plus "wire": the
    bytes the writer sent, when capture)."""
    lib = N.load()
    pattern = stream_pattern(wchunk)
    captured = bytearray() if capture else None

    srv = socket.create_server(("127.0.0.1", 0))
    port = srv.getsockname()[1]
    stats = {"writer": {}, "reader": {}}
    errors = []

    def timing(d):
        v = [C.c_double() for _ in range(4)]
        lib.sg_record_timing(*[C.byref(x) for x in v])
        for k, x in zip(("h2d_ms", "kernel_ms", "d2h_ms", "host_ms"), v):
            d[k] = d.get(k, 0.0) + x.value

    def writer():
        # two stages: this thread seals chunk c+1 (sg_write_records, GIL
        # released in the call) while a sender thread puts chunk c on the socket
        import queue

        try:
            enc = ChaCha20Poly1305(device).new_encryptor(KEY_C2S)
            sock = socket.create_connection(("127.0.0.1", port))
            sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
            nbuf = 3
            wires = [(C.c_uint8 * lib.sg_wire_bound(wchunk))() for _ in range(nbuf)]
            free, full = queue.Queue(), queue.Queue()
            for w in range(nbuf):
                free.put(w)
            d = stats["writer"]
            t_sock = [0.0]

            def sender():
                while True:
                    item = full.get()
                    if item is None:
                        return
                    w, ln = item
                    t0 = time.perf_counter()
                    sock.sendall(memoryview(wires[w])[:ln])
                    t_sock[0] += time.perf_counter() - t0
                    if captured is not None:
                        captured.extend(memoryview(wires[w])[:ln])
                    free.put(w)

            th = threading.Thread(target=sender)
            th.start()
            src = pattern.ctypes.data_as(C.c_void_p)
            wl = C.c_size_t(0)
            seq, sent = 0, 0
            while sent < total:
                n = min(wchunk, total - sent)
                w = free.get()
                nrec = N.check(lib.sg_write_records(enc._ptr, seq, 23, 3, 3, src, n, wires[w], len(wires[w]),
                                                    C.byref(wl)))
                timing(d)
                full.put((w, wl.value))
                seq += nrec
                sent += n
            full.put(None)
            th.join()
            sock.shutdown(socket.SHUT_WR)
            sock.close()
            d["socket_ms"] = t_sock[0] * 1e3
            d["records"] = seq
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("writer", repr(e)))

    def reader():
        # two stages: a receiver thread fills 8 MiB blocks from the socket while
        # this thread opens the complete records of the previous block
        import queue

        try:
            dec = ChaCha20Poly1305(device).new_decryptor(KEY_C2S)
            conn, _ = srv.accept()
            conn.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
            blk = 8 << 20
            blocks = queue.Queue(maxsize=4)
            t_sock = [0.0]

            def receiver():
                while True:
                    b = bytearray(blk)
                    mv, have = memoryview(b), 0
                    while have < blk:
                        t0 = time.perf_counter()
                        k = conn.recv_into(mv[have:], blk - have)
                        t_sock[0] += time.perf_counter() - t0
                        if k == 0:
                            break
                        have += k
                    blocks.put((b, have))
                    if have < blk:
                        blocks.put(None)
                        return

            th = threading.Thread(target=receiver)
            th.start()
            cap = 2 * blk + (64 << 10)
            buf = bytearray(cap)
            have = 0
            out = np.empty(cap, dtype=np.uint8)
            res = N.SgReadResult()
            seq, got, mism, t_verify = 0, 0, 0, 0.0
            d = stats["reader"]
            while True:
                item = blocks.get()
                if item is None:
                    break
                b, ln = item
                buf[have:have + ln] = memoryview(b)[:ln]
                have += ln
                src = (C.c_uint8 * have).from_buffer(buf)
                N.check(lib.sg_read_records(dec._ptr, seq, src, have, out.ctypes.data_as(C.c_void_p), cap,
                                            None, None, 1 << 20, C.byref(res)))
                del src
                timing(d)
                if res.error != N.SG_OK:
                    raise RuntimeError(f"record error {res.error} after {seq + res.records} records")
                # verify: the stream is the pattern repeated every wchunk bytes
                t1 = time.perf_counter()
                m, a = int(res.out_len), 0
                while a < m:
                    off = (got + a) % wchunk
                    ln2 = min(m - a, wchunk - off)
                    if not np.array_equal(out[a:a + ln2], pattern[off:off + ln2]):
                        mism += int(np.count_nonzero(out[a:a + ln2] != pattern[off:off + ln2]))
                    a += ln2
                got += m
                t_verify += time.perf_counter() - t1
                seq += res.records
                c = int(res.consumed)
                buf[:have - c] = buf[c:have]
                have -= c
            th.join()
            conn.close()
            if have:
                raise RuntimeError(f"{have} trailing bytes")
            d.update(socket_ms=t_sock[0] * 1e3, verify_ms=t_verify * 1e3, records=seq, bytes=got,
                     mismatched_bytes=mism)
        except Exception as e:  # pragma: no cover
            errors.append(("reader", repr(e)))

    t0 = time.perf_counter()
    tw, tr = threading.Thread(target=writer), threading.Thread(target=reader)
    tr.start()
    tw.start()
    tw.join()
    tr.join()
    wall = time.perf_counter() - t0
    srv.close()
    ok = not errors and stats["reader"].get("bytes") == total and stats["reader"].get("mismatched_bytes") == 0
    gib = total / 2**30
    per_gib = {side: {k.replace("_ms", "_ms_per_gib"): round(v / gib, 2) for k, v in stats[side].items()
                      if k.endswith("_ms")} for side in ("writer", "reader")}
    out = {
        "config": f"C4: {total} B application stream, TlsWriter/TlsReader batched GPU record layer over "
                  "loopback TCP, fixed keys (handshake bypassed)",
        "gib_per_s": round(total / wall / 2**30, 3), "wall_s": round(wall, 3), "correct": ok,
        "writer": {k: round(v, 1) if isinstance(v, float) else v for k, v in stats["writer"].items()},
        "reader": {k: round(v, 1) if isinstance(v, float) else v for k, v in stats["reader"].items()},
        "per_gib": per_gib,
        "errors": errors,
    }
    if capture:
        out["wire"] = bytes(captured)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30, help="application bytes (C4: 1 GiB)")
    ap.add_argument("--write-chunk", type=int, default=16 << 20, help="bytes per write_application_data call")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--json-out")
    ap.add_argument("--watchdog", type=float, default=0, help="dump every thread's stack and exit after this many s")
    args = ap.parse_args()
    if args.watchdog:
        import faulthandler

        faulthandler.dump_traceback_later(args.watchdog, exit=True)
    out = run(args.bytes, args.write_chunk, args.device)
    from suruga_amd import _native as N

    out["kernels"] = N.load().sg_build_info().decode()
    out["library"] = N.loaded_info()
    line = json.dumps(out)
    print(line)
    if args.json_out:
        Path(args.json_out).write_text(json.dumps(out, indent=1) + "\n")
    sys.exit(0 if out["correct"] else 1)


if __name__ == "__main__":
    main()
