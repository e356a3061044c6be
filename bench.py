#!/usr/bin/env python3
"""Benchmark: device-resident ChaCha20-Poly1305 seal+open over 16 KiB TLS records.

Metric (BASELINE.json): "GiB/s device-resident ChaCha20-Poly1305 over 16 KiB TLS
records, 1/2/4/8 GPUs".  One step = seal every record of the shard, then open
every sealed record (C1 of BASELINE.json: 2^20 x 16 KiB per GPU, one key,
sequential sequence numbers, TLS nonce/AD built on device).  value = plaintext
bytes processed by seal and open on all ranks / wall time of the timed region
(max over ranks), in GiB/s.  Weak scaling: each rank owns its own 2^20 records
(seq r*2^20 + i); there is no collective in the data path.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)
With --gpus N > 1 and no launcher environment (WORLD_SIZE unset) bench.py
starts the N rank processes itself (one per GPU, 127.0.0.1 rendezvous)
before anything touches a GPU, and exits with the worst rank's code.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
SIMDS_PER_CU = 4
SEED = 0x53555255
KEY = bytes(range(32))
METRIC = "GiB/s device-resident ChaCha20-Poly1305 over 16 KiB TLS records, 1/2/4/8 GPUs"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["c1", "c2"], default="c1",
                    help="c1: 16 KiB records, one key (the metric's config); c2: Zipf 64 B-16 KiB, 256 keys")
    ap.add_argument("--records", type=int, default=1 << 20, help="records per GPU (C1: 2^20)")
    ap.add_argument("--record-bytes", type=int, default=16384)
    # Sealed records (ct || tag, n + 16 bytes) start on 128-byte boundaries by
    # default: the record stream is non-temporal, and a record boundary inside
    # a 128-byte line costs a partial-line transfer (back to back
    # measured 1.2 % (C1) / 1.6 % (C2) slower, same box).  The padding is never
    # read or written and is not counted in any byte figure.
    ap.add_argument("--c2-ct-align", type=int, default=128,
                    help="C2: alignment of the sealed records (16 = back to back)")
    ap.add_argument("--c2-pt-align", type=int, default=64,
                    help="C2: alignment of the plaintext records (64 = back to back)")
    ap.add_argument("--ct-stride", type=int, default=0,
                    help="C1: bytes between sealed records (default: n + 16 rounded up to 128, i.e. 16512; "
                         "n + 16 = back to back)")
    ap.add_argument("--cpu-per-thread", type=int, default=64,
                    help="CPU baseline: records per thread in the sample (C2: 8x as many)")
    ap.add_argument("--cpu-seconds", type=float, default=2.5, help="min wall time of each CPU-baseline line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-bitexact", action="store_true",
                    help="skip the oracle tag fold / sample compare of the last step (C1 and C2)")
    ap.add_argument("--sg-records", type=int, default=16384,
                    help="records per rank moved by the separately timed RCCL scatter/gather (N > 1; 0 = off)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --records in total, split across ranks (default: weak, per rank)")
    ap.add_argument("--c2-steps", type=int, default=60,
                    help="C1 runs: timed steps of the C2 sub-record appended to the line (0 = none)")
    ap.add_argument("--energy-seconds", type=float, default=2.0,
                    help="length of the energy window after the event-timed steps (0 = no energy fields)")
    ap.add_argument("--record-path-bytes", type=int, default=1 << 30,
                    help="C4 host side after the device-resident lines: sg_write_records / sg_read_records over "
                         "this many application bytes from host memory (0: skip; rank 0 at N=1 only)")
    ap.add_argument("--traffic", default=None,
                    help="PMC-derived HBM traffic summary (tools/pmc_traffic.py)")
    return ap.parse_args()


def cpu_quota():
    """CPUs this process may use per the cgroup CPU quota (None: unlimited).
    On the GPU box the affinity mask lists every CPU of the host while the
    container is granted a share of them; threads beyond the share only
    time-slice (round 2's 256-thread baseline ran on a ~16-CPU share)."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()[:2]),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            if parse:
                q, per = parse(open(path).read())
                if q != "max":
                    return float(q) / float(per)
            else:
                q = int(open(path).read())
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                if q > 0:
                    return q / per
        except (OSError, ValueError):
            continue
    return None


def host_cpus():
    """(threads to use, affinity-mask CPUs, cgroup quota in CPUs or None)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cpu_quota()
    use = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return use, aff, quota


def cpu_baseline(args, n, lay=None):
    """CPU lines on the host cores, bounded samples; only the C calls are timed
    (buffers preallocated).  kind "port": the oracle (the reference's scalar
    algorithm restated in C); optimised_cpu: the same AEAD composed from
    OpenSSL's vectorised ChaCha20 / Poly1305 (SURVEY.md 8d's optional line).
    Both run on a persistent thread pool (oracle/so_pool.h), one contiguous
    slice of >= --cpu-per-thread records per thread, on the CPUs the cgroup
    quota grants (host_cpus).  C1: uniform 16 KiB TLS records; C2 (lay): the
    first records of the same Zipf layout with their connection keys."""
    import ctypes as C

    import numpy as np

    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_ffi import OsslLine  # checker/baseline only, never the measured path
    from oracle_ffi import oracle as get_oracle

    o = get_oracle()
    threads, aff, quota = host_cpus()
    ptr = lambda a, off=0: C.c_void_p(a.ctypes.data + off)  # noqa: E731
    if lay is None:
        count = max(args.cpu_per_thread * threads, 64)
        pt = np.empty(count * n, dtype=np.uint8)
        ct = np.empty(count * (n + 16), dtype=np.uint8)
        back = np.empty(count * n, dtype=np.uint8)
        for j in range(count):
            o.L.so_fill_record(SEED, j, ptr(pt, j * n), n)
        rec_bytes = lambda recs: recs * n  # noqa: E731
        desc = f"{n} B TLS records"
    else:
        # the first records of the C2 layout, whose mean record is ~2 KiB:
        # 8x the records per thread for a comparable slice of bytes
        count = min(lay.count, max(8 * args.cpu_per_thread * threads, 512))
        lens = np.ascontiguousarray(lay.lens[:count].astype(np.uint32))
        olens = np.ascontiguousarray(lens + np.uint32(16))
        io = np.ascontiguousarray(lay.in_off[:count].astype(np.uint64))
        oo = np.ascontiguousarray(lay.out_off[:count].astype(np.uint64))
        ki = np.ascontiguousarray(lay.key_index[:count].astype(np.uint32))
        sq = np.ascontiguousarray(lay.seq[:count].astype(np.uint64))
        kb = np.frombuffer(bytes(lay.keys), dtype=np.uint8).copy()
        pt_bytes = int(io[-1]) + int(lens[-1]) + 64
        pt = np.frombuffer(np.random.default_rng(SEED).bytes(pt_bytes), dtype=np.uint8).copy()
        ct = np.empty(int(oo[-1]) + int(lens[-1]) + 16 + 64, dtype=np.uint8)
        back = np.empty(pt_bytes, dtype=np.uint8)
        csum = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
        rec_bytes = lambda recs: int(csum[recs])  # noqa: E731
        desc = f"C2 Zipf TLS records (mean {csum[-1] / count:.0f} B), 256 connection keys"
    st = np.empty(count, dtype=np.uint8)

    def timed(seal, open_, recs, thr):
        reps, t = 0, 0.0
        while t < args.cpu_seconds or reps == 0:
            t0 = time.perf_counter()
            seal(recs, thr)
            bad = open_(recs, thr)
            t += time.perf_counter() - t0
            reps += 1
            assert bad == 0
        m = rec_bytes(recs) if lay is None else int(io[recs - 1]) + int(lens[recs - 1])
        if lay is None:
            assert np.array_equal(back[:m], pt[:m])
        else:
            assert all(np.array_equal(back[int(io[i]):int(io[i]) + int(lens[i])], pt[int(io[i]):int(io[i]) + int(lens[i])])
                       for i in range(0, recs, max(1, recs // 64)))
        return 2 * rec_bytes(recs) * reps / t / 2**30, reps

    if lay is None:
        def o_seal(recs, thr):
            o.L.so_seal_batch_tls(KEY, 0, ptr(pt), n, recs, ptr(ct), thr)

        def o_open(recs, thr):
            return o.L.so_open_batch_tls(KEY, 0, ptr(ct), n, recs, ptr(back), ptr(st), thr)
    else:
        def o_seal(recs, thr):
            o.L.so_batch_mixed(0, ptr(kb), ptr(ki), ptr(sq), ptr(lens), ptr(io), ptr(oo), ptr(pt), ptr(ct), None,
                               recs, thr)

        def o_open(recs, thr):
            return o.L.so_batch_mixed(1, ptr(kb), ptr(ki), ptr(sq), ptr(olens), ptr(oo), ptr(io), ptr(ct),
                                      ptr(back), ptr(st), recs, thr)

    one_recs = max(16, count // threads)  # one thread's slice of the multi-thread run
    gibs, reps = timed(o_seal, o_open, count, threads)
    one, _ = timed(o_seal, o_open, one_recs, 1)  # the reference is single-threaded per connection
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        L = OsslLine().L
        if lay is None:
            def s_seal(recs, thr):
                L.ossl_batch_tls(0, KEY, 0, ptr(pt), n, recs, ptr(ct), thr)

            def s_open(recs, thr):
                return L.ossl_batch_tls(1, KEY, 0, ptr(ct), n, recs, ptr(back), thr)
        else:
            def s_seal(recs, thr):
                L.ossl_batch_mixed(0, ptr(kb), ptr(ki), ptr(sq), ptr(lens), ptr(io), ptr(oo), ptr(pt), ptr(ct),
                                   recs, thr)

            def s_open(recs, thr):
                return L.ossl_batch_mixed(1, ptr(kb), ptr(ki), ptr(sq), ptr(olens), ptr(oo), ptr(io), ptr(ct),
                                          ptr(back), recs, thr)

        og, oreps = timed(s_seal, s_open, count, threads)
        o1, _ = timed(s_seal, s_open, one_recs, 1)
        ossl = {"value": round(og, 3), "unit": "GiB/s", "cores": threads, "single_thread_gibs": round(o1, 4),
                "scaling_efficiency": round(og / (o1 * threads), 3),
                "impl": "OpenSSL libcrypto ChaCha20 + EVP_MAC POLY1305 (fetched once, one context pair per thread) "
                        "composed per suruga's AEAD (oracle/ossl_aead.c)",
                "sample": f"{count} x {desc} seal+open, x{oreps} repetitions"}
    except (OSError, AssertionError) as e:
        ossl = {"unavailable": str(e)}
    return {
        "value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"{count} x {desc} seal+open, x{reps} repetitions, {threads} threads on a persistent pool "
                  f"(oracle/suruga_oracle.c, the reference's scalar algorithm)",
        "single_thread_gibs": round(one, 4),
        "scaling_efficiency": round(gibs / (one * threads), 3),
        "cpu": model or platform.processor(),
        "affinity_cpus": aff, "cgroup_cpu_quota": quota, "host_logical_cpus": os.cpu_count(),
        "cores_note": "threads = the CPUs the cgroup quota grants (affinity_cpus if unlimited); "
                      "scaling_efficiency = value / (single_thread_gibs x cores)",
        "optimised_cpu": ossl,
    }


def host_threads() -> int:
    """Threads for the oracle checkers: the CPUs this process may use."""
    return host_cpus()[0]


def bitexact_check(ct, n, count, seq0, cs=None):
    """Outside the timed region: the XOR-fold of every one of the batch's tags
    against the oracle's multithreaded fold of the same records (fill rule,
    seq = seq0 + i, chacha20_poly1305.rs:48-59), plus a byte-for-byte compare of
    a strided sample of whole records (ct || tag).  Test infrastructure only:
    the oracle checks, it is never the measured path."""
    import numpy as np

    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_ffi import oracle as get_oracle  # checker only

    o = get_oracle()
    rows = ct.view(count, cs or n + 16)[:, :n + 16]
    tags = rows[:, n:].cpu().numpy()
    fold = np.bitwise_xor.reduce(tags, axis=0).tobytes()
    t0 = time.perf_counter()
    ref_fold = o.tag_fold_tls(KEY, seq0, SEED, seq0, n, count, host_threads())
    fold_s = time.perf_counter() - t0
    idx = sorted(set([0, 1, count // 2, count - 1] + list(range(0, count, 4099))))
    sample_ok = True
    for i in idx:
        pt = o.fill_record(SEED, seq0 + i, n)
        exp = o.seal(KEY, (seq0 + i).to_bytes(8, "big"), pt, o.tls_ad(seq0 + i, n))
        sample_ok = sample_ok and rows[i].cpu().numpy().tobytes() == exp
    return {"bitexact_fold": fold == ref_fold, "fold_records": count, "bitexact_sample": sample_ok,
            "sample_records": len(idx), "oracle_fold_s": round(fold_s, 2)}


def bitexact_check_c2(lay, pt, ct, seq_off):
    """C2 counterpart of bitexact_check: the XOR-fold of all of the batch's tags
    (gathered from ct at out_off + len) against the oracle's multithreaded fold
    of the same records (the device plaintext copied to the host, each record
    sealed with its connection key and sequence number), plus a byte-for-byte
    compare of a strided sample of whole records.  Checker only."""
    import struct

    import numpy as np
    import torch

    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_ffi import oracle as get_oracle  # checker only

    o = get_oracle()
    count = lay.count
    seqs = lay.seq + np.uint64(seq_off)
    tag_at = torch.from_numpy((lay.out_off + lay.lens.astype(np.uint64)).view(np.int64)).to(ct.device)
    idx = (tag_at.view(-1, 1) + torch.arange(16, device=ct.device).view(1, 16)).view(-1)
    tags = ct[idx].view(count, 16).cpu().numpy()
    fold = np.bitwise_xor.reduce(tags, axis=0).tobytes()
    pt_h = pt.cpu().numpy()
    t0 = time.perf_counter()
    ref_fold = o.tag_fold_mixed(lay.keys, lay.key_index, seqs, lay.lens, lay.in_off, pt_h, host_threads())
    fold_s = time.perf_counter() - t0
    sample = sorted(set([0, 1, count // 2, count - 1] + list(range(0, count, 4099))))
    ok = True
    for i in sample:
        k = lay.keys[32 * int(lay.key_index[i]):32 * int(lay.key_index[i]) + 32]
        s, n, a, q = int(seqs[i]), int(lay.lens[i]), int(lay.in_off[i]), int(lay.out_off[i])
        exp = o.seal(k, struct.pack(">Q", s), pt_h[a:a + n].tobytes(), o.tls_ad(s, n))
        ok = ok and ct[q:q + n + 16].cpu().numpy().tobytes() == exp
    return {"bitexact_fold": fold == ref_fold, "fold_records": count, "bitexact_sample": ok,
            "sample_records": len(sample), "oracle_fold_s": round(fold_s, 2)}


def measure_record_path(args, bus):
    """The copy-inclusive rate (north star: "the rate including hipMemcpy to and
    from the GPU"; BASELINE.json configs[4]'s host side): sg_write_records /
    sg_read_records over --record-path-bytes of application data in host
    memory, 64 MiB per call, one direction at a time and both at once (writer
    and reader on two contexts and threads), from pageable buffers (the staged
    path) and from buffers registered with sg_host_register (zero-copy), wall
    clock around the calls, with the H2D / kernel / D2H / host-framing split
    per GiB (tools/record_path_bench.py).  Every byte read back is compared
    with the input, the duplex wire with the single-direction one, and a
    sample of the written records (first, every 4099th, last) with the
    oracle's TLS sealing of the same bytes (checker only).  Never `value`."""
    import struct

    import numpy as np

    sys.path.insert(0, str(ROOT / "tests"))
    sys.path.insert(0, str(ROOT / "tools"))
    from oracle_ffi import oracle as get_oracle  # checker only
    from record_path_bench import one

    o = get_oracle()
    rec = 16384
    wrec = 5 + rec + 16
    # on the CPUs of the card's NUMA node from here on (host buffers first
    # touched below, the copy threads created by the first record call)
    from suruga_amd import devmon

    prev = os.sched_getaffinity(0)
    cpus, how = devmon.pin_to_gpu_node(bus)

    def check_wire(data, wire, wlen):
        nrec = -(-data.size // rec)
        for r in sorted(set([0, nrec // 2, nrec - 1] + list(range(0, nrec, 4099)))):
            n = min(rec, data.size - r * rec)
            hdr = bytes([23, 3, 3]) + struct.pack(">H", n + 16)
            exp = hdr + o.seal(KEY, struct.pack(">Q", r), data[r * rec:r * rec + n].tobytes(), o.tls_ad(r, n))
            if wire[r * wrec:r * wrec + 5 + n + 16].tobytes() != exp:
                return False
        return True

    total = args.record_path_bytes
    runs = {}
    t0 = time.perf_counter()
    try:
        data = np.frombuffer(np.random.default_rng(0xC4).bytes(total), dtype=np.uint8).copy()
        for reg in (False, True):
            runs["registered" if reg else "pageable"] = one(total, 64 << 20, 0, reg, check_wire, data)
    finally:  # the timed C1 / C2 work before ran unpinned; so does whatever follows
        os.sched_setaffinity(0, prev)
    out = {"bytes": total, "call_bytes": 64 << 20, "copy_threads": int(os.environ.get("SG_COPY_THREADS", "8")),
           "note": "application GiB/s per direction from host memory, every copy inside; duplex.gibs counts both "
                   "directions' bytes; one key, seq from 0, content type 23, TLS 1.2 (tls.rs:126-130, 238-281)",
           **runs, "wall_s": round(time.perf_counter() - t0, 1)}
    out["correct"] = all(r["correct"] and r["duplex"]["correct"] and r["wire_sample_ok"] for r in runs.values())
    out["pinned"] = {"cpus": len(cpus) if cpus else None, "how": how}
    return out


def measure_scatter_gather(args, dist, backend, rank, world, dev, n, count, seq0, seal_b, lib, keys, ws, stream):
    """North star: RCCL over xGMI only to scatter inputs / gather outputs.
    Rank 0 holds S = --sg-records plaintext records for every rank, scatters
    them, each rank seals its slice, rank 0 gathers the sealed records back.
    Timed apart from the device-resident rate (best of 3, barrier + sync on
    both sides, MAX over ranks) and checked: every rank's received slice
    equals its own fill-rule records and rank 0 re-seals each gathered slice's
    plaintext and compares."""
    import ctypes as C

    import torch

    from suruga_amd import batch as B
    from suruga_amd import shard

    S = min(args.sg_records, count)
    # gloo rehearsals (several ranks on one card) move host tensors
    cdev = dev if backend == "nccl" else torch.device("cpu")
    mine = torch.empty(S * n, dtype=torch.uint8, device=cdev)
    sealed = torch.empty(S * (n + 16), dtype=torch.uint8, device=dev)
    src_chunks = gather_chunks = None
    seq_of = lambda r: r * args.records if not args.strong else shard.record_range(args.records, r, world)[0]  # noqa: E731
    if rank == 0:
        src_chunks, gather_chunks = [], []
        for r in range(world):
            t = torch.empty(S * n, dtype=torch.uint8, device=dev)
            B.fill_records(t, n, n, S, SEED, j0=seq_of(r))
            src_chunks.append(t.to(cdev))
            gather_chunks.append(torch.empty(S * (n + 16), dtype=torch.uint8, device=cdev))
    sync = torch.cuda.synchronize
    dd = dev if backend == "nccl" else None
    scatter_s = shard.timed_collective(dist, lambda: shard.scatter_records(dist, 0, mine, src_chunks), sync=sync,
                                       device=dd)
    mine_d = mine.to(dev)
    ok = bool(torch.equal(mine_d, torch.as_tensor(seal_b.inp[:S * n])))
    seal_s = B.Batch(count=S, keys=keys, inp=mine_d, out=sealed, uniform_len=n, in_stride=n, out_stride=n + 16,
                     seq0=seq0, workspace=ws, stream=stream).to_c()
    B.N.check(lib.sg_seal_batch(C.byref(seal_s)))
    torch.cuda.synchronize()
    sealed_c = sealed.to(cdev)
    gather_s = shard.timed_collective(dist, lambda: shard.gather_records(dist, 0, sealed_c, gather_chunks),
                                      sync=sync, device=dd)
    if rank == 0:
        check = torch.empty(S * (n + 16), dtype=torch.uint8, device=dev)
        for r in range(world):
            cs = B.Batch(count=S, keys=keys, inp=src_chunks[r].to(dev), out=check, uniform_len=n, in_stride=n,
                         out_stride=n + 16, seq0=seq_of(r), workspace=ws, stream=stream).to_c()
            B.N.check(lib.sg_seal_batch(C.byref(cs)))
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(check, gather_chunks[r].to(dev)))
    ok_all = sum_over_ranks(dist, 0.0 if ok else 1.0, dd) == 0.0
    moved_in, moved_out = (world - 1) * S * n, (world - 1) * S * (n + 16)  # bytes that cross the links
    return {"records_per_rank": S, "backend": "rccl" if backend == "nccl" else backend,
            "scatter_ms": round(scatter_s * 1e3, 3), "gather_ms": round(gather_s * 1e3, 3),
            "scatter_GBps": round(moved_in / scatter_s / 1e9, 2), "gather_GBps": round(moved_out / gather_s / 1e9, 2),
            "verified": ok_all,
            "note": "root rank 0 -> every rank and back, outside the device-resident value"}


def measure_scatter_gather_c2(args, dist, backend, rank, world, dev, lay, keys, stream):
    """C2 counterpart of measure_scatter_gather: rank 0 holds M = world x
    --sg-records mixed-size records (the first M of the Zipf layout, each with
    its connection key and sequence number), splits them into `world`
    contiguous byte-balanced ranges (shard.byte_balanced_ranges), scatters the
    plaintext bytes (padded to the largest slice), every rank seals its slice as
    one mixed batch, and rank 0 gathers the sealed slices and checks each
    against its own re-seal of the same records.  Every rank derives the
    slices' metadata from the shared layout; only record bytes travel."""
    import ctypes as C

    import numpy as np
    import torch

    from suruga_amd import batch as B
    from suruga_amd import shard

    M = min(args.sg_records * world, lay.count)
    lens = lay.lens[:M].astype(np.int64)
    rng = shard.byte_balanced_ranges(lens, world)
    in_off = lay.in_off[:M].astype(np.int64)
    # slice r: plaintext bytes [in_off[lo], end of record hi-1) of the layout; sealed records back to back (16-aligned)
    pt_span = [(int(in_off[lo]), int(in_off[hi - 1] + lens[hi - 1]) if hi > lo else int(in_off[lo])) for lo, hi in rng]
    pmax = max(b - a for a, b in pt_span)
    oslot = (lens + 16 + 15) // 16 * 16
    ct_len = [int(oslot[lo:hi].sum()) for lo, hi in rng]
    cmax = max(ct_len)
    cdev = dev if backend == "nccl" else torch.device("cpu")
    lib = B.N.load()

    def seal_slice(r, src_dev):
        lo, hi = rng[r]
        cnt = hi - lo
        out = torch.zeros(cmax, dtype=torch.uint8, device=dev)
        if cnt == 0:
            return out
        t64 = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.int64)).to(dev)  # noqa: E731
        t32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.int32)).to(dev)  # noqa: E731
        ioff = in_off[lo:hi] - in_off[lo]
        ooff = np.concatenate([[0], np.cumsum(oslot[lo:hi - 1])]).astype(np.int64)
        ws = torch.empty(B.workspace_size(cnt), dtype=torch.uint8, device=dev)
        b = B.Batch(count=cnt, keys=keys, inp=src_dev, out=out, lens=t32(lens[lo:hi]), max_len=int(lens[lo:hi].max()),
                    in_off=t64(ioff), out_off=t64(ooff), key_index=t32(lay.key_index[lo:hi]),
                    seq=t64(lay.seq[lo:hi].astype(np.int64)), workspace=ws, stream=stream).to_c()
        B.N.check(lib.sg_seal_batch(C.byref(b)))
        torch.cuda.synchronize()
        return out

    src_chunks = gather_chunks = None
    if rank == 0:
        full = torch.empty(pt_span[-1][1], dtype=torch.uint8, device=dev)
        B.fill_records(full, 0, full.numel(), 1, SEED, j0=0)
        src_chunks, gather_chunks = [], []
        for a, b_ in pt_span:
            t = torch.zeros(pmax, dtype=torch.uint8, device=dev)
            t[:b_ - a] = full[a:b_]
            src_chunks.append(t.to(cdev))
            gather_chunks.append(torch.empty(cmax, dtype=torch.uint8, device=cdev))
    mine = torch.empty(pmax, dtype=torch.uint8, device=cdev)
    sync = torch.cuda.synchronize
    dd = dev if backend == "nccl" else None
    scatter_s = shard.timed_collective(dist, lambda: shard.scatter_records(dist, 0, mine, src_chunks), sync=sync,
                                       device=dd)
    sealed = seal_slice(rank, mine.to(dev))
    sealed_c = sealed.to(cdev)
    gather_s = shard.timed_collective(dist, lambda: shard.gather_records(dist, 0, sealed_c, gather_chunks),
                                      sync=sync, device=dd)
    ok = True
    if rank == 0:
        for r in range(world):
            ok = ok and bool(torch.equal(seal_slice(r, src_chunks[r].to(dev))[:ct_len[r]],
                                         gather_chunks[r].to(dev)[:ct_len[r]]))
    ok_all = sum_over_ranks(dist, 0.0 if ok else 1.0, dd) == 0.0
    moved_in = sum(b - a for a, b in pt_span[1:])
    moved_out = sum(ct_len[1:])
    return {"records": M, "split": "byte_balanced_ranges", "ranges": [list(x) for x in rng],
            "backend": "rccl" if backend == "nccl" else backend,
            "scatter_ms": round(scatter_s * 1e3, 3), "gather_ms": round(gather_s * 1e3, 3),
            "scatter_GBps": round(moved_in / scatter_s / 1e9, 2), "gather_GBps": round(moved_out / gather_s / 1e9, 2),
            "verified": ok_all,
            "note": "root rank 0 -> every rank and back (slices padded to the largest), outside the device-resident value"}


def sum_over_ranks(dist, value, device=None):
    if dist is None:
        return value
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item())


def issue_roofline(dom, workload, count, cus, dom_ms, tj, isa, sclk_mhz):
    """The dominant launch against its VALU issue bound at the clock it ran at
    (VERDICT r3 item 2).  Model (profiles/r01_valu_issue_probes.md): a wave64
    VALU instruction costs 2 SIMD clocks when it is a v_add / v_xor of the
    lock-step ARX asm or any other full-rate opcode (paired with its SIMD
    partner wave), 4 otherwise (rotates and every half-rate instruction).  Instruction counts: the PMC
    SQ_INSTS_VALU of this build's profile (tj, per launch) split by the static
    census of the same sources (isa: tools/isa_census.py).  bound_ms = issue
    clocks per SIMD / sclk; frac = bound_ms / measured launch time (<= 1 when
    the model holds: the rest is stalls, barriers and launch tails).
    Full-rate opcodes outside the asm are priced at 2 as well: the measured
    cost of the feed-forward (124 v_add/v_xor per record, profiles/r04_ab:
    -1.5 % when removed) is the paired rate, not 4."""
    if not isa or not sclk_mhz:
        return {"bound": "valu", "unavailable": "no ISA census of this build" if not isa else "no sclk reading"}
    kern = isa["kernels"]
    simds = cus * SIMDS_PER_CU
    op = "true" if dom == "open" else "false"
    if workload == "c1":
        name = f"void sg::(anonymous namespace)::sg_wpr_kernel<{op}, true, 4u, false>(sg::KParams, sg::WprList)"
        k = kern.get(name)
        if k is None:
            return {"bound": "valu", "unavailable": f"{name} not in the census"}
        vpr = (tj or {}).get(f"{dom}_valu_per_record")
        src = "PMC SQ_INSTS_VALU per record (profile of this build)" if vpr else "static census (no PMC profile)"
        vpr = vpr or k["valu"]
        arx = k["arx_full"] + k["arx_rot"]
        oth = max(vpr - arx, 0.0)  # dynamic non-ARX VALU, split like the static census
        full_share = k["other_full"] / k["other_valu"] if k.get("other_valu") else 0.0
        clk_rec = 2 * k["arx_full"] + 4 * k["arx_rot"] + oth * (2 * full_share + 4 * (1 - full_share))
        clk = clk_rec * count / simds
        per = {"valu_per_record": round(vpr, 1), "arx_full_per_record": k["arx_full"],
               "arx_rot_per_record": k["arx_rot"], "other_valu_per_record": round(oth, 1),
               "other_full_rate_share": round(full_share, 3),
               "issue_clk_per_record": round(clk_rec, 1), "valu_source": src}
    else:
        byk = (tj or {}).get(f"{dom}_valu_by_kernel")
        if not byk:
            return {"bound": "valu", "unavailable": "no per-kernel PMC VALU counts of this build"}
        clk, per, miss = 0.0, {}, []
        for name, v in byk.items():
            k = kern.get(name)
            cpv = (k or {}).get("clk_per_valu_whole") or (k or {}).get("clk_per_valu")
            if not cpv:
                miss.append(name)
                continue
            clk += v * cpv / simds
            per[name] = {"valu": round(v), "clk_per_valu": cpv}
        per = {"kernels": per, "not_in_census": miss,
               "valu_source": "PMC SQ_INSTS_VALU per kernel and batch, priced with each kernel's static mix"}
    bound_ms = clk / (sclk_mhz * 1e3)
    return dict({"bound": "valu", "model": isa.get("model"), "sclk_mhz": sclk_mhz, "simds": simds,
                 "issue_bound_ms": round(bound_ms, 4), "avg_launch_ms": round(dom_ms, 4),
                 "frac": round(bound_ms / dom_ms, 4)}, **per)


def gather_over_ranks(dist, obj):
    """Every rank's `obj`, in rank order, on every rank (one entry without a group)."""
    if dist is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def rank_verdict(dist, mine: dict):
    """AND of every rank's correctness flags (rank 0 used to print
    its own).  `mine`: this rank's {"rank", "local_rank", "device",
    "roundtrip_ok", "bitexact_fold", "bitexact_sample"} (None = not checked).
    Returns (correct over all ranks, the per-rank list, the AND of each
    bit-exactness flag over the ranks that checked it)."""
    ranks = gather_over_ranks(dist, mine)
    correct = all(r["roundtrip_ok"] and r.get("bitexact_fold") is not False and r.get("bitexact_sample") is not False
                  for r in ranks)
    flags = {}
    for k in ("bitexact_fold", "bitexact_sample"):
        vals = [r.get(k) for r in ranks if r.get(k) is not None]
        flags[k] = all(vals) if vals else None
    return correct, ranks, flags


def correctness_fields(correct, ranks, flags, exact):
    """The line's correctness keys: rank 0's check details, overridden by the
    AND over every rank (a failing rank turns "correct" and its flag false)."""
    out = dict(exact or {})
    out.update({k: v for k, v in flags.items() if v is not None})
    out["correct"] = correct
    out["ranks"] = ranks
    return out


def exit_code(correct: bool) -> int:
    """Every rank exits 3 when any rank's check failed (0 otherwise)."""
    return 0 if correct else 3


def launch_ranks(args):
    """--gpus N without a launcher: start the N rank processes here, one per
    GPU (LOCAL_RANK r), with a 127.0.0.1 rendezvous, before this process makes
    any GPU call; wait for all of them and return the worst exit code (None:
    this process is itself a rank).  A rank that fails ends the others (its
    peers would wait at the next barrier forever)."""
    import signal
    import socket
    import subprocess

    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher set WORLD_SIZE={ws}")
        return None
    if args.gpus <= 1:
        return None
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []

    def forward(signum, _frame):  # a launcher stopped by a signal stops the ranks it started
        for pr in procs:
            if pr.poll() is None:
                pr.send_signal(signal.SIGTERM)
        raise SystemExit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env))
    rcs = [None] * len(procs)
    while any(rc is None for rc in rcs):
        for i, pr in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = pr.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, pr in enumerate(procs):  # the ranks this process started, by PID
                if rcs[i] is None:
                    pr.send_signal(signal.SIGTERM)
            for i, pr in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = pr.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        pr.kill()
                        rcs[i] = pr.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr, flush=True)
    return bad[0] if bad else 0


def make_workload(args, workload, count, seq0, dev, stream):
    """Device buffers and batch descriptors of one workload (C1: uniform 16 KiB
    records, one key; C2: the Zipf layout with 256 connection keys), inputs
    generated on the device."""
    import numpy as np
    import torch

    from suruga_amd import batch as B

    n = args.record_bytes
    w = {"workload": workload, "count": count, "seq0": seq0, "n": n, "lay": None, "cs": None}
    ws = torch.empty(B.workspace_size(count), dtype=torch.uint8, device=dev)
    status = torch.empty(count, dtype=torch.uint8, device=dev)
    if workload == "c1":
        keys = torch.tensor(list(KEY), dtype=torch.uint8, device=dev).view(1, 32)
        pt = torch.empty(count * n, dtype=torch.uint8, device=dev)
        cs = args.ct_stride or (n + 16 + 127) // 128 * 128
        if cs < n + 16 or cs % 16:
            raise SystemExit("--ct-stride must be >= n + 16 and a multiple of 16")
        ct = torch.empty(count * cs, dtype=torch.uint8, device=dev)
        back = torch.empty(count * n, dtype=torch.uint8, device=dev)
        B.fill_records(pt, n, n, count, SEED, j0=seq0)
        seal_b = B.Batch(count=count, keys=keys, inp=pt, out=ct, uniform_len=n, in_stride=n, out_stride=cs,
                         seq0=seq0, workspace=ws, stream=stream)
        open_b = B.Batch(count=count, keys=keys, inp=ct, out=back, uniform_len=n + 16, in_stride=cs,
                         out_stride=n, seq0=seq0, status=status, workspace=ws, stream=stream)
        w["payload_per_step"] = 2 * count * n
        w["alg"] = {"seal": (2 * n + 69) * count, "open": (2 * n + 70) * count}
        w["alg_read"] = {"seal": (n + 53) * count, "open": (n + 69) * count}  # R alone: pt|ct(+tag) + ad + nonce + key
        cfg = {"workload": f"C1: {count} x {n} B TLS records per GPU, one key, sequential seq, seal then open, "
                           "device-resident", "records_per_gpu": count, "record_bytes": n}
        cfg["layout"] = (f"plaintext records back to back ({n} B stride); sealed records (ct||tag) at a {cs} B "
                         f"stride" + (" (128-byte aligned slots)" if cs % 128 == 0 and cs != n + 16 else ""))
        w["cmp_args"] = (pt, n, back, n, n, count)
        w["cs"] = cs
    else:
        from suruga_amd import workloads as W

        lay = W.c2_layout(count, ct_align=args.c2_ct_align, pt_align=args.c2_pt_align)
        t64 = lambda a: torch.from_numpy(a.view(np.int64)).to(dev)  # noqa: E731
        t32 = lambda a: torch.from_numpy(a.view(np.int32)).to(dev)  # noqa: E731
        keys = torch.tensor(list(lay.keys), dtype=torch.uint8, device=dev).view(-1, 32)
        pt = torch.empty(lay.pt_bytes, dtype=torch.uint8, device=dev)
        ct = torch.empty(lay.ct_bytes, dtype=torch.uint8, device=dev)
        back = torch.empty(lay.pt_bytes, dtype=torch.uint8, device=dev)
        B.fill_records(pt, 0, lay.pt_bytes, 1, SEED, j0=seq0)
        if args.c2_pt_align != 64:  # padding between plaintext records: zero in pt and back (the compare is 64-byte granules)
            starts = torch.from_numpy(lay.in_off.view(np.int64)).to(dev)
            ln = torch.from_numpy(lay.lens.astype(np.int64)).to(dev)
            mark = torch.zeros(lay.pt_bytes + 1, dtype=torch.int32, device=dev)
            mark.index_add_(0, starts, torch.ones_like(starts, dtype=torch.int32))
            mark.index_add_(0, starts + ln, -torch.ones_like(starts, dtype=torch.int32))
            real = torch.cumsum(mark, 0)[:lay.pt_bytes] > 0
            pt[~real] = 0
            back.zero_()
        lens, olens = t32(lay.lens), t32(lay.lens + 16)
        in_off, out_off, kidx = t64(lay.in_off), t64(lay.out_off), t32(lay.key_index)
        seqs = t64(lay.seq + np.uint64(seq0 // 256))
        maxl = int(lay.lens.max())
        seal_b = B.Batch(count=count, keys=keys, inp=pt, out=ct, lens=lens, max_len=maxl, in_off=in_off,
                         out_off=out_off, key_index=kidx, seq=seqs, workspace=ws, stream=stream)
        open_b = B.Batch(count=count, keys=keys, inp=ct, out=back, lens=olens, max_len=maxl + 16, in_off=out_off,
                         out_off=in_off, key_index=kidx, seq=seqs, status=status, workspace=ws, stream=stream)
        w["payload_per_step"] = 2 * lay.payload
        w["alg"] = {"seal": 2 * lay.payload + 69 * count, "open": 2 * lay.payload + 70 * count}
        w["alg_read"] = {"seal": lay.payload + 53 * count, "open": lay.payload + 69 * count}
        cfg = {"workload": f"C2: {count} TLS records per GPU, Zipf(1.1) sizes 64 B-16 KiB (mean "
                           f"{lay.payload / count:.0f} B), 256 connection keys, seal then open, device-resident",
                           "records_per_gpu": count, "record_bytes": "zipf",
                           "layout": (f"plaintext records {args.c2_pt_align}-byte aligned"
                                      + (" (back to back)" if args.c2_pt_align == 64 else "")
                                      + f"; sealed records {args.c2_ct_align}-byte aligned")}
        w["cmp_args"] = (pt, 64, back, 64, 64, lay.pt_bytes // 64)  # 64-byte granules
        w["lay"] = lay
    w.update(keys=keys, pt=pt, ct=ct, back=back, ws=ws, status=status, seal_b=seal_b, open_b=open_b, cfg=cfg,
             seal_c=seal_b.to_c(), open_c=open_b.to_c())
    return w


def energy_fields(mon_e, tm_e, count, dom):
    """Energy per record at the power cap: the board power
    averaged over the second half of a >= --energy-seconds window of event-timed
    steps (power1_average is a running average that climbs from idle through a
    short run, so the first half is dropped), times each launch's event time in
    that same window, per record of the launch."""
    pw = (mon_e.get("board_power_w") or {}).get("mean")
    if not pw or not tm_e.get("seal_ms"):
        return {"unavailable": "no board power reading" if not pw else "no event-timed launches"}
    uj = lambda ms: round(pw * ms * 1e-3 / count * 1e6, 3)  # noqa: E731
    return {"board_power_w": pw, "sclk_mhz": (mon_e.get("sclk_mhz") or {}).get("mean"),
            "seal_ms": round(tm_e["seal_ms"], 4), "open_ms": round(tm_e["open_ms"], 4),
            "keying_ms": round(tm_e["keying_ms"], 4),
            "seal_uj_per_record": uj(tm_e["seal_ms"]), "open_uj_per_record": uj(tm_e["open_ms"]),
            "keying_uj_per_record": uj(tm_e["keying_ms"]),
            "energy_per_record_uj": uj(tm_e[f"{dom}_ms"]),
            "window_s": round(mon_e.get("window_s", 0.0), 3), "launches": int(tm_e.get("n_seal", 0)),
            "note": "board power (sysfs, mean of the window's second half) x event-timed launch time / records"}


def run_measurement(args, w, steps, warmup, dist, backend, rank, local, local_dev, dev, stream, sampler, lib, bus):
    """Warm-up, the timed region (barrier + sync on both sides, MAX over ranks),
    event-timed kernel times right after it, an energy window, and the checks of
    the last step (outside every timed region)."""
    import ctypes as C

    import torch

    from suruga_amd import batch as B
    from suruga_amd import shard

    seal_c, open_c = w["seal_c"], w["open_c"]

    def step():
        B.N.check(lib.sg_seal_batch(C.byref(seal_c)))
        B.N.check(lib.sg_open_batch(C.byref(open_c)))

    torch.cuda.synchronize()  # inputs and tables made on the default stream
    for _ in range(warmup):
        step()
    t_region0 = time.perf_counter()
    elapsed = shard.timed(dist, step, steps, sync=torch.cuda.synchronize,
                          device=dev if backend == "nccl" else None)
    t_region1 = time.perf_counter()

    # per-kernel device time with HIP events on the launch stream, right after
    # the timed steps while the GPU is still at its steady-state clock (round 2
    # took them after the CPU oracle fold, on a GPU that had idled for seconds)
    B.set_timing(True)
    t_ev0 = time.perf_counter()
    for _ in range(max(5, min(steps, 10))):
        step()
    tm = B.timing_read()  # (waits for the last event)
    t_ev1 = time.perf_counter()
    B.set_timing(False)
    # energy window (round 5): event-timed steps for >= --energy-seconds, the
    # board at its sustained power; its second half prices energy per record
    tm_e, mon_e = None, None
    if args.energy_seconds > 0:
        # steps per half window from the timed region's step time (the calls
        # are asynchronous: a wall-clock loop would only fill the queue)
        half = max(5, int(0.5 * args.energy_seconds / max(elapsed / steps, 1e-4)))
        t_e0 = time.perf_counter()
        for _ in range(half):  # first half: the board's running power average settles
            step()
        torch.cuda.synchronize()
        B.set_timing(True)
        t_h0 = time.perf_counter()
        for _ in range(half):
            step()
        tm_e = B.timing_read()  # (waits for the last event)
        t_h1 = time.perf_counter()
        B.set_timing(False)
        mon_e = sampler.summary(t_h0, t_h1)
        mon_e["window_s"] = t_h1 - t_e0
    mon = sampler.summary(t_region0, t_region1)
    # the clock of the event-timed steps, whose launch times the issue bound
    # prices (round 4: in a short run the clock still climbs through the timed
    # region, so its mean undercuts the clock the event-timed launches ran at)
    mon["event_steps_sclk_mhz"] = sampler.summary(t_ev0, t_ev1)["sclk_mhz"]

    # correctness of the last step (outside the timed region): every record
    # round-trips, and every tag and a sample of records equal the oracle's;
    # the verdict is the AND over all ranks
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    B.compare_records(*w["cmp_args"], mism, stream=stream)
    torch.cuda.synchronize()
    bad_status = int((w["status"] != 0).sum().item())
    roundtrip_ok = int(mism.item()) == 0 and bad_status == 0
    exact = None
    if not args.no_bitexact:
        torch.cuda.synchronize()
        exact = bitexact_check(w["ct"], w["n"], w["count"], w["seq0"], w["cs"]) if w["workload"] == "c1" else \
            bitexact_check_c2(w["lay"], w["pt"], w["ct"], w["seq0"] // 256)
    if os.environ.get("SG_BENCH_CORRUPT_RANK") == str(rank) and exact is not None:
        exact["bitexact_fold"] = False  # test hook (tests/test_bench_contract.py): a rank whose check fails
    mine = {"rank": rank, "local_rank": local, "device": local_dev, "pci_bus": bus, "roundtrip_ok": roundtrip_ok,
            "bitexact_fold": exact["bitexact_fold"] if exact else None,
            "bitexact_sample": exact["bitexact_sample"] if exact else None}
    correct, ranks, flags = rank_verdict(dist, mine)
    return {"elapsed": elapsed, "tm": tm, "mon": mon, "tm_e": tm_e, "mon_e": mon_e, "exact": exact,
            "correct": correct, "ranks": ranks, "flags": flags}


def kernel_fields(args, w, r, steps, world, dist, backend, dev, lib, props):
    """value, the dominant launch's HBM roofline (PMC traffic of the same build
    and layout), its VALU issue bound and the event-timed kernel times."""
    count, n, tm, mon = w["count"], w["n"], r["tm"], r["mon"]
    total_payload_per_step = w["payload_per_step"] * world if not args.strong else int(
        sum_over_ranks(dist, w["payload_per_step"], dev if backend == "nccl" else None))
    value = total_payload_per_step * steps / r["elapsed"] / 2**30
    ms_per_step = r["elapsed"] / steps * 1e3
    # dominant kernel's roofline (algorithmic bytes per launch):
    # seal R+W = 2n + 69 per record, open = 2n + 70
    dom = "open" if tm["open_ms"] >= tm["seal_ms"] else "seal"
    alg_bytes = w["alg"][dom]
    dom_ms = tm[f"{dom}_ms"]
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    achieved_read = w["alg_read"][dom] / (dom_ms * 1e-3) / 1e9
    # the event-timed kernels of one step against the wall-clock step
    kernel_sum_ms = tm["seal_ms"] + tm["open_ms"] + 2 * tm["keying_ms"]
    cfg = w["cfg"]
    traffic, traffic_src, tj = None, None, None
    # the PMC traffic summary of this exact kernel build and workload (the newest
    # profiles/traffic_*.json whose build string and record shape match)
    build = lib.sg_build_info().decode()
    cands = [Path(args.traffic)] if args.traffic else sorted(
        (ROOT / "profiles").glob("traffic_*.json"), key=lambda q: q.stat().st_mtime, reverse=True)
    for q in cands:
        try:
            tq = json.loads(q.read_text())
        except (ValueError, OSError):
            continue
        if tq.get("records") == count and tq.get("record_bytes") == cfg["record_bytes"] and \
                tq.get("kernels") == build and tq.get("layout") == cfg.get("layout") and \
                tq.get(f"{dom}_bytes_per_launch"):
            tj = tq
            traffic = tq.get(f"{dom}_bytes_per_launch")
            traffic_src = (f"profiles/{q.name}: rocprofv3 PMC FETCH_SIZE x 2 + WRITE_SIZE of this kernel build "
                           "and record layout in a separate profiling run (not this run)")
            break
    # the static ISA census of the loaded library's sources (tools/isa_census.py)
    from suruga_amd import batch as B

    provenance = B.N.loaded_info()
    isa = None
    isa_path = ROOT / "profiles" / f"isa_{provenance['source_hash']}.json"
    if isa_path.exists():
        try:
            isa = json.loads(isa_path.read_text())
        except ValueError:
            isa = None
    sclk = (mon.get("sclk_mhz") or {}).get("mean")
    sclk_ev = (mon.get("event_steps_sclk_mhz") or {}).get("mean") or sclk
    valu = issue_roofline(dom, w["workload"], count, props.multi_processor_count, dom_ms, tj, isa, sclk_ev)
    if valu.get("sclk_mhz") is not None:
        valu["sclk_window"] = "event-timed steps (the launches avg_launch_ms is taken from)"
    wpr_on = w["workload"] == "c1" and n == 16384 and lib.sg_set_lockstep(-1) == 1
    if w["workload"] == "c1":
        dom_kernel = f"sg_wpr_kernel<{dom.upper()}>" if wpr_on else f"sg_aead_kernel<{dom.upper()}, 256>"
        if dom == "open":  # (the open window also holds the failed-record scrub: one status byte per record)
            dom_kernel += " + sg_scrub_kernel"
        keying_note = "kernel_ms.keying: the sg_wpr_keying_kernel pre-pass, timed apart from the record launch"
    else:
        # the mixed batch's record window opens before the packed launch, so it
        # also holds the keying launches (side stream, beside the packed tail)
        dom_kernel = (f"sg_wpr_kernel<{dom.upper()}, J=2..4> + sg_pack_kernel<{dom.upper()}> + size classes + their "
                      "keying launches (one batch, from the packed launch to the last list)")
        keying_note = ("kernel_ms.keying: the tail memset, sg_classify_kernel and the population readback; the "
                       "keying launches are inside the seal/open window")
    energy = energy_fields(r["mon_e"], r["tm_e"], count, dom) if r["mon_e"] is not None else None
    return {
        "value": value, "ms_per_step": ms_per_step, "dom": dom, "build": build, "provenance": provenance,
        "sclk": sclk,
        "roofline": {"bound": "hbm", "kernel": dom_kernel,
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(dom_ms, 4),
                     # SURVEY.md 8(d)'s read-only variant (the north star's "HBM-read roofline")
                     "hbm_read": {"achieved": round(achieved_read, 1), "frac": round(achieved_read / HBM_PEAK_GBS, 4),
                                  "alg_read_bytes_per_launch": w["alg_read"][dom]}},
        "valu_roofline": valu,
        "kernel_ms": {"seal": round(tm["seal_ms"], 4), "open": round(tm["open_ms"], 4),
                      "keying": round(tm["keying_ms"], 4), "sum_per_step": round(kernel_sum_ms, 4),
                      "sum_vs_step": round(kernel_sum_ms / ms_per_step, 4),
                      "launches": int(tm.get("n_seal", 0)) + int(tm.get("n_open", 0)),
                      "note": "HIP events on the launch stream over steps run right after the timed region; "
                              + keying_note},
        "energy": energy,
        "records_per_s": round((args.records if args.strong else count * world) * steps / r["elapsed"], 1),
    }


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU; the process group only carries the timing protocol
    # (barriers + MAX of the elapsed time): RCCL ("nccl") by default, gloo for
    # rehearsing several ranks on one card (SG_DIST_BACKEND=gloo)
    backend = os.environ.get("SG_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if ndev else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    from suruga_amd import _build
    from suruga_amd import batch as B
    from suruga_amd import shard

    if not _build.LIB.exists():  # normally prebuilt in-tree; only rank 0 builds, the others wait
        if rank == 0:
            _build.build_library()
        if dist is not None:
            dist.barrier()
    n = args.record_bytes
    if args.strong:  # total work fixed: rank r owns a contiguous slice of --records
        lo, hi = shard.record_range(args.records, rank, world)
        count, seq0 = hi - lo, lo
    else:            # weak scaling (the metric's mode): --records per rank, seq r*records + i
        count, seq0 = args.records, rank * args.records
    # the batch calls run asynchronously on a stream of their own: on the NULL
    # (default) stream every call would end with a device sync (suruga_gpu.h)
    stream = torch.cuda.Stream(dev)
    w = make_workload(args, args.workload, count, seq0, dev, stream)
    lib = B.N.load()
    # the shader clock and board power (sysfs, plain reads on a background
    # thread from the warm-up to the end of the last measurement): the
    # issue-bound roofline is priced at the mean clock of the event-timed steps
    from suruga_amd import devmon

    props = torch.cuda.get_device_properties(dev)
    bus = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    sampler = devmon.Sampler(bus).start()
    r = run_measurement(args, w, args.steps, args.warmup, dist, backend, rank, local, local_dev, dev, stream,
                        sampler, lib, bus)
    kf = kernel_fields(args, w, r, args.steps, world, dist, backend, dev, lib, props)
    correct, ranks, flags, exact = r["correct"], r["ranks"], r["flags"], r["exact"]

    scatter_gather = None
    if world > 1 and args.sg_records > 0:
        try:  # a side measurement: a failure here is reported, not fatal to the device-resident line
            if args.workload == "c1":
                scatter_gather = measure_scatter_gather(args, dist, backend, rank, world, dev, n, count, seq0,
                                                        w["seal_b"], lib, w["keys"], w["ws"], stream)
            else:
                scatter_gather = measure_scatter_gather_c2(args, dist, backend, rank, world, dev, w["lay"], w["keys"],
                                                           stream)
        except (RuntimeError, ValueError) as e:
            scatter_gather = {"error": f"{type(e).__name__}: {e}"[:300]}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, n) if args.workload == "c1" else cpu_baseline(args, 0, w["lay"])

    # the C2 sub-record: after the C1 line's measurement,
    # the full Zipf batch of BASELINE.json configs[2] under the same protocol;
    # `value` stays C1's.  Its correctness joins the line's.
    c2 = None
    cfg1 = w["cfg"]
    if args.workload == "c1" and args.c2_steps > 0:
        del w
        torch.cuda.empty_cache()
        w2 = make_workload(args, "c2", count, seq0, dev, stream)
        r2 = run_measurement(args, w2, args.c2_steps, args.warmup, dist, backend, rank, local, local_dev, dev,
                             stream, sampler, lib, bus)
        k2 = kernel_fields(args, w2, r2, args.c2_steps, world, dist, backend, dev, lib, props)
        c2 = {"metric": "GiB/s device-resident ChaCha20-Poly1305 over Zipf 64 B-16 KiB TLS records (C2)",
              "value": round(k2["value"], 3), "unit": "GiB/s", "steps": args.c2_steps, "warmup": args.warmup,
              "ms_per_step": round(k2["ms_per_step"], 4), "config": w2["cfg"], "roofline": k2["roofline"],
              "valu_roofline": k2["valu_roofline"], "kernel_ms": k2["kernel_ms"], "energy": k2["energy"],
              "sclk_mhz": k2["sclk"], "records_per_s": k2["records_per_s"], "correct": r2["correct"],
              "ranks": r2["ranks"], **{kk: vv for kk, vv in (r2["exact"] or {}).items()},
              **{kk: vv for kk, vv in r2["flags"].items() if vv is not None}}
        correct = correct and r2["correct"]
        del w2
        torch.cuda.empty_cache()
    # the copy-inclusive rate of the record path: a side
    # measurement after the device-resident lines; its correctness joins the line's
    record_path = None
    if rank == 0 and world == 1 and args.record_path_bytes > 0:
        try:
            record_path = measure_record_path(args, bus)
            correct = correct and record_path["correct"]
        except (RuntimeError, OSError, ValueError) as e:
            record_path = {"error": f"{type(e).__name__}: {e}"[:300]}
    sampler.stop()
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(kf["value"], 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(kf["ms_per_step"], 4),
            "higher_is_better": True, "scaling": "strong" if args.strong else "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 records generated on device)",
            "config": dict(cfg1, parallelism=f"record-shard x{world}", kernels=kf["build"], library=kf["provenance"]),
            "roofline": kf["roofline"],
            "valu_roofline": kf["valu_roofline"],
            "sclk_mhz": kf["sclk"],
            "board_power_w": (r["mon"].get("board_power_w") or {}).get("last"),
            "energy_per_record_uj": (kf["energy"] or {}).get("energy_per_record_uj"),
            "energy": kf["energy"],
            "device_monitor": r["mon"],
            "kernel_ms": kf["kernel_ms"],
            "records_per_s": kf["records_per_s"],
            "cpu_baseline": cpu,
        }
        line.update(correctness_fields(r["correct"], ranks, flags, exact))
        line["correct"] = correct
        if scatter_gather is not None:
            line["scatter_gather"] = scatter_gather
        if c2 is not None:
            line["c2"] = c2
        if record_path is not None:
            line["record_path"] = record_path
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if exit_code(correct):
        sys.exit(exit_code(correct))


if __name__ == "__main__":
    main()
