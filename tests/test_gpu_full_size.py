"""Parity at BASELINE.json's full sizes (C1: 2^20 x 16 KiB; C2: 2^20 Zipf
records, 256 connection keys): every record round-trips on the device, and
the XOR-fold of all 2^20 tags equals the oracle's multithreaded fold of the
same records (oracle/suruga_oracle.c, a checker only), plus whole records of a
strided sample byte for byte.  The same checks bench.py makes outside its
timed region, here in the GPU suite the driver runs."""
import os
import struct

import numpy as np
import pytest

from test_gpu_parity import KEY, SEED, dev_bytes, tls_batch, torch_mod

pytestmark = pytest.mark.gpu


def _threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def test_c1_full_size_tag_fold(gpu, oracle):
    torch = torch_mod()
    from suruga_amd import batch as B

    count, n, seq0 = 1 << 20, 16384, 3
    pt, ct, back, st = tls_batch(count, n, seq0=seq0)
    mism = torch.zeros(1, dtype=torch.int64, device="cuda")
    B.compare_records(pt, n, back, n, n, count, mism)
    torch.cuda.synchronize()
    assert int(mism.item()) == 0 and int(st.sum().item()) == 0
    del back
    rows = ct.view(count, n + 16)
    fold = np.bitwise_xor.reduce(rows[:, n:].cpu().numpy(), axis=0).tobytes()
    assert fold == oracle.tag_fold_tls(KEY, seq0, SEED, 0, n, count, threads=_threads())
    for i in [0, 1, count // 2, count - 1] + list(range(7, count, 65537)):
        exp = oracle.seal(KEY, struct.pack(">Q", seq0 + i), oracle.fill_record(SEED, i, n), oracle.tls_ad(seq0 + i, n))
        assert rows[i].cpu().numpy().tobytes() == exp, i


def test_c2_full_size_tag_fold(gpu, oracle):
    torch = torch_mod()
    from suruga_amd import batch as B
    from suruga_amd import workloads as W

    lay = W.c2_layout(1 << 20, ct_align=128)
    count = lay.count
    gen = torch.Generator(device="cuda").manual_seed(11)
    pt = torch.randint(0, 256, (lay.pt_bytes,), dtype=torch.uint8, device="cuda", generator=gen)
    t64 = lambda a: torch.from_numpy(a.view(np.int64)).to("cuda")
    t32 = lambda a: torch.from_numpy(a.view(np.int32)).to("cuda")
    keys = dev_bytes(lay.keys).view(-1, 32)
    common = dict(count=count, keys=keys, key_index=t32(lay.key_index), seq=t64(lay.seq))
    maxl = int(lay.lens.max())
    ct = torch.zeros(lay.ct_bytes, dtype=torch.uint8, device="cuda")
    B.seal(B.Batch(inp=pt, out=ct, lens=t32(lay.lens), max_len=maxl, in_off=t64(lay.in_off),
                   out_off=t64(lay.out_off), **common))
    back = torch.zeros(lay.pt_bytes, dtype=torch.uint8, device="cuda")
    st = torch.full((count,), 0xFF, dtype=torch.uint8, device="cuda")
    B.open_(B.Batch(inp=ct, out=back, lens=t32(lay.lens + 16), max_len=maxl + 16, in_off=t64(lay.out_off),
                    out_off=t64(lay.in_off), status=st, **common))
    torch.cuda.synchronize()
    assert int(st.sum().item()) == 0
    # C2 plaintext records are back to back (lengths are multiples of 64, 64-byte
    # slots): the whole buffer comes back
    assert lay.pt_bytes == int(lay.lens.astype(np.uint64).sum()) and bool(torch.equal(back, pt))
    del back
    tag_at = t64(lay.out_off + lay.lens.astype(np.uint64))
    idx = (tag_at.view(-1, 1) + torch.arange(16, device="cuda").view(1, 16)).view(-1)
    fold = np.bitwise_xor.reduce(ct[idx].view(count, 16).cpu().numpy(), axis=0).tobytes()
    pt_h = pt.cpu().numpy()
    assert fold == oracle.tag_fold_mixed(lay.keys, lay.key_index, lay.seq, lay.lens, lay.in_off, pt_h,
                                         threads=_threads())
    for i in [0, 1, count // 2, count - 1] + list(range(5, count, 65537)):
        k = lay.keys[32 * int(lay.key_index[i]):32 * int(lay.key_index[i]) + 32]
        s, n, a, q = int(lay.seq[i]), int(lay.lens[i]), int(lay.in_off[i]), int(lay.out_off[i])
        exp = oracle.seal(k, struct.pack(">Q", s), pt_h[a:a + n].tobytes(), oracle.tls_ad(s, n))
        assert ct[q:q + n + 16].cpu().numpy().tobytes() == exp, (i, n)
