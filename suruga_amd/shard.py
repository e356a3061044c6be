"""Record sharding across GPUs.

Records are independent given (key, seq, ad), so N GPUs split a batch into
contiguous record ranges with no collective in the data path: each rank
seals/opens its own range with sequence numbers seq0 + lo .. seq0 + hi - 1
and its own copy of the key table.  Mixed-size batches (C2) are split by
bytes (prefix sum of lengths), not by record count.  The only communication is
the timing protocol of the benchmark: a barrier on both sides of the timed
region and a MAX over ranks of the elapsed time.

When the records start or end on one GPU (a host feeding one device), the
north star's "RCCL over xGMI only to scatter inputs / gather outputs" applies:
`scatter_records` / `gather_records` move equal byte slices between a root and
every rank (torch.distributed scatter/gather: RCCL send/recv over xGMI on
MI355X, gloo on CPU).  They sit outside the device-resident rate and are timed
on their own (`timed_collective`, bench.py "scatter_gather").
"""
from __future__ import annotations

import bisect
from typing import Sequence, Tuple


def record_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of `total` records for `rank`; sizes differ by <= 1."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def byte_balanced_ranges(lens: Sequence[int], world: int):
    """Split records into `world` contiguous ranges of ~equal payload bytes.

    Boundary r is the first record whose byte prefix reaches r/world of the
    total, so every range's payload differs from total/world by less than one
    record.  Returns [(lo, hi)] * world."""
    prefix = [0]
    for n in lens:
        prefix.append(prefix[-1] + int(n))
    total = prefix[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        i = bisect.bisect_left(prefix, target)
        # pick the closer of the two prefix points around the target
        if i > 0 and abs(prefix[i - 1] - target) <= abs(prefix[min(i, len(prefix) - 1)] - target):
            i -= 1
        cuts.append(max(cuts[-1], min(i, len(lens))))
    cuts.append(len(lens))
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def max_over_ranks(dist, value: float, device=None) -> float:
    """MAX of a per-rank float over the process group (the bench's clock)."""
    if dist is None:
        return value
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(dist, fn, steps: int, sync=None, device=None) -> float:
    """Run `fn` `steps` times bracketed by barrier + device sync on both sides;
    return the wall time, max over ranks."""
    import time

    if sync:
        sync()
    if dist:
        dist.barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    if sync:
        sync()
    if dist:
        dist.barrier()
    return max_over_ranks(dist, time.perf_counter() - t0, device)


def scatter_records(dist, src: int, out, chunks=None):
    """Rank `src` sends chunks[r] (one tensor per rank, same shape and dtype
    as `out`) to rank r; every rank receives its slice into `out`."""
    if dist is None:
        out.copy_(chunks[0])
        return out
    dist.scatter(out, scatter_list=chunks if dist.get_rank() == src else None, src=src)
    return out


def gather_records(dist, dst: int, inp, chunks=None):
    """Every rank sends `inp`; rank `dst` receives rank r's into chunks[r]."""
    if dist is None:
        chunks[0].copy_(inp)
        return chunks
    dist.gather(inp, gather_list=chunks if dist.get_rank() == dst else None, dst=dst)
    return chunks


def timed_collective(dist, fn, reps: int = 3, sync=None, device=None) -> float:
    """Best of `reps` runs of one collective, each bracketed like `timed`
    (barrier + device sync on both sides, MAX over ranks)."""
    return min(timed(dist, fn, 1, sync=sync, device=device) for _ in range(reps))
