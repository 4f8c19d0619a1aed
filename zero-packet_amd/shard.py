"""Multi-GPU sharding of a packet batch.

Every frame is an independent unit of PacketParser::parse
(/root/reference/src/packet/parser.rs:53 takes one byte slice and touches
nothing else), so a batch splits into contiguous frame ranges, one per rank
(one process per GPU, torch.distributed), with no data-path collective. The
only cross-rank traffic is the timing reduction (max over ranks) and,
optionally, gathering small per-rank summaries on the host.

    shard_bounds(lens, world)        contiguous frame ranges balanced by bytes
    local_shard(offs, lens, lo, hi)  byte window [b0, b1) + rebased offsets
    rank_shard(arena, offs, lens, rank, world)   both, applied to host arrays
"""
import numpy as np


def shard_bounds(lens, world):
    """Splits frames 0..n-1 into `world` contiguous ranges whose byte totals
    are as equal as possible: rank r gets [bounds[r], bounds[r+1]). Cuts are
    placed at the first frame whose exclusive byte prefix reaches r/world of
    the total (deterministic: every rank computes the same bounds)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    lens = np.asarray(lens, dtype=np.uint64)
    n = lens.size
    if n == 0:
        return [0] * (world + 1)
    excl = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1], out=excl[1:])
    total = int(excl[-1] + lens[-1])
    targets = [(total * r) // world for r in range(1, world)]
    cuts = np.searchsorted(excl, np.asarray(targets, dtype=np.uint64), side="left").tolist()
    return [0] + [int(c) for c in cuts] + [n]


def local_shard(offs, lens, lo, hi):
    """Byte window [b0, b1) of the arena that holds frames lo..hi-1 (any
    layout: gaps, overlap and order are allowed) and their offsets rebased to
    that window."""
    offs = np.asarray(offs, dtype=np.uint64)[lo:hi]
    lens = np.asarray(lens, dtype=np.uint32)[lo:hi]
    if offs.size == 0:
        return 0, 0, offs.copy(), lens.copy()
    b0 = int(offs.min())
    b1 = int((offs + lens.astype(np.uint64)).max())
    return b0, b1, offs - np.uint64(b0), lens.copy()


def rank_shard(arena, offs, lens, rank, world):
    """(arena slice, rebased offs, lens, (lo, hi)) of rank `rank`'s frames."""
    bounds = shard_bounds(lens, world)
    lo, hi = bounds[rank], bounds[rank + 1]
    b0, b1, o, ln = local_shard(offs, lens, lo, hi)
    return arena[b0:b1], o, ln, (lo, hi)
