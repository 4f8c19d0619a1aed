"""Per-batch counters over parse records (zp_stats_device).

    counts = stats.count(records)          # int64 device tensor [ZP_STATS_COUNT]
    stats.to_dict(counts)                  # {"ipv4": ..., "tcp": ..., "err:OK": ...}
    stats.combine([c0, c1, ...])           # the ranks' arrays summed on the host

Frames per presence bit of zp_record.flags (the nine PacketParser Options,
the IpInIp tag, both Option<ExtensionHeaders> and their slots) and frames per
zp_err code. Several batches accumulate into one array; the arrays of
several GPUs add up on the host (frames are independent, no exchange step).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .records import ERR_NAMES, EXT_SLOTS, RECORD_BYTES

FLAG_BITS = 24
FLAG_NAMES = (["ethernet", "arp", "ipv4", "ipv6", "ip_in_ip", "ip_in_ip_v6", "tcp", "udp",
               "icmpv4", "icmpv6", "ext", "inner_ext"] +
              [f"ext:{s}" for s in EXT_SLOTS] + [f"inner_ext:{s}" for s in EXT_SLOTS])
NAMES = FLAG_NAMES + [f"err:{e}" for e in ERR_NAMES]
COUNT = len(NAMES)                       # ZP_STATS_COUNT
assert len(FLAG_NAMES) == FLAG_BITS


def count(records, counts=None, stream=None):
    """Adds the counts of `records` (uint8 [n, 8] device tensor) into
    `counts` (int64 [COUNT] device tensor, zeroed when not given)."""
    if not records.is_cuda:
        raise RuntimeError("stats.count needs device records (no CPU fallback)")
    if (records.dtype != torch.uint8 or records.dim() != 2 or records.shape[1] != RECORD_BYTES
            or not records.is_contiguous()):
        raise ValueError(f"records must be a contiguous uint8 [n, {RECORD_BYTES}] tensor")
    if counts is None:
        counts = torch.zeros(COUNT, dtype=torch.int64, device=records.device)
    if (counts.numel() != COUNT or counts.dtype != torch.int64 or counts.device != records.device
            or not counts.is_contiguous()):
        raise ValueError(f"counts must be a contiguous int64 [{COUNT}] tensor on {records.device}")
    s = ctypes.c_void_p(stream) if stream is not None else \
        ctypes.c_void_p(torch.cuda.current_stream(records.device).cuda_stream)
    _lib.check(_lib.hip().zp_stats_device(records.data_ptr(), records.shape[0], counts.data_ptr(),
                                          s), "zp_stats_device")
    return counts


def to_dict(counts):
    c = counts.cpu().numpy() if isinstance(counts, torch.Tensor) else np.asarray(counts)
    return {name: int(v) for name, v in zip(NAMES, c)}


def combine(arrays):
    """Sums per-GPU count arrays on the host."""
    return np.sum([a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
                   for a in arrays], axis=0)
