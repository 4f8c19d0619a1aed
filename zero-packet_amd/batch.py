"""Device-resident batch API over torch tensors (torch = memory/streams only).

    arena  uint8  [B]       frames packed anywhere in one buffer
    offs   int64  [n]       frame start offsets (read as uint64)
    lens   int32  [n]       frame lengths (read as uint32)
    -> records uint8 [n, 8] (zp_record), ext uint8 [2, n, 16] (zp_ext_offsets:
       [0] the outer ipv6 extension chains, [1] the ip_in_ip ones; an entry
       is valid where the record's ZP_F_EXT / ZP_F_INNER_EXT bit is set,
       except an inline outer chain (ABI v6), which lives in its record:
       records_to_numpy rebuilds those entries)

parse_batch() enqueues the HIP kernel on torch's current stream of the
tensors' device, or on `stream` (zp_parse_batch_device). By default
(check=True) it first validates the descriptors with one device reduction on
that same stream and reads the result back, so the default call SYNCHRONISES
with the stream; check=False makes it enqueue-only. No CPU fallback: non-CUDA
tensors or a missing libzp_hip.so raise.
"""
import contextlib
import ctypes

import numpy as np
import torch

from . import _lib
from .records import EXT_BYTES, EXT_DTYPE, RECORD_BYTES, RECORD_DTYPE, expand_ext

CONFIGS = {"c1": 1, "c2": 2, "c3": 3, "c4": 4, "c5": 5, "c6": 6}
# zp_set_record_slots' automatic mode stores record codes from this many
# frames on (ZP_SLOT_MIN_FRAMES, zp_parse.hip)
RECORD_CODES_MIN_FRAMES = 1 << 21


def record_codes(n):
    """Whether a parse of n frames takes the record-code kernels under the
    process' zp_set_record_slots mode (0 auto, 1 always, 2 never) and, in
    the automatic mode, the current device's latest probe verdict."""
    lib = _lib.hip()
    mode = lib.zp_set_record_slots(0)
    lib.zp_set_record_slots(mode)
    if mode == 0 and n >= RECORD_CODES_MIN_FRAMES:
        return lib.zp_record_slots_state() == 1
    return mode == 1
SEED = 0x5EED2025


def _stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("zero-packet_amd batch API needs device tensors (no CPU fallback)")


def check_batch(arena, offs, lens, outs=(), bounds=True, stream=None):
    """Validates a device batch before a kernel reads it: dtypes, shapes,
    contiguity and device of every tensor, and (bounds=True) that every frame
    lies inside the arena: 0 <= offs[i], 0 <= lens[i], offs[i] + lens[i] <=
    arena.numel(). The kernels do not check descriptors on the device (a frame
    past the arena faults the GPU), so this is the Python API's guard; it
    costs one device reduction and one synchronisation. `outs` holds
    (tensor, row_bytes) pairs of outputs ([n, row_bytes] uint8, or any
    contiguous tensor of n * row_bytes bytes). The reduction runs on `stream`
    (a hipStream_t as int, the stream the kernel will be launched on) when
    given, so descriptors still being produced on it are read after they are
    written."""
    _need_cuda(arena, offs, lens)
    n = offs.numel()
    if arena.dtype != torch.uint8 or arena.dim() != 1 or not arena.is_contiguous():
        raise ValueError("arena must be a contiguous 1-D uint8 tensor")
    if offs.dtype != torch.int64 or lens.dtype != torch.int32:
        raise ValueError("offs must be int64 and lens int32")
    if lens.numel() != n or not offs.is_contiguous() or not lens.is_contiguous():
        raise ValueError("offs and lens must be contiguous with the same length")
    dev = arena.device
    for t, row in outs:
        if t is None:
            continue
        if not t.is_cuda or t.device != dev:
            raise ValueError(f"output tensor on {t.device}, arena on {dev}")
        if not t.is_contiguous() or t.numel() * t.element_size() != n * row:
            raise ValueError(f"output tensor must be contiguous with {n} x {row} bytes")
    for t in (offs, lens):
        if t.device != dev:
            raise ValueError(f"descriptor tensor on {t.device}, arena on {dev}")
    if bounds and n:
        on = (torch.cuda.stream(torch.cuda.ExternalStream(int(stream), device=dev))
              if stream is not None else contextlib.nullcontext())
        with on:
            lo = torch.minimum(offs.min(), lens.min().to(torch.int64))
            hi = (offs + lens.to(torch.int64)).max()
            lo, hi = torch.stack([lo, hi]).tolist()
        if lo < 0:
            raise ValueError("negative frame offset or length")
        if hi > arena.numel():
            raise ValueError(f"frame ends at byte {hi}, past the arena ({arena.numel()} bytes)")


def alloc_outputs(n, device, records=None, ext=None):
    """records uint8 [n, 8] and ext uint8 [2, n, 16] device tensors (the ones
    given are kept)."""
    if records is None:
        records = torch.empty((n, RECORD_BYTES), dtype=torch.uint8, device=device)
    if ext is None:
        ext = torch.empty((2, n, EXT_BYTES), dtype=torch.uint8, device=device)
    return records, ext


def parse_batch(arena, offs, lens, records=None, ext=None, stream=None, check=True):
    """Parses every frame; returns (records, ext) as uint8 device tensors.
    check=True (default) runs the descriptor bounds reduction (check_batch) on
    the launch stream and waits for it, so the call synchronises; check=False
    skips it for callers that validated the batch already and makes the call
    enqueue-only. Shapes and devices are always checked."""
    n = offs.numel()
    dev = arena.device
    if arena.is_cuda:
        records, ext = alloc_outputs(n, dev, records, ext)
    check_batch(arena, offs, lens, ((records, RECORD_BYTES), (ext, 2 * EXT_BYTES)), bounds=check,
                stream=stream)
    s = ctypes.c_void_p(stream) if stream is not None else _stream_ptr(dev)
    rc = _lib.hip().zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                          records.data_ptr(), ext.data_ptr(), s)
    _lib.check(rc, "zp_parse_batch_device")
    return records, ext


def generate(config, n, seed=SEED, first=0, device="cuda", pad=64):
    """Synthetic batch of BASELINE config `config` on the GPU: packets
    first..first+n-1, packed back to back. Returns (arena, offs, lens)."""
    cfg = CONFIGS.get(config, config)
    dev = torch.device(device)
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    s = _stream_ptr(dev)
    _lib.check(_lib.hip().zp_gen_lengths_device(cfg, seed, first, n, lens.data_ptr(), s),
               "zp_gen_lengths_device")
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    if n > 1:
        torch.cumsum(lens[:-1].to(torch.int64), 0, out=offs[1:])
    total = int(offs[-1].item() + lens[-1].item()) if n else 0
    arena = torch.zeros(total + pad, dtype=torch.uint8, device=dev)
    _lib.check(_lib.hip().zp_gen_frames_device(cfg, seed, first, n, arena.data_ptr(),
                                               offs.data_ptr(), lens.data_ptr(), s),
               "zp_gen_frames_device")
    return arena, offs, lens


def generate_host(config, n, seed=SEED, first=0, nthreads=0, pad=64):
    """CPU build of the same generator (libzp_host.so): numpy arrays."""
    cfg = CONFIGS.get(config, config)
    lens = np.empty(n, dtype=np.uint32)
    _lib.host().zp_host_gen_lengths(cfg, seed, first, n, lens.ctypes.data)
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(offs[-1] + lens[-1]) if n else 0
    arena = np.zeros(total + pad, dtype=np.uint8)
    _lib.host().zp_host_gen_frames(cfg, seed, first, n, arena.ctypes.data, offs.ctypes.data,
                                   nthreads)
    return arena, offs, lens


def record_err(records):
    """err codes of raw records (uint8 [n, 8], torch or numpy): bits 26-31 of
    the flags word, i.e. byte 3 >> 2 (include/zero_packet.h)."""
    return records[:, 3] >> 2


def record_flags(records):
    """ZP_F_* bits of raw records (uint8 [n, 8], torch): int32 [n]."""
    return records[:, 0:4].contiguous().view(torch.int32)[:, 0] & 0x00FFFFFF


def records_to_numpy(records, ext=None):
    """uint8 [n, 8] (device or host) -> structured numpy (RECORD_DTYPE) [n];
    with ext (uint8 [2, n, 16]) also the chains as EXT_DTYPE [2, n], the
    entries of inline outer chains (ABI v6, include/zero_packet.h) rebuilt
    from their records, so every entry a record flags is valid."""
    r = records.cpu().numpy() if isinstance(records, torch.Tensor) else records
    rec = np.ascontiguousarray(r).view(RECORD_DTYPE).reshape(-1)
    if ext is None:
        return rec
    e = ext.cpu().numpy() if isinstance(ext, torch.Tensor) else ext
    return rec, expand_ext(rec, np.ascontiguousarray(e).view(EXT_DTYPE).reshape(2, -1))
