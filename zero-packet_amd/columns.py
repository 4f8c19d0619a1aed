"""Column views over parsed frames (zp_extract_columns_device).

    cols = columns.extract(arena, offs, lens, records, names=("src_port", ...))

Each column is a device tensor of n entries (byte-array columns: [n, width]
uint8): the reader getters of every frame gathered into SoA form, so a
downstream consumer (flow table, filter, sampler) needs no host pass. Column
semantics and the reference getters they follow: include/zero_packet.h
(zp_col). Entry i is 0 when record i holds an error or the reader is absent.
"""
import collections
import ctypes

import numpy as np
import torch

from . import _lib
from .batch import alloc_outputs, check_batch
from .records import EXT_BYTES, RECORD_BYTES

# (name, torch dtype, elements per frame) in zp_col order.
COLUMNS = [
    ("dest_mac", torch.uint8, 6), ("src_mac", torch.uint8, 6),
    ("ethertype", torch.uint16, 1), ("vlan_tci", torch.uint16, 1),
    ("vlan_inner_tci", torch.uint16, 1), ("arp_oper", torch.uint16, 1),
    ("ip_version", torch.uint8, 1), ("src_addr", torch.uint8, 16),
    ("dest_addr", torch.uint8, 16), ("protocol", torch.uint8, 1), ("ttl", torch.uint8, 1),
    ("tos", torch.uint8, 1), ("ip_id", torch.uint32, 1), ("ip_len", torch.uint16, 1),
    ("inner_version", torch.uint8, 1), ("inner_src_addr", torch.uint8, 16),
    ("inner_dest_addr", torch.uint8, 16), ("inner_protocol", torch.uint8, 1),
    ("l4_proto", torch.uint8, 1), ("src_port", torch.uint16, 1), ("dest_port", torch.uint16, 1),
    ("tcp_seq", torch.uint32, 1), ("tcp_ack", torch.uint32, 1), ("tcp_flags", torch.uint8, 1),
    ("tcp_window", torch.uint16, 1), ("icmp_type", torch.uint8, 1),
    ("icmp_code", torch.uint8, 1), ("l4_checksum", torch.uint16, 1),
    ("payload_off", torch.uint32, 1),
]
NAMES = [c[0] for c in COLUMNS]
INDEX = {name: k for k, name in enumerate(NAMES)}
NUMPY_DTYPE = {torch.uint8: np.uint8, torch.uint16: np.uint16, torch.uint32: np.uint32}


def width(name):
    _, dt, k = COLUMNS[INDEX[name]]
    return k * torch.empty((), dtype=dt).element_size()


def _alloc(name, n, device):
    _, dt, k = COLUMNS[INDEX[name]]
    return torch.empty((n, k) if k > 1 else (n,), dtype=dt, device=device)


def extract(arena, offs, lens, records, names=None, out=None, stream=None, check=True):
    """Fills the requested columns (default: all) on the device; returns
    {name: tensor}. `out` may hold preallocated tensors. check: as in
    batch.parse_batch (descriptor bounds reduction)."""
    for t in (arena, offs, lens, records):
        if not t.is_cuda:
            raise RuntimeError("columns.extract needs device tensors (no CPU fallback)")
    n = offs.numel()
    check_batch(arena, offs, lens, ((records, RECORD_BYTES),), bounds=check)
    names = list(names) if names is not None else NAMES
    out = dict(out or {})
    ptrs = (ctypes.c_void_p * len(COLUMNS))()
    for name in names:
        if name not in out:
            out[name] = _alloc(name, n, arena.device)
        t = out[name]
        assert t.is_contiguous() and t.numel() * t.element_size() == n * width(name), name
        ptrs[INDEX[name]] = t.data_ptr()
    s = ctypes.c_void_p(stream) if stream is not None else \
        ctypes.c_void_p(torch.cuda.current_stream(arena.device).cuda_stream)
    rc = _lib.hip().zp_extract_columns_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                              records.data_ptr(), n, ptrs, s)
    _lib.check(rc, "zp_extract_columns_device")
    return {k: out[k] for k in names}


# Path choice of parse_with_columns(mode="auto") per workload key: the fused
# kernel (one pass) wins on most traffic, but plain IPv4 frames with wide
# column requests run faster as parse + extract (round 4/5: c3 with all 29
# columns +2-5 % fused; c4/c5/c6 -11 to -23 %). The library
# times both paths on the first call of a workload and keeps the faster one.
_AUTO_REPS = 2             # timed back-to-back runs per path (after one warm-up run)
_AUTO_MAX = 256            # workload keys remembered (least recently used dropped)
_AUTO_AGREE = 4            # arenas of one (device, columns, size octave) whose timings agree
_auto = collections.OrderedDict()
_agree = {}                # (device, columns, octave) -> the choices timed so far
auto_timings = 0           # first calls that timed both paths (diagnostics, tests)


def _auto_key(arena, n, names):
    # the arena buffer too: traffic of another shape arrives in another buffer
    # (c3 and c4 batches of one size want different paths, tools/cols_policy.py)
    return (arena.device.index, arena.data_ptr(), tuple(sorted(names)), max(n, 1).bit_length())


def reset_auto():
    """Forgets every choice of parse_with_columns(mode="auto") (the traffic in
    a reused arena changed shape): the next call of each workload times both
    paths again."""
    _auto.clear()
    _agree.clear()


def _remember(key, choice):
    _auto[key] = choice
    _auto.move_to_end(key)
    while len(_auto) > _AUTO_MAX:
        _auto.popitem(last=False)


def auto_choice(arena, n, names):
    """The path parse_with_columns(mode="auto") uses for this workload key
    (None before its first call)."""
    return _auto.get(_auto_key(arena, n, names))


def parse_with_columns(arena, offs, lens, names=None, records=None, ext=None, out=None,
                       stream=None, check=True, mode="auto"):
    """Records and the requested columns of every frame. Returns (records,
    ext, {name: tensor}); the results are the same on every path.
    mode: "fused" = zp_parse_batch_columns_device (one pass over the frames);
    "split" = zp_parse_batch_device then zp_extract_columns_device on the same
    stream; "auto" (default) = the faster of the two for this workload (device,
    arena buffer, column set, batch-size octave; reset_auto() forgets the
    choices): its first call runs each path once, then
    twice back to back between HIP events on the launch stream, keeps the
    faster, and synchronises; later calls of the workload run that path."""
    for t in (arena, offs, lens):
        if not t.is_cuda:
            raise RuntimeError("columns.parse_with_columns needs device tensors (no CPU fallback)")
    if mode not in ("auto", "fused", "split"):
        raise ValueError(f"mode {mode!r}: auto, fused or split")
    n = offs.numel()
    d = arena.device
    records, ext = alloc_outputs(n, d, records, ext)
    names = list(names) if names is not None else NAMES
    out = dict(out or {})
    ptrs = (ctypes.c_void_p * len(COLUMNS))()
    for name in names:
        if name not in out:
            out[name] = _alloc(name, n, d)
        ptrs[INDEX[name]] = out[name].data_ptr()
    check_batch(arena, offs, lens, [(records, RECORD_BYTES), (ext, 2 * EXT_BYTES)] +
                [(out[k], width(k)) for k in names], bounds=check)
    s = ctypes.c_void_p(stream) if stream is not None else \
        ctypes.c_void_p(torch.cuda.current_stream(d).cuda_stream)
    lib = _lib.hip()

    def fused():
        _lib.check(lib.zp_parse_batch_columns_device(arena.data_ptr(), offs.data_ptr(),
                                                     lens.data_ptr(), n, records.data_ptr(),
                                                     ext.data_ptr(), ptrs, s),
                   "zp_parse_batch_columns_device")

    def split():
        _lib.check(lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                             n, records.data_ptr(), ext.data_ptr(), s),
                   "zp_parse_batch_device")
        _lib.check(lib.zp_extract_columns_device(arena.data_ptr(), offs.data_ptr(),
                                                 lens.data_ptr(), records.data_ptr(), n, ptrs, s),
                   "zp_extract_columns_device")
    paths = {"fused": fused, "split": split}
    if mode != "auto":
        paths[mode]()
        return records, ext, {k: out[k] for k in names}
    key = _auto_key(arena, n, names)
    choice = _auto.get(key)
    shape = (key[0],) + key[2:]
    if choice is None and n:
        # A caller that hands over a fresh arena per batch: once the first
        # _AUTO_AGREE arenas of this shape agreed, new ones take that path
        # without timing it again.
        seen = _agree.get(shape, [])
        if len(seen) >= _AUTO_AGREE and len(set(seen)) == 1:
            choice = seen[0]
            _remember(key, choice)
    else:
        if choice is not None:
            _auto.move_to_end(key)
    if choice is None and n:
        # First call of this workload: each path once to warm up, then twice
        # back to back between two events (as a stream of calls runs), and
        # the faster is kept. Every run writes the same outputs.
        ts = torch.cuda.ExternalStream(stream, device=d) if stream is not None else \
            torch.cuda.current_stream(d)
        ms = {}
        for k in ("fused", "split"):
            paths[k]()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ts)
            for _ in range(_AUTO_REPS):
                paths[k]()
            b.record(ts)
            b.synchronize()
            ms[k] = a.elapsed_time(b)
        global auto_timings
        auto_timings += 1
        choice = min(ms, key=ms.get)
        _remember(key, choice)
        _agree.setdefault(shape, []).append(choice)
        if len(_agree[shape]) > 64:
            del _agree[shape][:-64]
        return records, ext, {k: out[k] for k in names}
    paths[choice or "fused"]()
    return records, ext, {k: out[k] for k in names}
