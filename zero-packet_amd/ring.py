"""Host-ring ingestion pipeline (zp_ring_*, include/zero_packet.h).

    ring = Ring(device=0, slots=4, slot_bytes=64 << 20)
    s = ring.acquire()                 # pinned host views: s.arena, s.offs, s.lens
    ... fill s.arena / s.offs[:n] / s.lens[:n] (a NIC ring would DMA here) ...
    ring.submit(s, n)                  # H2D -> parse -> D2H, asynchronous
    d = ring.wait()                    # oldest submitted slot, results in host memory
    use(d.records, d.ext)              # numpy RECORD_DTYPE [n], EXT_DTYPE [2, n]
    ring.release(d)

Frames start in host memory (README.md:85-115 of the reference feeds one
received frame at a time to PacketParser::parse, parser.rs:53); the ring
keeps several slots in flight so copies and the parse kernel overlap.
"""
import ctypes

import numpy as np

from . import _lib
from .records import EXT_DTYPE, RECORD_DTYPE


TIMEOUT = -4   # ZP_RING_TIMEOUT


class RingTimeout(RuntimeError):
    """A ring wait expired (ZP_RING_TIMEOUT)."""


class _SlotC(ctypes.Structure):
    _fields_ = [("id", ctypes.c_int32), ("arena", ctypes.c_void_p), ("offs", ctypes.c_void_p),
                ("lens", ctypes.c_void_p), ("arena_cap", ctypes.c_uint64),
                ("frames_cap", ctypes.c_uint64), ("records", ctypes.c_void_p),
                ("ext", ctypes.c_void_p), ("n", ctypes.c_uint64), ("seq", ctypes.c_uint64)]


def _np(ptr, dtype, count):
    if count == 0:
        return np.zeros(0, dtype)
    buf = (ctypes.c_uint8 * (count * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=count)


class Slot:
    """Numpy views over one slot's pinned buffers (valid until released)."""

    def __init__(self, c):
        self.id = c.id
        self.seq = c.seq
        self.n = c.n
        self.arena = _np(c.arena, np.uint8, c.arena_cap)
        self.offs = _np(c.offs, np.uint64, c.frames_cap)
        self.lens = _np(c.lens, np.uint32, c.frames_cap)
        self.records = _np(c.records, RECORD_DTYPE, c.n)
        self.ext = _np(c.ext, EXT_DTYPE, 2 * c.n).reshape(2, -1)   # [0] outer, [1] ip_in_ip


def _sigs(lib):
    if getattr(lib, "_ring_sigs", False):
        return lib
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32
    sp = ctypes.POINTER(_SlotC)
    for name, res, args in (("zp_ring_create", vp, [ctypes.c_int, u32, u64, u64]),
                            ("zp_ring_destroy", None, [vp]),
                            ("zp_ring_acquire", ctypes.c_int, [vp, sp, ctypes.c_int64]),
                            ("zp_ring_submit", ctypes.c_int, [vp, i32, u64]),
                            ("zp_ring_wait", ctypes.c_int, [vp, sp, ctypes.c_int64]),
                            ("zp_ring_release", ctypes.c_int, [vp, i32])):
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    lib._ring_sigs = True
    return lib


class Ring:
    def __init__(self, device=0, slots=4, slot_bytes=64 << 20, slot_frames=None):
        self.lib = _sigs(_lib.hip())
        self.slot_bytes = slot_bytes
        self.nslots = slots
        self.slot_frames = slot_frames or slot_bytes // 64 + 1
        self.h = self.lib.zp_ring_create(device, slots, slot_bytes, self.slot_frames)
        if not self.h:
            raise RuntimeError("zp_ring_create failed: " +
                               self.lib.zp_last_error().decode(errors="replace"))

    def close(self):
        if self.h:
            self.lib.zp_ring_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()

    def acquire(self, timeout_ms=-1):
        """Next FREE slot; raises RingTimeout when timeout_ms expires."""
        c = _SlotC()
        rc = self.lib.zp_ring_acquire(self.h, ctypes.byref(c), timeout_ms)
        if rc == TIMEOUT:
            raise RingTimeout(self.lib.zp_last_error().decode(errors="replace"))
        _lib.check(rc, "zp_ring_acquire")
        return Slot(c)

    def submit(self, slot, n):
        _lib.check(self.lib.zp_ring_submit(self.h, slot.id, n), "zp_ring_submit")

    def wait(self, timeout_ms=-1):
        """Oldest submitted slot with its records; raises RingTimeout."""
        c = _SlotC()
        rc = self.lib.zp_ring_wait(self.h, ctypes.byref(c), timeout_ms)
        if rc == TIMEOUT:
            raise RingTimeout(self.lib.zp_last_error().decode(errors="replace"))
        _lib.check(rc, "zp_ring_wait")
        return Slot(c)

    def poll(self):
        """wait() without blocking: a completed slot or None."""
        try:
            return self.wait(0)
        except RingTimeout:
            return None

    def release(self, slot):
        _lib.check(self.lib.zp_ring_release(self.h, slot.id), "zp_ring_release")

    def parse(self, arena, offs, lens, out=None, ext=None):
        """Runs a host batch through the ring: frames are copied into slots
        (cut at slot capacity), slots overlap in flight, records land in
        `out` (numpy RECORD_DTYPE [n]), chains in `ext` (EXT_DTYPE [2, n]).
        Returns (out, ext)."""
        arena = np.asarray(arena, np.uint8)
        offs = np.asarray(offs, np.uint64)
        lens = np.asarray(lens, np.uint32)
        n = len(offs)
        out = np.zeros(n, RECORD_DTYPE) if out is None else out
        ext = np.zeros((2, n), EXT_DTYPE) if ext is None else ext
        pending = []          # (first frame, count) per submitted slot, FIFO

        def drain_one():
            d = self.wait()
            i0, m = pending.pop(0)
            out[i0:i0 + m] = d.records
            ext[:, i0:i0 + m] = d.ext
            self.release(d)

        ends = offs + lens
        i = 0
        while i < n:
            # longest run [i, j) whose byte span fits a slot (vectorised over
            # a window of at most slot_frames frames)
            w_lo = np.minimum.accumulate(offs[i:i + self.slot_frames])
            w_hi = np.maximum.accumulate(ends[i:i + self.slot_frames])
            j = i + int(np.searchsorted((w_hi - w_lo) > self.slot_bytes, True))
            if j == i:
                raise ValueError(f"frame {i} does not fit a ring slot")
            lo, hi = int(w_lo[j - i - 1]), int(w_hi[j - i - 1])
            if len(pending) == self.nslots:   # single thread: free the oldest first
                drain_one()
            s = self.acquire()
            s.arena[:hi - lo] = arena[lo:hi]
            s.offs[:j - i] = offs[i:j] - lo
            s.lens[:j - i] = lens[i:j]
            self.submit(s, j - i)
            pending.append((i, j - i))
            i = j
        while pending:
            drain_one()
        return out, ext
