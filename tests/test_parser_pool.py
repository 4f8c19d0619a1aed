"""CPU: PacketParser.parse's context pool (parser.py), over a stand-in for the
C library (no device calls): contexts are created on the calling thread's
current device, one per concurrent caller, reused LIFO, frames past ONE_MAX
take the device's one large context, and quiesce() stops idle contexts only.
The real library runs the same paths in tests/test_gpu_parity.py
(test_parser_threads_and_current_device)."""
import threading
import time

import numpy as np
import pytest


class FakeLib:
    """zp_device_current / zp_ctx_create / zp_parse_one / zp_parse_one_config
    with the C signatures' meaning; zp_parse_one sleeps so calls overlap."""

    def __init__(self):
        self.device = 0
        self.created = []          # (handle, device, chunk)
        self.configured = []
        self.lock = threading.Lock()
        self.busy = set()
        self.overlap = 0
        self.bufs = {}             # context -> the (record, ext) addresses it was given

    def zp_device_current(self):
        return self.device

    def zp_ctx_create(self, device, chunk):
        with self.lock:
            h = 1000 + len(self.created)
            self.created.append((h, device, chunk))
        return h

    def zp_parse_one(self, ctx, frame, n, rec, ext):
        with self.lock:
            assert ctx not in self.busy, "a context served two calls at once"
            if n <= 64 << 10:      # pooled contexts (the large one gets a call's own)
                assert self.bufs.setdefault(ctx, (rec, ext)) == (rec, ext), "buffers moved"
            self.busy.add(ctx)
            self.overlap = max(self.overlap, len(self.busy))
        time.sleep(0.002)
        with self.lock:
            self.busy.discard(ctx)
        return 0

    def zp_parse_one_config(self, ctx, idle):
        self.configured.append(ctx)
        return 0

    def zp_last_error(self):
        return b""


@pytest.fixture
def fake(zp, monkeypatch):
    P = zp.parser
    lib = FakeLib()
    monkeypatch.setattr(zp._lib, "hip", lambda: lib)
    monkeypatch.setattr(zp._lib, "pyhip", lambda: lib)
    monkeypatch.setattr(P, "_POOLS", {})
    monkeypatch.setattr(P.PacketParser, "_from_words",
                        classmethod(lambda cls, f, w, o, x: ("ok", len(f))))
    return lib


def test_contexts_follow_current_device(zp, fake):
    P = zp.parser
    fake.device = 3
    assert P.PacketParser.parse(b"\0" * 60) == ("ok", 60)
    fake.device = 1
    P.PacketParser.parse(b"\0" * 60)
    assert [(d, c) for _, d, c in fake.created] == [(3, P.POOL_CHUNK), (1, P.POOL_CHUNK)]
    assert sorted(P._POOLS) == [1, 3]
    # reuse: no new context for a sequential caller
    P.PacketParser.parse(b"\0" * 60)
    assert len(fake.created) == 2


def test_threads_run_concurrently_on_own_contexts(zp, fake):
    P = zp.parser
    ths = [threading.Thread(target=lambda: [P.PacketParser.parse(b"\0" * 80) for _ in range(10)])
           for _ in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert fake.overlap >= 2                       # no global lock
    assert len(fake.created) <= 8
    pool = P._POOLS[0]
    assert sorted(pool.free) == sorted(pool.all)   # every lease returned
    # each context writes into record buffers of its own, kept across calls
    assert len(set(fake.bufs.values())) == len(fake.bufs) == len(pool.all)


def test_pool_bound_waits(zp, fake, monkeypatch):
    P = zp.parser
    monkeypatch.setattr(P, "POOL_MAX", 2)
    ths = [threading.Thread(target=lambda: [P.PacketParser.parse(b"\0" * 80) for _ in range(5)])
           for _ in range(6)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert len(fake.created) == 2 and fake.overlap == 2


def test_long_frames_take_the_large_context(zp, fake):
    P = zp.parser
    P.PacketParser.parse(b"\0" * (P.ONE_MAX + 1))
    P.PacketParser.parse(b"\0" * (P.ONE_MAX + 1))
    assert [c for _, _, c in fake.created] == [0]          # one 256 MiB-chunk context
    P.PacketParser.parse(b"\0" * P.ONE_MAX)
    assert [c for _, _, c in fake.created] == [0, P.POOL_CHUNK]


def test_quiesce_touches_idle_contexts_only(zp, fake):
    P = zp.parser
    P.PacketParser.parse(b"\0" * 64)
    pool = P._POOLS[0]
    held = pool.take()                                    # a call in flight elsewhere
    P.quiesce()
    assert held not in fake.configured
    assert set(fake.configured) == set(pool.free)
    pool.give(held)


def test_device_error_raises(zp, fake):
    P = zp.parser
    fake.device = -1
    with pytest.raises(RuntimeError):
        P.PacketParser.parse(b"\0" * 64)


def test_fast_record_path_equals_from_record(zp, golden):
    """PacketParser.parse rebuilds the common record (ordinary form, no
    extension chain) without from_record's general decode; on the golden
    packets and every config's frames both give the same parser (Debug
    text) or the same error."""
    import ctypes
    import oracle as orc
    P = zp.parser.PacketParser
    frames = [bytes.fromhex(fx["bytes"]) for fx in golden["fixtures"]]
    for c in ("c1", "c3", "c4", "c5", "c6"):
        a, o, l_ = zp.batch.generate_host(c, 800, first=77)
        frames += [a[int(x):int(x) + int(y)].tobytes() for x, y in zip(o, l_)]

    def res(fn):
        try:
            return fn().debug()
        except zp.parser.ZeroPacketError as e:
            return repr(e)
    kinds = set()
    for f in frames:
        err, r, x = orc.parse_one(f)
        pr = orc.pack(r, x)[0]
        ext = (ctypes.c_uint8 * 32)()
        ctypes.memmove(ext, x.tobytes(), 32)
        w, o = int(pr["flags"]), int(pr["offs"])
        kinds.add(bool(w >> 26 or w & (zp.records.F_EXT | zp.records.F_INNER_EXT)))
        assert res(lambda: P.from_record(f, pr, x)) == res(lambda: P._from_words(f, w, o, ext)), \
            f.hex()
    assert kinds == {False, True}                      # both paths were exercised
