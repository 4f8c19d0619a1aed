"""Host-ring ingestion pipeline (zp_ring_*).

CPU: geometry errors are refused before any device work.
GPU: batches fed through the ring (many wrap-arounds, ragged slot fills,
one producer and one consumer thread) give records byte-identical to the
oracle; misuse (frames outside the slot, release of a slot not held, wait
with nothing submitted) is refused with an error, not a fault.
"""
import threading

import numpy as np
import pytest

import oracle as orc


def test_ring_bad_geometry(zp):
    with pytest.raises(RuntimeError):
        zp.ring.Ring(device=0, slots=0, slot_bytes=1 << 20)
    with pytest.raises(RuntimeError):
        zp.ring.Ring(device=0, slots=4, slot_bytes=16)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,slots,slot_bytes", [("c5", 3, 1 << 20), ("c4", 2, 300_000),
                                                 ("c3", 4, 4 << 20)])
def test_ring_parse_matches_oracle(zp, cfg, slots, slot_bytes):
    arena, offs, lens = zp.batch.generate_host(cfg, 40000, first=555)
    want, wext = orc.parse_batch(arena, offs, lens)
    with zp.ring.Ring(0, slots, slot_bytes) as ring:
        got, gext = ring.parse(arena, offs, lens)
    assert got.tobytes() == orc.pack(want, wext).tobytes()
    assert zp.records.ext_match(gext, wext, want)


@pytest.mark.gpu
def test_ring_producer_consumer_threads(zp, golden):
    """A producer thread fills slots with ragged frame counts while the
    consumer thread drains them; sequence numbers come back in order."""
    import random
    from test_oracle_fuzz import mutate
    rng = random.Random(5)
    seeds = [bytes.fromhex(fx["bytes"]) for fx in golden["fixtures"]]
    frames = [mutate(rng, rng.choice(seeds)) for _ in range(3000)]
    batches, i = [], 0
    while i < len(frames):
        k = rng.randint(0, 97)
        batches.append(frames[i:i + k])
        i += k
    results = {}
    ring = zp.ring.Ring(0, 3, 64 << 10, 256)

    def producer():
        for b in batches:
            s = ring.acquire(20000)
            pos = 0
            for q, f in enumerate(b):
                pos += q % 3                   # gaps between frames
                s.arena[pos:pos + len(f)] = np.frombuffer(f, np.uint8)
                s.offs[q], s.lens[q] = pos, len(f)
                pos += len(f)
            ring.submit(s, len(b))

    def consumer():
        for k in range(len(batches)):
            d = ring.wait(20000) if k % 2 else None
            while d is None:
                d = ring.poll()
            results[d.seq] = d.records.copy()
            ring.release(d)

    tp = threading.Thread(target=producer, daemon=True)
    tc = threading.Thread(target=consumer, daemon=True)
    tp.start(); tc.start(); tp.join(60); tc.join(60)
    assert not tp.is_alive() and not tc.is_alive()
    assert sorted(results) == list(range(len(batches)))
    for seq, b in enumerate(batches):
        one = [orc.parse_one(f) for f in b]
        want = orc.pack(np.array([o[1] for o in one], orc.RECORD_DTYPE),
                        np.stack([o[2] for o in one], axis=1) if one
                        else np.zeros((2, 0), orc.EXT_DTYPE))
        assert results[seq].tobytes() == want.tobytes(), seq
    ring.close()


@pytest.mark.gpu
def test_ring_misuse(zp):
    ring = zp.ring.Ring(0, 2, 4096, 16)
    with pytest.raises(zp.ring.RingTimeout):
        ring.wait(50)                           # nothing submitted
    assert ring.poll() is None
    s = ring.acquire()
    s.offs[0], s.lens[0] = 4000, 200           # past the slot arena
    with pytest.raises(RuntimeError):
        ring.submit(s, 1)
    with pytest.raises(RuntimeError):
        ring.submit(s, 17)                     # over frame capacity
    with pytest.raises(RuntimeError):
        ring.release(s)                        # not DONE
    s1 = ring.acquire(10)                      # ring order: slot 1 ...
    assert s1.id == 1
    with pytest.raises(zp.ring.RingTimeout):
        ring.acquire(10)                       # ... then slot 0 again, still FILLING
    s.offs[0], s.lens[0] = 0, 64
    s.arena[:64] = 0
    ring.submit(s, 1)
    d = ring.wait()
    want = orc.parse_one_abi(bytes(64))[1]              # unknown ethertype 0: Ok, ethernet only
    assert d.n == 1 and d.records.tobytes() == want.tobytes()
    ring.release(d)
    ring.close()
