"""CPU: mutation fuzz in the style of fuzz/fuzz_targets/fuzz_target_1.rs —
the C oracle and the independent Python restatement agree on every record
for mutated golden and generated frames (and neither crashes)."""
import random

import numpy as np

import oracle as orc
import pyref
from test_oracle_golden import ERR


def rec_tuple(rec, ext):
    return orc.record_tuple(rec, ext)


def mutate(rng, frame):
    f = bytearray(frame)
    k = rng.random()
    if k < 0.5 and f:
        for _ in range(rng.randint(1, 3)):
            i = rng.randrange(min(len(f), 160))
            f[i] = rng.randrange(256)
    elif k < 0.7 and f:
        # header-structure bytes: ethertype / version / next-header / lengths
        i = rng.choice([12, 13, 14, 16, 17, 18, 20, 21, 22, 23]) % len(f)
        f[i] = rng.choice([0, 4, 6, 17, 41, 43, 44, 51, 58, 59, 60, 0x45, 0x60, 0x81, 0x86, 0xdd,
                           0x88, 0xa8, 0x08, 0x00, 0xff, 1, 2])
    elif k < 0.85:
        f = f[:rng.randrange(len(f) + 1)]
    else:
        f += bytes(rng.randrange(256) for _ in range(rng.randint(1, 40)))
    return bytes(f)


def test_fuzz_oracle_vs_pyref(zp, golden):
    rng = random.Random(1234)
    seeds = [bytes.fromhex(fx["bytes"]) for fx in golden["fixtures"]]
    for cfg in ("c3", "c4", "c5"):
        arena, offs, lens = zp.batch.generate_host(cfg, 40, first=777)
        seeds += [arena[o:o + l].tobytes() for o, l in zip(offs, lens)]
    errs = set()
    for it in range(4000):
        frame = mutate(rng, rng.choice(seeds))
        if rng.random() < 0.3:
            frame = mutate(rng, frame)
        _, rec, ext = orc.parse_one(frame)
        got = pyref.to_record_tuple(pyref.parse(frame), ERR)
        assert rec_tuple(rec, ext) == got, (it, frame.hex())
        errs.add(int(rec["err"]))
    # the fuzz reaches a broad set of error paths
    assert len(errs) >= 18, sorted(errs)


def test_fuzz_repaired_oracle_vs_pyref(zp, golden):
    """Mutations whose checksums are then refilled (tests/fuzzfix.py) get past
    the checksum checks into the field checks after them and into the accept
    path: the C oracle and the Python restatement still agree on every
    record, and the campaign reaches both outcomes broadly."""
    from fuzzfix import repair
    rng = random.Random(4321)
    seeds = [bytes.fromhex(fx["bytes"]) for fx in golden["fixtures"]]
    for cfg in ("c1", "c3", "c4", "c5", "c6"):
        arena, offs, lens = zp.batch.generate_host(cfg, 40, first=778)
        seeds += [arena[o:o + l].tobytes() for o, l in zip(offs, lens)]
    errs, ok = set(), 0
    for it in range(4000):
        frame = mutate(rng, rng.choice(seeds))
        if rng.random() < 0.3:
            frame = mutate(rng, frame)
        if rng.random() < 0.3 and len(frame) > 64:
            # L4 header fields of the common IPv4 shape (offsets 34-61)
            f = bytearray(frame)
            f[rng.randrange(34, 62)] = rng.choice([0, 1, 2, 4, 5, 15, 16, 0x40, 0x50, 0xF0, 255])
            frame = bytes(f)
        frame = repair(frame)
        _, rec, ext = orc.parse_one(frame)
        got = pyref.to_record_tuple(pyref.parse(frame), ERR)
        assert rec_tuple(rec, ext) == got, (it, frame.hex())
        errs.add(int(rec["err"]))
        ok += int(rec["err"]) == 0
    assert ok > 1000, ok
    assert len(errs) >= 15, sorted(errs)
    # past the checksums: the L4 field checks are reached
    for e in ("TCP_DATA_OFFSET", "UDP_LENGTH", "ICMPV4_TYPE", "ICMPV4_CODE"):
        assert ERR[e] in errs, e
