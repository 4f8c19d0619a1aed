"""Long campaign for the mixed-stack straight-line walk (fast_ip): c5 frames
with header bytes mutated (half with refilled checksums), only frames that
pass the path's wave probe kept, so whole waves take it; every record and
extension entry compared with the oracle. Outside the suite.

    python tools/fuzz_fast_ip.py [seeds] [frames per seed]
"""
import importlib
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 70000
    zp = importlib.import_module("zero-packet_amd")
    import oracle as orc
    from fuzzfix import repair
    from test_gpu_parity import _fast_ip_probe, assert_same, gpu_parse, pack
    vals = [0, 1, 4, 6, 17, 41, 43, 44, 51, 58, 59, 60, 0x45, 0x46, 0x40, 0x60, 0x65, 0x81, 0x00,
            0x86, 0xdd, 0x88, 0xa8, 0x08, 0xff, 5, 8, 128, 135]
    total = acc = 0
    for seed in range(seeds):
        rng = random.Random(1000 + seed)
        a, o, l_ = zp.batch.generate_host("c5", per, first=per * seed)
        frames = []
        for x, y in zip(o, l_):
            f = bytearray(a[int(x):int(x) + int(y)].tobytes())
            if rng.random() < 0.4:
                for _ in range(rng.randint(1, 3)):
                    j = rng.randrange(12, min(len(f), 130))
                    f[j] = rng.choice(vals) if rng.random() < 0.6 else rng.randrange(256)
                if rng.random() < 0.5:
                    f = bytearray(repair(bytes(f)))
            f = bytes(f)
            if _fast_ip_probe(f):
                frames.append(f)
        arena, offs, lens = pack(frames)
        want, wext = orc.parse_batch(arena, offs, lens)
        got, gext = gpu_parse(zp, arena, offs, lens, base_shift=seed % 16)
        assert_same(got, gext, want, wext)
        total += len(frames)
        acc += int((want["err"] == 0).sum())
        print(f"seed {seed}: {len(frames)} frames, {int((want['err'] == 0).sum())} accepted, "
              f"{len(set(want['err'].tolist()))} outcomes: byte-exact", flush=True)
    print(f"all {seeds} seeds byte-exact: {total} frames, {acc} accepted", flush=True)


if __name__ == "__main__":
    main()
