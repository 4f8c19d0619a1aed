"""Long GPU-vs-oracle fuzz run (not part of the test suite): many seeds of the
tests' mutation fuzzer, several base alignments, records byte for byte.
Usage: python tools/fuzz_long.py [rounds] [frames_per_round] [repair_p]
(repair_p: share of mutated frames whose checksums are refilled, tests/fuzzfix.py)"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as orc  # noqa: E402  (tests/oracle.py: the checker)
from test_gpu_parity import assert_same, fuzz_frames, gpu_parse, pack  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    repair_p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    zp = importlib.import_module("zero-packet_amd")
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "parse_golden.json")))
    t0 = time.time()
    for r in range(rounds):
        frames = fuzz_frames(zp, golden, count, 1000 + r, repair_p)
        arena, offs, lens = pack(frames, base_pad=r % 16)
        got, gext = gpu_parse(zp, arena, offs, lens, base_shift=(5 * r) % 16)
        want, wext = orc.parse_batch(arena, offs, lens)
        assert_same(got, gext, want, wext)
        acc = float((want["err"] == 0).mean())
        print(f"round {r}: {count} frames OK, {acc:.0%} accepted ({time.time() - t0:.0f} s)",
              flush=True)
    print("fuzz_long: all rounds identical", flush=True)


if __name__ == "__main__":
    main()
