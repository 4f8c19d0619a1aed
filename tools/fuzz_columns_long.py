"""Long GPU-vs-oracle column-view fuzz (not part of the test suite): the
tests' mutated frame corpus over many seeds, standalone and fused kernels.
Usage: python tools/fuzz_columns_long.py [rounds] [frames_per_round]"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as orc  # noqa: E402  (tests/oracle.py: the checker)
from test_columns import frames_corpus, pack  # noqa: E402


def main():
    import torch
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    zp = importlib.import_module("zero-packet_amd")
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "parse_golden.json")))
    d = torch.device("cuda:0")
    t0 = time.time()
    for r in range(rounds):
        arena, offs, lens = pack(frames_corpus(zp, golden, count, seed=100 + r))
        a = torch.from_numpy(arena).to(d)
        o = torch.from_numpy(offs.astype(np.int64)).to(d)
        l_ = torch.from_numpy(lens.astype(np.int32)).to(d)
        recs, _ = zp.batch.parse_batch(a, o, l_)
        got = zp.columns.extract(a, o, l_, recs)
        frecs, _, fcols = zp.columns.parse_with_columns(a, o, l_)
        torch.cuda.synchronize()
        assert torch.equal(frecs, recs), f"round {r}: fused records differ"
        want = orc.columns(arena, offs, lens, orc.parse_batch(arena, offs, lens)[0])
        for name in zp.columns.NAMES:
            assert np.array_equal(got[name].cpu().numpy(), want[name]), (r, name)
            assert np.array_equal(fcols[name].cpu().numpy(), want[name]), (r, "fused", name)
        print(f"round {r}: {count} frames OK ({time.time() - t0:.0f} s)", flush=True)
    print("fuzz_columns_long: all rounds identical", flush=True)


if __name__ == "__main__":
    main()
