"""Long GPU-vs-oracle builder fuzz (not part of the test suite): the tests'
random chains (valid and invalid, truncated buffers, random prior contents,
frames past the LDS staging; odd rounds with payloads up to 1.5 KB, copied
as a wave) over many seeds; every arena byte and result.
Usage: python tools/fuzz_builder_long.py [rounds] [chains_per_round]"""
import importlib
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_builder import random_chain, rb, run_oracle  # noqa: E402


def main():
    import torch
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    zp = importlib.import_module("zero-packet_amd")
    d = torch.device("cuda:0")
    t0 = time.time()
    for r in range(rounds):
        rng = random.Random(5000 + r)
        chains, lens, fills = [], [], []
        for _ in range(count):
            c, _, need = random_chain(zp, rng, valid=rng.random() < 0.6,
                                      pay_max=1500 if r % 2 else 120)
            x = rng.random()
            size = (rng.randrange(0, need + 1) if x < 0.15 else
                    rng.randrange(2000, 9000) if x < 0.2 else need + rng.randrange(0, 300))
            chains.append(c)
            lens.append(size)
            fills.append(np.array(rb(rng, size), np.uint8) if rng.random() < 0.5
                         else np.zeros(size, np.uint8))
        before, want, offs, lens_, wres, _ = run_oracle(zp, chains, lens, fill=fills,
                                                        align=r % 16, gap=r % 7)
        arena = torch.from_numpy(before).to(d)
        batch = zp.builder.BuildBatch()
        for c in chains:
            batch.add(c)
        got = batch.run(arena, torch.from_numpy(offs.astype(np.int64)).to(d),
                        torch.from_numpy(lens_.astype(np.int32)).to(d))
        torch.cuda.synchronize()
        assert arena.cpu().numpy().tobytes() == want.tobytes(), f"round {r}: bytes differ"
        assert got.tobytes() == wres.tobytes(), f"round {r}: results differ"
        print(f"round {r}: {count} chains OK ({time.time() - t0:.0f} s)", flush=True)
    print("fuzz_builder_long: all rounds identical", flush=True)


if __name__ == "__main__":
    main()
