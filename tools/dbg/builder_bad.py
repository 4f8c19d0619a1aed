"""Debug: the GPU builder vs the oracle on one test_gpu_builder_vs_oracle
configuration (seed big gap pay_max); prints what differs for bad frames."""
import importlib
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
zp = importlib.import_module("zero-packet_amd")
from test_builder import random_chain, run_oracle, rb  # noqa: E402

seed, big, gap, pay_max = (int(sys.argv[1]), sys.argv[2] == "1", int(sys.argv[3]), int(sys.argv[4]))
rng = random.Random(seed)
chains, lens, fills = [], [], []
for k in range(3000):
    valid = rng.random() < 0.6
    c, _, need = random_chain(zp, rng, valid=valid, pay_max=pay_max)
    r = rng.random()
    if r < 0.15:
        size = rng.randrange(0, need + 1)
    elif big and r < 0.3:
        size = rng.randrange(2000, 9000)
    else:
        size = need + rng.randrange(0, 300)
    chains.append(c); lens.append(size)
    fills.append(np.array(rb(rng, size), np.uint8) if rng.random() < 0.5 else np.zeros(size, np.uint8))
before, want, offs, lens_, wres, (ops, op_start, data) = run_oracle(zp, chains, lens, fill=fills, align=7, gap=gap)
d = torch.device("cuda:0")
arena = torch.from_numpy(before).to(d)
batch = zp.builder.BuildBatch()
for c in chains:
    batch.add(c)
got = batch.run(arena, torch.from_numpy(offs.astype(np.int64)).to(d),
                torch.from_numpy(lens_.astype(np.int32)).to(d))
torch.cuda.synchronize()
ga = arena.cpu().numpy()
ops = np.frombuffer(ops.tobytes(), np.uint8).reshape(-1, 64)
bad = [i for i, (o, l_) in enumerate(zip(offs, lens_)) if ga[o:o + l_].tobytes() != want[o:o + l_].tobytes()]
print("bad", len(bad))
for i in bad[:12]:
    o, l_ = int(offs[i]), int(lens_[i])
    diff = np.nonzero(ga[o:o + l_] != want[o:o + l_])[0]
    s0, s1 = int(op_start[i]), int(op_start[i + 1])
    kinds = [int(ops[k][0]) for k in range(s0, s1)]
    dl = [int(np.frombuffer(ops[k][28:32].tobytes(), np.uint32)[0]) for k in range(s0, s1)]
    b0 = [int(ops[k][1]) for k in range(s0, s1)]
    print(f"frame {i}: off {o} (mod16 {o % 16}) len {l_} err {int(wres[i]['err'])} gpu_err {int(got[i]['err'])} "
          f"hl {int(wres[i]['header_len'])} kinds {kinds} b0 {b0} data_len {dl} "
          f"ndiff {len(diff)} first {diff[:12].tolist()} last {diff[-3:].tolist()}")
    print("   want", want[o + diff[0]:o + diff[0] + 8].tolist(), "got", ga[o + diff[0]:o + diff[0] + 8].tolist())
