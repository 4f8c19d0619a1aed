import random, sys, importlib
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np, torch
zp = importlib.import_module("zero-packet_amd")
import test_builder as tb
rng = random.Random(1)
chains, lens, fills = [], [], []
for k in range(3000):
    valid = rng.random() < 0.6
    c, _, need = tb.random_chain(zp, rng, valid=valid)
    r = rng.random()
    size = rng.randrange(0, need + 1) if r < 0.15 else need + rng.randrange(0, 300)
    chains.append(c); lens.append(size)
    fills.append(np.array(tb.rb(rng, size), np.uint8) if rng.random() < 0.5 else np.zeros(size, np.uint8))
before, want, offs, lens_, wres, _ = tb.run_oracle(zp, chains, lens, fill=fills, align=7, gap=5)
d = torch.device("cuda:0")
arena = torch.from_numpy(before).to(d)
batch = zp.builder.BuildBatch()
for c in chains: batch.add(c)
got = batch.run(arena, torch.from_numpy(offs.astype(np.int64)).to(d), torch.from_numpy(lens_.astype(np.int32)).to(d))
torch.cuda.synchronize()
ga = arena.cpu().numpy()
nb = 0
for i, (o, l_) in enumerate(zip(offs, lens_)):
    g = ga[o:o+l_]; w = want[o:o+l_]
    if g.tobytes() != w.tobytes():
        nb += 1
        if nb <= 6:
            pos = np.nonzero(g != w)[0]
            print(i, "len", l_, "off%16", o % 16, "err", wres[i]["err"], "hl", wres[i]["header_len"], "kinds", [op[0] for op in chains[i].ops],
                  "diffpos", pos[:12].tolist(), "got", g[pos[:6]].tolist(), "want", w[pos[:6]].tolist(), "before", before[o:o+l_][pos[:6]].tolist())
print("bad", nb, "res equal", got.tobytes() == wres.tobytes())
