"""Record-code campaign (not part of the suite): c3 / c6 batches of 2M
frames with random header and payload bit flips in a random share of the
tiles (clean tiles take codes, mutated ones their records), parsed with
record codes always (zp_set_record_slots(1)) and never (2); the two must be
byte-identical, and a sample of each batch equal to the oracle.
Usage: python tools/fuzz_codes.py [rounds]"""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as orc  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    zp = importlib.import_module("zero-packet_amd")
    lib = zp._lib.hip()
    d = torch.device("cuda:0")
    n = 1 << 21
    total = 0
    for r in range(rounds):
        cfg = "c3" if r % 2 == 0 else "c6"
        arena, offs, lens = zp.batch.generate(cfg, n, first=1000003 * r, device=d)
        rng = np.random.default_rng(r)
        tiles = n // 64
        share = [0.01, 0.1, 0.5][r % 3]
        bad_tiles = np.nonzero(rng.random(tiles) < share)[0]
        k = int(len(bad_tiles))
        fr = bad_tiles * 64 + rng.integers(0, 64, k)
        o = offs[torch.from_numpy(fr).to(d)]
        l_ = lens[torch.from_numpy(fr).to(d)].to(torch.int64)
        pos = o + (torch.rand(k, device=d) * l_).to(torch.int64).clamp(max=l_ - 1)
        bit = torch.from_numpy(rng.integers(0, 8, k)).to(d).to(torch.uint8)
        arena[pos] ^= (torch.ones_like(bit) << bit)
        out = {}
        for mode in (1, 2):
            lib.zp_set_record_slots(mode)
            rec = torch.full((n, 8), 0xA5 if mode == 1 else 0x00, dtype=torch.uint8, device=d)
            zp.batch.parse_batch(arena, offs, lens, rec, check=False)
            torch.cuda.synchronize()
            out[mode] = rec
        lib.zp_set_record_slots(0)
        same = torch.equal(out[1], out[2])
        idx = np.sort(np.concatenate([rng.choice(n, 3000, replace=False), fr[:1000]]))
        so, sl = offs.cpu().numpy()[idx], lens.cpu().numpy()[idx]
        ah = arena.cpu().numpy()
        frames = [ah[int(a):int(a) + int(b)] for a, b in zip(so, sl)]
        pl = np.array([len(f) for f in frames], np.uint32)
        po = np.concatenate([[0], np.cumsum(pl[:-1].astype(np.int64))]).astype(np.uint64)
        pa = np.zeros(int(pl.sum()) + 64, np.uint8)
        for a, f in zip(po, frames):
            pa[int(a):int(a) + len(f)] = f
        want, wext = orc.parse_batch(pa, po, pl)
        w = orc.pack(want, wext).view(np.uint8).reshape(-1, 8)
        g = out[1].cpu().numpy()[idx]
        bad = int((g != w).any(1).sum())
        errs = int((zp.batch.record_err(out[1]) != 0).sum())
        total += n
        print(f"round {r} {cfg} share {share}: {k} mutated frames, {errs} error records, "
              f"codes == records: {same}, oracle sample {len(idx) - bad}/{len(idx)}", flush=True)
        assert same and bad == 0
    print(f"fuzz_codes: {total} frames, all identical", flush=True)


if __name__ == "__main__":
    main()
