"""Upper bound of walk-divergence removal: the same frames, regrouped so
that the frames of one wave share a header stack, timed against the
generator's order.

    python tools/sort_probe.py [--config c5] [--windows 256,4096,0]

Each frame gets a kind key from its parse record (outer IPv4/IPv6, IP-in-IP
tag, L4 type, extension chains). Inside windows of W consecutive frames
(0 = the whole batch) the frames are stably sorted by that key and the arena
is rebuilt packed in the new order on the GPU. The kernel is unchanged; only
the order of the input differs. Records of the sorted batch are checked
against the permuted records of the original one.
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from kbench import time_launches  # noqa: E402


def regroup(arena, offs, lens, perm, chunk=1 << 20):
    """arena2 packed in `perm` order (ragged gather in chunks of frames)."""
    dev = arena.device
    l2 = lens[perm].to(torch.int64)
    o2 = torch.zeros_like(l2)
    o2[1:] = torch.cumsum(l2[:-1], 0)
    total = int(o2[-1] + l2[-1])
    a2 = torch.zeros(total + 64, dtype=torch.uint8, device=dev)
    src_off = offs[perm]
    for lo in range(0, len(perm), chunk):
        hi = min(lo + chunk, len(perm))
        ln = l2[lo:hi]
        fr = torch.repeat_interleave(torch.arange(hi - lo, device=dev), ln)
        base = o2[lo]
        pos = torch.arange(int(ln.sum()), device=dev, dtype=torch.int64)
        within = pos + base - o2[lo:hi][fr]
        a2[base + pos] = arena[src_off[lo:hi][fr] + within]
    return a2, o2, l2.to(torch.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--packets", type=int, default=1 << 25)
    ap.add_argument("--windows", default="256,4096,0")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shuffle-tiles", action="store_true")
    args = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    lib = zp._lib.hip()
    dev = torch.device("cuda:0")
    n = args.packets
    arena, offs, lens = zp.batch.generate(args.config, n, device=dev)
    rec = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    ext = torch.empty((2, n, 16), dtype=torch.uint8, device=dev)
    nbytes = int(lens.to(torch.int64).sum())

    def run(a, o, l_):
        return lambda: lib.zp_parse_batch_device(a.data_ptr(), o.data_ptr(), l_.data_ptr(), n,
                                                 rec.data_ptr(), ext.data_ptr(), None)

    run(arena, offs, lens)()
    torch.cuda.synchronize()
    flags = rec[:, 0:4].contiguous().view(torch.int32)[:, 0].to(torch.int64)
    key = flags & 0xFFF                     # presence bits: stack shape and L4 type
    ref = rec.clone()
    base_ms = float(np.median(time_launches(run(arena, offs, lens), args.reps)))
    print(f"{args.config} generator order: {base_ms:.3f} ms  "
          f"{nbytes / base_ms / 1e6:.0f} GB/s", flush=True)
    for w in [int(x) for x in args.windows.split(",")]:
        W = n if w == 0 else w
        win = torch.arange(n, device=dev) // W
        perm = torch.argsort(win * 4096 + key, stable=True)
        if args.shuffle_tiles and w:
            # same tiles, random tile order inside each window: the kinds do
            # not land on the same XCD (workgroup b runs on XCD b % 8) in
            # every window
            t = perm[: n // W * W].view(n // W, W // 64, 64)
            g = torch.Generator(device=dev).manual_seed(7)
            order = torch.argsort(torch.rand(t.shape[:2], device=dev, generator=g), dim=1)
            t = torch.gather(t, 1, order[:, :, None].expand_as(t))
            perm = torch.cat([t.reshape(-1), perm[n // W * W:]])
        a2, o2, l2 = regroup(arena, offs, lens, perm)
        f = run(a2, o2, l2)
        f()
        torch.cuda.synchronize()
        same = torch.equal(rec[:, 4:8], ref[perm][:, 4:8]) and \
            torch.equal(rec[:, 0:4], ref[perm][:, 0:4])
        ms = []
        for _ in range(3):
            ms += time_launches(run(arena, offs, lens), args.reps // 2)
        base2 = float(np.median(ms))
        ms = []
        for _ in range(3):
            ms += time_launches(f, args.reps // 2)
        t = float(np.median(ms))
        print(f"{args.config} sorted in windows of {w or 'all'}{' (tiles shuffled)' if args.shuffle_tiles else ''}: {t:.3f} ms "
              f"(generator order {base2:.3f} ms, {100 * (t / base2 - 1):+.1f} %)  "
              f"flags/err match: {same}", flush=True)
        del a2, o2, l2, perm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
