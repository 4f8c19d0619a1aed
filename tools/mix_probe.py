"""Mixed traffic: tiles holding k IPv6 frames with extension chains (c4) among
64 - k IPv4 frames (c3), at random lanes. Times the parse with each variant
library (e.g. ZP_EXT_DENSE thresholds: from how many chains per wave all 64
extension entries are written as whole lines instead of only the flagged
ones) on the same batch.

    python tools/mix_probe.py --variants d8,d65 [--ks 4,8,12,16,24]
"""
import argparse
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from kbench import time_launches  # noqa: E402
from sort_probe import regroup  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=1 << 17)
    ap.add_argument("--ks", default="4,8,12,16,24")
    ap.add_argument("--variants", default="")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    dev = torch.device("cuda:0")
    libs = {"base": zp._lib.hip()}
    for v in filter(None, a.variants.split(",")):
        l = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzp_{v}.so"))
        l.zp_parse_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
            [ctypes.c_void_p] * 3
        libs[v] = l
    T = a.tiles
    n = 64 * T
    kmax = max(int(k) for k in a.ks.split(","))
    a3, o3, l3 = zp.batch.generate("c3", (64 - 1) * T, device=dev)
    a4, o4, l4 = zp.batch.generate("c4", kmax * T, device=dev)
    arena = torch.cat([a3, a4])
    offs = torch.cat([o3, o4 + a3.numel()])
    lens = torch.cat([l3, l4])
    del a3, a4
    torch.cuda.empty_cache()
    n3 = o3.numel()
    rec = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    ext = torch.empty((2, n, 16), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    for k in [int(x) for x in a.ks.split(",")]:
        # tile t: c4 frames k*t .. k*t+k-1 and c3 frames (64-k)*t .. at random lanes
        t = torch.arange(T, device=dev)
        src = torch.empty((T, 64), dtype=torch.int64, device=dev)
        src[:, :k] = n3 + k * t[:, None] + torch.arange(k, device=dev)
        src[:, k:] = (64 - k) * t[:, None] + torch.arange(64 - k, device=dev)
        order = torch.argsort(torch.rand((T, 64), device=dev, generator=g), dim=1)
        perm = torch.gather(src, 1, order).reshape(-1)
        a2, o2, l2 = regroup(arena, offs, lens, perm)
        ref_rec = ref_ext = None
        res = {name: [] for name in libs}
        for r in range(a.rounds):
            for name, l in libs.items():
                f = lambda l=l: l.zp_parse_batch_device(a2.data_ptr(), o2.data_ptr(),
                                                         l2.data_ptr(), n, rec.data_ptr(),
                                                         ext.data_ptr(), None)
                res[name] += time_launches(f, a.reps)
                if r == 0:
                    flags = rec[:, 0:4].contiguous().view(torch.int32)[:, 0]
                    has = (flags & (1 << 10)) != 0
                    if ref_rec is None:
                        ref_rec, ref_ext = rec.clone(), ext[0][has].clone()
                        assert int((zp.batch.record_err(rec) != 0).sum()) == 0
                    elif not (torch.equal(rec, ref_rec) and torch.equal(ext[0][has], ref_ext)):
                        print(f"  !! {name}: records or chains differ (k={k})", flush=True)
        nb = int(l2.to(torch.int64).sum())
        for name, ms in res.items():
            med = float(np.median(ms))
            print(f"k={k:2d} chains/wave {name:>6}: {med:.3f} ms  {nb / med / 1e6:6.0f} GB/s",
                  flush=True)
        del a2, o2, l2, perm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
