"""HBM write granularity: g bytes written per 128-B line (16-B stores), over
the same number of lines; if the time per line does not fall with g, partial
lines cost like whole ones (read-modify-write or line-granular writes).

    python tools/wgran.py [--gib 8]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from kbench import time_launches  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    mb = ctypes.CDLL(os.path.join(ROOT, "tools", "libmembw.so"))
    mb.membw_write.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    buf = torch.zeros(a.gib << 30, dtype=torch.uint8, device=dev)
    lines = buf.numel() // 128
    for nt in (0, 1):
        for lg16, off16 in ((3, 0), (2, 0), (2, 2), (2, 4), (1, 0), (1, 1), (1, 2), (0, 0),
                            (0, 1), (0, 3)):
            g = 16 << lg16
            f = lambda: mb.membw_write(buf.data_ptr(), lines, lg16, off16, nt, 4096, None)
            assert f() == 0
            ms = float(np.median(time_launches(f, a.reps)))
            print(f"nt={nt} {g:3d} B/line at +{16 * off16:3d}: {ms:7.3f} ms  "
                  f"{lines / ms / 1e6:6.2f} Glines/s  {lines * g / ms / 1e6:6.0f} GB/s written",
                  flush=True)


if __name__ == "__main__":
    main()
