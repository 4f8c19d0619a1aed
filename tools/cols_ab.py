"""A/B of the column-view kernels (standalone zp_extract_columns_device and
fused zp_parse_batch_columns_device) between the in-tree library and
tools/variants/libzc_<name>.so builds, interleaved in one process.
Usage: python tools/cols_ab.py prev[,other] [--configs c3,c5]"""
import argparse
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--configs", default="c3,c5")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    libs = [("base", zp._lib.hip())]
    for v in a.variants.split(","):
        libs.append((v, ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzc_{v}.so"))))
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    for _, l in libs:
        l.zp_extract_columns_device.argtypes = [vp, vp, vp, vp, u64, vp, vp]
        l.zp_parse_batch_columns_device.argtypes = [vp, vp, vp, u64, vp, vp, vp, vp]
    d = torch.device("cuda:0")
    s = torch.cuda.current_stream(d)
    for cfg in a.configs.split(","):
        n = {"c3": 1 << 24, "c4": 1 << 24, "c5": 1 << 25, "c2": 1 << 20}[cfg]
        arena, offs, lens = zp.batch.generate(cfg, n, device=d)
        rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
        ext = torch.empty((2, n, 16), dtype=torch.uint8, device=d)
        cols = [torch.empty(n * zp.columns.width(c), dtype=torch.uint8, device=d)
                for c in zp.columns.NAMES]
        ptrs = (ctypes.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
        zp.batch.parse_batch(arena, offs, lens, rec, ext, check=False)
        ref = None
        for name, l in libs:
            for label, fn in (
                    ("columns", lambda: l.zp_extract_columns_device(
                        arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), rec.data_ptr(), n,
                        ptrs, s.cuda_stream)),
                    ("fused", lambda: l.zp_parse_batch_columns_device(
                        arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, rec.data_ptr(),
                        ext.data_ptr(), ptrs, s.cuda_stream))):
                for c in cols:
                    c.zero_()
                assert fn() == 0
                torch.cuda.synchronize()
                got = torch.cat(cols)
                if ref is None:
                    ref = got.clone()
                same = bool(torch.equal(ref, got))
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.reps)]
                for x, y in ev:
                    x.record(s); fn(); y.record(s)
                torch.cuda.synchronize()
                ms = float(np.median([x.elapsed_time(y) for x, y in ev]))
                print(f"{cfg} {label:8s} [{name}]: {ms:.3f} ms{'' if same else '  COLUMNS DIFFER'}",
                      flush=True)
        del arena, offs, lens, rec, ext, cols, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
