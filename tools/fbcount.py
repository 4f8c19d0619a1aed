"""Diagnostic: fallback (past-window) chunk loads per frame of the walk, from
the ZP_DBG_FBCOUNT builds (tools/build_variants.sh fbcount...)."""
import ctypes
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    zp = importlib.import_module("zero-packet_amd")
    dev = torch.device("cuda:0")
    for cfg, n in (("c3", 1 << 22), ("c4", 1 << 22), ("c5", 1 << 22)):
        arena, offs, lens = zp.batch.generate(cfg, n, device=dev)
        rec = torch.empty((n, 8), dtype=torch.uint8, device=dev)
        ext = torch.empty((2, n, 16), dtype=torch.uint8, device=dev)
        for v in sys.argv[1].split(","):
            lib = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzp_{v}.so"))
            lib.zp_parse_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
                [ctypes.c_void_p] * 3
            lib.zp_dbg_fb_count.restype = ctypes.c_ulonglong
            lib.zp_dbg_fb_count()
            rep = getattr(lib, "zp_dbg_fb_repeat", None)
            if rep is not None:
                rep.restype = ctypes.c_ulonglong
                rep()
            lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                      rec.data_ptr(), ext.data_ptr(), None)
            torch.cuda.synchronize()
            c = lib.zp_dbg_fb_count()
            r = f", {rep()} of them repeats of a chunk the frame had loaded" if rep is not None else ""
            print(f"{cfg} {v}: {c} fallback chunk loads, {c / n:.3f} per frame{r}", flush=True)


if __name__ == "__main__":
    main()
