"""Record-store cost in the parse kernel's tile pattern by the records'
memory type (tools/membw.hip read_tiles with 8-B records): the
c5 and c3 tile sizes, records in hipMalloc / fine-grained / uncached /
contiguous device memory; then the parse kernel itself on c5 and c3 with its
records in each kind (same arena).

    python tools/rec_pattern.py
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KINDS = ["hipMalloc", "fine-grained", "uncached", "contiguous"]


def timed(fn, reps=10):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    fn()
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    mb = ctypes.CDLL(os.path.join(ROOT, "tools", "libmembw.so"))
    mb.membw_alloc.restype = ctypes.c_void_p
    mb.membw_alloc.argtypes = [ctypes.c_uint64, ctypes.c_int]
    mb.membw_free.argtypes = [ctypes.c_void_p]
    mb.membw_tiles.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                               ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]
    d = torch.device("cuda:0")
    buf = torch.randint(0, 255, (12 << 30,), dtype=torch.uint8, device=d)
    outs = {k: mb.membw_alloc((12 << 30) // 4096 * 64 * 8 + 4096, i) for i, k in enumerate(KINDS)}
    for label, region in (("c5 tile", 22672), ("c3 tile", 50016)):
        nb = buf.numel() // region * region
        ms = timed(lambda: mb.membw_tiles(buf.data_ptr(), buf.numel(), outs["hipMalloc"], region,
                                          0, 8960, None))
        print(f"tiles {label}: no records {ms:.3f} ms {nb / ms / 1e6:.0f} GB/s", flush=True)
        for k, p in outs.items():
            if not p:
                print(f"tiles {label}: {k}: allocation failed", flush=True)
                continue
            ms = timed(lambda: mb.membw_tiles(buf.data_ptr(), buf.numel(), p, region, 1, 8961,
                                              None))
            print(f"tiles {label}: 8-B records in {k:13s} {ms:.3f} ms {nb / ms / 1e6:.0f} GB/s",
                  flush=True)
    del buf
    torch.cuda.empty_cache()
    zp = importlib.import_module("zero-packet_amd")
    lib = zp._lib.hip()
    for cfg, n in (("c5", 1 << 25), ("c3", 1 << 24)):
        arena, offs, lens = zp.batch.generate(cfg, n, device=d)
        nbytes = int(lens.to(torch.int64).sum())
        ext = torch.empty((2, n, 16), dtype=torch.uint8, device=d)
        for k, p in outs.items():
            if not p:
                continue
            ms = timed(lambda: lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(),
                                                         lens.data_ptr(), n, p, ext.data_ptr(),
                                                         None))
            print(f"parse {cfg}: records in {k:13s} {ms:.3f} ms = {nbytes / ms / 1e6 / 8000:.3f} "
                  f"of 8 TB/s", flush=True)
        del arena, offs, lens, ext
        torch.cuda.empty_cache()
    for p in outs.values():
        if p:
            mb.membw_free(p)


if __name__ == "__main__":
    main()
