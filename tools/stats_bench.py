"""Timing of zp_stats_device over one c3 batch's records (16M x 8 B)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes
    zp = importlib.import_module("zero-packet_amd")
    variants = [v for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else []) if v]
    d = torch.device("cuda:0")
    n = 1 << 24
    arena, offs, lens = zp.batch.generate("c3", n, device=d)
    r, _ = zp.batch.parse_batch(arena, offs, lens)
    del arena
    c = zp.stats.count(r)
    s = torch.cuda.current_stream()
    libs = [("base", zp._lib.hip())]
    for v in variants:      # A/B builds of zp_stats.hip (tools/variants/libzs_<v>.so)
        libs.append((v, ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzs_{v}.so"))))
    for rnd in range(3):
        for name, lib in libs:
            ref = zp.stats.count(r)
            c.zero_()
            lib.zp_stats_device(ctypes.c_void_p(r.data_ptr()), ctypes.c_uint64(n),
                                ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(s.cuda_stream))
            torch.cuda.synchronize()
            assert torch.equal(c, ref), name
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(20)]
            for a, b in ev:
                a.record(s)
                lib.zp_stats_device(ctypes.c_void_p(r.data_ptr()), ctypes.c_uint64(n),
                                    ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(s.cuda_stream))
                b.record(s)
            torch.cuda.synchronize()
            ms = sorted(a.elapsed_time(b) for a, b in ev)[10]
            print(f"zp_stats_device [{name}], {n} records: {ms * 1e3:.1f} us, "
                  f"{n * 8 / ms / 1e6:.0f} GB/s of records, {n / ms / 1e6:.1f} Gpkt/s", flush=True)
    print(zp.stats.to_dict(zp.stats.count(r)), flush=True)


if __name__ == "__main__":
    main()
