"""Phase timing from the ZP_STAMPS diagnostic build (tools/variants/libzp_stamps*.so).
Shares, not absolute times, are meaningful (guide §7 'In-kernel stamps')."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ["desc+setup", "issue0", "stream", "walk+verdict"]
# builds with the tile_finish stamps (5: walk done, 6: verdict done)
NAMES_FINE = ["desc+setup", "issue0", "stream", "walk", "verdict", "stores"]
ORDER_FINE = [0, 1, 2, 3, 5, 6, 4]


def main():
    zp = importlib.import_module("zero-packet_amd")
    dev = torch.device("cuda:0")
    for variant in sys.argv[1].split(","):
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzp_{variant}.so"))
        lib.zp_parse_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
            [ctypes.c_void_p] * 3
        lib.zp_stamps_set.argtypes = [ctypes.c_void_p]
        for cfg in sys.argv[2].split(","):
            n = {"c3": 1 << 24, "c4": 1 << 24, "c5": 1 << 25, "c2": 1 << 20}[cfg]
            arena, offs, lens = zp.batch.generate(cfg, n, device=dev)
            rec = torch.empty((n, 8), dtype=torch.uint8, device=dev)
            ext = torch.empty((2, n, 16), dtype=torch.uint8, device=dev)
            nw = (n + 63) // 64
            buf = torch.zeros(nw * 8, dtype=torch.int64, device=dev)
            run = lambda: lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(),
                                                     lens.data_ptr(), n, rec.data_ptr(),
                                                     ext.data_ptr(), None)
            lib.zp_stamps_set(None)
            run(); run()
            lib.zp_stamps_set(ctypes.c_void_p(buf.data_ptr()))
            run()
            torch.cuda.synchronize()
            lib.zp_stamps_set(None)
            t = buf.view(nw, 8).cpu().numpy().astype(np.int64) * 10  # ns
            fine = bool((t[:, 5] > 0).all() and (t[:, 6] > 0).all())
            names = NAMES_FINE if fine else NAMES
            t = t[:, ORDER_FINE] if fine else t[:, :len(NAMES) + 1]
            d = np.diff(t, axis=1)
            life = t[:, -1] - t[:, 0]
            kern = t[:, -1].max() - t[:, 0].min()
            # average number of resident waves = sum(lifetimes) / kernel span
            print(f"{variant} {cfg}: kernel span {kern/1e6:.3f} ms, wave life mean "
                  f"{life.mean()/1e3:.1f} us (p50 {np.median(life)/1e3:.1f}, p99 "
                  f"{np.percentile(life, 99)/1e3:.1f}), mean resident waves "
                  f"{life.sum()/kern:.0f}", flush=True)
            print("   " + "  ".join(f"{nm} {d[:, i].mean()/1e3:.2f}us ({100*d[:, i].mean()/life.mean():.0f}%)"
                                     for i, nm in enumerate(names)), flush=True)
            del arena, offs, lens, rec, ext, buf
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
