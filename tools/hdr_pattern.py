"""The in-place builder's access pattern without its work (tools/membw.hip
hdr_tiles): one wave per tile of 64 frames, the tile read once by 1 KiB
nontemporal wave loads in groups of 8, then each lane writes back the whole
64-B sectors covering its frame's first `hdr` bytes (the builder's header
write-back). Store policies: plain / nt / write-through (agent-scope atomic
stores) / none / plain by the whole wave (coalesced) / plain without the
read. Next to it: the parse kernel and the builder on 4M c3
frames of the same box (tools/build_bench.py times the builder).

    python tools/hdr_pattern.py [--hdr 54,108]
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
import ucmem  # noqa: E402


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--hdr", default="54,108")
    ap.add_argument("--region", type=int, default=50016, help="tile bytes (c3: 64 x 781.5 B)")
    ap.add_argument("--gib", type=int, default=3, help="buffer (4M c3 frames = 3.28 GB)")
    ap.add_argument("--twophase", action="store_true",
                    help="also the write-back in two kernels: reads + a contiguous 64-B slot per "
                         "frame, then the slots read back and the sectors written")
    ap.add_argument("--uncached", action="store_true",
                    help="the buffer in uncached device memory (tools/ucmem.py)")
    ap.add_argument("--policies", default="3,1,0,2,4,5",
                    help="store policies to time (PMC passes: one or two)")
    ap.add_argument("--no-parse", action="store_true", help="skip the parse of 4M c3 frames")
    args = ap.parse_args()
    mb = ctypes.CDLL(os.path.join(ROOT, "tools", "libmembw.so"))
    mb.membw_hdr_tiles.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                   ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]
    d = torch.device("cuda:0")
    buf = torch.randint(0, 255, (args.gib << 30,), dtype=torch.uint8, device=d)
    if args.uncached:
        zp = importlib.import_module("zero-packet_amd")
        ub = ucmem.empty(buf.numel(), device=d)
        ub.copy_(buf)
        del buf
        buf = ub
        print("buffer in uncached device memory", flush=True)
    nb = buf.numel() // args.region * args.region
    names = {3: "read only", 1: "nt", 0: "plain", 2: "write-through", 4: "plain coop",
             5: "write only", 6: "plain paused", 7: "coop paused",
             8: "at frame start", 9: "at frame end"}
    pols = [int(x) for x in args.policies.split(",")]
    for hdr in [int(x) for x in args.hdr.split(",")]:
        # The write floor in absolute 64-B sectors: each lane writes the
        # 16-B chunks [s0, s1) of its tile (sectors relative to the tile base,
        # which is only 32-B aligned for odd tiles at region 50016)
        ntile = nb // args.region
        base = buf.data_ptr() + np.arange(ntile, dtype=np.int64) * args.region
        f = np.arange(64, dtype=np.int64) * (args.region // 64)
        s0, s1 = f & ~63, (f + hdr + 63) & ~63
        s1 = np.minimum(s1, args.region // 16 * 16)
        lo = (base[:, None] + s0[None, :]) // 64
        hi = (base[:, None] + s1[None, :] - 1) // 64
        sect = int((hi - lo + 1).sum())
        part = int(((base[:, None] + s0[None, :]) % 64 != 0).sum() +
                   ((base[:, None] + s1[None, :]) % 64 != 0).sum())
        wbytes = int((s1 - s0).sum()) * ntile
        print(f"hdr {hdr}: {ntile} tiles, written {wbytes / 1e6:.1f} MB in {sect} absolute 64-B "
              f"sectors = {sect * 64 / 1e6:.1f} MB ({part} partially covered sector ends)",
              flush=True)
        for pol in pols:
            name = names[pol]
            ms = timed(lambda: mb.membw_hdr_tiles(buf.data_ptr(), buf.numel(), args.region, hdr,
                                                  pol, 13 * 1024, None))
            print(f"hdr tiles region {args.region} hdr {hdr:4d} B {name:14s}: {ms:7.3f} ms "
                  f"read {nb / ms / 1e6:6.0f} GB/s", flush=True)
    if args.twophase:
        mb.membw_hdr_twophase.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_void_p]
        tmp = torch.empty(nb // args.region * 4096, dtype=torch.uint8, device=d)
        for hdr in [int(x) for x in args.hdr.split(",")]:
            for ph, name in ((3, "two phases"), (1, "phase 1 only"), (2, "phase 2 only")):
                ms = timed(lambda: mb.membw_hdr_twophase(buf.data_ptr(), buf.numel(), args.region,
                                                         hdr, tmp.data_ptr(), ph, None))
                print(f"hdr tiles region {args.region} hdr {hdr:4d} B {name:14s}: {ms:7.3f} ms",
                      flush=True)
        del tmp
    if args.no_parse:
        return
    zp = importlib.import_module("zero-packet_amd")
    n = 1 << 22
    arena, offs, lens = zp.batch.generate("c3", n, device=d)
    rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
    lib = zp._lib.hip()
    ms = timed(lambda: lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                                 n, rec.data_ptr(), None, None))
    print(f"parse 4M c3 frames ({int(lens.sum()) / 1e9:.2f} GB): {ms:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
