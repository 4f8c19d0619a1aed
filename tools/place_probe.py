"""Placement probe (measurement only): c3 parse time against where the
records buffer lies relative to the arena. One arena (generated once), one
records pool; the records pointer is carved at offsets within the pool, so
only the records' placement changes. Also the arena's own placement: copies
of the arena at offsets within a second pool (--arena-moves)."""
import argparse
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
zp = importlib.import_module("zero-packet_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 24)
    ap.add_argument("--offsets", default="0,64K,128K,256K,512K,1M,2M,3M,4M,6M,8M,12M,16M,24M,32M")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--arena-moves", default="",
                    help="offsets of arena copies within one pool (records fixed)")
    ap.add_argument("--arena-allocs", type=int, default=0,
                    help="separate allocations of arena copies (records fixed)")
    ap.add_argument("--hip-allocs", default="",
                    help="arena copies in hipMalloc / hipExtMallocWithFlags buffers: "
                         "comma list of default,contig")
    ap.add_argument("--dummy-first", type=int, default=0,
                    help="GiB allocated (and kept) before the arena is generated")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n = args.frames
    dummy = torch.empty(args.dummy_first << 30, dtype=torch.uint8, device=dev) if args.dummy_first else None
    arena, offs, lens = zp.batch.generate("c3", n, device=dev)
    ext = torch.empty((2, n, 16), dtype=torch.uint8, device=dev)

    def sz(x):
        m = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
        return int(x[:-1]) * m[x[-1]] if x[-1] in m else int(x)
    offsets = [sz(x) for x in args.offsets.split(",")]
    rec_bytes = n * 8
    pool = torch.empty(rec_bytes + max(offsets) + (1 << 20), dtype=torch.uint8, device=dev)
    lib = zp._lib.hip()
    s = torch.cuda.current_stream(dev)
    print(f"arena at {arena.data_ptr():#x} (mod 2M {arena.data_ptr() % (2 << 20):#x}), "
          f"records pool at {pool.data_ptr():#x}", flush=True)
    res = {o: [] for o in offsets}
    for _ in range(args.rounds):
        for o in offsets:
            rp = pool.data_ptr() + o
            def launch():
                zp._lib.check(lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                                        ctypes.c_void_p(rp), ext.data_ptr(),
                                                        ctypes.c_void_p(s.cuda_stream)), "parse")
            launch()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for a, b in ev:
                a.record(s); launch(); b.record(s)
            torch.cuda.synchronize()
            res[o].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
    total = int(lens.to(torch.int64).sum().item())
    nbytes = arena.numel()

    def timed(ap_, rp):
        def launch():
            zp._lib.check(lib.zp_parse_batch_device(ctypes.c_void_p(ap_), offs.data_ptr(), lens.data_ptr(), n,
                                                    ctypes.c_void_p(rp), ext.data_ptr(),
                                                    ctypes.c_void_p(s.cuda_stream)), "parse")
        launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.reps)]
        for a, b in ev:
            a.record(s); launch(); b.record(s)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))
    if args.arena_moves:
        moves = [sz(x) for x in args.arena_moves.split(",")]
        big = torch.empty(nbytes + max(moves), dtype=torch.uint8, device=dev)
        out = {m: [] for m in moves}
        for _ in range(args.rounds):
            for m in moves:
                big[m:m + nbytes].copy_(arena)
                torch.cuda.synchronize()
                out[m].append(timed(big.data_ptr() + m, pool.data_ptr()))
        for m in moves:
            ms = float(np.median(out[m]))
            print(f"arena copy at pool+{m:>11} (VA {big.data_ptr() + m:#x}): {ms:.3f} ms = "
                  f"{total / ms / 1e6 / 8000:.3f}  rounds {['%.3f' % x for x in out[m]]}", flush=True)
        del big
    if args.arena_allocs:
        copies = [arena]
        for _ in range(args.arena_allocs):
            copies.append(arena.clone())
        torch.cuda.synchronize()
        out = [[] for _ in copies]
        for _ in range(args.rounds):
            for i, c in enumerate(copies):
                out[i].append(timed(c.data_ptr(), pool.data_ptr()))
        for i, c in enumerate(copies):
            ms = float(np.median(out[i]))
            print(f"arena alloc {i} (VA {c.data_ptr():#x}): {ms:.3f} ms = {total / ms / 1e6 / 8000:.3f}  "
                  f"rounds {['%.3f' % x for x in out[i]]}", flush=True)
    if args.hip_allocs:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        hip.hipFree.argtypes = [ctypes.c_void_p]
        bufs = []
        for kind in args.hip_allocs.split(","):
            p = ctypes.c_void_p()
            rc = (hip.hipMalloc(ctypes.byref(p), nbytes) if kind == "default" else
                  hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, 0x4))
            if rc != 0:
                print(f"{kind}: allocation failed rc {rc}", flush=True)
                continue
            assert hip.hipMemcpy(p, ctypes.c_void_p(arena.data_ptr()), nbytes, 3) == 0   # device to device
            bufs.append((kind, p.value))
        out = [[] for _ in bufs]
        for _ in range(args.rounds):
            for i, (_, a) in enumerate(bufs):
                out[i].append(timed(a, pool.data_ptr()))
        for i, (kind, a) in enumerate(bufs):
            ms = float(np.median(out[i]))
            print(f"hip {kind} alloc (VA {a:#x}): {ms:.3f} ms = {total / ms / 1e6 / 8000:.3f}  "
                  f"rounds {['%.3f' % x for x in out[i]]}", flush=True)
        for _, a in bufs:
            hip.hipFree(ctypes.c_void_p(a))
    for o in offsets:
        ms = float(np.median(res[o]))
        print(f"records at pool+{o:>10} (rec-arena {(pool.data_ptr() + o - arena.data_ptr()) % (1 << 30):#x} mod 1G): "
              f"{ms:.3f} ms = {total / ms / 1e6 / 8000:.3f} of 8 TB/s  rounds {['%.3f' % x for x in res[o]]}",
              flush=True)


if __name__ == "__main__":
    main()
