"""Output (and input) memory kind A/B, one process, interleaved rounds
(DESIGN.md §4, round 5): the parse with its records + ext entries in ordinary
(torch / hipMalloc) or uncached device memory (tools/ucmem.py), and with the arena copied into uncached memory as well;
the fused parse + columns and the split path with the columns in either kind.

    python tools/uc_ab.py [--configs c3,c5,c4,c2,c6] [--columns]
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


def times(fn, reps):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c5,c4,c2,c6")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--columns", action="store_true")
    ap.add_argument("--arena-uc", action="store_true", help="also the arena in uncached memory")
    a = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    B = zp.batch
    lib = zp._lib.hip()
    d = torch.device("cuda:0")
    sizes = {"c2": 1 << 20, "c3": 1 << 24, "c4": 1 << 24, "c5": 1 << 25, "c6": 1 << 24}
    for cfg in a.configs.split(","):
        n = sizes[cfg]
        arena, offs, lens = B.generate(cfg, n, device=d)
        nbytes = int(lens.to(torch.int64).sum())
        outs = {"default": (torch.empty((n, 8), dtype=torch.uint8, device=d),
                            torch.empty((2, n, 16), dtype=torch.uint8, device=d)),
                "uncached": (ucmem.empty((n, 8), device=d), ucmem.empty((2, n, 16), device=d))}
        arenas = {"arena": arena}
        if a.arena_uc:
            au = ucmem.empty(arena.numel(), device=d)
            au.copy_(arena)
            arenas["arena_uc"] = au
        variants = [(f"{an}/rec_{k}", ar, r, e) for an, ar in arenas.items()
                    for k, (r, e) in outs.items()]
        res = {v[0]: [] for v in variants}
        ref = None
        for r in range(a.rounds):
            for name, ar, rec, ext in variants:
                fn = lambda ar=ar, rec=rec, ext=ext: lib.zp_parse_batch_device(
                    ar.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, rec.data_ptr(),
                    ext.data_ptr(), None)
                res[name] += times(fn, a.reps)
                if r == 0:
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = rec.clone()
                    elif not torch.equal(ref, rec):
                        print(f"  !! {cfg} {name}: records differ", flush=True)
        base = float(np.median(res[variants[0][0]]))
        for name, ms in res.items():
            med = float(np.median(ms))
            print(f"{cfg} parse {name:24s}: {med:8.4f} ms = {nbytes / med / 1e6 / 8000:.4f} of 8 TB/s"
                  f"  ({med / base - 1:+.1%})", flush=True)
        if a.columns and cfg != "c2":
            C = zp.columns
            for label, names in (("5tuple", ["src_addr", "dest_addr", "protocol", "src_port",
                                             "dest_port"]), ("all", C.NAMES)):
                cres = {}
                for kind in ("default", "uncached"):
                    rec, ext = outs[kind]
                    if kind == "default":
                        cols = {k: C._alloc(k, n, d) for k in names}
                    else:
                        cols = {}
                        for k in names:
                            _, dt, w = C.COLUMNS[C.INDEX[k]]
                            cols[k] = ucmem.empty((n, w) if w > 1 else (n,), dtype=dt, device=d)
                    ptrs = (ctypes.c_void_p * len(C.NAMES))()
                    for k in names:
                        ptrs[C.INDEX[k]] = cols[k].data_ptr()
                    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                    fused = lambda: lib.zp_parse_batch_columns_device(
                        arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, rec.data_ptr(),
                        ext.data_ptr(), ptrs, s)

                    def split():
                        lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(),
                                                  lens.data_ptr(), n, rec.data_ptr(),
                                                  ext.data_ptr(), s)
                        lib.zp_extract_columns_device(arena.data_ptr(), offs.data_ptr(),
                                                      lens.data_ptr(), rec.data_ptr(), n, ptrs, s)
                    cres[f"fused/{kind}"] = []
                    cres[f"split/{kind}"] = []
                    for r in range(a.rounds):
                        cres[f"fused/{kind}"] += times(fused, a.reps)
                        cres[f"split/{kind}"] += times(split, a.reps)
                    del cols
                line = "  ".join(f"{k} {float(np.median(v)):.3f}" for k, v in cres.items())
                print(f"{cfg} columns[{label}] ms: {line}", flush=True)
        del arena, offs, lens, outs, arenas, variants
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
