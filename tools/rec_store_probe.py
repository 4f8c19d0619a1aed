"""Record-store probe (lab): times tools/probes/rec_store.hip's modes over a
generated batch (the parse's tile pattern, descriptors included), interleaved
rounds in one process, beside the parse itself.

    python tools/rec_store_probe.py [--config c3] [--rounds 5]
"""
import argparse
import ctypes
import importlib
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MODES = {0: "no stores", 1: "nt 8 B x 64 at end (parse)", 2: "default policy at end",
         3: "nt before the loads", 4: "nt 16 B x 32 lanes", 5: "nt into a 2 MiB ring",
         6: "nt after half the loads", 7: "nt into the arena slice just read",
         8: "default policy into the 2 MiB ring", 9: "nt, two 4-B stores per lane",
         10: "nt records + nt ring (two stores)", 11: "2 store instructions (wide)",
         12: "4 store instructions", 13: "8 store instructions", 14: "16 store instructions",
         15: "records of 4 tiles by every 4th wave", 16: "records of 16 tiles by every 16th",
         17: "nt 4 B x 64 at end (a 4-B record)", 18: "nt 2 B x 64 at end (a 2-B record)",
         19: "nt low 4 B of each 8-B record", 20: "19 + high 4 B for every 4th lane",
         21: "64-B slot per tile, 16 x 4 B", 22: "64-B slot per tile, 4 x 16 B",
         "x": "expansion pass alone (slot -> 64 records)", "21x": "mode 21 + expansion pass"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--modes", default="", help="comma list of modes (default: all)")
    ap.add_argument("--variants", default="",
                    help="mode:tiles_per_wave:lds_bytes beside the modes at 1:8960")
    args = ap.parse_args()
    so = os.path.join(ROOT, "tools", "probes", "librec_store.so")
    src = os.path.join(ROOT, "tools", "probes", "rec_store.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                        "-o", so, src], check=True)
    lib = ctypes.CDLL(so)
    lib.rec_probe.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_void_p]
    zp = importlib.import_module("zero-packet_amd")
    d = torch.device("cuda:0")
    n = args.packets or {"c5": 1 << 25}.get(args.config, 1 << 24)
    a, o, l_ = zp.batch.generate(args.config, n, device=d)
    recs, ext = zp.batch.alloc_outputs(n, d)
    ring = torch.empty(64 * 4096 * 8, dtype=torch.uint8, device=d)
    wide = torch.empty(((n + 63) // 64) * 16 * 512, dtype=torch.uint8, device=d)
    sink = torch.zeros(1, dtype=torch.int32, device=d)
    scratch = a.clone()                                   # mode 7 writes into it
    s = torch.cuda.current_stream()
    nb = a.numel() // 16 * 16
    nbytes = int(l_.to(torch.int64).sum())

    lib.expand_probe.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]

    def run(m):
        if m in ("x", "21x"):
            if m == "21x":
                run(21)
            lib.expand_probe(recs.data_ptr(), n, ctypes.c_void_p(s.cuda_stream))
            return
        if m == "parse":
            zp.batch.parse_batch(a, o, l_, recs, ext, check=False)
            return
        mode, k, lds = (m, 1, 8960) if isinstance(m, int) else m
        src = scratch if mode == 7 else a
        lib.rec_probe(src.data_ptr(), nb, n, o.data_ptr(), l_.data_ptr(), recs.data_ptr(),
                      ring.data_ptr(), wide.data_ptr(), mode, k, lds, sink.data_ptr(),
                      ctypes.c_void_p(s.cuda_stream))
    extra = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",") if v]
    modes = [x if x in ("x", "21x") else int(x) for x in args.modes.split(",") if x] or list(MODES)
    if 0 not in modes:
        modes = [0] + modes
    keys = ["parse"] + modes + extra
    for k in keys:
        run(k)
    ms = {k: [] for k in keys}
    for _ in range(args.rounds):
        for k in keys:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(3)]
            for e0, e1 in ev:
                e0.record(s)
                run(k)
                e1.record(s)
            torch.cuda.synchronize()
            ms[k] += [e0.elapsed_time(e1) for e0, e1 in ev]
    base = float(np.median(ms[0]))
    print(f"{args.config}: {n} frames, {nbytes / 1e9:.2f} GB; medians over {3 * args.rounds} launches")
    for k in keys:
        med = float(np.median(ms[k]))
        name = "parse (zp_parse_kernel)" if k == "parse" else \
            f"mode {k}: {MODES[k]}" if isinstance(k, (int, str)) else \
            f"mode {k[0]}, {k[1]} tiles/wave, {k[2]} B LDS"
        print(f"  {name:42s} {med:8.4f} ms  {nbytes / (med * 1e-3) / 1e9:7.1f} GB/s  "
              f"+{med - base:7.4f} ms over no stores", flush=True)


if __name__ == "__main__":
    main()
