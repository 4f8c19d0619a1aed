"""Fused parse + columns (zp_parse_batch_columns_device) vs parse then columns
(zp_parse_batch_device + zp_extract_columns_device on the same stream), by
requested column bytes per frame, interleaved in one process (round 4,
DESIGN.md §11). Usage: python tools/cols_policy.py [--configs c3,c5]"""
import argparse
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SETS = {
    "ports+proto(5B)": ["protocol", "src_port", "dest_port"],
    "5tuple(37B)": ["src_addr", "dest_addr", "protocol", "src_port", "dest_port"],
    "5tuple+l4(47B)": ["src_addr", "dest_addr", "protocol", "src_port", "dest_port", "tcp_seq",
                       "tcp_ack", "tcp_flags", "l4_proto"],
    "l3l4(55B)": ["src_addr", "dest_addr", "protocol", "src_port", "dest_port", "tcp_seq",
                  "tcp_ack", "tcp_flags", "l4_proto", "ttl", "tos", "ip_id", "ip_len",
                  "ip_version"],
    "macs+l3l4(67B)": ["dest_mac", "src_mac", "src_addr", "dest_addr", "protocol", "src_port",
                       "dest_port", "tcp_seq", "tcp_ack", "tcp_flags", "l4_proto", "ttl", "tos",
                       "ip_id", "ip_len", "ip_version"],
    "all(73B)": None,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c5")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lib", default="", help="comma list of tools/variants/<name> builds whose "
                    "fused kernel is timed too (fused_<name>)")
    a = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    C = zp.columns
    lib = zp._lib.hip()
    vlibs = []
    for v in [x for x in a.lib.split(",") if x]:
        l = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", v, "libzp_hip.so"))
        l.zp_parse_batch_columns_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
            [ctypes.c_void_p] * 4
        vlibs.append((v, l))
    d = torch.device("cuda:0")
    s = torch.cuda.current_stream(d)
    for cfg in a.configs.split(","):
        n = {"c3": 1 << 24, "c4": 1 << 24, "c5": 1 << 25}[cfg]
        arena, offs, lens = zp.batch.generate(cfg, n, device=d)
        rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
        ext = torch.empty((2, n, 16), dtype=torch.uint8, device=d)
        for label, names in SETS.items():
            names = names or C.NAMES
            out = {k: C._alloc(k, n, d) for k in names}
            ptrs = (ctypes.c_void_p * len(C.NAMES))()
            for k in names:
                ptrs[C.INDEX[k]] = out[k].data_ptr()
            width = sum(C.width(k) for k in names)
            def fused():
                return lib.zp_parse_batch_columns_device(
                    arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, rec.data_ptr(),
                    ext.data_ptr(), ptrs, ctypes.c_void_p(s.cuda_stream))

            def split():
                rc = lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                               n, rec.data_ptr(), ext.data_ptr(),
                                               ctypes.c_void_p(s.cuda_stream))
                return rc or lib.zp_extract_columns_device(
                    arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), rec.data_ptr(), n, ptrs,
                    ctypes.c_void_p(s.cuda_stream))
            variants = [("fused", fused), ("split", split),
                        ("auto", lambda: C.parse_with_columns(arena, offs, lens, names=names,
                                                              records=rec, ext=ext, out=out,
                                                              check=False) and 0)]
            for v, l in vlibs:
                variants.append((f"fused_{v}", lambda l=l: l.zp_parse_batch_columns_device(
                    arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, rec.data_ptr(),
                    ext.data_ptr(), ptrs, ctypes.c_void_p(s.cuda_stream))))
            res = {v: [] for v, _ in variants}
            ref = None
            for r in range(a.rounds):
                for v, fn in variants:
                    assert not fn()
                    ev = [(torch.cuda.Event(enable_timing=True),
                           torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
                    for x, y in ev:
                        x.record(s); fn(); y.record(s)
                    torch.cuda.synchronize()
                    res[v] += [x.elapsed_time(y) for x, y in ev]
                    got = torch.cat([out[k].view(-1).view(torch.uint8) for k in names] + [rec.view(-1)])
                    if ref is None:
                        ref = got.clone()
                    elif not torch.equal(ref, got):
                        print(f"  !! {cfg} {label} {v}: results differ", flush=True)
            f, sp = (float(np.median(res[v])) for v in ("fused", "split"))
            extra = "".join(f"  {v} {float(np.median(res[v])):7.3f} ms ({float(np.median(res[v])) / sp:5.3f})"
                            for v, _ in variants[2:])
            extra += f"  [auto chose {C.auto_choice(arena, n, names)}]"
            print(f"{cfg} {label:18s} {width:3d} B/frame: fused {f:7.3f} ms  split {sp:7.3f} ms  "
                  f"fused/split {f / sp:5.3f}{extra}", flush=True)
            del out
        del arena, offs, lens, rec, ext
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
