"""Kernel A/B harness (one process, interleaved rounds; guide §5.4 rule 24).

    python tools/kbench.py [--configs c3,c2,c4,c5] [--variants base,...] [--membw]

Variants are extra builds of zp_parse.hip (tools/build_variants.sh) exposing
the same C ABI; each is timed with HIP events on the same resident batch.
"""
import argparse
import ctypes
import glob
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_launches(fn, reps):
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
    ap.add_argument("--configs", default="c3,c2,c4,c5")
    ap.add_argument("--variants", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--membw", action="store_true")
    ap.add_argument("--tiles", action="store_true",
                    help="read ceiling of the parse kernel's tile pattern (tools/membw.hip)")
    ap.add_argument("--no-base", action="store_true", help="time only --variants (PMC runs)")
    ap.add_argument("--columns", action="store_true", help="also time zp_extract_columns_device")
    ap.add_argument("--col-variants", default="",
                    help="A/B builds of zp_fields.hip (tools/variants/libzc_<name>.so), all columns")
    ap.add_argument("--c2cold", action="store_true",
                    help="c2 (1M x 64 B = 64 MiB, fits the 256 MiB MALL) warm vs cold: "
                         "8 rotating copies (512 MiB) so every launch reads from HBM")
    args = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    dev = torch.device("cuda:0")
    libs = {} if args.no_base else {"base": zp._lib.hip()}
    slot_mode = {}
    for v in [x for x in args.variants.split(",") if x]:
        if "@" in v:                               # "<lib>@<mode>": zp_set_record_slots(mode)
            base_v, m = v.split("@")
            l = libs["base"] if base_v == "base" else ctypes.CDLL(
                os.path.join(ROOT, "tools", "variants", f"libzp_{base_v}.so"))
            # (every entry point called with pointers needs its argtypes: a
            # ctypes default int argument truncates a pointer to 32 bits)
            l.zp_parse_batch_device.restype = ctypes.c_int
            l.zp_parse_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
                [ctypes.c_void_p] * 3
            l.zp_set_record_slots.restype = ctypes.c_int
            l.zp_set_record_slots.argtypes = [ctypes.c_int]
            libs[v] = l
            slot_mode[v] = int(m)
            continue
        so = os.path.join(ROOT, "tools", "variants", f"libzp_{v}.so")
        l = ctypes.CDLL(so)
        l.zp_parse_batch_device.restype = ctypes.c_int
        l.zp_parse_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
            [ctypes.c_void_p] * 3
        libs[v] = l
    try:
        rb = libs.get("base", zp._lib.hip())
        rb.zp_debug_resident_blocks.restype = ctypes.c_uint64
        print(f"resident blocks (persistent grid): {rb.zp_debug_resident_blocks()}", flush=True)
    except AttributeError:
        pass
    sizes = {"c1": 1 << 20, "c2": 1 << 20, "c3": 1 << 24, "c4": 1 << 24, "c5": 1 << 25,
             "c6": 1 << 24}
    if args.membw:
        mb = ctypes.CDLL(os.path.join(ROOT, "tools", "libmembw.so"))
        mb.membw_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        buf = torch.randint(0, 255, (13 << 30,), dtype=torch.uint8, device=dev)
        out = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
        for blocks in (2048, 4096, 8192, 16384):
            for nt in (0, 1):
                ms = time_launches(lambda: mb.membw_read(buf.data_ptr(), buf.numel(),
                                                         out.data_ptr(), blocks, nt, None), 10)
                print(f"membw read 13 GiB blocks={blocks} nt={nt}: "
                      f"{buf.numel() / (np.median(ms) * 1e-3) / 1e9:.0f} GB/s "
                      f"(min {min(ms):.3f} ms)", flush=True)
        mb.membw_region.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        rout = torch.zeros((13 << 30) // 1024 * 64, dtype=torch.int32, device=dev)
        for region in (16 << 10, 48 << 10, 192 << 10):
            for g in (4, 8, 16):
                ms = time_launches(lambda: mb.membw_region(buf.data_ptr(), buf.numel(),
                                                           rout.data_ptr(), region, g, None), 10)
                nbytes = buf.numel() // region * region
                print(f"membw region={region >> 10}KiB G={g}: "
                      f"{nbytes / (np.median(ms) * 1e-3) / 1e9:.0f} GB/s", flush=True)
        mb.membw_region2.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        names = {0: "1 wave/WG, G8", 1: "4 waves/WG, G8", 2: "4 waves interleaved, G8",
                 3: "8 waves interleaved, G8", 4: "8 waves interleaved, G4",
                 5: "1 wave/WG, G16"}
        for region in (48 << 10, 96 << 10):
            for mode, label in names.items():
                ms = time_launches(lambda: mb.membw_region2(buf.data_ptr(), buf.numel(),
                                                            rout.data_ptr(), region, mode, None), 10)
                nbytes = buf.numel() // region * region
                print(f"membw region2={region >> 10}KiB {label}: "
                      f"{nbytes / (np.median(ms) * 1e-3) / 1e9:.0f} GB/s", flush=True)
        del buf, rout
        torch.cuda.empty_cache()
    if args.tiles:
        # The parse kernel's access pattern without its work (tools/membw.hip
        # read_tiles): one wave per tile-sized region, 1 KiB loads in groups
        # of 8, 8,960 B of LDS per wave, and a 1 KiB record store per wave.
        mb = ctypes.CDLL(os.path.join(ROOT, "tools", "libmembw.so"))
        mb.membw_tiles.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
                                   ctypes.c_void_p]
        buf = torch.randint(0, 255, (12 << 30,), dtype=torch.uint8, device=dev)
        out = torch.zeros((12 << 30) // 4096 * 64 * 4 + 64, dtype=torch.int32, device=dev)
        for label, region in (("c5 tile (64 x 354.3 B)", 22672), ("c4 tile (64 x 797 B)", 51008),
                              ("c3 tile (64 x 781.6 B)", 50016), ("16 KiB", 16384),
                              ("c2 tile (64 x 64 B)", 4096)):
            for rec in (0, 1, 2):                 # no records, 16-B, 8-B records
                ms = time_launches(lambda: mb.membw_tiles(buf.data_ptr(), buf.numel(),
                                                          out.data_ptr(), region, rec > 0,
                                                          8960 + (rec == 2), None), 10)
                nbytes = buf.numel() // region * region
                print(f"tiles {label:24s} records={(0, 16, 8)[rec]}B: {np.median(ms):.3f} ms "
                      f"{nbytes / (np.median(ms) * 1e-3) / 1e9:.0f} GB/s", flush=True)
        del out
        # the copy pattern (builder payload pass): read + write the same bytes
        mb.membw_copy_tiles.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_void_p]
        half = (6 << 30)
        dst = torch.empty(half, dtype=torch.uint8, device=dev)
        for label, region in (("c3 tile", 50016), ("c5 tile", 22672)):
            ms = time_launches(lambda: mb.membw_copy_tiles(buf.data_ptr(), dst.data_ptr(), half,
                                                           region, None), 10)
            nbytes = half // region * region
            print(f"copy tiles {label:16s}: {np.median(ms):.3f} ms read {nbytes / 1e9:.2f} GB + "
                  f"write {nbytes / 1e9:.2f} GB = {2 * nbytes / (np.median(ms) * 1e-3) / 1e9:.0f} GB/s",
                  flush=True)
        del buf, dst
        torch.cuda.empty_cache()
    if args.c2cold:
        n = 1 << 20
        copies = [zp.batch.generate("c2", n, device=dev) for _ in range(8)]
        rec = torch.empty((n, 8), dtype=torch.uint8, device=dev)
        nbytes = int(copies[0][2].to(torch.int64).sum())
        c2libs = libs or {"base": zp._lib.hip()}
        for label, order in (("warm (same copy)", [0] * 8), ("cold (8 rotating copies)",
                                                            list(range(8)))):
            ms = {k: [] for k in c2libs}
            for r in range(args.rounds):          # the libs interleaved by round
                for name, lib in c2libs.items():
                    s = torch.cuda.current_stream()
                    ev = [(torch.cuda.Event(enable_timing=True),
                           torch.cuda.Event(enable_timing=True)) for _ in order]
                    for (a, b), k in zip(ev, order):
                        ar, of, ln = copies[k]
                        a.record(s)
                        lib.zp_parse_batch_device(ar.data_ptr(), of.data_ptr(), ln.data_ptr(), n,
                                                  rec.data_ptr(), None, None)
                        b.record(s)
                    torch.cuda.synchronize()
                    ms[name] += [a.elapsed_time(b) for a, b in ev]
            for name in c2libs:
                med = float(np.median(ms[name]))
                print(f"c2 {label} {name:>10s}: {med * 1e3:8.1f} us  {nbytes / med / 1e6:7.0f} GB/s  "
                      f"{n / med / 1e3:8.0f} Mpkt/s", flush=True)
        del copies
        torch.cuda.empty_cache()
    for cfg in [c for c in args.configs.split(",") if c]:
        label = cfg
        cfg, _, every = cfg.partition("~")         # "c3~2": every 2nd frame (gaps between frames)
        cfg, _, nn = cfg.partition(":")            # "c3:1048576": another batch size
        n = int(nn) if nn else sizes[cfg]
        arena, offs, lens = zp.batch.generate(cfg, n, device=dev)
        if every:
            offs, lens = offs[::int(every)].contiguous(), lens[::int(every)].contiguous()
            n = offs.numel()
        cfg = label
        # 16 B per frame: room for variants built with the ABI v2/v3 record
        rec = torch.empty((n, 16), dtype=torch.uint8, device=dev)
        ext = torch.empty((2, n, 16), dtype=torch.uint8, device=dev)
        nbytes = int(lens.to(torch.int64).sum())
        ref = None
        res = {k: [] for k in libs}
        for r in range(args.rounds):
            for name, l in libs.items():
                fn = lambda l=l: l.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(),
                                                          lens.data_ptr(), n, rec.data_ptr(),
                                                          ext.data_ptr(), None)
                if hasattr(l, "zp_set_record_slots"):
                    l.zp_set_record_slots(slot_mode.get(name, 0))
                if r == 0:
                    rec.fill_(0xA5)            # a build that stores no records shows as a diff
                res[name] += time_launches(fn, args.reps)
                if r == 0:
                    if ref is None:
                        ref = rec.clone()
                    elif not torch.equal(ref, rec):
                        print(f"  !! {name}: records differ from base on {cfg}", flush=True)
        for name, ms in res.items():
            med = float(np.median(ms))
            print(f"{cfg} {name:>12}: {med:8.3f} ms  {nbytes / med / 1e6:7.0f} GB/s  "
                  f"{n / med / 1e3:8.0f} Mpkt/s  (min {min(ms):.3f})", flush=True)
        rec = rec.view(-1)[:n * zp.records.RECORD_BYTES].view(n, zp.records.RECORD_BYTES)
        if args.columns:
            zp.batch.parse_batch(arena, offs, lens, rec, ext, check=False)
            for label, names in (("all", zp.columns.NAMES),
                                 ("5tuple", ["src_addr", "dest_addr", "protocol", "src_port",
                                             "dest_port"])):
                out = zp.columns.extract(arena, offs, lens, rec, names=names)
                ms = time_launches(lambda: zp.columns.extract(arena, offs, lens, rec, names=names, check=False,
                                                              out=out), args.reps * args.rounds)
                med = float(np.median(ms))
                wbytes = n * sum(zp.columns.width(c) for c in names)
                # records + descriptors + one staged 128-B header window per frame
                rbytes = n * (16 + 12 + 128)
                print(f"{cfg} columns[{label}]: {med:8.3f} ms  write {wbytes / med / 1e6:6.0f} GB/s"
                      f"  (write+read {(wbytes + rbytes) / med / 1e6:6.0f} GB/s)  "
                      f"{n / med / 1e3:8.0f} Mpkt/s", flush=True)
                ms = time_launches(lambda: zp.columns.parse_with_columns(
                    arena, offs, lens, names=names, records=rec, ext=ext, out=out, check=False),
                    args.reps * args.rounds)
                med = float(np.median(ms))
                print(f"{cfg} fused parse+columns[{label}]: {med:8.3f} ms  "
                      f"{(nbytes + wbytes) / med / 1e6:6.0f} GB/s (frames + columns)  "
                      f"{n / med / 1e3:8.0f} Mpkt/s", flush=True)
                del out
        if args.col_variants:
            zp.batch.parse_batch(arena, offs, lens, rec, ext, check=False)
            out = zp.columns.extract(arena, offs, lens, rec)
            ptrs = (ctypes.c_void_p * len(zp.columns.NAMES))()
            for k, name in enumerate(zp.columns.NAMES):
                ptrs[zp.columns.INDEX[name]] = out[name].data_ptr()
            ref = {k: v.clone() for k, v in out.items()}
            clibs = [("base", zp._lib.hip())] + [
                (v, ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzc_{v}.so")))
                for v in args.col_variants.split(",") if v]
            res = {k: [] for k, _ in clibs}
            s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            for r in range(args.rounds):
                for name, l in clibs:
                    fn = lambda l=l: l.zp_extract_columns_device(
                        ctypes.c_void_p(arena.data_ptr()), ctypes.c_void_p(offs.data_ptr()),
                        ctypes.c_void_p(lens.data_ptr()), ctypes.c_void_p(rec.data_ptr()),
                        ctypes.c_uint64(n), ptrs, s)
                    res[name] += time_launches(fn, args.reps)
                    if r == 0 and any(not torch.equal(ref[k], out[k]) for k in ref):
                        print(f"  !! {name}: columns differ from base on {cfg}", flush=True)
            for name, ms in res.items():
                print(f"{cfg} columns[all] {name:>10}: {float(np.median(ms)):8.3f} ms", flush=True)
            del out, ref
        del arena, offs, lens, rec, ext
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
