"""Does the placement of the arena change the c3 parse time?

One process, one c3 batch; the same bytes are copied into differently placed
allocations (fresh torch block, behind a large dummy block, at offsets inside
a larger block) and zp_parse_kernel is timed on each with HIP events.
Usage: python tools/alloc_probe.py [--steps K] [--config c3]
"""
import argparse
import ctypes
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
zp = importlib.import_module("zero-packet_amd")


def timeit(arena, offs, lens, records, inner, steps, base=None):
    s = torch.cuda.current_stream()
    for _ in range(3):
        zp.batch.parse_batch(arena, offs, lens, records, inner, check=False)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, b in ev:
        a.record(s)
        zp.batch.parse_batch(arena, offs, lens, records, inner, check=False)
        b.record(s)
    torch.cuda.synchronize()
    assert int((zp.batch.record_err(records) != 0).sum().item()) == 0
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return {"mean": round(sum(t) / len(t), 4), "min": round(t[0], 4),
            "med": round(t[len(t) // 2], 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--copies", type=int, default=6)
    ap.add_argument("--variants", default="", help="comma list of tools/variants/libzp_<name>.so")
    ap.add_argument("--no-check", action="store_true", help="time variants whose records differ (ablations)")
    ap.add_argument("--parse-only", action="store_true", help="no membw kernels (PMC runs)")
    ap.add_argument("--colocate", action="store_true",
                    help="arena and records in one allocation (several gaps and placements)")
    ap.add_argument("--move-records", action="store_true",
                    help="keep the arena, move the records buffer (and variants) instead")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    arena, offs, lens = zp.batch.generate(a.config, a.packets, device=dev)
    n = a.packets
    # one records allocation for the base and the variants (room for 16-B
    # records): the records' placement matters too
    vrec = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    records = vrec.view(-1)[:n * 8].view(n, 8)
    inner = torch.empty((2, n, 16), dtype=torch.uint8, device=dev)
    nb = arena.numel()
    mb = ctypes.CDLL(os.path.join(ROOT, "tools", "libmembw.so"))
    mb.membw_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    mb.membw_region2.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    variants = {}
    for v in filter(None, a.variants.split(",")):
        vl = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzp_{v}.so"))
        vl.zp_parse_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
            [ctypes.c_void_p] * 3
        variants[v] = vl
    out = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    rout = torch.zeros(nb // 1024 * 64 + 4096, dtype=torch.int32, device=dev)

    def bw(fn):
        s = torch.cuda.current_stream()
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.steps)]
        for x, y in ev:
            x.record(s)
            fn()
            y.record(s)
        torch.cuda.synchronize()
        t = sorted(x.elapsed_time(y) for x, y in ev)
        return round(t[len(t) // 2], 4)

    def probe(name, buf):
        r = timeit(buf, offs, lens, records, inner, a.steps)
        r["ptr"] = hex(buf.data_ptr())
        if variants:
            ref = records.clone()
            s = torch.cuda.current_stream()
            for vname, vl in variants.items():
                launch = lambda: vl.zp_parse_batch_device(buf.data_ptr(), offs.data_ptr(),
                                                          lens.data_ptr(), n, vrec.data_ptr(),
                                                          inner.data_ptr(),
                                                          ctypes.c_void_p(s.cuda_stream))
                vrec.zero_()
                launch()
                torch.cuda.synchronize()
                same = bool(torch.equal(vrec.view(-1)[:n * 8].view(n, 8), ref))
                r[vname] = bw(launch) if same or a.no_check else "RECORDS DIFFER"
            r["base_again"] = timeit(buf, offs, lens, records, inner, a.steps)["med"]
        if a.parse_only:
            print(json.dumps({name: r}), flush=True)
            return
        r["grid_ms"] = bw(lambda: mb.membw_read(buf.data_ptr(), nb, out.data_ptr(), 8192, 1, None))
        reg = 48 << 10
        r["region48_ms"] = bw(lambda: mb.membw_region2(buf.data_ptr(), nb // reg * reg,
                                                       rout.data_ptr(), reg, 0, None))
        print(json.dumps({name: r}), flush=True)

    if a.colocate:
        # arena and records in ONE allocation: records right after the arena
        # (2 MiB aligned, plus a gap), or right before it
        rb = n * 8
        al = 2 << 20
        for k in range(a.copies):
            for gap, before in ((0, False), (64 << 10, False), (al, False), (0, True)):
                body = (nb + al - 1) // al * al
                blk = torch.empty(body + gap + rb + al, dtype=torch.uint8, device=dev)
                if before:
                    rec2 = blk[:rb].view(n, 8)
                    a0 = (rb + gap + al - 1) // al * al
                    ar2 = blk[a0:a0 + nb]
                else:
                    ar2 = blk[:nb]
                    rec2 = blk[body + gap:body + gap + rb].view(n, 8)
                ar2.copy_(arena)
                r = timeit(ar2, offs, lens, rec2, inner, a.steps)
                sep = timeit(ar2, offs, lens, records, inner, a.steps)
                r["separate_records_med"] = sep["med"]
                r["arena_ptr"] = hex(ar2.data_ptr())
                r["rec_ptr"] = hex(rec2.data_ptr())
                print(json.dumps({f"copy{k} gap={gap >> 10}KiB "
                                  f"{'before' if before else 'after'}": r}), flush=True)
                del blk, ar2, rec2
            hold = torch.empty((k + 1) * (193 << 20), dtype=torch.uint8, device=dev)
            torch.cuda.empty_cache()
        return
    if a.move_records:
        hold = []
        for k in range(a.copies):
            hold.append(torch.empty(97 << 20, dtype=torch.uint8, device=dev))   # shift the next block
            rec2 = torch.empty((n, 8), dtype=torch.uint8, device=dev)
            r = timeit(arena, offs, lens, rec2, inner, a.steps)
            r["rec_ptr"] = hex(rec2.data_ptr())
            s = torch.cuda.current_stream()
            for vname, vl in variants.items():
                r[vname] = bw(lambda: vl.zp_parse_batch_device(
                    arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, rec2.data_ptr(),
                    inner.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
            print(json.dumps({f"records{k}": r}), flush=True)
            hold.append(rec2)
        return
    probe("base", arena)
    live = []
    for k in range(a.copies):
        blk = torch.empty(nb, dtype=torch.uint8, device=dev)
        blk.copy_(arena)
        live.append(blk)
        probe(f"copy{k}", blk)
    del live
    torch.cuda.empty_cache()
    for k in range(2):
        blk = torch.empty(nb, dtype=torch.uint8, device=dev)
        blk.copy_(arena)
        probe(f"realloc{k}", blk)
        del blk
        torch.cuda.empty_cache()
    probe("base_again", arena)

    # Raw HIP allocations: default and physically contiguous (hipDeviceMallocContiguous).
    hip = ctypes.CDLL("libamdhip64.so")
    lib = zp._lib.hip()
    for flags, label in ((4, "contig"), (0, "hipmalloc"), (4, "contig"), (0, "hipmalloc")):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nb), flags)
        if rc != 0:
            print(json.dumps({label: f"hipExtMallocWithFlags rc={rc}"}), flush=True)
            continue
        assert hip.hipMemcpy(p, ctypes.c_void_p(arena.data_ptr()), ctypes.c_size_t(nb), 3) == 0
        s = torch.cuda.current_stream()
        launch = lambda: lib.zp_parse_batch_device(p, offs.data_ptr(), lens.data_ptr(), n,
                                                   records.data_ptr(), inner.data_ptr(),
                                                   ctypes.c_void_p(s.cuda_stream))
        for _ in range(3):
            launch()
        r = {"parse_med": bw(launch), "ptr": hex(p.value)}
        assert int((zp.batch.record_err(records) != 0).sum().item()) == 0
        if not a.parse_only:
            r["region48_ms"] = bw(lambda: mb.membw_region2(p, nb // (48 << 10) * (48 << 10),
                                                           rout.data_ptr(), 48 << 10, 0, None))
        print(json.dumps({label: r}), flush=True)
        hip.hipFree(p)


if __name__ == "__main__":
    main()
