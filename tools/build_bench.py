"""Batched PacketBuilder throughput + full-size build -> parse round trip.

    python tools/build_bench.py [--frames 4194304] [--config c3]

Frames of a generated batch are rebuilt in place by chains
ethernet -> ipv4 -> tcp|udp|icmpv4 (payload None: the bytes already in the
buffer are the payload, so the chain writes headers and checksums only) with
fresh random header fields; every rebuilt frame must then parse Ok through
the parse kernel (the checksums the builder wrote verify). Algorithmic bytes
per frame: the frame is read once (the L4 checksum covers it) and the header
bytes are written.
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ucmem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-base", action="store_true",
                    help="time only the first of --variants (PMC passes of a variant)")
    ap.add_argument("--rounds", type=int, default=1,
                    help="interleaved timing rounds over the libs (median of the round medians)")
    ap.add_argument("--variants", default="", help="tools/variants/libzb_<name>.so builds to A/B")
    ap.add_argument("--payload", type=int, default=0,
                    help="copy min(P, room) payload bytes from the data blob into each frame "
                         "(set_payload(Some(..))); each frame from its own blob range")
    ap.add_argument("--shared-blob", action="store_true",
                    help="every frame copies from blob offset 0 (L2-resident source; round 2)")
    ap.add_argument("--oracle-sample", type=int, default=2000,
                    help="frames compared byte for byte with the oracle builder")
    ap.add_argument("--arena-mem", default="default", choices=["default", "uncached"],
                    help="the frames' buffer in ordinary or uncached device memory (round 5: "
                         "the header write-back's cost by memory kind)")
    ap.add_argument("--stamps", action="store_true",
                    help="phase shares from tools/variants/libzb_stamps.so (ZB_STAMPS build)")
    args = ap.parse_args()
    if args.stamps and "stamps" not in args.variants.split(","):
        args.variants = ",".join([v for v in args.variants.split(",") if v] + ["stamps"])
    zp = importlib.import_module("zero-packet_amd")
    B = zp.builder
    d = torch.device("cuda:0")
    n = args.frames
    arena, offs, lens = zp.batch.generate("c3", n, device=d)
    if args.arena_mem == "uncached":
        ua = ucmem.empty(arena.numel(), device=d)
        ua.copy_(arena)
        arena = ua
        print("arena in uncached device memory", flush=True)
    ln = lens.cpu().numpy().astype(np.int64)
    rng = np.random.default_rng(7)
    ops = np.zeros(3 * n, B.OP_DTYPE)
    eth, ip, l4 = ops[0::3], ops[1::3], ops[2::3]
    eth["kind"] = B.ETHERNET
    eth["src"][:, :6] = rng.integers(0, 256, (n, 6), dtype=np.uint8)
    eth["dst"][:, :6] = rng.integers(0, 256, (n, 6), dtype=np.uint8)
    eth["h"][:, 0] = 0x0800
    ip["kind"] = B.IPV4
    ip["b"][:, 0] = 4
    ip["b"][:, 1] = 5
    ip["b"][:, 5] = 64
    ip["h"][:, 0] = (ln - 14).astype(np.uint16)
    ip["h"][:, 1] = rng.integers(0, 65536, n, dtype=np.uint16)
    ip["src"][:, :4] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    ip["dst"][:, :4] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    which = rng.integers(0, 3, n)
    kinds = np.array([B.TCP, B.UDP, B.ICMPV4])[which]
    protos = np.array([6, 17, 1])[which]
    ip["b"][:, 6] = protos
    l4["kind"] = kinds
    l4["src"][:, :4] = ip["src"][:, :4]
    l4["dst"][:, :4] = ip["dst"][:, :4]
    l4["h"][:, 0] = rng.integers(1, 65536, n, dtype=np.uint16)
    l4["h"][:, 1] = rng.integers(1, 65536, n, dtype=np.uint16)
    tcp = which == 0
    l4["w"][tcp, 0] = rng.integers(0, 1 << 32, int(tcp.sum()), dtype=np.uint32)
    l4["b"][tcp, 0] = 5
    l4["b"][tcp, 2] = 0x18
    l4["h"][tcp, 2] = 65535
    udp = which == 1
    l4["h"][udp, 2] = (ln[udp] - 34).astype(np.uint16)
    icmp = which == 2
    l4["b"][icmp, 0] = 8
    l4["b"][icmp, 1] = 0
    l4["h"][icmp, 0] = 0
    l4["h"][icmp, 1] = 0
    for o in (eth, ip, l4):
        o["data_len"] = B.NO_DATA
    pay = np.zeros(n, np.int64)
    blob_bytes = 16
    if args.payload:
        start = np.where(tcp, 20, 8)
        pay = np.minimum(args.payload, ln - 34 - start)
        l4["data_len"] = pay.astype(np.uint32)
        if args.shared_blob:
            l4["data_off"] = 0
            blob_bytes = max(16, args.payload)
        else:                               # frame i copies blob[sum(pay[:i]) ...]: from HBM
            l4["data_off"] = (np.cumsum(pay) - pay).astype(np.uint32)
            blob_bytes = max(16, int(pay.sum()))
            assert blob_bytes < (1 << 32)
    t_ops = torch.from_numpy(ops.view(np.uint8)).to(d)
    t_start = torch.arange(0, 3 * n + 1, 3, dtype=torch.int32, device=d)
    t_data = torch.randint(0, 256, (blob_bytes,), dtype=torch.uint8, device=d)
    res = torch.zeros((n, 8), dtype=torch.uint8, device=d)
    import ctypes
    libs = [("base", zp._lib.hip())]
    for v in [x for x in args.variants.split(",") if x]:
        l_ = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"libzb_{v}.so"))
        l_.zp_build_batch_device.restype = ctypes.c_int
        l_.zp_build_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
            [ctypes.c_void_p] * 5
        libs.append((v, l_))
    if args.no_base:
        libs = libs[1:2]
    # The write floor at HBM granularity: every frame's written range
    # [A, A + headers + payload) rounded out to whole 64-B sectors (the
    # granularity of WRITE_SIZE / TCC_EA0_WRREQ), sectors shared by
    # neighbouring frames counted once.
    hlen = 14 + 20 + np.where(tcp, 20, 8)
    a0 = offs.cpu().numpy().astype(np.int64) + int(arena.data_ptr() % 64)
    s0, s1 = a0 // 64, (a0 + hlen + pay - 1) // 64
    order = np.argsort(s0)
    s0, s1 = s0[order], s1[order]
    prev_end = np.concatenate([[-1], np.maximum.accumulate(s1)[:-1]])
    sector_bytes = int(np.maximum(s1 - np.maximum(s0, prev_end + 1) + 1, 0).sum()) * 64
    exact_write = int(hlen.sum() + pay.sum())
    print(f"write floor: {exact_write / 1e9:.3f} GB of header/payload bytes, "
          f"{sector_bytes / 1e9:.3f} GB in whole 64-B sectors "
          f"({sector_bytes / exact_write:.2f} x)", flush=True)
    s = torch.cuda.current_stream(d)
    if args.stamps:
        # phase shares of the lane kernel from the ZB_STAMPS build
        # (tools/build_variants.sh "b-stamps:-DZB_STAMPS")
        l_ = dict(libs)["stamps"]
        l_.zb_stamps_set.argtypes = [ctypes.c_void_p]
        nw = (n + 63) // 64
        sb = torch.zeros(nw * 8, dtype=torch.int64, device=d)
        snap = arena.clone()
        for k in range(3):
            arena.copy_(snap)
            l_.zb_stamps_set(ctypes.c_void_p(sb.data_ptr()) if k == 2 else None)
            l_.zp_build_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                     t_ops.data_ptr(), t_start.data_ptr(), t_data.data_ptr(),
                                     res.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
        l_.zb_stamps_set(None)
        t = sb.view(nw, 8).cpu().numpy()[:, :6].astype(np.int64) * 10       # ns
        dd = np.diff(t, axis=1)
        life = t[:, 5] - t[:, 0]
        span = t[:, 5].max() - t[:, 0].min()
        names = ["stream", "chain", "copy pass 1", "copy pass 2", "write-back"]
        print(f"stamps P={args.payload}: span {span / 1e6:.3f} ms, wave life {life.mean() / 1e3:.1f} us, "
              f"resident {life.sum() / span:.0f}; " +
              "  ".join(f"{nm} {dd[:, i].mean() / 1e3:.2f}us ({100 * dd[:, i].mean() / life.mean():.0f}%)"
                        for i, nm in enumerate(names)), flush=True)
        arena.copy_(snap)
        del snap, sb
        libs = [x for x in libs if x[0] != "stamps"]
    snapshot = arena.clone()
    blob_read = int(pay.sum()) if args.payload and not args.shared_blob else 0
    errs = 0
    ref = None
    def launcher(lib):
        def launch():
            zp._lib.check(lib.zp_build_batch_device(arena.data_ptr(), offs.data_ptr(),
                                                    lens.data_ptr(), n, t_ops.data_ptr(),
                                                    t_start.data_ptr(), t_data.data_ptr(),
                                                    res.data_ptr(), s.cuda_stream),
                          "zp_build_batch_device")
        return launch
    for name, lib in libs:
        launch = launcher(lib)
        arena.copy_(snapshot)
        launch()
        torch.cuda.synchronize()
        if ref is None:
            ref = arena.clone()
        elif not torch.equal(ref, arena):
            print(f"  !! {name}: built bytes differ from base", flush=True)
        errs += int((res[:, 4] != 0).sum())
    times = {name: [] for name, _ in libs}
    for _ in range(args.rounds):
        for name, lib in libs:
            launch = launcher(lib)
            launch()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for a, b in ev:
                a.record(s); launch(); b.record(s)
            torch.cuda.synchronize()
            times[name].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
    for name, _ in libs:
        ms = float(np.median(times[name]))
        nbytes = int(ln.sum())
        hdr = exact_write
        opb = int(t_ops.numel() + t_start.numel() * 4)
        alg = nbytes + hdr + blob_read
        blob = " shared-blob" if args.shared_blob else ""
        print(f"build c3 x {n}{f' payload {args.payload}{blob}' if args.payload else ''} [{name}]: "
              f"{ms:.3f} ms  {n / ms / 1e3:.0f} Mpkt/s  "
              f"{alg / ms / 1e6:.0f} GB/s = {alg / ms / 1e6 / 8000:.3f} of 8 TB/s (frame read "
              f"{nbytes / 1e9:.2f} + header/payload write {hdr / 1e9:.2f} + blob read "
              f"{blob_read / 1e9:.2f} GB; {(alg + opb) / ms / 1e6:.0f} GB/s with the op reads)  "
              f"errors {errs}", flush=True)
    if args.oracle_sample:
        # a sample of the built frames against the oracle builder, from the
        # same prior bytes, ops and blob ranges
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle as orc
        idx = np.sort(rng.choice(n, min(n, args.oracle_sample), replace=False))
        o_h, l_h = offs.cpu().numpy()[idx], ln[idx]
        snap = snapshot.cpu().numpy()
        blob = t_data.cpu().numpy()
        a_s = np.zeros(int(l_h.sum()) + 64, np.uint8)
        so = np.concatenate([[0], np.cumsum(l_h)[:-1]]).astype(np.uint64)
        for k, (o, l_) in enumerate(zip(o_h, l_h)):
            a_s[int(so[k]):int(so[k]) + int(l_)] = snap[int(o):int(o) + int(l_)]
        ops_s = np.stack([eth[idx], ip[idx], l4[idx]], axis=1).reshape(-1).copy()
        res_s = orc.build_batch(a_s, so, l_h.astype(np.uint32), ops_s,
                                np.arange(0, 3 * len(idx) + 1, 3, dtype=np.uint32), blob)
        got = ref.cpu().numpy()             # the first launch from the snapshot
        bad = sum(1 for k, (o, l_) in enumerate(zip(o_h, l_h))
                  if got[int(o):int(o) + int(l_)].tobytes() !=
                  a_s[int(so[k]):int(so[k]) + int(l_)].tobytes())
        print(f"oracle sample: {len(idx) - bad}/{len(idx)} frames byte-identical, "
              f"{int((res_s[:, 4] != 0).sum())} oracle errors", flush=True)
        assert bad == 0
    recs, _ = zp.batch.parse_batch(arena, offs, lens)
    torch.cuda.synchronize()
    bad = int((zp.batch.record_err(recs) != 0).sum())
    print(f"round trip: {n - bad}/{n} rebuilt frames parse Ok", flush=True)
    assert errs == 0 and bad == 0


if __name__ == "__main__":
    main()
