"""PCIe-inclusive rate of the host-ring pipeline (zp_ring) vs the synchronous
host batch path (zp_parse_batch_host), on the same pinned c3 frames.

    python tools/ring_bench.py [--frames 2097152] [--slots 4] [--slot-mb 64]

Ring "prefilled": every slot's pinned arena already holds its frames (the NIC
DMA model: frames land in the pinned ring, nothing is copied by the host);
the timed loop only cycles submit -> wait -> release. Ring "memcpy": the
producer also copies each slot's frames from a host pool (a software ring).
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 21)
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--slot-mb", type=int, default=64)
    ap.add_argument("--passes", type=int, default=3)
    args = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    arena, offs, lens = zp.batch.generate_host("c3", args.frames)
    total = int(lens.sum(dtype=np.uint64))
    slot_bytes = args.slot_mb << 20
    ring = zp.ring.Ring(0, args.slots, slot_bytes)
    # cut the batch into slot-sized pieces once
    cuts, i = [], 0
    while i < len(offs):
        lo, j = int(offs[i]), i
        while j < len(offs) and int(offs[j] + lens[j]) - lo <= slot_bytes and j - i < ring.slot_frames:
            j += 1
        cuts.append((i, j, lo, int(offs[j - 1] + lens[j - 1])))
        i = j
    # prefilled: slot k holds piece k (ring order), resubmitted as-is each cycle
    nslots = args.slots
    slots = []
    for k in range(nslots):
        s = ring.acquire()
        slots.append(s)
    for k, s in enumerate(slots):
        i, j, lo, hi = cuts[k % len(cuts)]
        s.arena[:hi - lo] = arena[lo:hi]
        s.offs[:j - i] = offs[i:j] - lo
        s.lens[:j - i] = lens[i:j]
    bytes_per_slot = [int(lens[cuts[k % len(cuts)][0]:cuts[k % len(cuts)][1]].sum()) for k in range(nslots)]
    frames_per_slot = [cuts[k % len(cuts)][1] - cuts[k % len(cuts)][0] for k in range(nslots)]
    cycles = max(args.passes * len(cuts), 2 * nslots)
    # warm: one submit/wait of each slot
    for k, s in enumerate(slots):
        ring.submit(s, frames_per_slot[k])
    for _ in range(nslots):
        ring.release(ring.wait())
    t0 = time.perf_counter()
    nbytes = nfr = 0
    inflight = 0
    for c in range(cycles):
        k = c % nslots
        if inflight == nslots:
            ring.release(ring.wait())
            inflight -= 1
        s = ring.acquire()
        assert s.id == slots[k].id
        ring.submit(s, frames_per_slot[k])
        inflight += 1
        nbytes += bytes_per_slot[k]
        nfr += frames_per_slot[k]
    while inflight:
        ring.release(ring.wait())
        inflight -= 1
    dt = time.perf_counter() - t0
    print(f"ring prefilled  slots={nslots} x {args.slot_mb} MiB: {nbytes / dt / 1e9:6.2f} GB/s "
          f"{nfr / dt / 1e6:7.1f} Mpkt/s ({cycles} slot cycles)", flush=True)
    # memcpy producer: host copies each piece into the slot
    for p in range(1):
        t0 = time.perf_counter()
        out, _ = ring.parse(arena, offs, lens)
        dt = time.perf_counter() - t0
    print(f"ring memcpy     slots={nslots} x {args.slot_mb} MiB: {total / dt / 1e9:6.2f} GB/s "
          f"{len(offs) / dt / 1e6:7.1f} Mpkt/s", flush=True)
    ring.close()
    # synchronous host batch path on pinned memory, same frames
    host = torch.from_numpy(arena).pin_memory()
    recs = torch.empty((len(offs), 8), dtype=torch.uint8).pin_memory()
    lib = zp._lib.hip()
    ctx = lib.zp_ctx_create(0, 256 << 20)
    a = (ctx, host.data_ptr(), len(arena), offs.ctypes.data, lens.ctypes.data, len(offs),
         recs.data_ptr(), None)
    zp._lib.check(lib.zp_parse_batch_host(*a), "host")
    t0 = time.perf_counter()
    for _ in range(args.passes):
        zp._lib.check(lib.zp_parse_batch_host(*a), "host")
    dt = (time.perf_counter() - t0) / args.passes
    print(f"zp_parse_batch_host (2 x 256 MiB): {total / dt / 1e9:6.2f} GB/s "
          f"{len(offs) / dt / 1e6:7.1f} Mpkt/s", flush=True)
    lib.zp_ctx_destroy(ctx)
    assert (zp.records.rec_err(out) == 0).all()


if __name__ == "__main__":
    main()
