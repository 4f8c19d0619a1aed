"""Benchmark: device-resident batched PacketParser::parse on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--packets P]

One step = one zp_parse_batch_device launch over the whole per-GPU batch
(inputs already resident in HBM). Default workload: BASELINE config 3 — 16M
IPv4 frames, TCP/UDP/ICMPv4, lengths U[64,1500] (~13.1 GB, far past the
256 MiB Infinity Cache, so every step streams from HBM). Multi-GPU: one
process per GPU, each parses its own 16M-frame shard (packets
rank*P .. rank*P+P-1; weak scaling, no data-path collective). Rank 0 prints
one JSON line.

`python bench.py --gpus N` with N > 1 and no launcher around it starts the N
ranks itself: the parent spawns `torch.distributed.run --nproc-per-node N`
on this same command line before it touches the GPU, and relays rank 0's
JSON line. Under a launcher, --gpus must equal WORLD_SIZE.

--config c5 without --packets is config 5 itself: the 256M-frame IMIX stream
split into N contiguous shards, rank r parsing the r-th (strong scaling; at
N = 1 the whole 95 GB batch on one GPU).

Reported next to the GPU number:
  roofline      algorithmic bytes (sum of frame lengths) / mean kernel time
                from HIP events on the launch stream, vs 8.0 TB/s HBM peak
  cpu_baseline  the CPU oracle (a C port of the reference; the Rust original
                cannot be built here) on a bounded sample of the same frames
                (rank 0 at N = 1 only)
  h2d_d2h_inclusive  host-pinned frames -> H2D -> parse -> D2H (PCIe) rate on
                a 2M-frame sample (zp_parse_batch_host), every rank at once,
                frames summed over ranks / the slowest rank; never `value`;
                rejected frames reported, not asserted
  roofline.placement  the placement classes of the bench's own buffers: a
                plain streaming read of the arena, the parse's tile pattern
                over it, and that pattern with the 8-B record stores into the
                bench's records buffer
  config5       BASELINE config 5 in the same ranks after the headline: the
                256M-frame IMIX stream (--c5-frames) cut into N contiguous
                shards (strong scaling), its own timed loop of --steps
                launches, per-rank shards / rejected frames / roofline
                fraction (--no-c5 skips it)
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident Mpkt/s + GB/s, PacketParser::parse, 64-1500B mix"
HBM_PEAK_GBS = 8000.0
WORKLOADS = {
    "c1": "1M Eth+IPv4+UDP 64B (config 1/2 shape)",
    "c2": "1M Eth+IPv4+UDP 64B, 1x MI355X (config 2)",
    "c3": "16M IPv4 TCP/UDP/ICMPv4, U[64,1500]B (config 3)",
    "c4": "16M IPv6 + HBH/Routing/Fragment + VLAN/QinQ (config 4)",
    "c5": "IMIX 64/576/1500 7:4:1, IPv4/IPv6, 25% IP-in-IP (config 5 shard)",
    "c6": "16M mixed: c3/c4/c5 shapes + 1/16 ARP per packet (not a BASELINE config)",
}
DEFAULT_PACKETS = {"c1": 1 << 20, "c2": 1 << 20, "c3": 1 << 24, "c4": 1 << 24,
                   "c6": 1 << 24}
C5_TOTAL = 1 << 28          # config 5: one 256M-frame stream over all ranks


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_count(s):
    """'8M' -> 8388608, '256M' -> 268435456, '4096' -> 4096 (K/M/G = 2^10/20/30)."""
    s = str(s).strip()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(s[-1:].upper(), 1)
    return int(s[:-1] if mult > 1 else s) * mult


def host_cores():
    """CPU threads this process may use: the affinity mask, capped by the
    cgroup CPU quota when there is one (a GPU box shows the whole machine in
    its affinity mask but grants a share of it)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    threads = n if quota is None else max(1, min(n, int(quota)))
    return threads, n, quota


def spawn_ranks(n):
    """Runs this command line under torch.distributed.run with n ranks and
    relays rank 0's JSON line; returns the launcher's exit code. Called before
    anything touches the GPU (no exec from a GPU-initialised process)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] spawning {n} ranks: {' '.join(cmd)}")
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            print(line, flush=True)
        else:
            log(line)
    return p.returncode


def pmc_traffic(config, frames, nbytes):
    """HBM read bytes per launch from the committed PMC pass of this workload
    (tools/pmc_traffic.sh -> profiles/*_traffic_<config>.json), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_traffic_{config}.json")),
                       reverse=True):
        t = json.load(open(path))
        if t.get("frames_per_launch") == frames and t.get("algorithmic_bytes_per_launch") == nbytes:
            return int(t["read_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(zp, arena, offs, lens, sample_pkts, min_seconds):
    """Times the oracle (C port, every core of this process' CPU share) on the
    first `sample_pkts` frames, copied to host memory."""
    from tests import oracle as orc   # the checker, used here only as the baseline
    m = min(sample_pkts, offs.numel())
    o = offs[:m].cpu().numpy().astype(np.uint64)
    ln = lens[:m].cpu().numpy().astype(np.uint32)
    end = int(o[-1] + ln[-1])
    a = arena[:end].cpu().numpy()
    cores, visible, quota = host_cores()
    threads = int(os.environ.get("ZP_CPU_THREADS", cores))
    orc.parse_batch(a, o[:1024], ln[:1024], threads)          # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        rec, _ = orc.parse_batch(a, o, ln, threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    assert (rec["err"] == 0).all()
    sec = dt / reps
    # the same port on one core, on the first eighth of the sample
    m1 = max(1, m // 8)
    reps1, t1 = 0, time.perf_counter()
    while True:
        orc.parse_batch(a, o[:m1], ln[:m1], 1)
        reps1 += 1
        dt1 = time.perf_counter() - t1
        if dt1 >= min_seconds / 2:
            break
    sec1 = dt1 / reps1
    return {"value": round(m / sec / 1e6, 3), "unit": "Mpkt/s", "cores": threads,
            "cpus_in_affinity_mask": visible, "cgroup_cpu_quota": quota,
            "kind": "port", "gb_per_s": round(float(ln.sum()) / sec / 1e9, 3),
            "value_1core": round(m1 / sec1 / 1e6, 3),
            "gb_per_s_1core": round(float(ln[:m1].sum()) / sec1 / 1e9, 3),
            "sample": f"first {m} frames of the timed batch ({float(ln.sum())/1e9:.2f} GB), "
                      f"{reps} passes, oracle/zp_oracle.c with {threads} threads; 1-core: "
                      f"first {m1} frames, {reps1} passes"}


def pcie_inclusive(zp, arena, offs, lens, sample_pkts, barrier=lambda: None):
    """Host-pinned frames through zp_parse_batch_host (H2D + parse + D2H).
    Every rank runs it at once between two barriers (each GPU has its own host
    link); returns this rank's (frames, bytes, seconds per pass)."""
    m = min(sample_pkts, offs.numel())
    o = offs[:m].cpu().numpy().astype(np.uint64)
    ln = lens[:m].cpu().numpy().astype(np.uint32)
    end = int(o[-1] + ln[-1])
    host = torch.empty(end, dtype=torch.uint8).pin_memory()
    host.copy_(arena[:end])
    recs = torch.empty((m, zp.records.RECORD_BYTES), dtype=torch.uint8).pin_memory()
    lib = zp._lib.hip()
    ctx = lib.zp_ctx_create(torch.cuda.current_device(), 256 << 20)
    args = (ctx, host.data_ptr(), end, o.ctypes.data, ln.ctypes.data, m, recs.data_ptr(), None)
    zp._lib.check(lib.zp_parse_batch_host(*args), "zp_parse_batch_host")   # warm
    barrier()
    reps, t0 = 3, time.perf_counter()
    for _ in range(reps):
        zp._lib.check(lib.zp_parse_batch_host(*args), "zp_parse_batch_host")
    sec = (time.perf_counter() - t0) / reps
    barrier()
    lib.zp_ctx_destroy(ctx)
    errs = int((zp.batch.record_err(recs) != 0).sum().item())
    return m, end, sec, errs


PCIE_PATH = "pinned host -> H2D -> kernel -> D2H records, 2 streams x 256 MiB chunks"


def placement_probe(zp, arena, offs, lens, records, kernel_ms, reps=5):
    """The placement classes of the bench's own buffers, measured beside the
    parse on the launch stream (HIP events, interleaved rounds, medians):
      read      a plain grid-stride streaming read of the whole arena
                (zp_probe_read_device): the arena's placement;
      tiles     the parse's tile pattern, reads only (zp_probe_tiles_device:
                one wave per 64-frame slice with a parse wave's LDS, the
                tile's descriptors, then its slice of the arena);
      tiles_rec the same plus the 8-B record stores into the bench's records
                buffer: tiles_rec - tiles is what the record stores cost on
                this records placement;
      tiles_code the same with record codes (zp_probe_tiles_codes_device: a
                byte per frame, then the expansion kernel), the pattern of
                the parse when it stores codes (zp_set_record_slots, the
                automatic mode from 2M frames).
    parse_over_* = the parse kernel's mean time / the probe's."""
    import ctypes
    lib = zp._lib.hip()
    sink = torch.zeros(1, dtype=torch.int32, device=arena.device)
    stream = torch.cuda.current_stream(arena.device)
    nb = arena.numel() // 16 * 16
    n = offs.numel()
    s = ctypes.c_void_p(stream.cuda_stream)
    od, ld = offs.data_ptr(), lens.data_ptr()
    probes = {
        "read": lambda: lib.zp_probe_read_device(arena.data_ptr(), nb, sink.data_ptr(), s),
        "tiles": lambda: lib.zp_probe_tiles_device(arena.data_ptr(), nb, n, od, ld, None,
                                                   sink.data_ptr(), s),
        "tiles_rec": lambda: lib.zp_probe_tiles_device(arena.data_ptr(), nb, n, od, ld,
                                                       records.data_ptr(), sink.data_ptr(), s),
        "tiles_code": lambda: lib.zp_probe_tiles_codes_device(arena.data_ptr(), nb, n, od, ld,
                                                              records.data_ptr(), sink.data_ptr(),
                                                              s),
    }
    for f in probes.values():
        zp._lib.check(f(), "placement probe")
    ms = {k: [] for k in probes}
    for _ in range(reps):
        for k, f in probes.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            f()
            b.record(stream)
            ms[k].append((a, b))
    torch.cuda.synchronize()
    med = {k: float(np.median([a.elapsed_time(b) for a, b in v])) for k, v in ms.items()}
    return {"arena_bytes": nb, "read_ms": round(med["read"], 4),
            "read_gbs": round(nb / (med["read"] * 1e-3) / 1e9, 1),
            "tiles_ms": round(med["tiles"], 4), "tiles_rec_ms": round(med["tiles_rec"], 4),
            "record_store_ms": round(med["tiles_rec"] - med["tiles"], 4),
            "parse_over_read": round(kernel_ms / med["read"], 4),
            "parse_over_tiles": round(kernel_ms / med["tiles"], 4),
            "parse_over_tiles_rec": round(kernel_ms / med["tiles_rec"], 4),
            "tiles_code_ms": round(med["tiles_code"], 4),
            "parse_over_tiles_code": round(kernel_ms / med["tiles_code"], 4),
            "arena_va_mod_1g": arena.data_ptr() % (1 << 30),
            "records_va_mod_1g": records.data_ptr() % (1 << 30),
            "probe": "zp_probe_read_device: grid-stride nt 16-B loads, 2048 x 256 lanes; "
                     "zp_probe_tiles_device: one wave per 64-frame slice, its 64 descriptors, "
                     "nt 16-B loads, tiles_rec + 64 nt 8-B stores per wave into the bench's "
                     "records; zp_probe_tiles_codes_device: tiles + a 64-B code store per full "
                     "tile, then the record expansion kernel"}


def gather_rows(row, world, rank, dev):
    """Every rank's float64 row as a [world, len(row)] numpy array (one
    all-reduce of a zero-padded table; no data-path collective)."""
    t = torch.zeros((world, len(row)), dtype=torch.float64, device=dev)
    t[rank] = torch.tensor(row, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def config5_leg(zp, total, steps, warmup, world, rank, dev, barrier, coll_dev):
    """BASELINE config 5 in the same ranks: the `total`-frame IMIX stream cut
    into `world` contiguous shards, rank r parsing frames [total*r/world,
    total*(r+1)/world) (strong scaling: the job is fixed, N shares it). Timed
    like the headline: barrier + synchronise around exactly `steps` launches,
    max over ranks."""
    first, end = total * rank // world, total * (rank + 1) // world
    n = end - first
    arena, offs, lens = zp.batch.generate("c5", n, first=first, device=dev)
    records, ext = zp.batch.alloc_outputs(n, dev)
    nbytes = int(lens.to(torch.int64).sum().item())
    zp.batch.parse_batch(arena, offs, lens, records, ext, check=True)
    torch.cuda.synchronize()
    errs = int((zp.batch.record_err(records) != 0).sum().item())
    for _ in range(warmup):
        zp.batch.parse_batch(arena, offs, lens, records, ext, check=False)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        ev[k][0].record(stream)
        zp.batch.parse_batch(arena, offs, lens, records, ext, check=False)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kmean = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    del arena, offs, lens, records, ext
    torch.cuda.empty_cache()
    rows = gather_rows([first, end, nbytes, errs, kmean, elapsed], world, rank, coll_dev)
    t = float(rows[:, 5].max())
    job_bytes = int(rows[:, 2].sum())
    # HBM bytes per launch from the committed PMC pass of the whole stream on
    # one GPU (tools/pmc_traffic.sh <round> c5), when this run is that workload
    traffic, traffic_src = pmc_traffic("c5", n, nbytes) if world == 1 else (None, None)
    return {
        "traffic": traffic, "traffic_source": traffic_src,
        "workload": WORKLOADS["c5"].replace(" shard", "") + f", {total} frames split {world} ways",
        "frames_total": total, "bytes_total": job_bytes, "scaling": "strong",
        "steps": steps, "warmup": warmup, "ms_per_step": round(t / steps * 1e3, 4),
        "mpkt_s": round(total * steps / t / 1e6, 2),
        "gb_s": round(job_bytes * steps / t / 1e9, 2),
        "shards": [[int(a), int(b)] for a, b in rows[:, 0:2]],
        "rejected_per_rank": [int(x) for x in rows[:, 3]],
        "kernel_ms_per_rank": [round(float(x), 4) for x in rows[:, 4]],
        "frac_per_rank": [round(float(b) / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                          for b, k in zip(rows[:, 2], rows[:, 4])],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--packets", type=int, default=0, help="frames per GPU (default: config)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pcie", action="store_true")
    ap.add_argument("--c5-frames", type=str, default=str(C5_TOTAL),
                    help="frames of the config-5 stream split over the ranks (e.g. 8M)")
    ap.add_argument("--no-c5", action="store_true", help="skip the config-5 leg")
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed even at N = 1 (under a launcher): runs the "
                         "RCCL init / barrier / all-reduce path of the multi-GPU line on one GPU")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(spawn_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        log(f"[bench] --gpus {args.gpus} but the launcher started "
            f"WORLD_SIZE={os.environ['WORLD_SIZE']} ranks")
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    # One rank per GPU over RCCL. More ranks than GPUs (a rehearsal of the N>1
    # path on a smaller box) share devices and synchronise over gloo.
    shared = world > ndev
    local_dev = local % ndev if shared else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    dist_on = world > 1 or (args.dist and "WORLD_SIZE" in os.environ)
    if dist_on:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if dist_on:
            if shared:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local_dev])

    zp = importlib.import_module("zero-packet_amd")
    if args.config == "c5" and not args.packets:
        # config 5: contiguous 1/world shards of one 256M-frame stream
        first, end = C5_TOTAL * rank // world, C5_TOTAL * (rank + 1) // world
        n, job_frames, scaling = end - first, C5_TOTAL, "strong"
    else:
        n = args.packets or DEFAULT_PACKETS[args.config]
        first, job_frames, scaling = rank * n, n * world, "weak"
    t0 = time.perf_counter()
    arena, offs, lens = zp.batch.generate(args.config, n, first=first, device=dev)
    records, ext = zp.batch.alloc_outputs(n, dev)
    torch.cuda.synchronize()
    total_bytes = int(lens.to(torch.int64).sum().item())
    log(f"[rank {rank}] generated {n} frames, {total_bytes/1e9:.2f} GB in "
        f"{time.perf_counter()-t0:.1f}s")

    # One checked parse (descriptor bounds, shapes) whatever --warmup is: the
    # rejected-frame check below reads its records.
    zp.batch.parse_batch(arena, offs, lens, records, ext, check=True)
    torch.cuda.synchronize()
    errs = int((zp.batch.record_err(records) != 0).sum().item())
    assert errs == 0, f"{errs} frames rejected (generator/kernel mismatch)"
    for _ in range(args.warmup):
        zp.batch.parse_batch(arena, offs, lens, records, ext, check=False)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        zp.batch.parse_batch(arena, offs, lens, records, ext, check=False)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kms = [a.elapsed_time(b) for a, b in ev]
    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared else dev)
    job_bytes = torch.tensor([total_bytes], dtype=torch.int64, device="cpu" if shared else dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(job_bytes, op=dist.ReduceOp.SUM)
    elapsed = float(t.item())
    job_bytes = int(job_bytes.item())

    traffic, traffic_src = pmc_traffic(args.config, n, total_bytes)
    ms_step = elapsed / args.steps * 1e3
    mpkts = job_frames * args.steps / elapsed / 1e6
    gbs = job_bytes * args.steps / elapsed / 1e9
    kmean = float(np.mean(kms))
    achieved = total_bytes / (kmean * 1e-3) / 1e9

    out = {
        "metric": METRIC, "value": round(mpkts, 2), "unit": "Mpkt/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (zp_gen: deterministic frames with valid checksums)",
        "gb_per_s": round(gbs, 2),
        "config": {"workload": WORKLOADS[args.config], "config": args.config,
                   "frames_per_gpu": n, "bytes_per_gpu": total_bytes,
                   "job_frames": job_frames, "job_bytes": job_bytes,
                   "mean_frame_bytes": round(total_bytes / n, 2),
                   "parallelism": f"dp{world} (independent shards, no collective)"
                                  + (" [ranks share GPUs: rehearsal only]" if shared else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": ("zp_parse_slots_kernel + zp_rec_expand_kernel (record codes)"
                                if zp.batch.record_codes(n) else "zp_parse_kernel"),
                     "kernel_ms_mean": round(kmean, 4), "kernel_ms_min": round(min(kms), 4),
                     "algorithmic_bytes_per_launch": total_bytes},
    }
    coll_dev = "cpu" if shared else dev
    out["roofline"]["placement"] = placement_probe(zp, arena, offs, lens, records, kmean)
    if not args.no_pcie:
        # every rank's host path at once: frames of all ranks / the slowest rank
        m, nb, sec, perr = pcie_inclusive(zp, arena, offs, lens, 1 << 21, barrier)
        rows = gather_rows([m, nb, sec, perr], world, rank, coll_dev)
        t = float(rows[:, 2].max())
        out["h2d_d2h_inclusive"] = {
            "mpkt_per_s": round(float(rows[:, 0].sum()) / t / 1e6, 2),
            "gb_per_s": round(float(rows[:, 1].sum()) / t / 1e9, 2),
            "sample_frames": int(rows[:, 0].sum()), "ranks": world,
            "per_rank_gb_per_s": [round(float(b) / s / 1e9, 2) for b, s in rows[:, 1:3]],
            "rejected_frames": int(rows[:, 3].sum()),
            "path": PCIE_PATH + ("; all ranks concurrently, summed" if world > 1 else "")}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(zp, arena, offs, lens, args.cpu_sample,
                                           args.cpu_seconds)
        # vs_baseline stays null: BASELINE.md has no published number for
        # this metric. The ratio to the CPU leg of this run is reported
        # beside it instead.
        out["vs_cpu_baseline"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    if args.config != "c5" and not args.no_c5:
        # BASELINE config 5 (256M-frame IMIX over the N GPUs, strong scaling)
        # in the same ranks, so every 1/2/4/8-GPU line carries it
        del arena, offs, lens, records, ext
        torch.cuda.empty_cache()
        out["config5"] = config5_leg(zp, parse_count(args.c5_frames), args.steps, args.warmup,
                                     world, rank, dev, barrier, coll_dev)
        # rejected frames are reported (rejected_per_rank), not asserted: the
        # generator writes valid frames, so a nonzero count is a finding
    if dist_on:
        out["config"]["dist_backend"] = dist.get_backend()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
