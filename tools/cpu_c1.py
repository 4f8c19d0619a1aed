"""BASELINE config 1: 1M fixed Eth+IPv4+UDP 64-B frames through the CPU
oracle (the C restatement of PacketParser::parse; the Rust reference cannot
be built here), on every core this process may use and on one core.

    python tools/cpu_c1.py [--seconds 5]

Prints one JSON line. The frames are the host generator's config-1 batch
(the same bytes the GPU parses as config 2); every frame must parse Ok.
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def timed(fn, seconds):
    fn()                                            # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        out = fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return dt / reps, reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=5.0)
    args = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    import bench
    import oracle as orc
    n = args.frames
    arena, offs, lens = zp.batch.generate_host("c1", n)
    cores, visible, quota = bench.host_cores()
    out = {"config": "c1: 1M Eth+IPv4+UDP 64B through the CPU oracle (plumbing, no GPU)",
           "frames": n, "bytes": int(lens.sum()), "cpus_in_affinity_mask": visible,
           "cgroup_cpu_quota": quota, "kind": "port (oracle/zp_oracle.c, C restatement)"}
    for label, threads in (("all_cores", cores), ("one_core", 1)):
        sec, reps, (rec, _) = timed(lambda: orc.parse_batch(arena, offs, lens, threads),
                                    args.seconds)
        assert (rec["err"] == 0).all(), "generator/oracle mismatch"
        out[label] = {"threads": threads, "ms": round(sec * 1e3, 3),
                      "mpkt_per_s": round(n / sec / 1e6, 2),
                      "gb_per_s": round(float(lens.sum()) / sec / 1e9, 3), "passes": reps}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
