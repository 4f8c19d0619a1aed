"""zp_parse_one latency (per-frame PacketParser::parse through the GPU):
builds tools/latency/parse_one_main.cpp against libzp_hip.so and runs it with
1 and 8 threads (one zp_ctx each) on generated c3 frames; then
PacketParser.parse (the Python facade, one pooled context per concurrent
call) from 1 and 8 Python threads.

    python tools/parse_one_latency.py [--calls 3000] [--py-threads 1,8]
"""
import argparse
import importlib
import os
import json
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3000)
    ap.add_argument("--threads", default="1,8")
    ap.add_argument("--modes", default="5000,0",
                    help="zp_parse_one_config idle_us per run: >0 resident server, 0 launch per call")
    ap.add_argument("--lib", default="", help="directory of another libzp_hip.so build (A/B)")
    ap.add_argument("--py-threads", default="1,8", help="Python facade thread counts ('' = skip)")
    ap.add_argument("--lives", default="0", help="server life per run in us (test hook; 0 = default)")
    args = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    a, o, l_ = zp.batch.generate_host("c3", 256)
    frames = "".join(a[x:x + y].tobytes().hex() + "\n" for x, y in zip(o, l_))
    lib = os.path.abspath(args.lib) if args.lib else os.path.join(ROOT, "zero-packet_amd")
    exe = os.path.join(ROOT, "tools", "latency", "parse_one" + ("_ab" if args.lib else ""))
    subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"),
                    "-o", exe, os.path.join(ROOT, "tools", "latency", "parse_one_main.cpp"),
                    "-L" + lib, "-lzp_hip", "-Wl,-rpath," + lib], check=True)
    runs = [(m, t, lf) for m in args.modes.split(",") for t in args.threads.split(",")
            for lf in (args.lives.split(",") if m != "0" else ["0"])]
    for m, t, lf in runs:
        if True:
            r = subprocess.run([exe, t, str(args.calls), m, lf], input=frames, capture_output=True,
                               text=True, timeout=300)
            print(r.stdout.strip() or r.stderr[-2000:], flush=True)
            if r.returncode:
                sys.exit(r.returncode)
    frames_b = [a[x:x + y].tobytes() for x, y in zip(o, l_)]
    for t in [int(x) for x in args.py_threads.split(",") if x]:
        py_threads(zp, frames_b, t, args.calls)


def py_threads(zp, frames, threads, calls):
    """PacketParser.parse from `threads` Python threads, `calls` each."""
    P = zp.parser.PacketParser
    for f in frames[:64]:                                   # warm the pool's servers
        P.parse(f)
    lat = [[] for _ in range(threads)]
    go = threading.Barrier(threads + 1)

    def run(t):
        P.parse(frames[t])                                  # this thread's pool context
        go.wait()
        for k in range(calls):
            t0 = time.perf_counter()
            P.parse(frames[(k * 7 + t) % len(frames)])
            lat[t].append(time.perf_counter() - t0)
    ths = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    go.wait()
    t0 = time.perf_counter()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    allv = sorted(x for v in lat for x in v)
    print(json.dumps({"api": "PacketParser.parse (Python)", "threads": threads,
                      "calls": len(allv), "p50_us": round(1e6 * allv[len(allv) // 2], 2),
                      "p99_us": round(1e6 * allv[int(len(allv) * 0.99)], 2),
                      "calls_per_s": round(len(allv) / dt)}), flush=True)


if __name__ == "__main__":
    main()
