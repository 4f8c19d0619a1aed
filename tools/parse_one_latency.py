"""zp_parse_one latency (per-frame PacketParser::parse through the GPU):
builds tools/latency/parse_one_main.cpp against libzp_hip.so and runs it with
1 and 8 threads (one zp_ctx each) on generated c3 frames.

    python tools/parse_one_latency.py [--calls 3000]
"""
import argparse
import importlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3000)
    ap.add_argument("--threads", default="1,8")
    ap.add_argument("--modes", default="5000,0",
                    help="zp_parse_one_config idle_us per run: >0 resident server, 0 launch per call")
    ap.add_argument("--lib", default="", help="directory of another libzp_hip.so build (A/B)")
    args = ap.parse_args()
    zp = importlib.import_module("zero-packet_amd")
    a, o, l_ = zp.batch.generate_host("c3", 256)
    frames = "".join(a[x:x + y].tobytes().hex() + "\n" for x, y in zip(o, l_))
    lib = os.path.abspath(args.lib) if args.lib else os.path.join(ROOT, "zero-packet_amd")
    exe = os.path.join(ROOT, "tools", "latency", "parse_one" + ("_ab" if args.lib else ""))
    subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"),
                    "-o", exe, os.path.join(ROOT, "tools", "latency", "parse_one_main.cpp"),
                    "-L" + lib, "-lzp_hip", "-Wl,-rpath," + lib], check=True)
    for m in args.modes.split(","):
        for t in args.threads.split(","):
            r = subprocess.run([exe, t, str(args.calls), m], input=frames, capture_output=True,
                               text=True, timeout=300)
            print(r.stdout.strip() or r.stderr[-2000:], flush=True)
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
