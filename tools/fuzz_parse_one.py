"""Long zp_parse_one campaign (not part of the test suite): the tests'
mutation fuzzer's frames (raw and with refilled checksums) through one
context's resident server wave, one call per frame, every record and chain
entry compared with the oracle's; every round also switches the context to
one launch per call for a slice of the frames and back, and waits past the
server's idle timeout once, so the server leaves and is relaunched.
With threads > 1 (round 6: the device's shared server) the frames of a
round are split over that many threads with a context each; besides, one
thread stops the device's server now and then (zp_parse_one_config) and
another creates and destroys a context between its frames, while the others
keep calling.
Usage: python tools/fuzz_parse_one.py [rounds] [frames_per_round] [threads]"""
import threading
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as orc  # noqa: E402  (tests/oracle.py: the checker)
from test_gpu_parity import fuzz_frames  # noqa: E402


def threaded(zp, golden, rounds, count, threads):
    lib = zp._lib.hip()
    t0 = time.time()
    total = [0] * threads
    bad = []

    def worker(t, frames):
        rec = np.zeros(1, zp.records.RECORD_DTYPE)
        ext = np.zeros((2, 16), np.uint8)
        ctx = lib.zp_ctx_create(0, 1 << 20)
        try:
            for i, f in enumerate(frames):
                if t == 1 and i % 997 == 500:
                    lib.zp_parse_one_config(ctx, 5000)    # stops the device's server
                if t == 2 and i % 1499 == 700:            # a context comes and goes
                    lib.zp_ctx_destroy(ctx)
                    ctx = lib.zp_ctx_create(0, 1 << 20)
                buf = ctypes.create_string_buffer(f, max(len(f), 1))
                rc = lib.zp_parse_one(ctx, ctypes.addressof(buf), len(f), rec.ctypes.data,
                                      ext.ctypes.data)
                err, wrec, wext = orc.parse_one(f)
                if rc != err or rec.tobytes() != orc.pack(wrec, wext).tobytes() or \
                        ext.tobytes() != wext.view(np.uint8).tobytes():
                    bad.append((t, i, rc, err, f.hex()))
                    return
                total[t] += 1
        finally:
            lib.zp_ctx_destroy(ctx)
    for r in range(rounds):
        frames = fuzz_frames(zp, golden, count, 7000 + r, 0.5 if r % 2 else 0.0)
        ths = [threading.Thread(target=worker, args=(t, frames[t::threads]))
               for t in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if bad:
            raise SystemExit(f"round {r}: {bad[:3]}")
        print(f"round {r}: {len(frames)} frames on {threads} threads OK "
              f"({time.time() - t0:.0f} s)", flush=True)
    print(f"fuzz_parse_one: {sum(total)} calls on {threads} threads identical to the oracle",
          flush=True)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    zp = importlib.import_module("zero-packet_amd")
    if threads > 1:
        golden = json.load(open(os.path.join(ROOT, "tests", "golden", "parse_golden.json")))
        return threaded(zp, golden, rounds, count, threads)
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "parse_golden.json")))
    lib = zp._lib.hip()
    ctx = lib.zp_ctx_create(0, 0)
    rec = np.zeros(1, zp.records.RECORD_DTYPE)
    ext = np.zeros((2, 16), np.uint8)
    t0 = time.time()
    total = acc = 0
    try:
        for r in range(rounds):
            frames = fuzz_frames(zp, golden, count, 5000 + r, 0.5 if r % 2 else 0.0)
            lib.zp_parse_one_config(ctx, 5000)
            for i, f in enumerate(frames):
                if i == count // 2:
                    time.sleep(0.02)                      # past the 5-ms idle timeout
                if i == 3 * count // 4:
                    lib.zp_parse_one_config(ctx, 0)       # one launch per call ...
                if i == 3 * count // 4 + 200:
                    lib.zp_parse_one_config(ctx, 5000)    # ... and back to the server
                buf = ctypes.create_string_buffer(f, max(len(f), 1))
                rc = lib.zp_parse_one(ctx, ctypes.addressof(buf), len(f), rec.ctypes.data,
                                      ext.ctypes.data)
                err, wrec, wext = orc.parse_one(f)
                if rc != err or rec.tobytes() != orc.pack(wrec, wext).tobytes() or \
                        ext.tobytes() != wext.view(np.uint8).tobytes():
                    raise SystemExit(f"round {r} frame {i}: rc {rc} vs {err}, frame {f.hex()}")
                acc += err == 0
            total += len(frames)
            print(f"round {r}: {len(frames)} frames OK ({time.time() - t0:.0f} s)", flush=True)
    finally:
        lib.zp_ctx_destroy(ctx)
    print(f"fuzz_parse_one: {total} calls identical to the oracle, {acc / total:.0%} accepted",
          flush=True)


if __name__ == "__main__":
    main()
