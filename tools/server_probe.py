"""zp_parse_one server timing probe: the device clock rate the host converts
its idle/life bounds with, the stall hook's real length, and how long a
torch.cuda.synchronize() waits with the server idle or under traffic, per
server life (test hooks of libzp_hip.so).

    python tools/server_probe.py
"""
import ctypes
import importlib
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    zp = importlib.import_module("zero-packet_amd")
    torch.zeros(1, device="cuda")
    lib = zp._lib.hip()
    a, o, l_ = zp.batch.generate_host("c5", 256, first=5)
    frames = [a[int(x):int(x) + int(y)].tobytes() for x, y in zip(o, l_)]
    bufs = [ctypes.create_string_buffer(f, len(f)) for f in frames]
    rec = np.zeros(1, zp.records.RECORD_DTYPE)
    ext = np.zeros((2, 16), np.uint8)
    ctx = lib.zp_ctx_create(0, 1 << 20)

    def call(i):
        return lib.zp_parse_one(ctx, ctypes.addressof(bufs[i]), len(frames[i]), rec.ctypes.data,
                                ext.ctypes.data)
    # stall hook: a give-up of 500 us behind stalls of 10 and 40 ms
    for stall in (10000, 40000):
        lib.zp__one_test_hooks(ctx, 0, 500, stall)
        t0 = time.perf_counter()
        rc = call(0)
        print(json.dumps({"probe": "stall", "stall_us": stall, "rc": rc,
                          "call_ms": round(1e3 * (time.perf_counter() - t0), 3)}), flush=True)
    lib.zp__one_test_hooks(ctx, 0, 10_000_000, 0)
    # idle server: one call, then a sync after a short gap
    for life in (1000, 5000):
        lib.zp__one_test_hooks(ctx, life, 0, 0)
        w = []
        for k in range(10):
            call(k)
            time.sleep(0.0002)
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            w.append(time.perf_counter() - t0)
        print(json.dumps({"probe": "idle_server_sync", "life_us": life,
                          "wait_ms": [round(1e3 * x, 3) for x in w]}), flush=True)
    sys.setswitchinterval(5e-5)
    for life in (200, 1000, 3000):
        lib.zp__one_test_hooks(ctx, life, 0, 0)
        stop = threading.Event()
        n = [0]

        def caller():
            k = 0
            while not stop.is_set():
                call(k % len(frames))
                k += 1
            n[0] = k
        th = threading.Thread(target=caller)
        th.start()
        time.sleep(0.1)
        w = []
        for k in range(10):
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            w.append(time.perf_counter() - t0)
            time.sleep(0.05)
        stop.set()
        th.join()
        st = np.zeros(3, np.uint64)
        lib.zp__one_stats(ctx, st.ctypes.data)
        print(json.dumps({"probe": "traffic_sync", "life_us": life, "calls": n[0],
                          "launches_rotations_relaunches": [int(x) for x in st],
                          "wait_ms": [round(1e3 * x, 3) for x in w]}), flush=True)
    lib.zp_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
