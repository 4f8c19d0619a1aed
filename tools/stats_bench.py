"""Timing of zp_stats_device over one c3 batch's records (16M x 16 B)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    zp = importlib.import_module("zero-packet_amd")
    d = torch.device("cuda:0")
    n = 1 << 24
    arena, offs, lens = zp.batch.generate("c3", n, device=d)
    r, _ = zp.batch.parse_batch(arena, offs, lens)
    del arena
    c = zp.stats.count(r)
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(20)]
    for a, b in ev:
        a.record(s)
        zp.stats.count(r, counts=c)
        b.record(s)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)[10]
    print(f"zp_stats_device, {n} records: {ms * 1e3:.1f} us, {n * 16 / ms / 1e6:.0f} GB/s of "
          f"records, {n / ms / 1e6:.1f} Gpkt/s", flush=True)
    print(zp.stats.to_dict(zp.stats.count(r)), flush=True)


if __name__ == "__main__":
    main()
