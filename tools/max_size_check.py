"""One GPU, the whole 256M-frame IMIX of BASELINE config 5 (≈95 GB of frames,
arena offsets far past 2^32, 4M workgroups): every frame accepted, a random
sample byte-exact vs the oracle, and the kernel time. Not part of the suite
(it needs ~110 GB of HBM). Usage: python tools/max_size_check.py [frames]"""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as orc  # noqa: E402  (tests/oracle.py: the checker)
from test_gpu_parity import assert_same, pack  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 20
    zp = importlib.import_module("zero-packet_amd")
    d = torch.device("cuda:0")
    t0 = time.time()
    arena, offs, lens = zp.batch.generate("c5", n, device=d)
    torch.cuda.synchronize()
    nbytes = int(lens.to(torch.int64).sum().item())
    print(f"generated {n} frames, {nbytes / 1e9:.1f} GB in {time.time() - t0:.1f} s", flush=True)
    rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
    ext = torch.empty((2, n, 16), dtype=torch.uint8, device=d)
    zp.batch.parse_batch(arena, offs, lens, rec, ext, check=False)
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(s)
    zp.batch.parse_batch(arena, offs, lens, rec, ext, check=False)
    ev[1].record(s)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1])
    bad = int((zp.batch.record_err(rec) != 0).sum().item())
    print(f"parse: {ms:.2f} ms, {nbytes / ms / 1e6:.0f} GB/s, {n / ms / 1e3:.0f} Mpkt/s, "
          f"rejected {bad}", flush=True)
    assert bad == 0
    g = torch.Generator(device=d).manual_seed(5)
    idx = torch.cat([torch.randint(0, n, (3000,), device=d, generator=g),
                     torch.arange(n - 1000, n, device=d)])      # the last frames too
    so, sl = offs[idx].cpu().numpy(), lens[idx].cpu().numpy()
    frames = [arena[int(o):int(o) + int(l)].cpu().numpy().tobytes() for o, l in zip(so, sl)]
    sa, sof, sle = pack(frames)
    want, wext = orc.parse_batch(sa, sof, sle)
    got, gext = zp.batch.records_to_numpy(rec[idx], ext[:, idx])
    assert_same(got, gext, want, wext)
    print(f"max_size_check: OK (last offset {int(offs[-1].item()):,})", flush=True)


if __name__ == "__main__":
    main()
