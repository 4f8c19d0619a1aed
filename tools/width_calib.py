"""FETCH_SIZE calibration by load width (tools/membw.hip membw_width): reads a
4 GiB buffer (> the 256 MiB Infinity Cache) once per launch with dword,
dwordx2, dwordx4 loads and the builder's 5-dword blob pattern, 3 launches
each. Run under rocprofv3 --pmc (tools/pmc_width.sh); the known byte count
per launch fixes each width's FETCH_SIZE factor."""
import ctypes
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "libmembw.so")
SRC = os.path.join(ROOT, "tools", "membw.hip")


def main():
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SRC):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                        "-o", SO, SRC], check=True)
    mb = ctypes.CDLL(SO)
    mb.membw_width.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                               ctypes.c_int, ctypes.c_void_p]
    nbytes = 4 << 30
    buf = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
    out = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for w in (1, 2, 4, 8, 16, 5):
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            assert mb.membw_width(buf.data_ptr(), nbytes, out.data_ptr(), w, 8192, s) == 0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        print(f"width {w}: {nbytes} B per launch, {nbytes / dt / 1e9:.0f} GB/s (wall)", flush=True)
    # write-allocate probe: copy 2 GiB with 0 / 1 / 4 of every line's 8 chunks left unwritten
    mb.membw_copy_gap.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_void_p]
    half = nbytes // 2
    for gap in (0, 1, 4):
        for _ in range(3):
            assert mb.membw_copy_gap(buf.data_ptr(), buf.data_ptr() + half, half, gap, 8192, s) == 0
        torch.cuda.synchronize()
        print(f"copy_gap {gap}: {half} B src, {half * (8 - gap) // 8} B written per launch",
              flush=True)


if __name__ == "__main__":
    sys.exit(main())
