"""One zp_parse_kernel launch per variant library, in order, for PMC passes
(instruction counts per variant are deterministic: no timing noise).
Usage: rocprofv3 --pmc SQ_INSTS_VALU ... -- python3 tools/pmc_variants.py c5 base,fakewalk,...
Then: python3 tools/pmc_variants.py --report <counter_collection.csv> base,fakewalk,..."""
import csv
import ctypes
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def report(path, names):
    rows = [r for r in csv.DictReader(open(path)) if "zp_parse_kernel" in r["Kernel_Name"]]
    by = {}
    for r in rows:
        by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)
    for name, i in zip(names, ids[-len(names):]):
        print(f"{name:12s} " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(by[i].items())))


def main():
    if sys.argv[1] == "--report":
        report(sys.argv[2], sys.argv[3].split(","))
        return
    import torch
    zp = importlib.import_module("zero-packet_amd")
    cfg, names = sys.argv[1], sys.argv[2].split(",")
    n = {"c2": 1 << 20, "c3": 1 << 24, "c4": 1 << 24, "c5": 1 << 25}[cfg]
    d = torch.device("cuda:0")
    arena, offs, lens = zp.batch.generate(cfg, n, device=d)
    rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
    ext = torch.empty((2, n, 16), dtype=torch.uint8, device=d)
    for name in names:
        lib = zp._lib.hip() if name == "base" else ctypes.CDLL(
            os.path.join(ROOT, "tools", "variants", f"libzp_{name}.so"))
        if name != "base":
            lib.zp_parse_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + \
                [ctypes.c_void_p] * 3
        lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                  rec.data_ptr(), ext.data_ptr(), None)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
