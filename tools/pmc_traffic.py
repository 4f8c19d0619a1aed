"""Turns a rocprofv3 --pmc TCC_EA0_RDREQ_sum/TCC_EA0_WRREQ_sum pass over
bench.py into per-launch HBM bytes of zp_parse_kernel.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is
TCC_EA0_RDREQ x 64 B and reports exactly half of the bytes of a wide
streaming read, i.e. read bytes = RDREQ x 128 B (calibrated here with a known
13 GiB read, tools/pmc_calib.sh). Writes: WRREQ x 64 B (matches the 32-B
records exactly)."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402


def main():
    d, cfg, out = sys.argv[1], sys.argv[2], sys.argv[3]
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    s = summarize(paths)
    rd = s[("zp_parse_kernel", "TCC_EA0_RDREQ_sum")]
    wr = s[("zp_parse_kernel", "TCC_EA0_WRREQ_sum")]
    bench = [l for l in open(os.path.join(d, "bench.log")) if l.startswith("{")]
    b = json.loads(bench[-1]) if bench else {}
    res = {
        "kernel": "zp_parse_kernel", "config": cfg,
        "frames_per_launch": b.get("config", {}).get("frames_per_gpu"),
        "algorithmic_bytes_per_launch": b.get("roofline", {}).get("algorithmic_bytes_per_launch"),
        "dispatches": rd[1],
        "TCC_EA0_RDREQ_sum_per_launch": rd[0], "TCC_EA0_WRREQ_sum_per_launch": wr[0],
        "read_bytes_per_launch": rd[0] * 128, "write_bytes_per_launch": wr[0] * 64,
        "method": "rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -- python3 bench.py "
                  "(own pass, no tracing); read = RDREQ x 128 B, write = WRREQ x 64 B (gfx950)",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
