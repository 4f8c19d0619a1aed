"""Turns a rocprofv3 --pmc TCC_EA0_RDREQ_sum/TCC_EA0_WRREQ_sum pass over
bench.py into per-launch HBM bytes of the parse: zp_parse_kernel, or with
record codes (zp_set_record_slots, from 2M frames of traffic with code
tiles) zp_parse_slots_kernel + zp_rec_expand_kernel (one of each per
launch), whichever path most launches took.

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
    names = [k for k in ("zp_parse_kernel", "zp_parse_slots_kernel", "zp_rec_expand_kernel")
             if (k, "TCC_EA0_RDREQ_sum") in s]
    per = {k: {"RDREQ": s[(k, "TCC_EA0_RDREQ_sum")][0], "WRREQ": s[(k, "TCC_EA0_WRREQ_sum")][0],
               "dispatches": s[(k, "TCC_EA0_RDREQ_sum")][1]} for k in names}
    # the path most launches took (the automatic mode probes the other now
    # and then)
    main_k = max((k for k in ("zp_parse_kernel", "zp_parse_slots_kernel") if k in per),
                 key=lambda k: per[k]["dispatches"])
    launch = [main_k] + (["zp_rec_expand_kernel"] if main_k == "zp_parse_slots_kernel" else [])
    rd = (sum(per[k]["RDREQ"] for k in launch), per[main_k]["dispatches"])
    wr = (sum(per[k]["WRREQ"] for k in launch), per[main_k]["dispatches"])
    bench = [l for l in open(os.path.join(d, "bench.log")) if l.startswith("{")]
    b = json.loads(bench[-1]) if bench else {}
    res = {
        "kernel": " + ".join(launch), "config": cfg, "per_kernel": per,
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
