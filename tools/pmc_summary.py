"""Per-kernel mean-per-dispatch counter values from rocprofv3 --pmc CSVs.
    python tools/pmc_summary.py <dir-with-*_counter_collection.csv> [...]"""
import collections
import csv
import glob
import os
import sys


def summarize(paths):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0]
            per[(name, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {}
    for (name, ctr), d in sorted(per.items()):
        out[(name, ctr)] = (sum(d.values()) / len(d), len(d))
    return out


if __name__ == "__main__":
    paths = []
    for a in sys.argv[1:]:
        paths += glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True)
    for (name, ctr), (v, k) in summarize(paths).items():
        print(f"{name:40s} {ctr:28s} {v:14.5g}  (dispatches {k})")
