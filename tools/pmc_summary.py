#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs under gpurun_out/pmc_*: per kernel dispatch (in launch
order), the counter values of the render kernels.  Usage: tools/pmc_summary.py [DIR...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    dirs = sys.argv[1:] or sorted(glob.glob(os.path.join("gpurun_out", "pmc_*")))
    for d in dirs:
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = list(csv.DictReader(open(f)))
        per = defaultdict(dict)
        names = {}
        for r in rows:
            k = r["Kernel_Name"]
            if not any(s in k for s in ("render", "sample", "mega", "batch")):
                continue
            did = int(r.get("Dispatch_Id", 0))
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[did] = k.split("(")[0]
        print(f"== {d}")
        for did in sorted(per):
            vals = "  ".join(f"{c}={v:.4g}" for c, v in sorted(per[did].items()))
            print(f"  #{did} {names[did]}: {vals}")


if __name__ == "__main__":
    main()
