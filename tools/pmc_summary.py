#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV outputs (gpurun_out/pmc_*/...counter_collection.csv): per kernel
name, the mean over dispatches of each counter (summed over the per-XCD/per-SE dimensions)."""
import collections
import csv
import glob
import os
import sys


def main(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(float)
        names = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            acc[names[d]][c].append(v)
    for k, cs in acc.items():
        short = k.replace("(anonymous namespace)::", "").split("(")[0][:80]
        print(short)
        for c, vs in sorted(cs.items()):
            print(f"    {c:28s} mean {sum(vs) / len(vs):16.4g}   n={len(vs)}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
