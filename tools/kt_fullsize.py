#!/usr/bin/env python3
"""Kernel-trace summary of the fast kernel's FULL-SIZE launches only (the bench's timed steps), from
a rocprofv3 --kernel-trace CSV: rocprofv3's own --stats table averages every launch of a kernel,
the bench's small sample / parity launches included, so its mean is not the timed step's.  A launch
counts as full size when it takes at least half of the longest launch of the same kernel.

    python3 tools/kt_fullsize.py gpurun_out/kt_C3/kt_kernel_trace.csv [--bench profiles/..._bench.json]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--bench", default=None, help="the bench line of the same command (kernel_ms_avg beside)")
    ap.add_argument("--kernel", default="pe_fast_kernel")
    a = ap.parse_args()
    by = {}
    for r in csv.DictReader(open(a.trace)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
        by.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for name, ms in by.items():
        big = [x for x in ms if x >= 0.5 * max(ms)]
        out[name] = {"launches": len(ms), "full_size_launches": len(big), "full_size_mean_ms": round(statistics.mean(big), 4),
                     "full_size_min_ms": round(min(big), 4), "full_size_max_ms": round(max(big), 4),
                     "all_launches_mean_ms": round(statistics.mean(ms), 4)}
    if a.bench:
        b = json.loads(open(a.bench).read().strip().splitlines()[-1])
        out["bench_kernel_ms_avg (HIP events, timed steps)"] = b["roofline"]["kernel_ms_avg"]
        out["bench_workload"] = b["config"]["workload"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
