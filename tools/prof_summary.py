#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output directory (rocpd .db or CSV) as text."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    # the rocpd top_kernels view reports microseconds; normalise to ns like the CSV
    return [(n, int(k), float(t) * 1e3, float(a) * 1e3, float(p)) for n, k, t, a, p in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r["Percentage"])))
    return out


def main(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    print(f"rocprofv3 --kernel-trace --stats summary ({os.path.basename((csvs or dbs)[0])})")
    print(f"{'calls':>6} {'avg_ms':>12} {'total_ms':>12} {'pct':>7}  kernel")
    for n, k, t, a, p in rows:
        print(f"{k:>6} {a / 1e6:>12.3f} {t / 1e6:>12.3f} {p:>6.2f}%  {n}")


if __name__ == "__main__":
    main(sys.argv[1])
