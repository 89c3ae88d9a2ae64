#!/usr/bin/env python3
"""HBM traffic of one launch of the fast kernel from the rocprofv3 --pmc passes of tools/pmc.sh
(FETCH_SIZE and WRITE_SIZE in their own runs), corrected as /opt/skills/guides/MI355X_MICROARCH.md
(HBM section) prescribes: both counters are kB; FETCH_SIZE reports half of the bytes of a wide
streaming read on gfx950 and is doubled.  Prints the JSON that bench.py reports as
roofline.traffic (profiles/<round>_pmc_<config>.json)."""
import argparse
import collections
import csv
import glob
import json
import os


def per_dispatch(root, group, counter):
    vals = collections.defaultdict(float)
    names = {}
    for path in glob.glob(os.path.join(root, f"pmc_{group}", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                key = (path, r["Dispatch_Id"])
                vals[key] += float(r["Counter_Value"])
                names[key] = r["Kernel_Name"]
    out = collections.defaultdict(list)
    for k, v in vals.items():
        out[names[k]].append(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--config", required=True)
    ap.add_argument("--pairs", type=int, required=True)
    a = ap.parse_args()
    fetch = per_dispatch(a.root, "fetch", "FETCH_SIZE")
    write = per_dispatch(a.root, "write", "WRITE_SIZE")
    kern = [k for k in fetch if "pe_fast_kernel" in k]
    assert kern, "no pe_fast_kernel dispatches"
    k = max(kern, key=lambda x: max(fetch[x]))  # the full-job kernel (the paths leg runs other variants)
    # the bench launches the kernel on the full job and on smaller host packs / parity samples:
    # keep the full-size launches (within half of the largest)
    big_f = [v for v in fetch[k] if v >= 0.5 * max(fetch[k])]
    big_w = [v for v in write[k] if v >= 0.5 * max(write[k])]
    f_kb = sum(big_f) / len(big_f)
    w_kb = sum(big_w) / len(big_w)
    traffic = (2 * f_kb + w_kb) * 1024
    print(json.dumps({
        "config": a.config, "pairs": a.pairs, "kernel": k.replace("(anonymous namespace)::", "").split("(")[0],
        "dispatches": len(big_f), "FETCH_SIZE_kB": round(f_kb, 1), "WRITE_SIZE_kB": round(w_kb, 1),
        "traffic_bytes": int(traffic),
        "correction": "traffic = 2 x FETCH_SIZE + WRITE_SIZE (kB x 1024); FETCH_SIZE doubled on gfx950 "
                      "(MI355X_MICROARCH.md, HBM [CDNA4]); Infinity-Cache hits are included",
    }, indent=1))


if __name__ == "__main__":
    main()
