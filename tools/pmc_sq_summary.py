#!/usr/bin/env python3
"""Summarise tools/pmc_sq.sh (SQ / GRBM counter passes + kernel trace) per config into
profiles/<round>_sq_<cfg>.json: per full-size launch of the fast kernel, the mean of every
counter (summed over the per-XCD / per-SE dimensions), the kernel-trace duration, and derived
figures:
  * valu_per_tile      -- SQ_INSTS_VALU / tiles (a tile = one wave's 32 pairs or 64 reads)
  * kernel_cycles      -- GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs): the launch in
                          shader-clock cycles, whatever clock the chip held while profiled
  * valu_issue_frac    -- SQ_INSTS_VALU x 2 cycles (a wave64 VALU issues over 2 cycles on a
                          SIMD-32, MI355X_MICROARCH.md) / (1024 SIMDs x kernel_cycles)
  * wait_frac / inst_stall_frac / active_frac -- SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
                          SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (disjoint, sum ~ 1)
  * lds_busy_frac      -- SQ_LDS_IDX_ACTIVE / (256 CUs x kernel_cycles) (LDS-array cycles; the
                          counter's units are taken as cycles per CU, uncalibrated)
Usage: python3 tools/pmc_sq_summary.py gpurun_out/sq --round r03 --pairs 100000000 [--out profiles]"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def counters(root, cfg, group):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for path in glob.glob(os.path.join(root, f"{cfg}_{group}", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                key = (path, r["Dispatch_Id"])
                vals[key][r["Counter_Name"]] += float(r["Counter_Value"])
                names[key] = r["Kernel_Name"]
    return vals, names


def fast_launches(vals, names, probe):
    keys = [k for k in vals if "pe_fast_kernel" in names[k]]
    if not keys:
        return {}, None
    big = max(vals[k].get(probe, 0.0) for k in keys)
    keys = [k for k in keys if vals[k].get(probe, 0.0) >= 0.5 * big]  # the full-size launches
    out = {}
    for c in vals[keys[0]]:
        out[c] = sum(vals[k][c] for k in keys) / len(keys)
    return out, names[keys[0]]


def trace_ms(root, cfg):
    ds = []
    # (pmc_sq.sh's own trace, or profile_round.sh's beside the counter directory: gpurun_out/kt_<cfg>)
    paths = glob.glob(os.path.join(root, f"{cfg}_kt", "**", "*kernel_trace.csv"), recursive=True) or \
        glob.glob(os.path.join(os.path.dirname(os.path.normpath(root)), f"kt_{cfg}", "**", "*kernel_trace.csv"), recursive=True)
    for path in paths:
        with open(path) as f:
            for r in csv.DictReader(f):
                if "pe_fast_kernel" in r["Kernel_Name"]:
                    ds.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    if not ds:
        return None, 0
    big = [d for d in ds if d >= 0.5 * max(ds)]
    return statistics.median(big), len(big)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--round", required=True)
    ap.add_argument("--pairs", type=int, default=100_000_000)
    ap.add_argument("--out", default="profiles")
    ap.add_argument("--configs", default="C3 C4 C5")
    a = ap.parse_args()
    for cfg in a.configs.split():
        merged, kname = {}, None
        for g, probe in (("issue", "SQ_INSTS_VALU"), ("lds", "SQ_INSTS_LDS")):
            v, n = counters(a.root, cfg, g)
            m, k = fast_launches(v, n, probe)
            for c, x in m.items():
                merged.setdefault(c, x)  # GRBM_GUI_ACTIVE: from the first pass
            kname = kname or k
        if not merged:
            print(f"{cfg}: no counters")
            continue
        ms, nk = trace_ms(a.root, cfg)
        paired = cfg != "C2"
        tiles = -(-a.pairs // (32 if paired else 64))
        cyc = merged.get("GRBM_GUI_ACTIVE", 0.0) / 8
        d = {
            "config": cfg, "pairs" if paired else "reads": a.pairs, "tiles": tiles,
            "kernel": (kname or "").replace("(anonymous namespace)::", "").split("(")[0],
            "kernel_ms_trace": round(ms, 3) if ms else None, "trace_launches": nk,
            "counters_per_launch": {c: round(x, 1) for c, x in sorted(merged.items())},
        }
        if cyc:
            d["kernel_cycles"] = round(cyc)
            d["effective_clock_GHz_profiled"] = round(cyc / (ms * 1e6), 3) if ms else None
            valu = merged.get("SQ_INSTS_VALU")
            if valu:
                d["valu_per_tile"] = round(valu / tiles, 1)
                d["valu_issue_frac"] = round(valu * 2 / (1024 * cyc), 4)
            if "SQ_LDS_IDX_ACTIVE" in merged:
                d["lds_busy_frac"] = round(merged["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 4)
            if "SQ_INSTS_LDS" in merged:
                d["lds_per_tile"] = round(merged["SQ_INSTS_LDS"] / tiles, 1)
            if "SQ_INSTS_SALU" in merged:
                d["salu_per_tile"] = round(merged["SQ_INSTS_SALU"] / tiles, 1)
        wc = merged.get("SQ_WAVE_CYCLES")
        if wc:
            for c, k in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "inst_stall_frac"),
                         ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if c in merged:
                    d[k] = round(merged[c] / wc, 4)
        d["note"] = ("counters summed over XCDs/SEs per dispatch, mean over the full-size launches of the "
                     "profiled bench command (tools/pmc_sq.sh); SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are "
                     "quad-cycles summed over waves; valu_issue_frac = VALU x 2 / (1024 SIMDs x kernel_cycles)")
        path = os.path.join(a.out, f"{a.round}_sq_{cfg}.json")
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
        print(json.dumps(d))


if __name__ == "__main__":
    main()
