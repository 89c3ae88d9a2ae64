#!/usr/bin/env python3
"""Profiling aid: where the e2e raw-stream pipeline leaves the copy engines idle.

Reads the rocprofv3 kernel and memory-copy traces of tools/gpu_e2e_trace.sh and prints the
H2D / D2H / kernel busy time, the idle stretches of the copy engines (neither direction busy)
longer than --min-gap microseconds, and what ran on the GPU during each (kernel names)."""
import argparse
import csv
import glob
import os


def load(root, pat):
    rows = []
    for p in glob.glob(os.path.join(root, "**", pat), recursive=True):
        with open(p) as f:
            rows += list(csv.DictReader(f))
    return rows


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/e2e_trace")
    ap.add_argument("--min-gap", type=float, default=200.0)
    ap.add_argument("--show", type=int, default=25)
    a = ap.parse_args()
    ker = load(a.root, "*kernel_trace.csv")
    cpy = load(a.root, "*memory_copy_trace.csv")
    kiv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?")) for r in ker]
    h2d, d2h = [], []
    for r in cpy:
        d = (r.get("Direction") or r.get("Kind") or "").upper()
        iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        (h2d if "HOST_TO_DEVICE" in d or "H2D" in d else d2h if "DEVICE_TO_HOST" in d or "D2H" in d else []).append(iv)
    t0 = min([x[0] for x in kiv] + [x[0] for x in h2d + d2h])
    t1 = max([x[1] for x in kiv] + [x[1] for x in h2d + d2h])
    # the pipeline's span: from the first window copy to the last output copy
    s0, s1 = min(x[0] for x in h2d), max(x[1] for x in d2h)
    busy = lambda iv: sum(b - a for a, b in union([(max(x[0], s0), min(x[1], s1)) for x in iv if x[1] > s0 and x[0] < s1]))
    cu = union(h2d + d2h)
    print(f"trace {1e-6 * (t1 - t0):.1f} ms, pipeline span {1e-6 * (s1 - s0):.1f} ms: H2D busy {1e-6 * busy(h2d):.1f}, "
          f"D2H busy {1e-6 * busy(d2h):.1f}, copies (either) {1e-6 * busy(h2d + d2h):.1f}, "
          f"kernels {1e-6 * busy([x[:2] for x in kiv]):.1f} ms; {len(h2d)} H2D, {len(d2h)} D2H copies")
    gaps = [(cu[i][1], cu[i + 1][0]) for i in range(len(cu) - 1) if cu[i + 1][0] - cu[i][1] > a.min_gap * 1e3]
    tot = sum(b - a for a, b in gaps)
    print(f"{len(gaps)} copy-idle stretches > {a.min_gap:.0f} us inside the span: {1e-6 * tot:.1f} ms")
    for g0, g1 in gaps[: a.show]:
        ks = [k for k in kiv if k[1] > g0 and k[0] < g1]
        names = {}
        for k in ks:
            n = k[2].split("(")[0].split("::")[-1][:32]
            names[n] = names.get(n, 0) + 1e-3 * (min(k[1], g1) - max(k[0], g0))
        top = ", ".join(f"{n} {v:.0f}us" for n, v in sorted(names.items(), key=lambda x: -x[1])[:4])
        print(f"  at {1e-6 * (g0 - s0):8.2f} ms: {1e-3 * (g1 - g0):7.0f} us idle; kernels: {top or '-'}")


if __name__ == "__main__":
    main()
