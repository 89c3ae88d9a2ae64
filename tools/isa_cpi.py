#!/usr/bin/env python3
"""Profiling aid: static average issue cycles per VALU instruction of each BASELINE workload's
fast-kernel instantiation (the tile loop of tools/isa_budget.py, priced with the gfx950 opcode
costs of profiles/r04_micro_opcost2.txt), as JSON for bench.py's roofline.valu.issue_frac.

    hipcc -std=c++17 -O3 --offload-arch=gfx950 --offload-device-only -S -gline-tables-only \\
          -Iinclude fqtool_amd/csrc/pe_fast.hip -o /tmp/pe_fast_g.s
    python tools/isa_cpi.py /tmp/pe_fast_g.s > profiles/r06_isa_cpi.json

A static mix weights every instruction of the loop once (rare hand-off paths included), so this is
an estimate of the dynamic average, not a measurement of it."""
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# workload -> pe_fast_kernel<LEAN, PAIRED, MERGE, XTRA, FIX> (the FIX twin: row stride 160)
KERNELS = {"C2": "ILb1ELb0ELb0ELb0ELb1E", "C3": "ILb1ELb1ELb0ELb0ELb1E", "C4": "ILb0ELb1ELb1ELb0ELb1E",
           "C5": "ILb0ELb1ELb0ELb0ELb1E"}


def main(asm):
    out = {}
    for cfg, k in KERNELS.items():
        r = subprocess.run([sys.executable, os.path.join(HERE, "isa_budget.py"), asm, "pe_fast_kernel" + k,
                            "--costs", os.path.join(HERE, "..", "profiles", "r04_micro_opcost2.txt")],
                           capture_output=True, text=True, check=True)
        tot = [l for l in r.stdout.splitlines() if l.startswith("total")][0].split()
        valu_loop, cyc_loop = float(tot[-2]), float(tot[-1])
        out[cfg] = {"kernel": "pe_fast_kernel" + k, "valu_static_loop": valu_loop, "cycles_static_loop": cyc_loop,
                    "cycles_per_valu": round(cyc_loop / valu_loop, 3)}
    out["note"] = ("static: every VALU of the tile loop priced once with the measured gfx950 opcode costs "
                   "(4 waves per SIMD), tools/isa_cpi.py")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
