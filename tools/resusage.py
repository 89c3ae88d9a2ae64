#!/usr/bin/env python3
"""Per-kernel register / spill table from hipcc -Rpass-analysis=kernel-resource-usage (stdin)."""
import re, subprocess, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|TotalSGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]):\s*(\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        dm = subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()
        dm = dm.replace("(anonymous namespace)::", "").split("(")[0]
        cur = {"name": dm}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
for r in rows:
    print(f"{r['name'][:70]:70s} V={r.get('VGPRs'):>4} S={r.get('TotalSGPRs'):>4} scratch={r.get('ScratchSize'):>4} "
          f"occ={r.get('Occupancy')} sspill={r.get('SGPRs Spill')} vspill={r.get('VGPRs Spill')}")
