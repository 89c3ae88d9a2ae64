#!/usr/bin/env python3
"""Profiling aid: spill-related instructions (scratch, v_readlane / v_writelane, s_nop) per loop depth
in one kernel of a gfx950 .s file.  python tools/loopspill.py file.s 'pe_fast_kernelILb0ELb1ELb1ELb0ELb1E'"""
import collections, re, sys
path, sym = sys.argv[1], sys.argv[2]
on, depth, cnt = False, 0, collections.Counter()
for ln in open(path):
    if not on:
        on = ln.startswith("_Z") and sym in ln.split(":")[0]
        continue
    if ln.startswith(".Lfunc_end"):
        break
    if ln.startswith(".LBB") or ln.startswith("; %bb"):
        d = re.search(r"Depth=(\d+)", ln)
        depth = int(d.group(1)) if d else 0
        continue
    s = ln.strip()
    if not s or s.startswith((".", ";")):
        continue
    op = s.split()[0]
    if op.startswith("scratch_") or op in ("v_readlane_b32", "v_writelane_b32", "s_nop"):
        cnt[(op, depth)] += 1
for (op, d), n in sorted(cnt.items()):
    print(f"depth {d}  {op:24s} {n}")
