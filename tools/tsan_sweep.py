#!/usr/bin/env python3
"""Every golden e2e case through the ThreadSanitizer build of the host pipeline (tests/tsan_util.py)
at -w 4 and -w 16 with two engines (one for -d): outputs checked against the reference's, TSan
reports counted.  python tools/tsan_sweep.py > profiles/r04_tsan_sweep.txt"""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import e2e_util as E  # noqa: E402
import tsan_util as T  # noqa: E402

T.build()
total = 0
for case in E.ok_cases():
    for w in (4, 16):
        with tempfile.TemporaryDirectory() as d:
            t0 = time.time()
            err, n = T.run_case(case, d, w, devices=2)
            total += n
            print(f"{case:30s} -w {w:2d}  outputs = reference  TSan reports {n}  ({time.time() - t0:.1f}s)", flush=True)
            if n:
                print(err[-8000:], flush=True)
print(f"total TSan reports: {total}")
