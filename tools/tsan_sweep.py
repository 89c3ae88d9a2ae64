#!/usr/bin/env python3
"""Every golden e2e case through the ThreadSanitizer build of the host pipeline (tests/tsan_util.py):
host packs at -w 4 and -w 16 on two engines (one for -d), then the raw stream (plain inputs, 4 KiB
first window, 7-pair packs) with the engine's output text on three and four engines and with the
records-only egress on one engine (FQ_RAW_EGRESS=host, byte ranges and copied): outputs checked
against the reference's, TSan reports counted.
python tools/tsan_sweep.py > profiles/r05_tsan_sweep.txt   (SWEEP=raw: the raw-stream part only)"""
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
skip_rest = False
for case in E.ok_cases() if os.environ.get("SWEEP", "all") != "raw" else []:
    for w in (4, 16):
        with tempfile.TemporaryDirectory() as d:
            t0 = time.time()
            err, n = T.run_case(case, d, w, devices=2)
            total += n
            print(f"{case:30s} -w {w:2d}  outputs = reference  TSan reports {n}  ({time.time() - t0:.1f}s)", flush=True)
            if n:
                print(err[-8000:], flush=True)
# raw stream: the engine's output text on three and four engines; records-only egress (one engine)
# as byte ranges of the windows (zc) and copied
for case in E.ok_cases():
    for egress, devices in (("text", 3), ("text", 4), ("zc", 1), ("copy", 1)):
        if egress != "text" or devices != 3:
            if skip_rest:  # (options that keep the case off the raw stream: one run says so)
                continue
        env = {"FQ_RAW_WINDOW0": "4096"}
        if egress != "text":
            env.update(FQ_RAW_EGRESS="host", FQ_RAW_ZC="1" if egress == "zc" else "0")
        with tempfile.TemporaryDirectory() as d:
            t0 = time.time()
            err, n = T.run_case(case, d, 4, devices=devices, mode="raw", env_extra=env, pack_pairs=7)
            total += n
            path = (f"raw stream on {devices} engines" if f"raw stream on {devices} engines" in err else
                    "raw, records-only" if "records-only egress" in err else
                    "raw stream, 1 engine" if "raw stream" in err else "host packs (options)")
            skip_rest = path == "host packs (options)"
            print(f"{case:30s} raw egress {egress:4s} ({path:24s})  outputs = reference  TSan reports {n}  ({time.time() - t0:.1f}s)", flush=True)
            if n:
                print(err[-8000:], flush=True)
print(f"total TSan reports: {total}")
