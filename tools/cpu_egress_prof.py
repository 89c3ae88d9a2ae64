#!/usr/bin/env python3
"""Profiling aid (CPU only): the host formatter's cost per egress mode, with the CPU stand-in engine
(build/cpuhost/fqtool; test infrastructure) processing the packs.  The stand-in is slower than the
GPU, so the pipeline is engine-bound here; what this measures is the tool's own "format" stamp (the
formatter thread: records-only formatting, adapter-entry counting) on the same synthetic workload as
bench.py's e2e leg (C3 options).

    python tools/cpu_egress_prof.py [--pairs 1000000] [--workers 8]
"""
import argparse
import ctypes
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--variants", default=";FQ_RAW_EGRESS=host;FQ_RAW_EGRESS=host FQ_RAW_ZC=0")
    args = ap.parse_args()
    import torch

    from fqtool_amd import abi
    from oracle_lib import load_oracle

    subprocess.run(["make", "-s", "-C", REPO, "cpuhost"], check=True)
    oracle = load_oracle()
    n = args.pairs
    bufs = [torch.empty(abi.batch_bytes(n, bench.STRIDE), dtype=torch.uint8) for _ in range(4)]
    lens = [torch.empty(n, dtype=torch.int16) for _ in range(2)]
    b = abi.FqBatch()
    b.n, b.stride = n, bench.STRIDE
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    first = 10 ** 12
    oracle.orc_synth_fill(ctypes.byref(b), bench.SEED, first, bench.READ_LEN)
    tmp = tempfile.mkdtemp(prefix="fqegress_")
    try:
        ins = bench.write_fastq_fast(bufs, n, first, tmp)
        tool = os.path.join(REPO, "build", "cpuhost", "fqtool")
        for v in args.variants.split(";"):
            env = dict(os.environ)
            for tok in v.split():
                k, val = tok.split("=", 1)
                env[k] = val
            cmd = [tool, "-i", ins[0], "-I", ins[1], "-o", "/dev/null", "-O", "/dev/null", "-q", "-a", "--detect_pe_adapter",
                   "-g", "-w", str(args.workers), "-J", os.path.join(tmp, "r.json"), "-H", os.path.join(tmp, "r.html")]
            p = subprocess.run(cmd, capture_output=True, text=True, env=env)
            line = [l for l in p.stderr.splitlines() if "fqtool-amd:" in l]
            m = re.search(r"format ([0-9.]+) s", line[-1]) if line else None
            print(f"{v or 'text egress':40s} rc={p.returncode} format {m.group(1) if m else '?'} s   "
                  + (line[-1].split("ended:")[1][:200] if line and "ended:" in line[-1] else p.stderr[-300:]), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
