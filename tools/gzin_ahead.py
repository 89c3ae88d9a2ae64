#!/usr/bin/env python3
"""Profiling aid: the fqtool binary on two single-member gzip -6 FASTQ inputs (bench.py's e2e_gzin
shape: synthetic 2x150 pairs, bench.gzip_single_member), options -q -a --detect_pe_adapter -g,
outputs /dev/null, with FQ_PARGZ_AHEAD (chunks each inflater may decode ahead of the reader, per
thread) and OMP_NUM_THREADS (the tool gives each mate's inflater half of it) swept; runs alternate
between the settings.  --quals binned: pargz_speed's reads (4 binned quality values); gauss: qualities
clamp(N(36 - 0.06 i, 3), 2, 41) as SURVEY 8(d)'s generator (the bench's high-entropy case).  Prints
one JSON line per run.

    python tools/gzin_ahead.py [--pairs 10000000] [--ahead 2,6] [--omp 16] [--quals binned|gauss] [--repeat 3]
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def synth_gauss(path, reads, L=150, seed=7):
    import numpy as np
    rng = np.random.default_rng(seed)
    head = b"@SYN:1:1101:"
    step = 1 << 18
    mean = 36 - 0.06 * np.arange(L)
    with open(path, "wb") as f:
        for lo in range(0, reads, step):
            k = min(step, reads - lo)
            idx = np.arange(lo, lo + k)
            name = np.array([b"%s%05d:%07d 1:N:0:ACGTACGT\n" % (head, i % 100000, i // 100000) for i in idx])
            nl = len(name[0])
            rec = np.empty((k, nl + L + 3 + L + 1), np.uint8)
            rec[:, :nl] = np.frombuffer(b"".join(name), np.uint8).reshape(k, nl)
            rec[:, nl:nl + L] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, (k, L))]
            rec[:, nl + L:nl + L + 3] = np.frombuffer(b"\n+\n", np.uint8)
            q = np.clip(np.rint(rng.normal(mean, 3.0, (k, L))), 2, 41).astype(np.uint8) + 33
            rec[:, nl + L + 3:nl + 2 * L + 3] = q
            rec[:, -1] = 10
            f.write(rec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=10_000_000)
    ap.add_argument("--ahead", default="2,6")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--omp", default="16")
    ap.add_argument("--gz-threads", default="0", help="FQ_GZ_THREADS values (inflate threads per file; 0: half of OMP_NUM_THREADS)")
    ap.add_argument("--quals", default="binned", choices=["binned", "gauss"])
    a = ap.parse_args()
    import bench
    import pargz_speed
    tmp = tempfile.mkdtemp(prefix="gzin_")
    try:
        t0 = time.time()
        ins = []
        for m in range(2):
            fq = os.path.join(tmp, f"r{m + 1}.fq")
            if a.quals == "binned":
                pargz_speed.synth_fastq(fq, a.pairs, seed=11 + m)
            else:
                synth_gauss(fq, a.pairs, seed=11 + m)
            bench.gzip_single_member(fq, fq + ".gz")
            os.remove(fq)
            ins.append(fq + ".gz")
        print(json.dumps({"pairs": a.pairs, "quals": a.quals, "gz_GB": round(sum(os.path.getsize(p) for p in ins) / 1e9, 3),
                          "made_s": round(time.time() - t0, 1), "affinity_cpus": len(os.sched_getaffinity(0)),
                          "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}), flush=True)
        tool = os.path.join(REPO, "fqtool_amd", "bin", "fqtool")
        cmd = [tool, "-i", ins[0], "-I", ins[1], "-o", "/dev/null", "-O", "/dev/null", "-q", "-a", "--detect_pe_adapter",
               "-g", "-w", "16", "-J", os.path.join(tmp, "r.json"), "-H", os.path.join(tmp, "r.html")]
        subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)  # (warm-up)
        for rep in range(a.repeat):
            for ah, omp, gt in [(x, y, z) for x in a.ahead.split(",") for y in a.omp.split(",") for z in a.gz_threads.split(",")]:
                time.sleep(2.0)
                t0 = time.perf_counter()
                p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                                   env=dict(os.environ, FQ_PARGZ_AHEAD=ah, OMP_NUM_THREADS=omp, FQ_GZ_THREADS=gt))
                dt = time.perf_counter() - t0
                line = ([l for l in p.stderr.splitlines() if "fqtool-amd:" in l] or [""])[-1]

                def stamp(key):
                    mm = re.search(key + r" ([0-9.]+) s", line)
                    return float(mm.group(1)) if mm else None
                print(json.dumps({"ahead_per_thread": int(ah), "omp_num_threads": int(omp), "gz_threads": int(gt), "rep": rep, "rc": p.returncode, "wall_s": round(dt, 3),
                                  "Mreads_s": round(2 * a.pairs / dt / 1e6, 2), "first_pack_at_s": stamp("first pack submitted at"),
                                  "pipeline_done_at_s": stamp("pipeline done at"), "window_reads_s": stamp("window reads")}),
                      flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
