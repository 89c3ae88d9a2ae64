#!/usr/bin/env python3
"""Profiling aid: the host feed's ceiling -- how fast the fqtool binary's host side (window reader
pread into staging, one thread per engine with RawMulti's ordered enqueue / launch, the formatter
hand-off, the writers) moves plain FASTQ when its G engines cost nothing (tools/micro/null_engine.cpp,
loaded through LD_LIBRARY_PATH in place of the GPU engine).  No GPU is used; run it on the GPU box's
host to measure that box's cores and page cache.

    python tools/host_feed.py [--pairs 20000000] [--engines 1,2,4,8] [--workers 16] [--out null|file]

Options -q -g (no -a: the adapter detection pre-pass needs the GPU).  Input: fixed-width synthetic records (326 bytes per read: a 20-byte name, 150 bp), repeated blocks,
written once to a temp directory (page cache).  Prints one JSON line per run: wall, input GB/s,
Mreads/s, and the tool's own stage times (window reads, reader waiting for a stage, pipeline done).
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
READ_LEN = 150
NAME_LEN = 20
REC = 1 + NAME_LEN + 1 + READ_LEN + 1 + 2 + READ_LEN + 1  # '@' name '\n' seq '\n' '+\n' qual '\n'


def build_null_engine():
    out = os.path.join(REPO, "build", "nullhost")
    os.makedirs(out, exist_ok=True)
    lib = os.path.join(out, "libfqengine.so")
    src = os.path.join(REPO, "tools", "micro", "null_engine.cpp")
    if not os.path.exists(lib) or os.path.getmtime(lib) < os.path.getmtime(src):
        subprocess.run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-I" + os.path.join(REPO, "include"), "-o", lib, src],
                       check=True)
    return out


def write_fastq(path, pairs, mate):
    """fixed-width records from one repeated 4096-record block (the null engine reads nothing)"""
    import random
    rnd = random.Random(12345 + mate)
    blk = []
    for i in range(4096):
        seq = "".join(rnd.choice("ACGT") for _ in range(READ_LEN))
        qual = "".join(chr(33 + rnd.randrange(2, 41)) for _ in range(READ_LEN))
        blk.append(f"@r{i:0{NAME_LEN - 1}d}\n{seq}\n+\n{qual}\n")
    block = "".join(blk).encode()
    assert len(block) == 4096 * REC
    with open(path, "wb") as f:
        full, rest = divmod(pairs, 4096)
        big = block * 16
        for _ in range(full // 16):
            f.write(big)
        for _ in range(full % 16):
            f.write(block)
        f.write(block[:rest * REC])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=20_000_000)
    ap.add_argument("--engines", default="1,2,4,8")
    ap.add_argument("--workers", default="16", help="comma list of -w values")
    ap.add_argument("--out", default="null", choices=["null", "file"])
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--egress", default="text", help="comma list: text (engine output text), host (records-only, "
                    "byte ranges), hostcopy (records-only, copied); host* run on one engine only")
    args = ap.parse_args()
    libdir = build_null_engine()
    tool = os.path.join(REPO, "fqtool_amd", "bin", "fqtool")
    tmp = tempfile.mkdtemp(prefix="fqfeed_")
    try:
        t0 = time.time()
        ins = [os.path.join(tmp, "r1.fq"), os.path.join(tmp, "r2.fq")]
        for m, p in enumerate(ins):
            write_fastq(p, args.pairs, m)
        gb = 2 * args.pairs * REC / 1e9
        print(json.dumps({"input_GB": round(gb, 3), "pairs": args.pairs, "written_s": round(time.time() - t0, 1),
                          "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
                          "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}), flush=True)
        env = dict(os.environ, LD_LIBRARY_PATH=libdir, FQ_NULL_REC1=str(REC), FQ_NULL_REC2=str(REC), FQ_NULL_LEN=str(READ_LEN),
                   FQ_TIMING_MONO="1")
        runs = []
        for eg in args.egress.split(","):
            for w in [int(x) for x in args.workers.split(",")]:
                for g in [int(x) for x in args.engines.split(",")]:
                    if eg == "text" or g == 1:
                        runs.append((eg, w, g))
        for eg, w, g in runs:
                env_run = dict(env)
                if eg != "text":
                    env_run.update(FQ_RAW_EGRESS="host", FQ_RAW_ZC="1" if eg == "host" else "0")
                outs = ["/dev/null", "/dev/null"] if args.out == "null" else [os.path.join(tmp, "o1.fq"), os.path.join(tmp, "o2.fq")]
                cmd = [tool, "-i", ins[0], "-I", ins[1], "-o", outs[0], "-O", outs[1], "-q", "-g", "-w", str(w),
                       "--devices", ",".join(["0"] * g), "-J", os.path.join(tmp, "r.json"), "-H", os.path.join(tmp, "r.html")]
                for rep in range(args.repeat):
                    time.sleep(1.0)
                    t0 = time.monotonic()  # (CLOCK_MONOTONIC, as the tool's steady_clock stamps)
                    p = subprocess.run(cmd, capture_output=True, text=True, env=env_run)
                    t1 = time.monotonic()
                    dt = t1 - t0
                    if p.returncode != 0:
                        print(json.dumps({"engines": g, "workers": w, "error": p.stderr[-1500:]}), flush=True)
                        break
                    log = [l for l in p.stderr.splitlines() if "fqtool-amd:" in l]
                    mono = [l for l in p.stderr.splitlines() if "fqtool-amd mono:" in l]
                    line = log[-1] if log else ""
                    mm = re.search(r"t0 ([0-9.]+) end ([0-9.]+)", mono[-1]) if mono else None
                    # process start -> the pipeline's t0 (exec, engines' libraries), and the last log line
                    # -> the process reaped (the exit's unmapping of windows and packs)
                    before_t0 = round(float(mm.group(1)) - t0, 3) if mm else None
                    after_end = round(t1 - float(mm.group(2)), 3) if mm else None
                    def stamp(key):
                        mm = re.search(key + r" ([0-9.]+) s", line)
                        return float(mm.group(1)) if mm else None
                    print(json.dumps({"engines": g, "workers": w, "out": args.out, "egress": eg, "rep": rep, "wall_s": round(dt, 3),
                                      "input_GB_s": round(gb / dt, 2), "Mreads_s": round(2 * args.pairs / dt / 1e6, 1),
                                      "window_reads_s": stamp("window reads"),
                                      "reader_waiting_for_stage_s": stamp("reader waiting for a stage"),
                                      "pipeline_done_at_s": stamp("pipeline done at"),
                                      "first_pack_at_s": stamp("first pack submitted at"),
                                      "format_s": stamp("format"),
                                      "engines_ready_at_s": stamp("engines ready at"),
                                      "start_to_t0_s": before_t0, "log_to_exit_s": after_end,
                                      "path": "raw stream on %d engines" % g if "raw stream on" in line else
                                              ("raw stream" if "raw stream" in line else "other")}), flush=True)
                    for f in outs:
                        if f != "/dev/null" and os.path.exists(f):
                            os.remove(f)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
