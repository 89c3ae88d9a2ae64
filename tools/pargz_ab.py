#!/usr/bin/env python3
"""Profiling aid: inflate speed of host-library builds side by side (variants of pargz.cpp built into
build/pargz_ab/<name>.so, e.g. other table sizes), each drained in its own process through
fqh_gz_drain on one gzip -6 file of SURVEY 8(d)-style reads (tools/gzin_ahead.synth_gauss), runs
alternating between the builds.  Prints one JSON line per run.

    python tools/pargz_ab.py [--reads 3000000] [--threads 1,16] [--repeat 3] [--builds base,lit10]
"""
import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def drain_child(lib, gz, threads):
    lib = ctypes.CDLL(lib)
    lib.fqh_gz_drain.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t,
                                 ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_double)]
    n, ok, sec = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_double()
    rc = lib.fqh_gz_drain(gz.encode(), 1 << 20, threads, 0, ctypes.byref(n), ctypes.byref(ok), ctypes.byref(sec))
    print(json.dumps({"rc": rc, "bytes": n.value, "ok": ok.value, "s": sec.value}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=3_000_000)
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--builds", default=None)
    ap.add_argument("--child", nargs=3, default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:
        drain_child(a.child[0], a.child[1], int(a.child[2]))
        return
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench
    import gzin_ahead
    libs = sorted(glob.glob(os.path.join(REPO, "build", "pargz_ab", "*.so")))
    if a.builds:
        libs = [os.path.join(REPO, "build", "pargz_ab", b + ".so") for b in a.builds.split(",")]
    tmp = tempfile.mkdtemp(prefix="pargzab_")
    fq, gz = os.path.join(tmp, "r.fq"), os.path.join(tmp, "r.fq.gz")
    gzin_ahead.synth_gauss(fq, a.reads)
    bench.gzip_single_member(fq, gz)
    text = os.path.getsize(fq)
    os.remove(fq)
    print(json.dumps({"reads": a.reads, "text_bytes": text, "gz_bytes": os.path.getsize(gz)}), flush=True)
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.join(REPO, "fqtool_amd", "lib"))
    try:
        for rep in range(a.repeat):
            for t in [int(x) for x in a.threads.split(",")]:
                for lib in libs:
                    p = subprocess.run([sys.executable, __file__, "--child", lib, gz, str(t)], capture_output=True, text=True,
                                       env=env, timeout=300)
                    r = json.loads(p.stdout.strip().splitlines()[-1])
                    print(json.dumps({"build": os.path.basename(lib)[:-3], "threads": t, "rep": rep,
                                      "ok": r["ok"] == 1 and r["bytes"] == text, "MB_s": round(text / r["s"] / 1e6, 1)}), flush=True)
    finally:
        os.remove(gz)
        os.rmdir(tmp)


if __name__ == "__main__":
    main()
