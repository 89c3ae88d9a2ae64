#!/usr/bin/env python3
"""Inflate speed of one single-member gzip FASTQ file: zlib's gzread in the reference's 1 MiB
calls (one thread) against the parallel inflater (fqtool_amd/host/pargz.cpp) on 1..N threads,
through the host library's speed probe (fqh_gz_drain: 1 MiB calls into one buffer, discarded).  The file is
synthetic FASTQ in bench.py's record format (random bases, qualities from a skewed alphabet),
compressed by bench.gzip_single_member at level 6.

  python tools/pargz_speed.py [--reads N] [--threads 1,4,8,16] [--out JSON]"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def synth_fastq(path, reads, L=150, seed=7):
    import numpy as np
    rng = np.random.default_rng(seed)
    head = b"@SYN:1:1101:"
    step = 1 << 18
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
            q = np.frombuffer(b"F:,#", np.uint8)[rng.choice(4, (k, L), p=[0.80, 0.12, 0.06, 0.02])]
            rec[:, nl + L + 3:nl + 2 * L + 3] = q
            rec[:, -1] = 10
            f.write(rec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=4_000_000)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    lib = ctypes.CDLL(os.path.join(REPO, "fqtool_amd", "lib", "libfqhost.so"))
    lib.fqh_gz_drain.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t,
                                 ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_double)]

    def drain(path, threads):
        n, ok, sec = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_double()
        rc = lib.fqh_gz_drain(path.encode(), 1 << 20, threads, 0, ctypes.byref(n), ctypes.byref(ok), ctypes.byref(sec))
        return rc, n.value, ok.value, sec.value

    tmp = tempfile.mkdtemp(prefix="pargz_")
    src, gz = os.path.join(tmp, "r1.fq"), os.path.join(tmp, "r1.fq.gz")
    t0 = time.perf_counter()
    synth_fastq(src, a.reads)
    bench.gzip_single_member(src, gz)
    text = os.path.getsize(src)
    os.remove(src)
    res = {"reads": a.reads, "text_bytes": text, "gz_bytes": os.path.getsize(gz),
           "made_s": round(time.perf_counter() - t0, 1), "affinity_cpus": len(os.sched_getaffinity(0))}
    print(f"[pargz_speed] {a.reads} reads, {text / 1e9:.2f} GB text, {res['gz_bytes'] / 1e9:.2f} GB gzip", flush=True)
    rc, n, ok, dt = drain(gz, 0)
    assert rc == 0 and n == text and ok == 1, (rc, n, ok)
    res["zlib_gzread_MB_s"] = round(text / dt / 1e6, 1)
    print(f"[pargz_speed] zlib gzread: {text / dt / 1e6:.1f} MB/s", flush=True)
    for t in [int(x) for x in a.threads.split(",")]:
        rc, n, ok, dt = drain(gz, t)
        assert rc == 1 and n == text and ok == 1, (rc, n, ok)
        res[f"pargz_{t}t_MB_s"] = round(text / dt / 1e6, 1)
        res[f"pargz_{t}t_Mreads_s"] = round(a.reads / dt / 1e6, 2)
        print(f"[pargz_speed] parallel, {t} threads: {text / dt / 1e6:.1f} MB/s ({a.reads / dt / 1e6:.2f} Mreads/s)",
              flush=True)
    os.remove(gz)
    os.rmdir(tmp)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
