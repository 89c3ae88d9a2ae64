#!/usr/bin/env python3
"""Profiling aid: stage timing of the adapter-detection pre-pass (host/evaluator.cpp) on a
synthetic C3 FASTQ pair of PAIRS pairs.  FQH_DETECT_TIMING=1 makes detect_adapter print its
stage times.  On the CPU (no GPU) the k-mer work runs on the oracle backend (tests/e2e_util.py),
so only the host stages are meaningful there; on the GPU box it uses fq_kmer_* (kmer.hip).
  python3 tools/detect_timing.py [--cpu]"""
import ctypes, os, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import numpy as np
from fqtool_amd import abi


def write_pair(oracle, n, d):
    from batch_util import synth_pack
    paths = [os.path.join(d, "r1.fq"), os.path.join(d, "r2.fq")]
    step = 1 << 16
    with open(paths[0], "wb") as f1, open(paths[1], "wb") as f2:
        for lo in range(0, n, step):
            k = min(step, n - lo)
            pk = synth_pack(oracle, k, True, first=lo)
            for m, f in ((1, f1), (2, f2)):
                seq, qual, ln = getattr(pk, "seq%d" % m), getattr(pk, "qual%d" % m), getattr(pk, "len%d" % m)
                out = []
                for i in range(k):
                    L = int(ln[i])
                    out.append(b"@r%d %d:N\n" % (lo + i, m) + seq[i, :L].tobytes() + b"\n+\n" + qual[i, :L].tobytes() + b"\n")
                f.write(b"".join(out))
    return paths


def main():
    from oracle_lib import load_oracle
    import e2e_util as E
    oracle = load_oracle()
    n = int(os.environ.get("PAIRS", 300000))
    d = tempfile.mkdtemp(prefix="fqdet_")
    t0 = time.time()
    paths = write_pair(oracle, n, d)
    print(f"wrote {n} pairs in {time.time() - t0:.1f}s", file=sys.stderr)
    host = abi.load_host()
    if "--cpu" in sys.argv:
        be = E.oracle_kmer_backend(oracle)
        host.fqh_set_kmer_backend(ctypes.addressof(be))
    os.environ["FQH_DETECT_TIMING"] = "1"
    buf = ctypes.create_string_buffer(256)
    for p in paths:
        t0 = time.time()
        rc = host.fqh_detect_adapter(p.encode(), 0, buf, 256)
        print(f"{os.path.basename(p)}: rc {rc} adapter {buf.value.decode()!r} {time.time() - t0:.3f}s", flush=True)


if __name__ == "__main__":
    main()
