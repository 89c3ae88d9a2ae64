"""Debug helper (GPU box): run one golden e2e case through the session API twice -- CPU oracle and
HIP engine -- and report where the outputs and per-read records differ."""
import ctypes
import difflib
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import e2e_util as E  # noqa: E402
from fqtool_amd import abi  # noqa: E402
from oracle_lib import load_oracle  # noqa: E402


def main():
    case, mode = sys.argv[1], sys.argv[2]
    max_n = int(sys.argv[3]) if len(sys.argv) > 3 else 4000
    os.environ["FQ_ENGINE_GENERAL_ONLY"] = "1" if mode == "general" else "0"
    host = abi.load_host()
    eng = abi.load_engine()
    orc = load_oracle()
    recs = {"oracle": [], "engine": []}
    oproc = E.oracle_process(orc)

    def mk(tag):
        def process(p, b, nres, mc):
            if tag == "oracle":
                res, acc = oproc(p, b, nres, mc)
            else:
                if os.environ.get("FQ_DBG_IDX") and not recs[tag]:
                    p.reserved[1] = int(os.environ["FQ_DBG_IDX"]) + 1
                h = ctypes.c_void_p()
                assert eng.fq_engine_create(ctypes.byref(p), 0, max(b.n, 1), b.stride, ctypes.byref(h)) == 0
                res = np.zeros(nres, dtype=np.dtype(abi.RESULT_DTYPE_FIELDS))
                assert eng.fq_engine_process(h, ctypes.byref(b), res.ctypes.data) == 0
                acc = np.zeros(eng.fq_engine_acc_words(h), np.uint64)
                assert eng.fq_engine_read_acc(h, acc.ctypes.data, acc.size) == 0
                eng.fq_engine_destroy(h)
            recs[tag].append((res.copy(), acc.copy()))
            return res, acc
        return process

    dirs = {}
    for tag in ("oracle", "engine"):
        d = tempfile.mkdtemp()
        dirs[tag] = d
        E.run_session(host, E.argv_for("fqtool", case, d), mk(tag), max_n=max_n)
    for k, ((ro, ao), (re_, ae)) in enumerate(zip(recs["oracle"], recs["engine"])):
        bo, be = ro.view(np.uint8), re_.view(np.uint8)
        if not np.array_equal(bo, be):
            bad = np.nonzero((bo != be).reshape(-1, 16).any(axis=1))[0]
            print("pack", k, "records differ at", bad[:10])
            for i in bad[:5]:
                print("  oracle", ro[i], "engine", re_[i])
        if not np.array_equal(ao, ae):
            print("pack", k, "acc differs at", np.nonzero(ao != ae)[0][:10])
    for f in sorted(os.listdir(dirs["oracle"])):
        a = open(os.path.join(dirs["oracle"], f), "rb").read()
        b = open(os.path.join(dirs["engine"], f), "rb").read() if os.path.exists(os.path.join(dirs["engine"], f)) else None
        if a != b:
            print("file", f, "differs", len(a), None if b is None else len(b))
            if b is not None and f.endswith(".fq"):
                da = a.decode(errors="replace").splitlines()
                db = b.decode(errors="replace").splitlines()
                for line in list(difflib.unified_diff(da, db, lineterm="", n=2))[:30]:
                    print("   ", line[:200])


if __name__ == "__main__":
    main()
