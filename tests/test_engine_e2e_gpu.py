"""The HIP engine against the CPU oracle on every end-to-end golden input and command line
(tests/golden/e2e): the packs the tool builds from the real FASTQ files, with the engine
parameters the tool derives from each command line, in both dispatch modes (gfx950 fast
kernels with per-tile hand-off, and the general kernel only).  Per-read records and every
accumulator word must be identical; a mismatch reports the read it happened on."""
import ctypes
import os

import numpy as np
import pytest

import e2e_util as E
from fqtool_amd import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def host():
    return abi.load_host()


@pytest.fixture(scope="module")
def eng():
    return abi.load_engine()


def engine_vs_oracle(eng, orc, mode):
    oracle_process = E.oracle_process(orc)

    def process(p, b, nres, mc):
        res_o, acc_o = oracle_process(p, b, nres, mc)
        os.environ["FQ_ENGINE_GENERAL_ONLY"] = "1" if mode == "general" else "0"
        h = ctypes.c_void_p()
        rc = eng.fq_engine_create(ctypes.byref(p), 0, max(b.n, 1), b.stride, ctypes.byref(h))
        assert rc == 0, eng.fq_engine_last_error(None)
        try:
            res_e = np.zeros_like(res_o)
            assert eng.fq_engine_process(h, ctypes.byref(b), res_e.ctypes.data) == 0, eng.fq_engine_last_error(h)
            acc_e = np.zeros(eng.fq_engine_acc_words(h), np.uint64)
            assert eng.fq_engine_read_acc(h, acc_e.ctypes.data, acc_e.size) == 0
        finally:
            eng.fq_engine_destroy(h)
        if not np.array_equal(res_o, res_e):
            bad = np.nonzero(res_o != res_e)[0]
            i = int(bad[0])
            mates = 2 if b.seq2 else 1
            pair, mate = divmod(i, mates)
            lens = [ctypes.cast(b.len1, ctypes.POINTER(ctypes.c_uint16))[pair]]
            if mates == 2:
                lens.append(ctypes.cast(b.len2, ctypes.POINTER(ctypes.c_uint16))[pair])
            rows = [E.read_row(b, m, pair, lens[m]) for m in range(mates)]
            raise AssertionError(f"{len(bad)} records differ; first record {i} (pair {pair} mate {mate}): "
                                 f"oracle={res_o[i]} engine={res_e[i]} "
                                 f"mate-records oracle={res_o[pair*mates:pair*mates+mates]} "
                                 f"engine={res_e[pair*mates:pair*mates+mates]} reads={rows}")
        if not np.array_equal(acc_o, acc_e):
            bad = np.nonzero(acc_o != acc_e)[0]
            raise AssertionError(f"{len(bad)} accumulator words differ; first {bad[:8]}: "
                                 f"oracle={acc_o[bad[:8]]} engine={acc_e[bad[:8]]}")
        return res_e, acc_e
    return process


@pytest.mark.parametrize("mode", ["fast", "general"])
@pytest.mark.parametrize("case", E.ok_cases())
def test_engine_matches_oracle_on_golden_inputs(case, mode, host, eng, oracle, tmp_path):
    try:
        report = E.run_session(host, E.argv_for("fqtool", case, str(tmp_path)), engine_vs_oracle(eng, oracle, mode),
                               max_n=4000, dup_engine=lambda k: E.OracleDup(oracle, k))
    finally:
        os.environ.pop("FQ_ENGINE_GENERAL_ONLY", None)
    E.check_outputs(case, str(tmp_path), report)
