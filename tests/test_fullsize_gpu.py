"""Full-size parity: the HIP engine over tens of millions of HBM-resident synthetic pairs, every
result record and every accumulator word against the CPU restatement over the same pairs
(oracle run on a host thread pool, tests/sample_parity.py).

The batch sizes make every persistent workgroup walk thousands of tiles (long LDS accumulation
runs before the flush), and end in a ragged tile.  Reference semantics: the whole
processPairEnd / processSingleEnd loop body per pack (src/peprocessor.cpp:261-508,
src/seprocessor.cpp:290-388) and the end-of-run merge of the per-thread accumulators
(src/peprocessor.cpp:179-217).  Integer/byte work: bit-exact.
"""
import ctypes
import time

import numpy as np
import pytest

from fqtool_amd import abi
from batch_util import config
from sample_parity import check_sample, device_batch, engine_run, first_diff, host_copy, oracle_parallel

pytestmark = pytest.mark.gpu

STRIDE, L, SEED = 160, 150, 20261015


@pytest.fixture(scope="module")
def eng_lib():
    return abi.load_engine()


def synth_device(lib, torch, n, paired, first):
    dev = torch.device("cuda:0")
    planes = [torch.empty(abi.batch_bytes(n, STRIDE), dtype=torch.uint8, device=dev)
              for _ in range(4 if paired else 2)]
    lens = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2 if paired else 1)]
    b = device_batch(planes, lens, n, STRIDE, paired)
    assert lib.fq_synth_fill_device(ctypes.byref(b), SEED, first, L, None) == 0
    torch.cuda.synchronize()
    return planes, lens


@pytest.mark.parametrize("name,n", [("C2", 20_000_017), ("C3", 20_000_017), ("C3", 100_000_000), ("C4", 20_000_017),
                                    ("C5", 20_000_017), ("C3b", 20_000_021), ("PE_all", 4_000_005),
                                    ("PE_correct", 4_000_005), ("PE_correct_x", 4_000_005), ("PE_correct_merge", 4_000_005), ("PE_umi_merge", 4_000_005), ("PE_correct_front", 4_000_005), ("PE_correct_umi_merge", 4_000_005),
                                    ("PE_umi_x", 4_000_005)])
def test_fullsize_parity(eng_lib, oracle, name, n):
    import torch

    p = config(name, max_cycles=320 if name in ("C4", "PE_correct_merge", "PE_umi_merge", "PE_correct_umi_merge") else 256)
    paired = bool(p.paired)
    t0 = time.time()
    planes, lens = synth_device(eng_lib, torch, n, paired, first=3 * 10**9)
    # (inputs copied first: -c rewrites corrected bases and qualities in place, as the reference's
    # BaseCorrector does to its Read objects)
    hp, l1, l2 = host_copy(torch, planes, lens, paired)
    eres, eacc = engine_run(eng_lib, torch, p, planes, lens, n, STRIDE, paired, 0)
    got = eres.cpu().numpy().view(np.dtype(abi.RESULT_DTYPE_FIELDS))
    del planes, lens, eres
    torch.cuda.empty_cache()
    t1 = time.time()
    ores, oacc = oracle_parallel(oracle, p, hp, l1, l2, n, STRIDE)
    print(f"{name}: {n} {'pairs' if paired else 'reads'}; engine+copies {t1 - t0:.1f}s, oracle {time.time() - t1:.1f}s")
    nbad, i = first_diff(got, ores)
    assert nbad == 0, f"{nbad} records differ; first #{i}: oracle={ores[i]} engine={got[i]}"
    nbad, i = first_diff(eacc, oacc)
    assert nbad == 0, f"{nbad} accumulator words differ; first word {i}: oracle={oacc[i]} engine={eacc[i]}"
    # every read is counted once by FilterResult and once by the pre-filter Stats
    assert int(oacc[abi.FQ_ACC_FILTER:abi.FQ_ACC_FILTER + 32].sum()) == n * (2 if paired else 1)


def test_sample_checker_catches_a_wrong_record(eng_lib, oracle):
    """The bench's parity_sample leg over a 2 M-pair batch: green on the engine's own records,
    red once one sampled record is corrupted."""
    import torch

    p = config("C3", max_cycles=256)
    n = 2_000_003
    planes, lens = synth_device(eng_lib, torch, n, True, first=7 * 10**9)
    res, _ = engine_run(eng_lib, torch, p, planes, lens, n, STRIDE, True, 0)
    ok = check_sample(eng_lib, oracle, torch, p, planes, lens, res, n, STRIDE, 200_000)
    assert ok["ok"], ok
    assert ok["pairs"] >= 200_000
    res.view(-1, 32)[n - 1, 2] ^= 0x10  # last (ragged) tile, always sampled: read-1 record's code
    bad = check_sample(eng_lib, oracle, torch, p, planes, lens, res, n, STRIDE, 200_000)
    assert not bad["ok"] and not bad["full_run_records_equal"] and bad["sample_run_acc_equal"]
