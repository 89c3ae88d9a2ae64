"""Duplication analysis (-d) on the GPU (fq_dup_*, dup.hip) against the CPU restatement of
Duplicate (reference src/duplicate.cpp:46-166), which the -d e2e fixtures pin to the reference.

Bit-exact: the statAll histogram, GC sums and totals must be identical.  Covers several packs
in order (the per-key state carries across packs), duplicated pairs inside one pack (the sort +
per-key walk), reads too short / with N (skipped), SE and PE, and two tables fed interleaved
packs then merged (the multi-engine path of the tool)."""
import ctypes

import numpy as np
import pytest

from fqtool_amd import abi
from batch_util import Pack, config, edge_pack, synth_pack

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng_lib():
    return abi.load_engine()


def with_duplicates(pk, rng, frac=0.3):
    """Copy the key bases / 32-mer of earlier reads into later ones, with some variation."""
    n = pk.n
    for i in rng.choice(np.arange(1, n), int(n * frac), replace=False):
        j = int(rng.integers(0, i))
        pk.seq1[i, :16] = pk.seq1[j, :16]
        if pk.paired:
            if rng.random() < 0.7:
                pk.seq2[i, :32] = pk.seq2[j, :32]
        elif rng.random() < 0.7:
            L = int(pk.len1[i])
            Lj = int(pk.len1[j])
            if L >= 37 and Lj >= 37:
                pk.seq1[i, L - 37:L - 5] = pk.seq1[j, Lj - 37:Lj - 5]
    return pk


def oracle_stat(oracle, packs, paired, keylen, hist_size):
    d = oracle.orc_dup_create(keylen)
    try:
        for pk in packs:
            oracle.orc_dup_add_batch(d, ctypes.byref(pk.batch()), int(paired))
        hist, gcs, tot = np.zeros(hist_size, np.uint64), np.zeros(hist_size, np.uint64), np.zeros(2, np.uint64)
        oracle.orc_dup_stat(d, hist_size, hist.ctypes.data, gcs.ctypes.data, tot.ctypes.data)
        return hist, gcs, tot
    finally:
        oracle.orc_dup_destroy(d)


def engine_stat(lib, packs, p, keylen, hist_size, n_tables=1):
    """Packs dealt round-robin over n_tables engines, each with its own table; tables merged."""
    dups, engines = [], []
    try:
        for _ in range(n_tables):
            d = ctypes.c_void_p()
            assert lib.fq_dup_create(0, keylen, ctypes.byref(d)) == 0
            dups.append(d)
            h = ctypes.c_void_p()
            assert lib.fq_engine_create(ctypes.byref(p), 0, max(pk.n for pk in packs), 160, ctypes.byref(h)) == 0
            engines.append(h)
            assert lib.fq_engine_set_dup(h, d) == 0
        for k, pk in enumerate(packs):
            h = engines[k % n_tables]
            res = pk.result_array()
            assert lib.fq_engine_submit(h, ctypes.byref(pk.batch()), res.ctypes.data, k) == 0, lib.fq_engine_last_error(h)
            assert lib.fq_engine_poll(h, 1, None) == 1
        for d in dups[1:]:
            assert lib.fq_dup_merge(dups[0], d) == 0
        hist, gcs, tot = np.zeros(hist_size, np.uint64), np.zeros(hist_size, np.uint64), np.zeros(2, np.uint64)
        assert lib.fq_dup_stat(dups[0], hist_size, hist.ctypes.data, gcs.ctypes.data, tot.ctypes.data) == 0
        return hist, gcs, tot
    finally:
        for h in engines:
            lib.fq_engine_destroy(h)
        for d in dups:
            lib.fq_dup_destroy(d)


def check(a, b):
    for x, y, what in zip(a, b, ("histogram", "GC sums", "totals")):
        assert np.array_equal(x, y), "%s differ: oracle %s engine %s" % (what, x[:12], y[:12])


@pytest.mark.parametrize("paired", [True, False])
@pytest.mark.parametrize("n_tables", [1, 3])
def test_dup_synthetic_packs(eng_lib, oracle, paired, n_tables):
    rng = np.random.default_rng(5)
    packs = [with_duplicates(synth_pack(oracle, 3000 + 17 * k, paired, first=9000 * k), rng) for k in range(5)]
    p = config("C3" if paired else "C2", max_cycles=256)
    want = oracle_stat(oracle, packs, paired, 12, 32)
    assert want[0][2:].sum() > 0  # some keys counted more than once
    check(want, engine_stat(eng_lib, packs, p, 12, 32, n_tables))


@pytest.mark.parametrize("keylen,hist_size", [(12, 2), (13, 8), (15, 5)])
def test_dup_edge_packs(eng_lib, oracle, keylen, hist_size):
    rng = np.random.default_rng(keylen)
    packs = [with_duplicates(edge_pack(2500, True, seed=31 + k), rng, 0.5) for k in range(3)]
    p = config("C3", max_cycles=256)
    want = oracle_stat(oracle, packs, True, keylen, hist_size)
    check(want, engine_stat(eng_lib, packs, p, keylen, hist_size, 2))
