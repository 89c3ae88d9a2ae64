"""The adapter-detection k-mer work on the GPU (fq_kmer_*, kmer.hip) against the CPU
restatement of Evaluator::evaluateAdapterSeq's loops (reference src/evaluator.cpp:265-279,
:392-405): identical 10-mer histograms and seed occurrence sets, on the reference's testdata
reads and on hostile reads (N, lowercase, IUPAC, reads shorter than the window range).
End to end, the detected adapters are checked by the td_pe_detect / synth_pe_c3 fixtures."""
import ctypes
import gzip
import os

import numpy as np
import pytest

from fqtool_amd import abi
from batch_util import edge_pack

pytestmark = pytest.mark.gpu
INPUTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "inputs")


@pytest.fixture(scope="module")
def eng_lib():
    return abi.load_engine()


def _testdata_reads():
    with gzip.open(os.path.join(INPUTS, "r2.fq.gz")) as f:
        lines = f.read().split(b"\n")
    return [lines[i] for i in range(1, len(lines), 4)]


def edge_reads():
    pk = edge_pack(4000, True, stride=176, seed=3)
    return [bytes(pk.seq1[i, :pk.len1[i]]) for i in range(pk.n)] + [bytes(pk.seq2[i, :pk.len2[i]]) for i in range(pk.n)]


def readset(reads):
    seq = np.frombuffer(b"".join(reads), np.uint8).copy()
    off = np.zeros(len(reads) + 1, np.uint32)
    off[1:] = np.cumsum([len(r) for r in reads])
    return seq, off


@pytest.mark.parametrize("source", ["testdata", "edge"])
@pytest.mark.parametrize("tail", [1, 4])
def test_kmer_histogram_and_seeds(eng_lib, oracle, source, tail):
    reads = _testdata_reads() if source == "testdata" else edge_reads()
    seq, off = readset(reads)
    n = len(reads)
    k, first = 10, 20
    g, o = ctypes.c_void_p(), ctypes.c_void_p()
    assert eng_lib.fq_kmer_open(0, seq.ctypes.data, off.ctypes.data, n, ctypes.byref(g)) == 0
    assert oracle.orc_kmer_open(0, seq.ctypes.data, off.ctypes.data, n, ctypes.byref(o)) == 0
    try:
        cg = np.zeros(1 << 20, np.uint32)
        co = np.zeros(1 << 20, np.uint32)
        assert eng_lib.fq_kmer_count(g, k, first, tail, cg.ctypes.data) == 0
        assert oracle.orc_kmer_count(o, k, first, tail, co.ctypes.data) == 0
        assert co.sum() > 0 and np.array_equal(cg, co)
        for seed in list(np.argsort(co)[-5:]) + [0, 12345]:
            cap = int(co[seed])
            og, oo = np.zeros(cap + 1, np.uint64), np.zeros(cap + 1, np.uint64)
            ng, no = ctypes.c_size_t(), ctypes.c_size_t()
            assert eng_lib.fq_kmer_find(g, k, first, tail, int(seed), og.ctypes.data, cap + 1, ctypes.byref(ng)) == 0
            assert oracle.orc_kmer_find(o, k, first, tail, int(seed), oo.ctypes.data, cap + 1, ctypes.byref(no)) == 0
            assert ng.value == no.value == cap
            assert np.array_equal(np.sort(og[:cap]), np.sort(oo[:cap]))
    finally:
        eng_lib.fq_kmer_close(g)
        oracle.orc_kmer_close(o)
