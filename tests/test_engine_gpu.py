"""Parity of the HIP engine (libfqengine.so, through its C-ABI) with the CPU restatement.

Every per-read result record and every accumulator word must be identical (integer/byte
work: bit-exact, no tolerance).  Runs on the MI355X box only (`-m gpu`).
"""
import ctypes

import numpy as np
import pytest

from fqtool_amd import abi
from batch_util import (AD1, AD2, ALL_CONFIGS, Pack, adapter_pack, config, edge_pack, polyx_pack, polyx_params, run_oracle,
                        synth_pack)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng_lib():
    return abi.load_engine()


@pytest.fixture(params=["fast", "general"])
def mode(request, monkeypatch):
    """Run each parity case through the default dispatch (gfx950 fast kernels, handing single
    pairs / reads to the general kernel) and through the general kernel only."""
    monkeypatch.setenv("FQ_ENGINE_GENERAL_ONLY", "1" if request.param == "general" else "0")
    return request.param


def make_engine(lib, p, max_batch=8192, max_stride=160):
    h = ctypes.c_void_p()
    rc = lib.fq_engine_create(ctypes.byref(p), 0, max_batch, max_stride, ctypes.byref(h))
    assert rc == 0, lib.fq_engine_last_error(None)
    return h


def run_engine(lib, p, pk):
    h = make_engine(lib, p, max_batch=max(pk.n, 1), max_stride=pk.stride)
    try:
        res = pk.result_array()
        b = pk.batch()
        rc = lib.fq_engine_process(h, ctypes.byref(b), res.ctypes.data)
        assert rc == 0, lib.fq_engine_last_error(h)
        acc = np.zeros(lib.fq_engine_acc_words(h), np.uint64)
        rc = lib.fq_engine_read_acc(h, acc.ctypes.data, acc.size)
        assert rc == 0, lib.fq_engine_last_error(h)
        return res, acc
    finally:
        lib.fq_engine_destroy(h)


def assert_same(p, res_o, acc_o, res_e, acc_e):
    if not np.array_equal(res_o, res_e):
        bad = np.nonzero(res_o != res_e)[0]
        i = int(bad[0])
        raise AssertionError(f"{len(bad)} result records differ; first #{i}: oracle={res_o[i]} engine={res_e[i]}")
    if not np.array_equal(acc_o, acc_e):
        bad = np.nonzero(acc_o != acc_e)[0]
        raise AssertionError(f"{len(bad)} accumulator words differ; first idx {bad[:8]}: "
                             f"oracle={acc_o[bad[:8]]} engine={acc_e[bad[:8]]}")


@pytest.mark.parametrize("name", ALL_CONFIGS)
def test_synthetic_parity(eng_lib, oracle, name, mode):
    p = config(name, max_cycles=512)
    pk = synth_pack(oracle, 6000, bool(p.paired), first=12345)
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("paired", [True, False])
@pytest.mark.parametrize("mask,max_mm,per,req", [(0b11111, 5, 8, 10), (0b01101, 5, 8, 10), (0b10000, 2, 3, 6),
                                                 (0b00001, 1, 1, 3), (0b01111, 0, 8, 10), (0b00000, 5, 8, 1),
                                                 (0b01111, 5, 20, 16)])
def test_polyx_tails(eng_lib, oracle, paired, mask, max_mm, per, req):
    """The fast kernels decide most polyX scans on the code column (polyx_no_trim) and run the
    scalar restatement for the rest: both against the oracle on homopolymer tails."""
    p = polyx_params(paired, mask, max_mm, per, req)
    pk = polyx_pack(4000, paired, seed=mask * 131 + max_mm * 7 + per + req)
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("stride", [160, 336])
@pytest.mark.parametrize("ads", [(AD1, AD2), (AD1[:20], AD2[:21]), (AD1[:19], AD2[:16]),
                                 ("AGATCGGAAGAGCNCACGTCTG", "agatcggaagagcgtcgtgtag"), (AD1 + AD2, AD2[:8])])
@pytest.mark.parametrize("name", ["C3b", "SE_adapter", "PE_correct_x", "PE_merge_q"])
def test_adapter_by_sequence(eng_lib, oracle, name, ads, stride):
    """trimBySequence at every offset kind (adapter_pack) with adapters the fast kernels filter
    on the code columns (>= 20 upper-case ACGT bytes) and ones they search byte by byte (shorter,
    with an N, lower case), on both column builds."""
    p = config(name, max_cycles=512)
    abi.set_adapter(p, 1, ads[0])
    if p.paired:
        abi.set_adapter(p, 2, ads[1])
    pk = adapter_pack(5003, bool(p.paired), ads[0], ads[1], stride=stride, seed=len(ads[0]) * 7 + len(ads[1]) + stride)
    res_o, acc_o = run_oracle(oracle, p, pk)
    flags = res_o["flags"]
    assert ((flags & abi.FQ_RF_AD_SEQ) != 0).sum() > pk.n // 20
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("name", ALL_CONFIGS)
def test_edge_case_parity(eng_lib, oracle, name, mode):
    p = config(name, max_cycles=512)
    pk = edge_pack(3000, bool(p.paired), seed=hash(name) & 0xFFFF)
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("name", ["C3", "C3b", "C4", "C5", "PE_all", "C2", "SE_all"])
def test_mixed_fast_and_handoff_tiles(eng_lib, oracle, name):
    """Mostly clean synthetic tiles plus scattered tiles with IUPAC bases, quality bytes >= 128
    and over-long reads: the fast kernel hands those pairs to the general kernel."""
    p = config(name, max_cycles=512)
    paired = bool(p.paired)
    n = 8001 if paired else 8033  # a ragged last tile
    pk = synth_pack(oracle, n, paired, first=555, stride=176)
    rng = np.random.default_rng(3)
    m2 = (pk.seq2, pk.qual2, pk.len2) if paired else (pk.seq1, pk.qual1, pk.len1)
    for i in rng.choice(n, 40, replace=False):
        kind = i % 3
        if kind == 0:
            pk.seq1[i, rng.integers(0, 150)] = ord("R")
        elif kind == 1:
            m2[1][i, rng.integers(0, 150)] = 200
        else:
            m2[0][i, 150:170] = ord("A")
            m2[1][i, 150:170] = ord("I")
            m2[2][i] = 170
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("stride", [160, 336])
@pytest.mark.parametrize("name", ["C3", "C4", "C5", "PE_all", "C2", "SE_all"])
def test_dense_per_pair_handoff(eng_lib, oracle, name, stride):
    """The fast kernels hand over single pairs (single-end: reads), not whole tiles: ~12 % of the
    pairs hold a lowercase base, an IUPAC code, a quality byte >= 128 or an over-long read in
    either mate or both, one whole tile goes over, and the last tile is ragged.  The pairs kept on
    the fast path share their tiles (and LDS statistics) with the handed-over ones.  Stride 160
    runs the 160-position build, stride 336 the 320-position build (reads of 330 bases go over)."""
    p = config(name, max_cycles=512)
    paired = bool(p.paired)
    n = 12_345
    pk = synth_pack(oracle, n, paired, first=97, stride=stride)
    rng = np.random.default_rng(29)
    mates = [(pk.seq1, pk.qual1, pk.len1)] + ([(pk.seq2, pk.qual2, pk.len2)] if paired else [])
    picks = rng.choice(n, n // 8, replace=False)
    picks = np.concatenate([picks, np.arange(64 * 3, 64 * 4)])  # one whole tile (both layouts)
    for k, i in enumerate(picks):
        which = [mates[k % len(mates)]] if k % 5 else mates  # every fifth: both mates
        for s, q, ln in which:
            kind = (k // 2) % 4
            if kind == 0:
                s[i, rng.integers(0, 150)] = ord("a") + 2 * (k % 3)  # a, c, e
            elif kind == 1:
                s[i, rng.integers(0, 150)] = ord("Y")
            elif kind == 2:
                q[i, rng.integers(0, 150)] = 129 + k % 100
            elif stride == 160:
                s[i, rng.integers(0, 150)] = ord("n")
            else:
                s[i, 150:330] = ord("G")
                q[i, 150:330] = ord("F")
                ln[i] = 330
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("stride", [160, 336])
@pytest.mark.parametrize("name", ["C3", "C3b", "C4", "C5", "PE_all", "PE_correct", "PE_correct_merge", "PE_umi_x", "C2",
                                  "SE_all"])
def test_lowercase_bases(eng_lib, oracle, name, stride):
    """Soft-masked reads: lowercase a c g t stay on the fast kernels (a per-base flag beside the
    codes) -- stretches anywhere in either mate, lowercase polyG / polyX tails, lowercase adapter
    copies, lowercase in the overlap of truly overlapping pairs -- next to a few hard bytes ('n',
    IUPAC) that still go to the general kernel.  Byte semantics as the reference: the reverse
    complement upper-cases them (src/seq.h:24-48), Stats buckets byte & 7 (src/stats.cpp:249),
    passFilter counts 'N' only, polyG/polyX/adapter/complexity compare bytes."""
    p = config(name, max_cycles=512)
    paired = bool(p.paired)
    n = 7001
    pk = synth_pack(oracle, n, paired, first=4242, stride=stride)
    rng = np.random.default_rng(41)
    mates = [(pk.seq1, pk.len1)] + ([(pk.seq2, pk.len2)] if paired else [])
    acgt = np.zeros(256, bool)
    acgt[[ord(c) for c in "ACGT"]] = True
    for m, (s, ln) in enumerate(mates):
        ad = (AD1 if m == 0 else AD2).lower().encode()
        for i in range(n):
            L = int(ln[i])
            u = rng.random()
            if u < 0.25:  # a stretch
                a = int(rng.integers(0, L))
                b = min(L, a + int(rng.integers(1, 61)))
            elif u < 0.32:  # the tail (polyG / polyX / adapter region)
                a, b = L - int(rng.integers(1, 31)), L
            elif u < 0.36 and L > 60:  # a lowercase adapter copy
                k = int(rng.integers(20, L - 10))
                t = ad[: L - k]
                s[i, k:k + len(t)] = np.frombuffer(t, np.uint8)
                continue
            elif u < 0.39:  # a lowercase polyG tail
                g = int(rng.integers(5, 40))
                s[i, max(0, L - g):L] = ord("g")
                continue
            elif u < 0.41:  # a hard byte: the pair goes over
                s[i, int(rng.integers(0, L))] = ord("n") if rng.random() < 0.5 else ord("R")
                continue
            else:
                continue
            a = max(a, 0)
            row = s[i, a:b]
            row[acgt[row]] |= 0x20
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("stride", [160, 336])
@pytest.mark.parametrize("name", ["C3", "C3b", "C4", "C5", "PE_all", "C2", "SE_all"])
def test_iupac_bases(eng_lib, oracle, name, stride):
    """IUPAC codes and other bytes outside ACGTN (R Y K M S W B D H V, 'n', 'X', '.') stay on the fast
    kernels (code 3 with the N bit and the flag bit beside the codes): anywhere in either mate,
    several per read, inside polyG tails and the overlap of truly overlapping pairs, next to
    lowercase bases.  Byte semantics as the reference: the reverse complement makes them 'N'
    (src/seq.h:24-48), Stats buckets byte & 7 (src/stats.cpp:249, classes 0, 2 and 5 included),
    passFilter counts only 'N' (src/filter.cpp:18), overlap / polyG / polyX / adapters compare
    bytes.  The merge variant and the low-complexity filter hand such pairs over."""
    p = config(name, max_cycles=512)
    paired = bool(p.paired)
    n = 6007
    pk = synth_pack(oracle, n, paired, first=777, stride=stride)
    rng = np.random.default_rng(53)
    mates = [(pk.seq1, pk.len1)] + ([(pk.seq2, pk.len2)] if paired else [])
    codes = np.frombuffer(b"RYKMSWBDHVnX.", np.uint8)
    for m, (s, ln) in enumerate(mates):
        for i in range(n):
            L = int(ln[i])
            u = rng.random()
            if u < 0.08:  # a few exotic bytes anywhere
                for _ in range(int(rng.integers(1, 4))):
                    s[i, int(rng.integers(0, L))] = codes[int(rng.integers(0, len(codes)))]
            elif u < 0.10:  # in the tail (polyG / polyX / adapter region)
                s[i, L - int(rng.integers(1, 20))] = codes[int(rng.integers(0, len(codes)))]
            elif u < 0.11:  # next to lowercase bases
                a = int(rng.integers(0, max(1, L - 20)))
                row = s[i, a:a + 20]
                row[np.isin(row, np.frombuffer(b"ACGT", np.uint8))] |= 0x20
                s[i, a + 10] = ord("R")
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("name", ["C3", "C2", "PE_correct", "PE_umi", "C4"])
def test_index_filtered_pairs(eng_lib, oracle, name, mode):
    """fq_batch.flags: pairs the host's index filter dropped count only in the pre-filter stats
    (src/peprocessor.cpp:283-286); the flags travel with the pack in both dispatch modes."""
    p = config(name, max_cycles=512)
    pk = synth_pack(oracle, 5000, bool(p.paired), first=4321)
    rng = np.random.default_rng(11)
    pk.flags = (rng.random(pk.n) < 0.2).astype(np.uint8) * abi.FQ_BF_INDEX_FILTERED
    res_o, acc_o = run_oracle(oracle, p, pk)
    mates = 2 if p.paired else 1
    assert ((res_o["flags"].reshape(-1, mates)[:, 0] & abi.FQ_RF_INDEX_FILTERED) != 0).sum() == int(pk.flags.astype(bool).sum())
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


def test_correction_counts(eng_lib, oracle):
    """-c on hostile reads corrects bases (the oracle is pinned to the reference by the
    td_pe_correct / edge_pe_correct e2e fixtures); the engine agrees on every record and word."""
    p = config("PE_correct", max_cycles=512)
    pk = edge_pack(6000, True, seed=99)
    res_o, acc_o = run_oracle(oracle, p, pk)
    tail = abi.acc_tail_offset(p.insert_size_max, p.max_cycles)
    assert acc_o[tail + abi.FQ_ACC_TAIL_CORRECTED_BASES] > 0
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


def test_empty_pack(eng_lib, oracle):
    p = config("C3", max_cycles=256)
    pk = Pack(0, 160, True)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert not acc_e.any()


def test_device_synth_matches_host(eng_lib, oracle):
    import torch

    n, stride, L = 5000, 160, 150
    dev = torch.device("cuda:0")
    bufs = [torch.zeros(abi.batch_bytes(n, stride), dtype=torch.uint8, device=dev) for _ in range(4)]
    lens = [torch.zeros(n, dtype=torch.int16, device=dev) for _ in range(2)]
    b = abi.FqBatch()
    b.n, b.stride = n, stride
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    assert eng_lib.fq_synth_fill_device(ctypes.byref(b), 20261015, 777, L, None) == 0
    torch.cuda.synchronize()
    pk = synth_pack(oracle, n, True, first=777, L=L, stride=stride)
    got = [abi.untile_rows(t.cpu().numpy(), n, stride)[:, :L] for t in bufs]
    exp = [pk.seq1[:, :L], pk.qual1[:, :L], pk.seq2[:, :L], pk.qual2[:, :L]]
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)
    assert (lens[0].cpu().numpy() == L).all() and (lens[1].cpu().numpy() == L).all()


def test_device_path_accumulates_like_host_path(eng_lib, oracle):
    """process_device on HBM-resident synthetic data == oracle on the same bytes, split over
    several launches (accumulation across calls)."""
    import torch

    p = config("C3", max_cycles=256)
    n, stride, L = 20000, 160, 150
    dev = torch.device("cuda:0")
    bufs = [torch.zeros(abi.batch_bytes(n, stride), dtype=torch.uint8, device=dev) for _ in range(4)]
    lens = [torch.zeros(n, dtype=torch.int16, device=dev) for _ in range(2)]
    res_d = torch.zeros(n * 2 * 16, dtype=torch.uint8, device=dev)
    b = abi.FqBatch()
    b.n, b.stride = n, stride
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    assert eng_lib.fq_synth_fill_device(ctypes.byref(b), 99, 0, L, None) == 0
    torch.cuda.synchronize()
    h = make_engine(eng_lib, p, max_batch=0, max_stride=0)
    try:
        half = n // 2 // abi.TILE_READS * abi.TILE_READS  # sub-batches start on a tile boundary
        for lo, hi in ((0, half), (half, n)):
            sub = abi.FqBatch()
            sub.n, sub.stride = hi - lo, stride
            sub.seq1, sub.qual1 = b.seq1 + lo * stride, b.qual1 + lo * stride
            sub.seq2, sub.qual2 = b.seq2 + lo * stride, b.qual2 + lo * stride
            sub.len1, sub.len2 = b.len1 + lo * 2, b.len2 + lo * 2
            assert eng_lib.fq_engine_process_device(h, ctypes.byref(sub), res_d.data_ptr() + lo * 32, None) == 0
        assert eng_lib.fq_engine_sync(h) == 0
        acc = np.zeros(eng_lib.fq_engine_acc_words(h), np.uint64)
        assert eng_lib.fq_engine_read_acc(h, acc.ctypes.data, acc.size) == 0
    finally:
        eng_lib.fq_engine_destroy(h)
    pk = synth_pack(oracle, n, True, seed=99, L=L, stride=stride)
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e = res_d.cpu().numpy().view(res_o.dtype)
    assert_same(p, res_o, acc_o, res_e, acc)


def test_too_long_read_is_rejected(eng_lib, oracle):
    p = config("C3", max_cycles=100)
    pk = synth_pack(oracle, 10, True)
    h = make_engine(eng_lib, p, max_batch=10, max_stride=160)
    try:
        res = pk.result_array()
        rc = eng_lib.fq_engine_process(h, ctypes.byref(pk.batch()), res.ctypes.data)
        assert rc == -4
    finally:
        eng_lib.fq_engine_destroy(h)


def test_null_mate_after_full_pairs(eng_lib, oracle, mode):
    """Regression: a pair whose read 2 is NULL must not see read 2 as present because the lane
    processed a full pair in its previous tile (the mate-presence shuffle once ran only in the
    lanes whose own read survived).  The first 2 tiles of every wave have both mates good, the
    rest have an all-N read 2 that cut_front trims to NULL."""
    p = config("PE_all", max_cycles=512)
    p.cut_front = 1
    n = 32 * 4096 * 3
    pk = synth_pack(oracle, n, True, first=777)
    bad = slice(32 * 4096, None)
    pk.seq2[bad, :150] = ord("N")
    pk.qual2[bad, :150] = ord("#")
    res_o, acc_o = run_oracle(oracle, p, pk)
    assert (res_o["flags"][1::2][32 * 4096:] & abi.FQ_RF_NULL).all()
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


def test_async_submit_poll_pipeline(eng_lib, oracle):
    """fq_engine_submit / fq_engine_poll: more packs than pipeline slots, pinned and pageable
    host buffers, an empty pack and a ragged one; packs come back in submission order with the
    oracle's records, and the accumulator is the sum over all packs (the reference's per-worker
    accumulation over disjoint packs, src/peprocessor.cpp:546-566)."""
    p = config("C3b", max_cycles=256)
    sizes = [5000, 0, 4097, 31, 6000, 1, 5000]
    packs = [synth_pack(oracle, n, True, first=100_000 * k) for k, n in enumerate(sizes)]
    h = make_engine(eng_lib, p, max_batch=max(sizes), max_stride=160)
    pinned = []
    try:
        outs, batches = [], []
        for k, pk in enumerate(packs):
            if k % 2 == 0:  # page-locked records
                ptr = ctypes.c_void_p()
                nbytes = max(1, pk.n * 2 * 16)
                assert eng_lib.fq_host_alloc(nbytes, ctypes.byref(ptr)) == 0
                pinned.append(ptr)
                buf = (ctypes.c_uint8 * nbytes).from_address(ptr.value)
                res = np.frombuffer(buf, dtype=np.dtype(abi.RESULT_DTYPE_FIELDS), count=pk.n * 2)
            else:
                res = pk.result_array()
            outs.append(res)
            batches.append(pk.batch())
        got = []
        for k, pk in enumerate(packs):
            assert eng_lib.fq_engine_submit(h, ctypes.byref(batches[k]), outs[k].ctypes.data if outs[k].size else
                                            ctypes.addressof(ctypes.c_uint8()), 1000 + k) == 0, \
                eng_lib.fq_engine_last_error(h)
            seq = ctypes.c_uint64()
            if eng_lib.fq_engine_poll(h, 0, ctypes.byref(seq)) == 1:
                got.append(seq.value)
        res_dummy = packs[0].result_array()
        assert eng_lib.fq_engine_process(h, ctypes.byref(batches[0]), res_dummy.ctypes.data) != 0  # packs pending
        while eng_lib.fq_engine_pending(h) > 0:
            seq = ctypes.c_uint64()
            assert eng_lib.fq_engine_poll(h, 1, ctypes.byref(seq)) == 1
            got.append(seq.value)
        assert got == [1000 + k for k in range(len(packs))]
        assert eng_lib.fq_engine_poll(h, 1, None) == 0
        acc = np.zeros(eng_lib.fq_engine_acc_words(h), np.uint64)
        assert eng_lib.fq_engine_read_acc(h, acc.ctypes.data, acc.size) == 0
        want_acc = np.zeros_like(acc)
        for k, pk in enumerate(packs):
            res_o, acc_o = run_oracle(oracle, p, pk)
            assert np.array_equal(outs[k], res_o), f"pack {k}"
            want_acc += acc_o
        assert np.array_equal(acc, want_acc)
    finally:
        eng_lib.fq_engine_destroy(h)
        for ptr in pinned:
            eng_lib.fq_host_free(ptr)


@pytest.mark.parametrize("name", ALL_CONFIGS)
@pytest.mark.parametrize("L,stride", [(250, 256), (300, 304)])
def test_long_read_parity(eng_lib, oracle, name, L, stride):
    """2x250 / 2x300 rows run on the 320-position build of the fast kernels (pe_fast_long.hip;
    -m on its 4-wave merge variant)."""
    p = config(name, max_cycles=640)
    pk = synth_pack(oracle, 3000, bool(p.paired), first=777, L=L, stride=stride)
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)


@pytest.mark.parametrize("name", ALL_CONFIGS)
@pytest.mark.parametrize("stride", [320, 336])
def test_long_edge_parity(eng_lib, oracle, name, stride, mode):
    """Ragged/hostile reads up to the row stride: tiles with a read beyond 320 bp (stride 336) are
    handed to the general kernel by the long build."""
    p = config(name, max_cycles=704)
    pk = edge_pack(2000, bool(p.paired), stride=stride, seed=(hash(name) + stride) & 0xFFFF)
    res_o, acc_o = run_oracle(oracle, p, pk)
    res_e, acc_e = run_engine(eng_lib, p, pk)
    assert_same(p, res_o, acc_o, res_e, acc_e)
