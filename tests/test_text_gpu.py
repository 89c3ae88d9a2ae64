"""FASTQ-text packs (fq_engine_submit_text: GPU-side ingest and egress) against the oracle.

The engine builds the batch planes from the FASTQ bytes and writes the output FASTQ of the
records that pass; its per-read records and accumulator must equal the oracle's on the same
pack, and its output text must equal Read::toString of every passing record (both mates of a
passing pair for PE), in input order (src/read.h:166-168, src/peprocessor.cpp:402-403,
src/seprocessor.cpp:337-350).  Records carry CRLF terminators, named strand lines and ragged
lengths so the per-record offsets of the index are exercised."""
import ctypes
import random

import numpy as np
import pytest

from batch_util import config, edge_pack, run_oracle, synth_pack
from fqtool_amd import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    return abi.load_engine()


def fastq_text(pk, mate, rng):
    """The pack's reads of one mate as FASTQ bytes + fq_text_rec index + the expected record parts."""
    seqs, quals, lens = getattr(pk, "seq%d" % mate), getattr(pk, "qual%d" % mate), getattr(pk, "len%d" % mate)
    parts, recs, names, strands = [], [], [], []
    off = 0
    for i in range(pk.n):
        L = int(lens[i])
        name = b"@r%d/%d extra:%d" % (i, mate, rng.randint(0, 99999))
        strand = b"+" if rng.random() < 0.8 else b"+r%d" % i
        eol = b"\r\n" if rng.random() < 0.1 else b"\n"
        seq, qual = seqs[i, :L].tobytes(), quals[i, :L].tobytes()
        name_off = off
        seq_off = name_off + len(name) + len(eol)
        strand_off = seq_off + L + len(eol)
        qual_off = strand_off + len(strand) + len(eol)
        rec = name + eol + seq + eol + strand + eol + qual + eol
        parts.append(rec)
        recs.append((name_off, seq_off, strand_off, qual_off, len(name), len(strand), L, 0))
        names.append(name)
        strands.append(strand)
        off += len(rec)
    text = np.frombuffer(b"".join(parts), np.uint8).copy()
    return text, np.array(recs, dtype=np.dtype(abi.TEXT_REC_DTYPE)), names, strands


def expected_out(pk, res, paired, texts):
    outs = [bytearray(), bytearray()]
    for i in range(pk.n):
        rs = [res[2 * i], res[2 * i + 1]] if paired else [res[i]]
        ok = all((int(r["flags"]) & (abi.FQ_RF_NULL | abi.FQ_RF_INDEX_FILTERED)) == 0 and int(r["code"]) == 0 for r in rs)
        if not ok:
            continue
        for m, r in enumerate(rs):
            _, _, names, strands = texts[m]
            seq = getattr(pk, "seq%d" % (m + 1))[i]
            qual = getattr(pk, "qual%d" % (m + 1))[i]
            a, n = int(r["start"]), int(r["len"])
            outs[m] += names[i] + b"\n" + seq[a:a + n].tobytes() + b"\n" + strands[i] + b"\n" + qual[a:a + n].tobytes() + b"\n"
    return [bytes(o) for o in outs]


def run_text(lib, p, pk, texts, seq_no=7):
    paired = bool(p.paired)
    h = ctypes.c_void_p()
    assert lib.fq_engine_create(ctypes.byref(p), 0, pk.n, pk.stride, ctypes.byref(h)) == 0, \
        lib.fq_engine_last_error(None).decode()
    try:
        tb = abi.FqTextBatch()
        tb.n, tb.stride = pk.n, pk.stride
        outbufs = []
        out = abi.FqTextOut()
        for m in range(2 if paired else 1):
            text, recs = texts[m][0], texts[m][1]
            tb.text[m], tb.text_bytes[m], tb.rec[m] = text.ctypes.data, text.size, recs.ctypes.data
            ob = np.zeros(text.size + 16, np.uint8)
            outbufs.append(ob)
            out.text[m] = ob.ctypes.data
        res = pk.result_array()
        assert lib.fq_engine_submit_text(h, ctypes.byref(tb), res.ctypes.data, ctypes.byref(out), seq_no) == 0, \
            lib.fq_engine_last_error(h).decode()
        seq = ctypes.c_uint64()
        assert lib.fq_engine_poll(h, 1, ctypes.byref(seq)) == 1, lib.fq_engine_last_error(h).decode()
        assert seq.value == seq_no
        acc = np.zeros(lib.fq_engine_acc_words(h), np.uint64)
        assert lib.fq_engine_read_acc(h, acc.ctypes.data, acc.size) == 0
        got = [outbufs[m][: out.bytes[m]].tobytes() for m in range(len(outbufs))]
        return res, acc, got
    finally:
        lib.fq_engine_destroy(h)


@pytest.mark.parametrize("cfg", ["C3", "C5", "PE_all", "C2", "SE_all"])
@pytest.mark.parametrize("source", ["synth", "edge"])
def test_text_pack_matches_oracle(lib, oracle, cfg, source):
    paired = cfg not in ("C2", "SE_all")
    p = config(cfg, max_cycles=512)
    pk = synth_pack(oracle, 6000, paired, first=91) if source == "synth" else edge_pack(3000, paired)
    rng = random.Random(5)
    texts = [fastq_text(pk, m, rng) for m in ((1, 2) if paired else (1,))]
    res_o, acc_o = run_oracle(oracle, p, pk)
    res, acc, got = run_text(lib, p, pk, texts)
    assert np.array_equal(res, res_o)
    assert np.array_equal(acc, acc_o)
    exp = expected_out(pk, res_o, paired, texts)
    for m in range(len(got)):
        assert got[m] == exp[m], f"mate {m + 1}: output text differs"


def test_text_pack_last_record_without_terminator(lib, oracle):
    """An input whose last line lacks its terminator: the output still ends the record with one."""
    p = config("C3", max_cycles=512)
    pk = synth_pack(oracle, 500, True, first=3)
    rng = random.Random(9)
    texts = [fastq_text(pk, m, rng) for m in (1, 2)]
    for m in range(2):  # drop the final "\n" (and a "\r" before it)
        t = texts[m][0]
        cut = 2 if t.size >= 2 and t[-2] == 13 else 1
        texts[m] = (t[:-cut].copy(),) + texts[m][1:]
    res_o, _ = run_oracle(oracle, p, pk)
    res, _, got = run_text(lib, p, pk, texts)
    assert np.array_equal(res, res_o)
    exp = expected_out(pk, res_o, True, texts)
    assert got == exp


def test_text_pack_refuses_discard_unmerged(lib, oracle):
    # -m runs on text packs (the merged stream, tests/test_host_e2e.py); with --discard_unmerged the
    # unmerged pairs go to out1 / out2 instead, which only the host packs write
    p = config("C4", max_cycles=512)
    p.discard_unmerged = 1
    pk = synth_pack(oracle, 64, True)
    rng = random.Random(1)
    texts = [fastq_text(pk, m, rng) for m in (1, 2)]
    h = ctypes.c_void_p()
    assert lib.fq_engine_create(ctypes.byref(p), 0, pk.n, pk.stride, ctypes.byref(h)) == 0
    try:
        tb = abi.FqTextBatch()
        tb.n, tb.stride = pk.n, pk.stride
        out = abi.FqTextOut()
        keep = [np.zeros(texts[m][0].size + 16, np.uint8) for m in range(2)]
        for m in range(2):
            tb.text[m], tb.text_bytes[m], tb.rec[m] = texts[m][0].ctypes.data, texts[m][0].size, texts[m][1].ctypes.data
            out.text[m] = keep[m].ctypes.data
        res = pk.result_array()
        assert lib.fq_engine_submit_text(h, ctypes.byref(tb), res.ctypes.data, ctypes.byref(out), 1) == abi.FQ_E_INVALID
    finally:
        lib.fq_engine_destroy(h)
