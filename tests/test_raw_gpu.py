"""Raw FASTQ streams (fq_engine_raw_*: record indexing on the GPU) against the oracle.

The input bytes of each mate go over in windows of random sizes that split records anywhere, the
mates' windows independent of each other; the engine carries the bytes after each pack's last
record into the next window, cuts the plain records (four '\\n'-terminated lines, FqReader::read
of src/fqreader.cpp:160-195) and pairs the mates (FqReaderPair::read, :254-267).  Over the whole
stream the packs' output text must equal Read::toString of every passing record in input order,
the accumulator must equal the oracle's over all pairs, and the trimmed-adapter entries must be
FilterResult's strings (src/filterresult.cpp:138-157).  A record that is not plain ends the stream
at the pair before it, at the exact byte offsets where the host reader resumes."""
import ctypes
import random
import zlib
from collections import Counter

import numpy as np
import pytest

from batch_util import config, edge_pack, run_oracle, synth_pack
from fqtool_amd import abi
from test_text_gpu import expected_out

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    return abi.load_engine()


def plain_fastq(pk, mate, rng, irregular_at=None):
    """Plain FASTQ bytes of one mate (names of random length), the record byte offsets, and the
    names / strands expected_out needs.  irregular_at: that record's sequence line ends in CRLF."""
    seqs, quals, lens = getattr(pk, "seq%d" % mate), getattr(pk, "qual%d" % mate), getattr(pk, "len%d" % mate)
    parts, names, strands, offs = [], [], [], []
    off = 0
    for i in range(pk.n):
        L = int(lens[i])
        name = b"@r%d/%d" % (i, mate) + b"x" * rng.randint(0, 40)
        strand = b"+" if rng.random() < 0.7 else b"+r%d" % i
        eol1 = b"\r\n" if i == irregular_at else b"\n"
        rec = name + b"\n" + seqs[i, :L].tobytes() + eol1 + strand + b"\n" + quals[i, :L].tobytes() + b"\n"
        offs.append(off)
        parts.append(rec)
        names.append(name)
        strands.append(strand)
        off += len(rec)
    offs.append(off)
    return np.frombuffer(b"".join(parts), np.uint8).copy(), offs, names, strands


def adapter_strings(res, pk, p, paired):
    out = [Counter(), Counter()]
    for i in range(pk.n):
        for m in range(2 if paired else 1):
            r = res[2 * i + m] if paired else res[i]
            if not (int(r["flags"]) & (abi.FQ_RF_AD_OVERLAP | abi.FQ_RF_AD_SEQ)) or int(r["ad_len"]) == 0:
                continue
            a, n = int(r["ad_pos"]), int(r["ad_len"])
            if int(r["flags"]) & abi.FQ_RF_AD_NEG:
                s = bytes(p.adapter2 if m else p.adapter1)[a:a + n]
            else:
                s = getattr(pk, "seq%d" % (m + 1))[i, a:a + n].tobytes()
            out[m][s] += 1
    return out


def decode_entries(buf, adapter):
    c, o = Counter(), 0
    while o + 3 <= len(buf):
        n = buf[o] | (buf[o + 1] << 8)
        if buf[o + 2]:
            pos = buf[o + 3] | (buf[o + 4] << 8)
            c[adapter[pos:pos + n]] += 1
            o += 5
        else:
            c[bytes(buf[o + 3:o + 3 + n])] += 1
            o += 3 + n
    assert o == len(buf)
    return c


def run_raw(lib, p, texts, max_batch, stride, rng, wcap=60000, ccap=600000):
    """Drives the raw protocol like the tool: enqueue window k+1, launch window k, poll; empty
    windows drain the carry once all bytes are sent.  Returns (pairs per pack, output text per
    mate, adapter entry counts per mate, accumulator, stop info)."""
    mates = len(texts)
    h = ctypes.c_void_p()
    assert lib.fq_engine_create(ctypes.byref(p), 0, max_batch, stride, ctypes.byref(h)) == 0, \
        lib.fq_engine_last_error(None).decode()
    keep = []
    try:
        assert lib.fq_engine_raw_begin(h, wcap, ccap) == 0, lib.fq_engine_last_error(h).decode()
        pos = [0, 0]
        starts = []  # per enqueued window: (start, n) per mate
        frac = [0.0]  # the mates advance through their inputs at about the same rate (the caller's
        #               job: the device carry holds only the imbalance), each split at random bytes

        def enqueue(empty=False):
            w = abi.FqRawWindow()
            win = []
            frac[0] = min(1.0, frac[0] + rng.uniform(0.2, 1.0) * wcap * 0.8 / max(t.size for t in texts))
            for m in range(mates):
                want = int(frac[0] * texts[m].size) - pos[m] + rng.randint(-3000, 3000)
                n = 0 if empty else max(0, min(want, wcap, texts[m].size - pos[m]))
                if frac[0] >= 1.0 and not empty:
                    n = min(wcap, texts[m].size - pos[m])
                w.bytes[m] = texts[m].ctypes.data + pos[m] if n else None
                w.n[m] = n
                win.append((pos[m], n))
                pos[m] += n
            assert lib.fq_engine_raw_enqueue(h, ctypes.byref(w)) == 0, lib.fq_engine_last_error(h).decode()
            starts.append(win)

        def more():
            return any(pos[m] < texts[m].size for m in range(mates))

        packs, outs, ads, stop = [], [bytearray(), bytearray()], [Counter(), Counter()], None
        adapters = [bytes(p.adapter1), bytes(p.adapter2)]
        pending = []
        enqueue()
        k = 0
        while True:
            if more() and len(starts) - k < 2:
                enqueue()
            r = abi.FqRawResult()
            o = abi.FqRawOut()
            bufs = []
            for m in range(mates):
                tb = np.zeros(ccap + wcap + 4 * max_batch + 64, np.uint8)
                bufs += [tb, tb]
                o.text.text[m] = tb.ctypes.data
            assert lib.fq_engine_raw_launch(h, ctypes.byref(r), ctypes.byref(o), k) == 0, lib.fq_engine_last_error(h).decode()
            pending.append((k, o, bufs))
            keep.append(bufs)
            packs.append(r.pairs)
            seq = ctypes.c_uint64()
            while len(pending) > 2:
                assert lib.fq_engine_poll(h, 1, ctypes.byref(seq)) == 1, lib.fq_engine_last_error(h).decode()
                kk, oo, bb = pending.pop(0)
                assert seq.value == kk
                for m in range(mates):
                    nb = oo.text.bytes[m]
                    outs[m] += bb[2 * m][:nb].tobytes()
                    ads[m] += decode_entries(bb[2 * m][nb:nb + oo.adapter_bytes[m]].tobytes(), adapters[m])
            left = any(r.carry[m] for m in range(mates))
            win = starts[k]
            k += 1
            last = not more() and len(starts) == k
            exhausted = any(pos[m] == texts[m].size for m in range(mates))
            if r.stop or (r.pairs == 0 and exhausted) or (last and not (left and r.pairs > 0)):
                stop = (bool(r.stop), [win[m][0] + win[m][1] - r.carry[m] for m in range(mates)], r.pairs)
                break
            if last:
                enqueue(empty=True)
        seq = ctypes.c_uint64()
        for kk, oo, bb in pending:
            assert lib.fq_engine_poll(h, 1, ctypes.byref(seq)) == 1, lib.fq_engine_last_error(h).decode()
            assert seq.value == kk
            for m in range(mates):
                nb = oo.text.bytes[m]
                outs[m] += bb[2 * m][:nb].tobytes()
                ads[m] += decode_entries(bb[2 * m][nb:nb + oo.adapter_bytes[m]].tobytes(), adapters[m])
        assert lib.fq_engine_sync(h) == 0
        acc = np.zeros(lib.fq_engine_acc_words(h), np.uint64)
        assert lib.fq_engine_read_acc(h, acc.ctypes.data, acc.size) == 0
        return packs, [bytes(x) for x in outs[:mates]], ads[:mates], acc, stop
    finally:
        lib.fq_engine_destroy(h)


@pytest.mark.parametrize("cfg", ["C3", "C5", "PE_all", "C2", "SE_all"])
@pytest.mark.parametrize("source", ["synth", "edge"])
@pytest.mark.parametrize("max_batch", [4096, 97])
def test_raw_stream_matches_oracle(lib, oracle, cfg, source, max_batch):
    paired = cfg not in ("C2", "SE_all")
    p = config(cfg, max_cycles=512)
    pk = synth_pack(oracle, 3000, paired, first=17) if source == "synth" else edge_pack(2000, paired)
    if source == "edge":  # an empty sequence line is not plain: give those reads one base
        for i in range(pk.n):
            for m in ((1, 2) if paired else (1,)):
                if int(getattr(pk, "len%d" % m)[i]) == 0:
                    pk.set(i, m, b"N", b"#")
    rng = random.Random(zlib.crc32(("%s/%s/%d" % (cfg, source, max_batch)).encode()))
    texts = [plain_fastq(pk, m, rng) for m in ((1, 2) if paired else (1,))]
    stride = 320 if source == "edge" else 160
    # reads longer than the engine's stride are not plain: keep every read within it here
    assert int(pk.len1.max()) <= stride and (not paired or int(pk.len2.max()) <= stride)
    res_o, acc_o = run_oracle(oracle, p, pk)
    packs, outs, ads, acc, stop = run_raw(lib, p, [t[0] for t in texts], max_batch, stride, rng)
    assert sum(packs) == pk.n and max(packs) <= max_batch, packs
    assert stop[0] is False
    assert np.array_equal(acc, acc_o)
    exp = expected_out(pk, res_o, paired, [(None, None, t[2], t[3]) for t in texts])
    for m in range(len(outs)):
        assert outs[m] == exp[m], f"mate {m + 1}: output text differs"
    want = adapter_strings(res_o, pk, p, paired)
    for m in range(len(ads)):
        assert ads[m] == want[m], f"mate {m + 1}: adapter strings differ"


@pytest.mark.parametrize("mate", [1, 2])
def test_raw_stream_stops_at_irregular_record(lib, oracle, mate):
    """A CRLF line end (the reference folds "\\r\\n" by its buffer rule) makes record 1234 irregular:
    the stream ends with pair 1233 and reports each mate's offset of record 1234."""
    p = config("C3", max_cycles=512)
    pk = synth_pack(oracle, 3000, True, first=5)
    rng = random.Random(31 + mate)
    bad = 1234
    texts = [plain_fastq(pk, m, rng, irregular_at=bad if m == mate else None) for m in (1, 2)]
    packs, outs, _, acc, stop = run_raw(lib, p, [t[0] for t in texts], 4096, 160, rng)
    assert stop[0] is True or stop[2] == 0
    assert sum(packs) == bad
    assert stop[1] == [texts[0][1][bad], texts[1][1][bad]]
    sub = synth_pack(oracle, bad, True, first=5)
    res_o, acc_o = run_oracle(oracle, p, sub)
    assert np.array_equal(acc, acc_o)
    exp = expected_out(sub, res_o, True, [(None, None, t[2][:bad], t[3][:bad]) for t in texts])
    assert outs == exp


def test_raw_stream_unequal_mates_stop_at_the_shorter(lib, oracle):
    """Mate 2 has 200 records fewer: the pairs end with the shorter mate; the host reader resumes
    at mate 1's next record (and reports the reference's error there)."""
    p = config("C3", max_cycles=512)
    pk = synth_pack(oracle, 2500, True, first=8)
    rng = random.Random(4)
    t1 = plain_fastq(pk, 1, rng)
    t2 = plain_fastq(pk, 2, rng)
    short = 2300
    packs, _, _, _, stop = run_raw(lib, p, [t1[0], t2[0][:t2[1][short]].copy()], 4096, 160, rng)
    assert sum(packs) == short
    assert stop[1] == [t1[1][short], t2[1][short]]
