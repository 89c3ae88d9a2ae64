"""Helpers shared by the parity tests: numpy-backed fq_batch packs and config presets."""
import ctypes
import random

import numpy as np

from fqtool_amd import abi

AD1 = "AGATCGGAAGAGCACACGTCTGAACTCCAGTCA"
AD2 = "AGATCGGAAGAGCGTCGTGTAGGGAAAGAGTGT"


class Pack:
    """A pack as (n, stride) row arrays; batch() lays them out as the engine's fq_batch planes
    (chunk-interleaved tiles, include/fqengine.h) and keeps those buffers alive."""

    def __init__(self, n, stride, paired):
        self.n, self.stride, self.paired = n, stride, paired
        self.seq1 = np.zeros((n, stride), np.uint8)
        self.qual1 = np.zeros((n, stride), np.uint8)
        self.len1 = np.zeros(n, np.uint16)
        if paired:
            self.seq2 = np.zeros((n, stride), np.uint8)
            self.qual2 = np.zeros((n, stride), np.uint8)
            self.len2 = np.zeros(n, np.uint16)

    def set(self, i, mate, seq, qual):
        assert len(seq) == len(qual) <= self.stride
        s = getattr(self, "seq%d" % mate)
        q = getattr(self, "qual%d" % mate)
        s[i, : len(seq)] = np.frombuffer(seq, np.uint8)
        q[i, : len(qual)] = np.frombuffer(qual, np.uint8)
        getattr(self, "len%d" % mate)[i] = len(seq)

    flags = None  # optional per-pair FQ_BF_* flags (np.uint8, n)

    def planes(self):
        return ("seq1", "qual1", "seq2", "qual2") if self.paired else ("seq1", "qual1")

    def batch(self):
        self._tiled = {k: abi.tile_rows(getattr(self, k)) for k in self.planes()}
        b = abi.FqBatch()
        b.n, b.stride = self.n, self.stride
        b.seq1, b.qual1, b.len1 = self._tiled["seq1"].ctypes.data, self._tiled["qual1"].ctypes.data, self.len1.ctypes.data
        if self.paired:
            b.seq2, b.qual2, b.len2 = self._tiled["seq2"].ctypes.data, self._tiled["qual2"].ctypes.data, self.len2.ctypes.data
        if self.flags is not None:
            b.flags = self.flags.ctypes.data
        return b

    def load_batch(self):
        """Copy the planes of the last batch() back into the row arrays (after a fill)."""
        for k in self.planes():
            getattr(self, k)[:] = abi.untile_rows(self._tiled[k], self.n, self.stride)

    def result_array(self):
        return np.zeros(self.n * (2 if self.paired else 1), dtype=np.dtype(abi.RESULT_DTYPE_FIELDS))


def synth_pack(oracle, n, paired, seed=20261015, first=0, L=150, stride=160):
    pk = Pack(n, stride, paired)
    b = pk.batch()
    oracle.orc_synth_fill(ctypes.byref(b), seed, first, L)
    pk.load_batch()
    return pk


def rand_read(rng, n):
    seq = bytes(rng.choice(b"ACGTN" if rng.random() < 0.9 else b"ACGTNacgtRYK") for _ in range(n))
    qual = bytes(33 + rng.randint(2, 41) if rng.random() > 0.02 else rng.choice([25, 32, 126, 200])
                 for _ in range(n))
    return seq, qual


def edge_pack(n, paired, stride=160, seed=7):
    """Ragged and hostile reads: empty, very short, all-N, exotic bytes, polyG runs, adapters."""
    rng = random.Random(seed)
    pk = Pack(n, stride, paired)
    for i in range(n):
        for m in ((1, 2) if paired else (1,)):
            L = rng.choice([0, 1, 3, 4, 5, 10, 29, 30, 31, 49, 50, 51, 100, 149, 150, 151, stride])
            seq, qual = rand_read(rng, L)
            kind = rng.random()
            if kind < 0.1:
                seq = b"N" * L
            elif kind < 0.2 and L > 20:
                g = rng.randint(1, L)
                seq = seq[: L - g] + b"G" * g
            elif kind < 0.35 and L > 40:
                ad = (AD1 if m == 1 else AD2).encode()
                k = rng.randint(0, L - 1)
                seq = (seq[:k] + ad + b"G" * L)[:L]
            pk.set(i, m, seq, qual)
    if paired:  # make ~1/3 of the pairs truly overlapping
        for i in range(0, n, 3):
            L = int(pk.len1[i])
            if L < 40:
                continue
            comp = bytes.maketrans(b"ACGTacgt", b"TGCATGCA")
            s1 = bytes(pk.seq1[i, :L])
            ins = rng.randint(L // 2, L + 60)
            frag = s1 + bytes(rng.choice(b"ACGT") for _ in range(max(0, ins - L)))
            frag = frag[:ins]
            r2 = frag.translate(comp)[::-1][:L]
            r2 = (r2 + AD2.encode() + b"G" * L)[:L]
            pk.set(i, 2, r2, bytes(pk.qual2[i, :L]))
    return pk


def adapter_pack(n, paired, ad1, ad2, stride=160, seed=5):
    """Reads holding a copy of their mate's adapter at every kind of offset trimBySequence tests
    (src/adaptertrimmer.cpp:29-90): its tail at the read start (pos -1 .. -6), anywhere inside,
    cut off by the read end (pos up to L - 5 and beyond), with 0 .. allowance + 2 substitutions
    (another base, 'N', the same letter in lower case), decoys with too many mismatches ahead of a
    real copy, random lengths 0-stride.  Mates are independent random sequence, so almost no pair
    overlaps and the by-sequence search runs on nearly every read."""
    rng = random.Random(seed)
    pk = Pack(n, stride, paired)
    lens = [0, 1, 4, 5, 6, 8, 15, 16, 17, 19, 20, 21, 31, 32, 33, 40, 63, 64, 65, 100, 127, 145, 149, 150, 151, stride]
    for i in range(n):
        for m in ((1, 2) if paired else (1,)):
            ad = (ad1 if m == 1 else ad2).encode()
            L = rng.choice(lens)
            seq = bytearray(rng.choice(b"ACGT") for _ in range(L))
            copies = rng.choice([0, 1, 1, 1, 2])
            for c in range(copies):
                if L == 0 or not ad:
                    break
                pos = rng.randint(-min(6, len(ad) - 1), L - 1) if rng.random() < 0.6 else rng.randint(max(-6, L - 20), L - 1)
                start = max(0, -pos)
                piece = bytearray(ad[start:])
                at = max(0, pos)
                piece = piece[: L - at]
                if not piece:
                    continue
                allowed = min(L - pos, len(ad)) // 8
                subs = rng.randint(0, allowed + 2) if c == copies - 1 else allowed + 1 + rng.randint(0, 3)
                for _ in range(subs):
                    k = rng.randrange(len(piece))
                    kind = rng.random()
                    if kind < 0.6:
                        piece[k] = rng.choice([b for b in b"ACGT" if b != piece[k]])
                    elif kind < 0.8:
                        piece[k] = ord("N")
                    else:
                        piece[k] = piece[k] | 0x20
                seq[at:at + len(piece)] = piece
            if L and rng.random() < 0.05:
                seq[rng.randrange(L)] = ord("N")
            qual = bytes(33 + rng.randint(10, 40) for _ in range(L))
            pk.set(i, m, bytes(seq), qual)
    return pk


def polyx_pack(n, paired, stride=160, seed=11):
    """Reads ending in a homopolymer tail (A, T, C, G or N) of 1-24 bases with 0-3 substitutions at
    random tail positions, ahead of which sits random sequence: polyX scans that break before, at
    and after the compare requirement and the first allowance step (src/polyx.cpp:45-101)."""
    rng = random.Random(seed)
    pk = Pack(n, stride, paired)
    for i in range(n):
        for m in ((1, 2) if paired else (1,)):
            L = rng.choice([8, 12, 16, 30, 75, 100, 149, 150])
            seq = bytearray(bytes(rng.choice(b"ACGT") for _ in range(L)))
            x = rng.choice(b"ATCGN")
            t = min(L, rng.randint(1, 24))
            for k in range(L - t, L):
                seq[k] = x
            for _ in range(rng.choice([0, 0, 1, 1, 2, 3])):
                k = rng.randint(max(0, L - t - 2), L - 1)
                seq[k] = rng.choice(b"ACGTN")
            qual = bytes(33 + rng.randint(20, 40) for _ in range(L))
            pk.set(i, m, bytes(seq), qual)
    return pk


def polyx_params(paired, mask, max_mm, per, compare_req, max_cycles=512):
    p = abi.default_params(paired=paired, max_cycles=max_cycles)
    p.qual_filter_enabled = 1
    p.polyx_enabled = 1
    p.polyx_mask, p.polyx_max_mismatch, p.polyx_one_mismatch_per, p.polyx_compare_req = mask, max_mm, per, compare_req
    return p


def config(name, max_cycles=256):
    """Parameter presets: the BASELINE configs plus extra option coverage."""
    paired = name not in ("C2", "SE_adapter", "SE_all", "SE_umi", "SE_correct")
    p = abi.default_params(paired=paired, max_cycles=max_cycles)
    p.qual_filter_enabled = 1  # every config has -q
    if name == "C2":
        pass
    elif name in ("C1", "C3"):
        p.adapter_trimming = 1
        p.polyg_enabled = 1
    elif name == "C3b":
        p.adapter_trimming = 1
        p.polyg_enabled = 1
        abi.set_adapter(p, 1, AD1)
        abi.set_adapter(p, 2, AD2)
    elif name == "C4":
        p.adapter_trimming = 1
        p.polyg_enabled = 1
        p.cut_right = 1
        p.merge_enabled = 1
    elif name == "C5":
        p.adapter_trimming = 1
        p.polyg_enabled = 1
        p.polyx_enabled = 1
        p.cut_right = 1
    elif name == "PE_all":
        p.adapter_trimming = 1
        abi.set_adapter(p, 1, AD1[:20])
        abi.set_adapter(p, 2, "AGATCGGAAGAGC")
        p.polyg_enabled = 1
        p.polyx_enabled = 1
        p.polyx_mask = 0b01101
        p.cut_front = 1
        p.cut_tail = 1
        p.cut_front_window, p.cut_tail_window = 3, 5
        p.cut_front_quality, p.cut_tail_quality = 25, 15
        p.trim_front1, p.trim_tail1, p.trim_front2, p.trim_tail2 = 2, 1, 0, 3
        p.max_len1, p.max_len2 = 120, 0
        p.length_filter_enabled, p.min_len, p.max_len = 1, 30, 140
        p.complexity_enabled, p.complexity_threshold = 1, 0.4
        p.avg_qual_limit = 25.5
        p.n_base_limit = 3
    elif name == "PE_merge_discard":
        p.merge_enabled = 1
        p.discard_unmerged = 1
        p.cut_right = 1
        p.cut_right_window = 7
        p.length_filter_enabled = 1
        p.overlap_diff_limit, p.overlap_require = 3, 20
    elif name == "SE_adapter":
        p.adapter_trimming = 1
        abi.set_adapter(p, 1, AD1)
        p.polyg_enabled = 1
        p.polyx_enabled = 1
        p.cut_right = 1
    elif name == "SE_all":
        p.adapter_trimming = 1
        abi.set_adapter(p, 1, "AGATCGGA")
        p.polyx_enabled = 1
        p.polyx_mask = 0b11111
        p.cut_front = p.cut_tail = 1
        p.trim_front1, p.trim_tail1 = 3, 2
        p.length_filter_enabled, p.min_len, p.max_len = 1, 20, 100
        p.complexity_enabled = 1
        p.low_qual_base_limit = 10
    elif name == "PE_merge_q":  # merge with polyX, adapters by sequence, maxLen, a short overlap requirement
        p.merge_enabled = 1
        p.adapter_trimming = p.polyg_enabled = p.polyx_enabled = 1
        abi.set_adapter(p, 1, AD1[:16])
        p.max_len2 = 120
        p.overlap_diff_limit, p.overlap_require = 5, 12
        p.avg_qual_limit = 20.0
        p.length_filter_enabled, p.min_len = 1, 40
    elif name == "PE_correct":  # -c with the C3 options
        p.adapter_trimming = p.polyg_enabled = 1
        p.correction_enabled = 1
    elif name == "PE_correct_all":  # -c ahead of adapters by sequence, polyX, merge
        p.adapter_trimming = p.polyg_enabled = p.polyx_enabled = 1
        abi.set_adapter(p, 1, AD1)
        p.correction_enabled = 1
        p.merge_enabled = 1
        p.cut_right = 1
    elif name == "PE_correct_merge":  # -c with the config-4 options (the merge variant's -c instantiation)
        p.adapter_trimming = p.polyg_enabled = 1
        p.cut_right = 1
        p.merge_enabled = 1
        p.correction_enabled = 1
    elif name == "PE_merge_complexity":  # -m with the low-complexity filter (merged reads: both parts + junction)
        p.adapter_trimming = p.polyg_enabled = 1
        p.merge_enabled = 1
        p.complexity_enabled, p.complexity_threshold = 1, 0.745
        p.n_base_limit = 2
    elif name == "PE_correct_front":  # -c with front trimming (pre/post Stats: the fix-up in the pre block)
        p.adapter_trimming = p.polyg_enabled = 1
        p.correction_enabled = 1
        p.cut_front, p.cut_front_window, p.cut_front_quality = 1, 4, 20
        p.trim_front1, p.trim_tail1, p.trim_front2 = 2, 1, 5
    elif name == "PE_correct_umi_merge":  # -c, UMI in both reads and -m (the merge variant's -c/UMI code)
        p.adapter_trimming = p.polyg_enabled = 1
        p.correction_enabled = 1
        p.merge_enabled = 1
        p.cut_right = 1
        p.umi_front1, p.umi_front2 = 8, 4
    elif name == "PE_correct_x":  # -c with the config-5 options (the fast kernels' -c variant)
        p.adapter_trimming = p.polyg_enabled = p.polyx_enabled = 1
        abi.set_adapter(p, 1, AD1)
        p.cut_right = 1
        p.correction_enabled = 1
    elif name == "PE_umi":  # UMI in both reads (trimFront after the pre-filter stats)
        p.adapter_trimming = p.polyg_enabled = p.polyx_enabled = 1
        p.cut_front = 1
        p.umi_front1, p.umi_front2 = 10, 7
    elif name == "PE_umi_x":  # UMI in both reads with the config-5 options (cut_right scan on the cut read)
        p.adapter_trimming = p.polyg_enabled = p.polyx_enabled = 1
        abi.set_adapter(p, 2, AD2)
        p.cut_right = 1
        p.umi_front1, p.umi_front2 = 8, 12
    elif name == "PE_umi_merge":  # UMI in both reads with the config-4 options (pre/post Stats in the merge variant)
        p.adapter_trimming = p.polyg_enabled = 1
        p.cut_right = 1
        p.merge_enabled = 1
        p.umi_front1, p.umi_front2 = 9, 6
    elif name == "SE_correct":  # -c on single-end input: a no-op, as in SingleEndProcessor
        p.adapter_trimming = p.polyg_enabled = 1
        abi.set_adapter(p, 1, AD1)
        p.correction_enabled = 1
    elif name == "SE_umi":
        p.polyg_enabled = 1
        p.cut_tail = 1
        p.umi_front1 = 12
    elif name == "PE_cutRF":  # cut_right (w=3, staged scan) after forced front/tail trims
        p.adapter_trimming = p.polyg_enabled = 1
        p.cut_right, p.cut_right_window, p.cut_right_quality = 1, 3, 28
        p.trim_front1, p.trim_tail1, p.trim_front2, p.trim_tail2 = 5, 2, 3, 7
    elif name.startswith("PE_cutR"):  # cut_right alone (removed-mode stats), window w
        w = int(name[7:])
        p.adapter_trimming = p.polyg_enabled = 1
        p.cut_right, p.cut_right_window, p.cut_right_quality = 1, w, 30
    elif name.startswith("PE_cut"):  # both forward window scans from unaligned starts, window w
        w = int(name[6:])
        p.adapter_trimming = p.polyg_enabled = 1
        p.cut_front, p.cut_front_window, p.cut_front_quality = 1, max(1, w // 2), 15
        p.cut_right, p.cut_right_window, p.cut_right_quality = 1, w, 28
        p.trim_front1, p.trim_front2 = 1, 3
    else:
        raise KeyError(name)
    return p


ALL_CONFIGS = ["C2", "C3", "C3b", "C4", "C5", "PE_all", "PE_merge_discard", "SE_adapter", "SE_all",
               "PE_cut1", "PE_cut4", "PE_cut11", "PE_cut40", "PE_cutR1", "PE_cutR2", "PE_cutR5", "PE_cutRF", "PE_merge_q",
               "PE_correct", "PE_correct_all", "PE_correct_merge", "PE_correct_x", "PE_umi", "PE_umi_x", "PE_umi_merge",
               "PE_correct_front", "PE_correct_umi_merge", "PE_merge_complexity", "SE_correct", "SE_umi"]


def run_oracle(oracle, p, pk):
    res = pk.result_array()
    acc = np.zeros(abi.acc_words(p.insert_size_max, p.max_cycles), np.uint64)
    b = pk.batch()
    rc = oracle.orc_process_batch(ctypes.byref(p), ctypes.byref(b), res.ctypes.data, acc.ctypes.data)
    assert rc == 0, rc
    return res, acc
