"""Pins the CPU restatement (oracle/fq_oracle.c) against the reference itself.

tests/golden/kat_*.tsv hold crafted + random inputs and the answers of the UNMODIFIED
reference functions (compiled from /root/reference/src, see tests/golden/make_kat.py).
Every case must match exactly.
"""
import ctypes
import os

import pytest

from fqtool_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_cases(kind):
    rows = []
    with open(os.path.join(GOLDEN, f"kat_{kind}.tsv"), "rb") as f:
        for raw in f:
            cols = raw.rstrip(b"\n").split(b"\t")
            sep = cols.index(b"|")
            inp = [b"" if c == b"~" else c for c in cols[:sep]]
            ans = [b"" if c == b"~" else c for c in cols[sep + 1:]]
            rows.append((inp, ans))
    assert rows
    return rows


def nums(s):
    return [float(x) for x in s.decode().split(",")]


def ci():
    return ctypes.c_int(0)


def test_pass_filter(oracle):
    for inp, ans in load_cases("pass"):
        p = abi.default_params()
        v = nums(inp[1])
        p.qual_filter_enabled, p.length_filter_enabled = int(v[0]), int(v[1])
        p.low_qual_limit, p.low_qual_base_limit, p.n_base_limit = int(v[2]) + 33, int(v[3]), int(v[4])
        p.avg_qual_limit, p.min_len, p.max_len = v[5], int(v[6]), int(v[7])
        p.complexity_enabled, p.complexity_threshold = int(v[8]), v[9]
        is_null = inp[2] == b"NULL"
        s, q = (b"", b"") if is_null else (inp[2], inp[3])
        got = oracle.orc_pass_filter(ctypes.byref(p), s, q, len(s), int(is_null))
        assert got == int(ans[0]), (inp, ans, got)


def test_trim_and_cut(oracle):
    for inp, ans in load_cases("cut"):
        p = abi.default_params()
        v = [int(x) for x in nums(inp[1])]
        p.cut_front, p.cut_right, p.cut_tail = v[2], v[3], v[4]
        p.cut_front_window, p.cut_right_window, p.cut_tail_window = v[5], v[6], v[7]
        p.cut_front_quality, p.cut_right_quality, p.cut_tail_quality = v[8], v[9], v[10]
        s, q = inp[2], inp[3]
        st, ln = ci(), ci()
        nonnull = oracle.orc_trim_and_cut(ctypes.byref(p), s, q, len(s), v[0], v[1], ctypes.byref(st),
                                          ctypes.byref(ln))
        if ans[0] == b"NULL":
            assert nonnull == 0, (inp, ans)
        else:
            assert nonnull == 1, (inp, ans)
            a, b = st.value, st.value + ln.value
            assert (s[a:b], q[a:b]) == (ans[0], ans[1]), (inp, ans, a, b)


def test_polyg(oracle):
    for inp, ans in load_cases("polyg"):
        v = [int(x) for x in nums(inp[1])]
        s = inp[2]
        bases = ci()
        n = oracle.orc_trim_polyg(s, len(s), v[0], v[1], v[2], ctypes.byref(bases))
        reads = 1 if bases.value >= 0 else 0
        got_bases = bases.value if bases.value >= 0 else 0
        assert (s[:n], reads, got_bases) == (ans[0], int(ans[1]), int(ans[2])), (inp, ans)


def test_polyx(oracle):
    for inp, ans in load_cases("polyx"):
        v = [int(x) for x in nums(inp[1])]
        s = inp[2]
        mask = sum(1 << i for i, c in enumerate(b"ATCGN") if c in inp[6])
        poly, bases = ci(), ci()
        n = oracle.orc_trim_polyx(s, len(s), mask, v[0], v[1], v[2], ctypes.byref(poly), ctypes.byref(bases))
        counts = [[0, 0] for _ in range(5)]
        if poly.value >= 0:
            counts[poly.value] = [1, bases.value]
        exp_counts = [[int(x) for x in c.split(b",")] for c in ans[1:6]]
        assert (s[:n], counts) == (ans[0], exp_counts), (inp, ans)


def test_overlap(oracle):
    for inp, ans in load_cases("overlap"):
        v = [int(x) for x in nums(inp[1])]
        s1, s2 = inp[2], inp[4]
        ov = oracle.orc_analyze(s1, len(s1), s2, len(s2), v[0], v[1])
        got = (ov.overlapped, ov.offset, ov.overlap_len, ov.diff)
        assert got == tuple(int(x) for x in ans[:4]), (inp, ans, got)


def revcomp(s):
    comp = {ord("A"): b"T", ord("a"): b"T", ord("T"): b"A", ord("t"): b"A", ord("C"): b"G",
            ord("c"): b"G", ord("G"): b"C", ord("g"): b"C"}
    return b"".join(comp.get(c, b"N") for c in reversed(s))


def merged_name(name, len1, len2):
    """OverlapAnalysis::merge naming (reference src/overlapanalysis.cpp:93-101)."""
    pos = name.find(b" ")
    tag = b"_merged_%d_%d" % (len1, len2)
    if pos < 0:
        return tag
    head = name[: pos - 1] if pos >= 1 else name
    return head + tag + name[pos:]


def test_merge(oracle):
    for inp, ans in load_cases("merge"):
        v = [int(x) for x in nums(inp[1])]
        s1, q1, s2, q2, name = inp[2], inp[3], inp[4], inp[5], inp[6]
        ov = oracle.orc_analyze(s1, len(s1), s2, len(s2), v[0], v[1])
        if not ov.overlapped or ov.overlap_len == 0:
            assert ans[0] == b"NULL", (inp, ans)
            continue
        ol = ov.overlap_len
        l1 = ol + max(0, ov.offset)
        l2 = len(s2) - ol if ov.offset > 0 else 0
        seq = s1[:l1] + revcomp(s2)[ol:ol + l2]
        qual = q1[:l1] + q2[::-1][ol:ol + l2]
        assert (merged_name(name, l1, l2), seq, qual) == (ans[0], ans[1], ans[2]), (inp, ans)


def test_trim_by_sequence(oracle):
    for inp, ans in load_cases("adseq"):
        s, ad = inp[2], inp[6]
        pos = ci()
        found = oracle.orc_trim_by_sequence(s, len(s), ad, len(ad), ctypes.byref(pos))
        if not found:
            assert (0, s) == (int(ans[0]), ans[1]), (inp, ans)
            assert int(ans[2]) == 0
            continue
        pp = pos.value
        rec = ad[-pp:] if pp < 0 else s[pp:]
        new = b"" if pp < 0 else s[:pp]
        reads = 1 if rec else 0
        assert (1, new, reads, len(rec), rec) == (int(ans[0]), ans[1], int(ans[2]), int(ans[3]), ans[4]), \
            (inp, ans)


def test_trim_by_overlap(oracle):
    for inp, ans in load_cases("adov"):
        v = [int(x) for x in nums(inp[1])]
        s1, s2 = inp[2], inp[4]
        ov = oracle.orc_analyze(s1, len(s1), s2, len(s2), v[0], v[1])
        ol = ov.overlap_len
        if ov.diff <= 5 and ov.overlapped and ov.offset < 0 and ol > len(s1) // 3:
            got = (1, s1[:ol], s2[:ol], 2, (len(s1) - ol) + (len(s2) - ol), s1[ol:], s2[ol:])
        else:
            got = (0, s1, s2, 0, 0, b"", b"")
        exp = (int(ans[0]), ans[1], ans[2], int(ans[3]), int(ans[4]), ans[5], ans[6])
        assert got == exp, (inp, ans)
