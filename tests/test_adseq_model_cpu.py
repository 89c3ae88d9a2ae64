"""Host-side model of the fast kernels' trimBySequence filter (pe_fast.hip `adseq_search`).

The kernel rejects offsets with a code-level lower bound before running the reference's byte
test (src/adaptertrimmer.cpp:29-90).  This checks the argument the kernel relies on, in plain
Python on random and adapter-laden reads: with 2-bit codes (A C T G = 0 1 2 3 from (byte >> 1) & 3,
N read as G's code, a lower-case base as its upper-case letter's), the bound never exceeds the
byte mismatch count, so the first offset the filtered search accepts is the reference's.
The GPU parity of the kernel itself is tests/test_engine_gpu.py::test_adapter_by_sequence.
"""
import random


def ref_trim_by_sequence(r, ad):
    """The reference loop (src/adaptertrimmer.cpp:29-70), returning pos or None."""
    rlen, alen = len(r), len(ad)
    if alen < 4:
        return None
    start = -4 if alen >= 16 else -3 if alen >= 12 else -2 if alen >= 8 else 0
    for pos in range(start, rlen - 4):
        cmplen = min(rlen - pos, alen)
        allowed = cmplen // 8
        mm = 0
        ok = True
        for i in range(max(0, -pos), cmplen):
            if ad[i] != r[i + pos]:
                mm += 1
                if mm > allowed:
                    ok = False
                    break
        if ok:
            return pos
    return None


def code(b):
    return 3 if b in (ord("N"), ord("n")) else ((b & ~0x20) >> 1) & 3


def bound(r, ad, j0, k, m):
    """Code mismatches of read positions j0 .. j0+m-1 against adapter positions k .. k+m-1."""
    return sum(code(r[j0 + j]) != code(ad[k + j]) for j in range(m))


def filtered_search(r, ad):
    n, alen = len(r), len(ad)
    assert alen >= 20 and all(c in b"ACGT" for c in ad)

    def exact(pos):
        cmplen = min(n - pos, alen)
        allowed = cmplen // 8
        return sum(ad[i] != r[i + pos] for i in range(max(0, -pos), cmplen)) <= allowed

    for pos in range(-4, 0):
        if pos >= n - 4:
            return None
        if bound(r, ad, 0, -pos, min(n, 16)) <= min(n - pos, alen) // 8 and exact(pos):
            return pos
    if n >= 16:
        K = alen // 8 + 1
        for pos in range(0, n - 15):
            if bound(r, ad, pos, 0, 16) < K and exact(pos):
                return pos
    for pos in range(max(0, n - 15), n - 4):
        m = n - pos
        if bound(r, ad, pos, 0, m) <= m // 8 and exact(pos):
            return pos
    return None


def test_filtered_search_equals_reference_loop():
    rng = random.Random(1)
    hits = 0
    for t in range(3000):
        alen = rng.choice([20, 21, 24, 33, 34, 40, 64])
        ad = bytes(rng.choice(b"ACGT") for _ in range(alen))
        n = rng.choice([0, 1, 4, 5, 6, 10, 15, 16, 17, 20, 21, 40, 100, 150])
        r = bytearray(rng.choice(b"ACGTN" if rng.random() < 0.3 else b"ACGT") for _ in range(n))
        if n and rng.random() < 0.8:
            pos = rng.randint(-6, n - 1)
            piece = bytearray(ad[max(0, -pos):])[: n - max(0, pos)]
            for _ in range(rng.randint(0, 6)):
                if piece:
                    k = rng.randrange(len(piece))
                    piece[k] = rng.choice([ord("N"), piece[k] | 0x20, rng.choice(b"ACGT")])
            r[max(0, pos):max(0, pos) + len(piece)] = piece
        r = bytes(r)
        want = ref_trim_by_sequence(r, ad)
        assert filtered_search(r, ad) == want, (r, ad)
        hits += want is not None
    assert hits > 500
