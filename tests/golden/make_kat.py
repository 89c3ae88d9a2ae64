#!/usr/bin/env python3
"""Generate the per-function known-answer vectors tests/golden/kat_<kind>.tsv.

Inputs are seeded crafted + random cases (edge cases SURVEY.md 8(c) asks for: empty reads,
reads shorter than the window / than 30 / than 50, all-N, lowercase and IUPAC bytes,
exactly 5 mismatches at i=49 vs i=50 of an overlap, adapters of length 3/4/8/12/16/33,
polyG tails of length 10 +/- 1, extreme quality bytes).  Answers come from the UNMODIFIED
reference functions, compiled from /root/reference/src into oracle/_ref/ref_kat by
oracle/Makefile.ref (our harness source: oracle/harness/ref_kat.cpp).  Run in the
development container only:

    make -f oracle/Makefile.ref -j8 && python3 tests/golden/make_kat.py

Each output line is: <input columns...> TAB '|' TAB <reference answer columns...>
"""
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_kat")

ADAPTER1 = "AGATCGGAAGAGCACACGTCTGAACTCCAGTCA"
ADAPTER2 = "AGATCGGAAGAGCGTCGTGTAGGGAAAGAGTGT"


def enc(s):
    return s if s else "~"


def rand_seq(rng, n, alphabet="ACGT", n_rate=0.01, exotic=0.0):
    out = []
    for _ in range(n):
        r = rng.random()
        if r < n_rate:
            out.append("N")
        elif r < n_rate + exotic:
            out.append(rng.choice("acgtnRYKMSWBDHV.-"))
        else:
            out.append(rng.choice(alphabet))
    return "".join(out)


def rand_qual(rng, n, lo=2, hi=41, bad_tail=False, exotic=0.0):
    q = []
    tail_start = rng.randint(max(0, n - 40), n) if bad_tail else n + 1
    for i in range(n):
        if rng.random() < exotic:
            q.append(chr(rng.choice([25, 32, 33, 34, 35, 60, 74, 75, 90, 126])))
        elif i >= tail_start:
            q.append(chr(33 + rng.randint(2, 12)))
        else:
            q.append(chr(33 + rng.randint(lo, hi)))
    return "".join(q)


def revcomp(s):
    comp = {"A": "T", "C": "G", "G": "C", "T": "A", "a": "T", "c": "G", "g": "C", "t": "A"}
    return "".join(comp.get(c, "N") for c in reversed(s))


def mutate(rng, s, k):
    s = list(s)
    for _ in range(k):
        if not s:
            break
        i = rng.randrange(len(s))
        s[i] = rng.choice([c for c in "ACGT" if c != s[i]])
    return "".join(s)


def case(kind, params, s1="", q1="", s2="", q2="", extra=""):
    return "\t".join([kind, params, enc(s1), enc(q1), enc(s2), enc(q2), enc(extra)])


def gen_pass(rng):
    out = []
    out.append(case("pass", "1,0,15,22,5,0,15,0,0,0.3", "NULL", ""))
    for n in [0, 1, 2, 14, 15, 16, 30, 150, 151]:
        s = rand_seq(rng, n)
        out.append(case("pass", "1,1,15,22,5,0,15,0,1,0.3", s, rand_qual(rng, n)))
    for _ in range(600):
        n = rng.choice([rng.randint(0, 40), rng.randint(0, 160), 150])
        s = rand_seq(rng, n, n_rate=rng.choice([0, 0.01, 0.05, 0.5]), exotic=rng.choice([0, 0, 0.05]))
        if rng.random() < 0.1:
            s = "A" * n if rng.random() < 0.5 else ("AC" * n)[:n]
        q = rand_qual(rng, n, lo=rng.choice([0, 2, 15]), hi=rng.choice([20, 30, 41]),
                      bad_tail=rng.random() < 0.3, exotic=rng.choice([0, 0, 0.02]))
        p = [rng.choice([0, 1, 1]), rng.choice([0, 1]), rng.choice([0, 15, 20, 30, 60]),
             rng.choice([0, 5, 22, 40]), rng.choice([0, 5, 10]),
             rng.choice([0, 0, 20, 25.5, 30, 33.25]), rng.choice([0, 15, 50]),
             rng.choice([0, 0, 100, 140]), rng.choice([0, 1]), rng.choice([0.0, 0.3, 0.5, 0.75, 1.0])]
        out.append(case("pass", ",".join(str(x) for x in p), s, q))
    return out


def gen_cut(rng):
    out = []
    for _ in range(900):
        n = rng.choice([rng.randint(0, 12), rng.randint(0, 160), 150])
        s = rand_seq(rng, n, n_rate=rng.choice([0, 0.02, 0.3]))
        if n and rng.random() < 0.3:
            k = rng.randint(0, min(n, 6))
            s = "N" * k + s[k:]
        if n and rng.random() < 0.3:
            k = rng.randint(0, min(n, 6))
            s = s[: n - k] + "N" * k
        q = rand_qual(rng, n, lo=rng.choice([0, 2, 20, 28, 28]), hi=rng.choice([30, 41, 41]),
                      bad_tail=rng.random() < 0.5, exotic=rng.choice([0, 0, 0.03]))
        if n and rng.random() < 0.3:
            k = rng.randint(0, n)
            q = "".join(chr(33 + rng.randint(0, 10)) for _ in range(k)) + q[k:]
        front = rng.choice([0, 0, 0, 0, 1, 3, 10, 200])
        tail = rng.choice([0, 0, 0, 0, 1, 5, 30, 200])
        flags = [rng.choice([0, 1]) for _ in range(3)]
        w = [rng.choice([1, 2, 4, 4, 10, 50]) for _ in range(3)]
        qq = [rng.choice([1, 15, 20, 20, 30, 36]) for _ in range(3)]
        p = [front, tail] + flags + w + qq
        out.append(case("cut", ",".join(str(x) for x in p), s, q))
    return out


def gen_polyg(rng):
    out = []
    for _ in range(700):
        n = rng.choice([0, 1, 2, 9, 10, 11, rng.randint(0, 160), 150, 150])
        g = rng.choice([0, 1, 9, 10, 11, rng.randint(0, n + 1), n])
        g = min(g, n)
        s = rand_seq(rng, n - g) + "G" * g
        if g and rng.random() < 0.5:
            s = mutate(rng, s[: n - g], 0) + mutate(rng, "G" * g, rng.randint(1, 4))
        if rng.random() < 0.1:
            s = s.lower()
        p = rng.choice([[1, 10, 10], [10, 1, 10], [rng.randint(0, 20), rng.randint(0, 12), rng.randint(1, 12)]])
        out.append(case("polyg", ",".join(str(x) for x in p), s, rand_qual(rng, n)))
    return out


def gen_polyx(rng):
    out = []
    for _ in range(700):
        n = rng.choice([0, 1, 5, 9, 10, 11, rng.randint(0, 160), 150])
        base = rng.choice("ATCGN")
        g = min(n, rng.choice([0, 1, 9, 10, 11, rng.randint(0, n + 1)]))
        s = rand_seq(rng, n - g) + mutate(rng, base * g, rng.randint(0, 3) if base != "N" else 0)
        if rng.random() < 0.05:
            s = s.lower()
        chars = "".join(c for c in "ATCGN" if rng.random() < 0.6)
        p = [rng.choice([10, 10, 0, 1, 5, 20]), rng.choice([1, 1, 2, 5, 0]), rng.choice([10, 10, 8, 1, 3])]
        out.append(case("polyx", ",".join(str(x) for x in p), s, rand_qual(rng, n), extra=chars))
    return out


def make_pair(rng, L1, L2, ins, err1=0, err2=0, ad=True):
    frag = rand_seq(rng, max(ins, 0), n_rate=0.002)
    r1 = frag[:L1]
    if len(r1) < L1:
        r1 += (ADAPTER1 if ad else "") + "G" * L1
        r1 = r1[:L1]
    r2 = revcomp(frag)[:L2]
    if len(r2) < L2:
        r2 += (ADAPTER2 if ad else "") + "G" * L2
        r2 = r2[:L2]
    return mutate(rng, r1, err1), mutate(rng, r2, err2)


def gen_overlap(rng, kind="overlap"):
    out = []
    for _ in range(900 if kind == "overlap" else 400):
        L1 = rng.choice([150, 150, 100, rng.randint(0, 160), rng.randint(0, 40)])
        L2 = rng.choice([150, 150, L1, rng.randint(0, 160), rng.randint(0, 40)])
        ins = rng.choice([rng.randint(20, 320), rng.randint(100, 200), rng.randint(150, 280)])
        r1, r2 = make_pair(rng, L1, L2, ins, rng.choice([0, 0, 1, 3, 4, 5, 6, 10]),
                           rng.choice([0, 0, 1, 3, 5]))
        if rng.random() < 0.05:
            r1 = r1.lower()
        if rng.random() < 0.05:
            r2 = r2.lower()
        p = rng.choice([[5, 30], [5, 30], [5, 30], [rng.randint(0, 10), rng.randint(0, 60)]])
        out.append(case(kind, ",".join(str(x) for x in p), r1, rand_qual(rng, len(r1)), r2,
                        rand_qual(rng, len(r2))))
    # exactly 5 mismatches placed around position 49/50 of an otherwise perfect overlap
    for pos5 in [45, 48, 49, 50, 51, 55]:
        for L in [150, 60, 51, 50, 49]:
            frag = rand_seq(rng, L, n_rate=0)
            r1 = frag
            r2 = revcomp(frag)
            rc2 = list(revcomp(r2))
            for k in [0, 10, 20, 30, pos5][: 5]:
                if k < L:
                    rc2[k] = "A" if rc2[k] != "A" else "C"
            r2 = revcomp("".join(rc2))
            out.append(case(kind, "5,30", r1, rand_qual(rng, L), r2, rand_qual(rng, L)))
    return out


def gen_merge(rng):
    out = []
    names = ["@NS500511:211:HGMYTBGX9:1:11101:4574:1050 1:N:0:TAGTTCC", "@noSpaceName", "@ x", "@a b c",
             "@SYN:1:1101:1:2 1:N:0:ACGTACGT"]
    for c in gen_overlap(rng, "merge"):
        f = c.split("\t")
        f[6] = rng.choice(names)
        out.append("\t".join(f))
    return out


def gen_adseq(rng):
    out = []
    for _ in range(900):
        n = rng.choice([0, 3, 4, 5, 8, 20, rng.randint(0, 160), 150, 150])
        alen = rng.choice([0, 3, 4, 5, 7, 8, 11, 12, 15, 16, 20, 33, 33, 33])
        ad = rng.choice([ADAPTER1, ADAPTER2, rand_seq(rng, 40, n_rate=0)])[:alen]
        if rng.random() < 0.05:
            ad = ad.lower()
        pos = rng.choice([rng.randint(-4, n), rng.randint(max(0, n - 40), n + 1), -4, -3, -2, -1, 0])
        if pos >= 0:
            s = rand_seq(rng, pos) + ad + rand_seq(rng, n)
        else:
            s = ad[-pos:] + rand_seq(rng, n)
        s = mutate(rng, s[:n], rng.choice([0, 0, 1, 2, 5]))
        if rng.random() < 0.05:
            s = s.lower()
        out.append(case("adseq", str(rng.choice([0, 1])), s, rand_qual(rng, len(s)), extra=ad))
    return out


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the harness first: make -f oracle/Makefile.ref -j8")
    rng = random.Random(20261015)
    gens = {"pass": gen_pass, "cut": gen_cut, "polyg": gen_polyg, "polyx": gen_polyx,
            "overlap": gen_overlap, "merge": gen_merge, "adseq": gen_adseq,
            "adov": lambda r: [c.replace("overlap", "adov", 1) for c in gen_overlap(r, "overlap")[:500]]}
    for kind, g in gens.items():
        cases = g(rng)
        res = subprocess.run([HARNESS], input="\n".join(cases) + "\n", capture_output=True, text=True,
                             check=True)
        answers = res.stdout.rstrip("\n").split("\n")
        assert len(answers) == len(cases), (kind, len(answers), len(cases))
        path = os.path.join(HERE, f"kat_{kind}.tsv")
        with open(path, "w") as f:
            for c, a in zip(cases, answers):
                a_cols = a.split("\t")[2:]
                f.write(c + "\t|\t" + "\t".join(a_cols) + "\n")
        print(f"{kind}: {len(cases)} cases -> {os.path.relpath(path, REPO)}")


if __name__ == "__main__":
    main()
