#!/usr/bin/env python3
"""Golden vectors for the JSON number formatter: how the reference's vendored JSON writer
(nlohmann 3.5.0 dump(), compiled from /root/reference/src/json.hpp into oracle/_ref/ref_grisu by
oracle/Makefile.ref; harness source oracle/harness/ref_grisu.cpp) prints each double.
Inputs: seeded ratios of integers (the report's quality / content curves and rates), random bit
patterns, powers of ten, integers, boundaries, subnormals, zeros.  Output:
tests/golden/grisu2_vectors.tsv (hex bits TAB reference text).  Development container only."""
import os
import random
import struct
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def bits(x):
    return "%016x" % struct.unpack("<Q", struct.pack("<d", x))[0]


def main():
    rng = random.Random(20261015)
    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 0.1, 0.2, 0.3, 1e15, 1e16, 1e-4, 1e-5, 1.5e-5, 123456789012345.0,
            1234567890123456.0, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, float("inf"),
            float("nan"), 9007199254740993.0, 0.30000000000000004, 36.77, 2.0 / 3.0]
    for k in range(-30, 30):
        vals.append(10.0 ** k)
        vals.append(3 * 10.0 ** k)
    for _ in range(20000):  # quality means, content ratios, rates
        den = rng.randint(1, 10 ** rng.randint(1, 9))
        num = rng.randint(0, den * rng.choice([1, 1, 41, 100]))
        vals.append(num / den)
    for _ in range(20000):  # arbitrary finite doubles
        b = rng.getrandbits(64)
        x = struct.unpack("<d", struct.pack("<Q", b))[0]
        if x == x and abs(x) != float("inf"):
            vals.append(x)
    for _ in range(5000):
        vals.append(float(rng.randint(-10 ** 17, 10 ** 17)))
    inp = "\n".join(bits(v) for v in vals) + "\n"
    out = subprocess.run([os.path.join(REPO, "oracle", "_ref", "ref_grisu")], input=inp, capture_output=True,
                         text=True, check=True).stdout
    with open(os.path.join(HERE, "grisu2_vectors.tsv"), "w") as f:
        f.write(out)
    print(len(vals), "vectors")


if __name__ == "__main__":
    main()
