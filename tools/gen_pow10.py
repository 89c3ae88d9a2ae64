#!/usr/bin/env python3
"""Emit the cached powers of ten used by Grisu2 (fqtool_amd/host/json.cpp): for k = -300..324
step 8, the 64-bit significand f and binary exponent e with f * 2^e ~= 10^k, 2^63 <= f < 2^64,
rounded to nearest (exact rational arithmetic)."""
from fractions import Fraction


def table():
    rows = []
    for k in range(-300, 325, 8):
        v = Fraction(10) ** k
        e = v.numerator.bit_length() - v.denominator.bit_length() - 64
        scale = lambda e: Fraction(2) ** e if e >= 0 else Fraction(1, 2 ** (-e))
        while v / scale(e) >= 2 ** 64:
            e += 1
        while v / scale(e) < 2 ** 63:
            e -= 1
        f = int(v / scale(e) + Fraction(1, 2))
        if f >= 2 ** 64:
            f >>= 1
            e += 1
        rows.append((f, e, k))
    return rows


if __name__ == "__main__":
    for f, e, k in table():
        print("    {0x%016XULL, %d, %d}," % (f, e, k))
