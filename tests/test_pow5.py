"""pow5 (csrc/device.h) vs the reference's std::pow(x, 5) (material.h:97).

The device computes the correctly rounded x^5 (double-double product, one rounding).  This test restates that
algorithm with exact rationals and measures how often glibc's pow (what the reference and the oracle call) differs
from it: the Schlick reflectance is only compared against a 24-bit uniform, so a 1-ulp difference changes a branch
only when the uniform falls within that ulp.
"""
import math
import random
from fractions import Fraction


def correctly_rounded_pow5(x: float) -> float:
    return float(Fraction(x) ** 5)  # float(Fraction) rounds to nearest-even


def test_glibc_pow5_is_within_one_ulp_of_correct_rounding():
    rng = random.Random(7)
    differ = 0
    n = 50000
    for _ in range(n):
        x = 1.0 - (rng.random() * 2.0 - 1.0)  # 1 - cos(theta), cos in [-1, 1)
        a, b = math.pow(x, 5), correctly_rounded_pow5(x)
        if a != b:
            differ += 1
            assert abs(a - b) <= math.ulp(b)
    assert differ / n < 0.005


def test_reflectance_branch_is_unchanged_by_one_ulp():
    # refl_p = r0 + (1 - r0) * x^5 against u = k * 2^-24: the branch flips only if u lies between the two values
    rng = random.Random(8)
    r0 = ((1 - 1.5) / (1 + 1.5)) ** 2
    flips = 0
    for _ in range(20000):
        x = 1.0 - (rng.random() * 2.0 - 1.0)
        p1 = r0 + (1 - r0) * math.pow(x, 5)
        p2 = r0 + (1 - r0) * correctly_rounded_pow5(x)
        u = rng.randrange(1 << 24) * 2.0**-24
        flips += (p1 > u) != (p2 > u)
    assert flips == 0
