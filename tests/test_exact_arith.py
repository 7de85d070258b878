"""Exact-arithmetic shortcuts of the device code (csrc/device.h), restated with rationals.

* div_rcp: x / a as q = RN(x * RN(1/a)), corrected by one fma residual step (Markstein) -- must equal the IEEE
  division bit for bit (sphere roots, camera-ray s/t).
* pow5 vs the reference's std::pow(x, 5) (material.h:97).  The device computes the correctly rounded x^5 (double-double product, one rounding).  This test restates that
algorithm with exact rationals and measures how often glibc's pow (what the reference and the oracle call) differs
from it: the Schlick reflectance is only compared against a 24-bit uniform, so a 1-ulp difference changes a branch
only when the uniform falls within that ulp.
"""
import math
import random
from fractions import Fraction


def fma(a: float, b: float, c: float) -> float:
    return float(Fraction(a) * Fraction(b) + Fraction(c))  # one rounding


def div_rcp(x: float, a: float, inv_a: float) -> float:  # csrc/device.h div_rcp
    q = x * inv_a
    return fma(fma(-q, a, x), inv_a, q)


def test_div_rcp_equals_division():
    rng = random.Random(5)
    cases = []
    for _ in range(20000):  # |d|^2 of traced rays against root numerators
        a = rng.uniform(1e-3, 100.0) * 2.0 ** rng.randint(-40, 8)
        cases.append((rng.uniform(-100, 100), a))
    for _ in range(5000):  # divisors with all-ones / minimal significands, numerators near powers of two
        a = ((1 << 53) - 1 - rng.randint(0, 200)) * 2.0 ** (-52 + rng.randint(-6, 6))
        b = ((1 << 52) + rng.randint(0, 200)) * 2.0 ** (-52 + rng.randint(-6, 6))
        x = ((1 << 53) - 1 - rng.randint(0, 50)) * 2.0 ** (-52 + rng.randint(-3, 3))
        cases += [(x, a), (x, b), (-x, a)]
    for w in (2, 3, 7, 400, 1919, 1920, 4096):  # gen_ray: (i + u) / (W - 1)
        for i in range(0, w, max(1, w // 50)):
            cases.append((i + rng.randrange(1 << 24) * 2.0**-24, float(w - 1)))
    for x, a in cases:
        assert div_rcp(x, a, 1.0 / a) == x / a, (x.hex(), a.hex())


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


def fastdiv_make(d: int):  # csrc/kernels.hip FastDiv::make
    l = 0
    while l < 32 and (1 << l) < d:
        l += 1
    return ((1 << 32) * ((1 << l) - d)) // d + 1, l


def test_fastdiv_equals_integer_division():
    rng = random.Random(9)
    divisors = [1, 2, 3, 7, 8, 16, 64, 135, 240, 1920, 32400, 2073600, (1 << 31) - 1, 1 << 31]
    divisors += [rng.randint(1, 1 << 31) for _ in range(200)]
    for d in divisors:
        m, l = fastdiv_make(d)
        assert 0 < m < (1 << 32)
        for n in [0, 1, d - 1, d, d + 1, (1 << 31) - 1] + [rng.randrange(1 << 31) for _ in range(500)]:
            if 0 <= n < (1 << 31):
                assert (((m * n) >> 32) + n) >> l == n // d, (d, n)


PCG_A, PCG_C, M64 = 6364136223846793005, 1442695040888963407, (1 << 64) - 1


def pcg_jump(steps: int):  # csrc/device.h pcg_jump: s -> a s + c after `steps` LCG steps
    a, c = 1, 0
    for _ in range(steps):
        a, c = (a * PCG_A) & M64, (c * PCG_A + PCG_C) & M64
    return a, c


def test_pcg_jump_table_matches_stepping():
    """coop_unit_sphere's helpers jump a stream ahead by 3 j draws; the affine map must equal 3 j LCG steps."""
    rng = random.Random(10)
    for _ in range(20):
        s0 = rng.getrandbits(64)
        s = s0
        for j in range(64):
            a, c = pcg_jump(3 * j)
            assert (a * s0 + c) & M64 == s, j
            for _ in range(3):
                s = (s * PCG_A + PCG_C) & M64
