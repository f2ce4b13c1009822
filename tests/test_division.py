"""The kernels' shared-divisor quotient (device_core.inc div_y / div3): y = RN(1/d) once,
then q0 = RN(n*y), q = RN(q0 - RN(d*q0 - n)*y) per numerator, claimed bit-identical to the IEEE
division n / d (Markstein's correction; the reference divides component by component, tuple.rs:95-98,
light.rs:60-61).  fma is emulated exactly with rational arithmetic (Fraction -> float rounds to
nearest, ties to even), so this checks the claim on the CPU for the magnitudes the renders use."""
import math
import random
from fractions import Fraction as F

import pytest


def fma(a, b, c):
    if a == 0.0 or b == 0.0:  # signed-zero semantics of a*b + c with an exact zero product
        return (a * b) + c
    r = F(a) * F(b) + F(c)
    if r == 0:
        return 0.0  # exact zero sum of non-zero terms is +0 in round-to-nearest
    return float(r)


def div_y(n, d, y):
    q0 = n * y
    return fma(-fma(d, q0, -n), y, q0)


def same(a, b):
    return a == b and math.copysign(1.0, a) == math.copysign(1.0, b)


@pytest.mark.parametrize("seed", range(4))
def test_div_y_matches_ieee_division(seed):
    rnd = random.Random(seed)
    for _ in range(6000):
        d = math.ldexp(rnd.random() + 0.5, rnd.randint(-40, 40))  # positive divisors (norms, distances)
        n = math.ldexp(rnd.random() * 2.0 - 1.0, rnd.randint(-45, 45))
        y = 1.0 / d
        assert same(div_y(n, d, y), n / d), (n, d)


def test_div_y_signed_zeros_and_unit_vectors():
    rnd = random.Random(7)
    for n in (0.0, -0.0):
        for d in (1.0, 3.0, 0.1, 1e30):
            assert same(div_y(n, d, 1.0 / d), n / d)
    for _ in range(4000):  # normalize(v): every component over |v|
        v = [rnd.uniform(-10, 10) for _ in range(3)]
        m = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
        y = 1.0 / m
        for c in v:
            assert same(div_y(c, m, y), c / m)


def test_area_cell_offsets():
    """(col + u) / level for every level up to RR_MAX_AREA_LEVEL (1024, rray.h), u with 32 random bits
    (jitter_value), including the extreme cells (col 0 with u = 0, col level-1 with u just below 1).
    Markstein's theorem covers every level (y = RN(1/level), q0 faithful, the residual exact in one fma);
    the samples check the implementation of it."""
    rnd = random.Random(11)
    for level in range(1, 1025):
        y = 1.0 / level
        cases = [(0, 0.0), (level - 1, (2**32 - 1) / 4294967296.0)]
        cases += [(rnd.randrange(level), rnd.getrandbits(32) * (1.0 / 4294967296.0))
                  for _ in range(40 if level <= 64 else 8)]
        for col, u in cases:
            n = col + u
            assert same(div_y(n, float(level), y), n / level), (level, col, u)
