"""The oracle's fused multiply-add emulation (oracle/fma.py) is the correctly rounded
a*b + c the HIP Hopper step computes with v_fma_f64 (envs.h fmad): checked against
exact rational arithmetic (Python's float(Fraction) rounds half-to-even)."""
from fractions import Fraction

import numpy as np

from oracle import fma as F


def _exact(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def test_fma_emulation_is_correctly_rounded():
    rng = np.random.default_rng(7)
    N = 6000
    a = rng.standard_normal(N) * 2.0 ** rng.integers(-30, 30, N)
    b = rng.standard_normal(N) * 2.0 ** rng.integers(-30, 30, N)
    c = rng.standard_normal(N) * 2.0 ** rng.integers(-60, 60, N)
    q = N // 6
    c[:q] = -(a[:q] * b[:q]) * (1 + rng.standard_normal(q) * 1e-15)  # near-cancellation
    c[q:2 * q] = -(a[q:2 * q] * b[q:2 * q])                            # the rounded product
    # products of 27-bit integers plus half-integers: ties and exact cases
    a[-q:] = rng.integers(1, 2 ** 27, q).astype(float)
    b[-q:] = rng.integers(1, 2 ** 27, q).astype(float)
    c[-q:] = rng.integers(-2 ** 53, 2 ** 53, q).astype(float) * 0.5
    got = F.fma(a, b, c)
    want = np.array([_exact(x, y, z) for x, y, z in zip(a, b, c)])
    np.testing.assert_array_equal(got, want)
    # differs from the unfused expression somewhere (the test exercises rounding)
    assert np.any(got != a * b + c)


def test_fma_scalar_and_plain_mode():
    assert F.fma(0.1, 10.0, -1.0) == _exact(0.1, 10.0, -1.0)
    with F.plain():
        assert F.fma(0.1, 10.0, -1.0) == 0.1 * 10.0 - 1.0
    assert F.EXACT
