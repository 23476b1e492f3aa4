"""Floating-point identities the kernels rely on to stay bit-identical to the oracle.

* rollout.hip `div_count`: a mean over n envs divides by n; when n = 2^k the kernel
  multiplies by the exact 2^-k instead.  Both are IEEE operations on the same real value
  x / 2^k, rounded once, so the results are identical -- including quotients in the
  subnormal range, signed zeros, infinities and NaN.
* scan.hip `gae_full_kernel`: a chunk's multipliers B = (gl*kk)*B over its steps are
  gl^L when no step breaks the chunk; the power is formed by the same sequence of
  multiplications, so it equals the per-step product bit for bit (kk in {0, 1}).
"""
import numpy as np


def test_division_by_power_of_two_equals_multiplication_by_its_reciprocal():
    rng = np.random.default_rng(0)
    x = np.concatenate([
        rng.standard_normal(200000) * 10.0 ** rng.integers(-300, 300, 200000),
        rng.standard_normal(1000) * 1e-310,             # subnormal inputs
        np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 1.7976931348623157e308]),
    ])
    for k in (0, 1, 6, 12, 13, 20, 52, 60):
        n = float(2 ** k)
        q_div = x / n
        q_mul = x * np.ldexp(1.0, -k)
        same = (q_div == q_mul) | (np.isnan(q_div) & np.isnan(q_mul))
        assert same.all(), k
        # signed zeros too
        assert (np.signbit(q_div) == np.signbit(q_mul)).all(), k


def test_chunk_multiplier_power_equals_per_step_products():
    for gl in (0.995 * 0.97, 0.99 * 0.95, 0.9999, 0.5, 1.0):
        for L in (1, 2, 4, 8, 16, 32):
            B = 1.0
            for _ in range(L):
                B = (gl * 1.0) * B  # gae_scan_kernel: B = gl * kk * B, kk = 1
            p = 1.0
            for _ in range(L):
                p = gl * p  # gae_full_kernel's glL
            assert B == p
