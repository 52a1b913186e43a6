"""rx_fdiv.h's shared-divisor division (rx_recip once per divisor, rx_div per quotient) against the compiler's FP64
`n / d` on the device, bitwise: random operands across the exponent range the viscous kernels' quotients can take, the
signed zeros, infinities and NaNs (v_div_fixup's cases), and quotients the two sequences round the same way only when
v_div_scale leaves the operands unscaled; since round 6 the guarded rx_div<true> (build knob
RX_FDIV_GUARD) against `/` over every operand — tiny and denormal numerators, huge and denormal divisors, overflowing
and denormal quotients — which it hands to the compiler's division. Uses tests/native/libfdiv_check.so (built by __graft_entry__.build()).
Requires an MI355X."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libfdiv_check.so")


def divide(n, d, guarded=False):
    assert os.path.exists(LIB), "tests/native/libfdiv_check.so is not built (make -C tests/native)"
    lib = C.CDLL(LIB)
    fn = lib.fdiv_check_guarded if guarded else lib.fdiv_check
    n = np.ascontiguousarray(n, dtype=np.float64)
    d = np.ascontiguousarray(d, dtype=np.float64)
    ref, fast = np.empty_like(n), np.empty_like(n)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    assert fn(p(n), p(d), p(ref), p(fast), C.c_int(len(n))) == 0
    return ref, fast


def random_operands(rng, count, lo, hi):
    m = rng.uniform(1.0, 2.0, count) * rng.choice([-1.0, 1.0], count)
    return np.ldexp(m, rng.integers(lo, hi, count))


def test_fdiv_matches_the_hardware_division_in_range():
    rng = np.random.default_rng(20261018)
    count = 1 << 20
    n = random_operands(rng, count, -900, 700)
    d = random_operands(rng, count, -900, 700)
    # the range v_div_scale leaves alone: |n| >= 2^-969, d normal with 1/d normal, |n / d| in [2^-1022, 2^767]
    e = np.frexp(n)[1] - np.frexp(d)[1]
    keep = (e > -1000) & (e < 760)
    n, d = n[keep], d[keep]
    # the viscous kernels' typical magnitudes too (fractions, densities, lengths, mechanism constants)
    n = np.concatenate([n, rng.uniform(-1e3, 1e3, 1 << 16), rng.uniform(0, 1, 1 << 16) ** 8])
    d = np.concatenate([d, rng.uniform(1e-6, 1e3, 1 << 16), rng.uniform(1e-3, 1, 1 << 16)])
    ref, fast = divide(n, d)
    bad = ref.view(np.uint64) != fast.view(np.uint64)
    assert not bad.any(), (int(bad.sum()), n[bad][:4], d[bad][:4], ref[bad][:4], fast[bad][:4])


def test_fdiv_special_values():
    vals = np.array([0.0, -0.0, 1.0, -1.0, 3.0, -7.5, 1e-30, -2e30, np.inf, -np.inf, np.nan])
    n, d = np.meshgrid(vals, vals, indexing="ij")
    n, d = n.ravel(), d.ravel()
    ref, fast = divide(n, d)
    nan = np.isnan(ref)
    assert np.array_equal(nan, np.isnan(fast))
    # signed zeros and infinities: the same bits (v_div_fixup applies the sign); NaN payloads are not compared
    assert np.array_equal(ref[~nan].view(np.uint64), fast[~nan].view(np.uint64)), (n[~nan], d[~nan])


def test_guarded_fdiv_matches_the_hardware_division_everywhere():
    """Round 6: rx_div<true> is `n / d` for every operand pair, not only where v_div_scale leaves them unscaled: random
    exponents over the whole double range (denormals included), tiny numerators next to the 2^-969 threshold, divisors
    at the 2^-200 / 2^52 window edges, quotients that overflow or go denormal."""
    rng = np.random.default_rng(20261019)
    count = 1 << 19
    n = random_operands(rng, count, -1074, 1024)
    d = random_operands(rng, count, -1074, 1024)
    edge_n = random_operands(rng, count, -975, -963)      # around the numerator threshold
    edge_d = np.concatenate([random_operands(rng, count // 2, -203, -197), random_operands(rng, count // 2, 49, 55)])
    tiny = np.ldexp(rng.uniform(1, 2, count), rng.integers(-1074, -1022, count))  # denormal numerators
    n = np.concatenate([n, edge_n, rng.uniform(-1, 1, count), tiny, rng.uniform(1e-3, 1, count)])
    d = np.concatenate([d, rng.uniform(1e-3, 1e3, count), edge_d, rng.uniform(1e-6, 1, count),
                        np.ldexp(rng.uniform(1, 2, count), rng.integers(-1074, -1022, count))])
    ref, fast = divide(n, d, guarded=True)
    nan = np.isnan(ref)
    assert np.array_equal(nan, np.isnan(fast))
    bad = ref[~nan].view(np.uint64) != fast[~nan].view(np.uint64)
    assert not bad.any(), (int(bad.sum()), n[~nan][bad][:4], d[~nan][bad][:4])
