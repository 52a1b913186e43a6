// Division by a shared divisor, bit for bit the hardware FP64 division the compiler emits for `n / d`.
//
// gfx950's `n / d` is an 11-instruction sequence (v_div_scale x2, v_rcp_f64, four FMAs refining the reciprocal y of d,
// q = n y, r = fma(-d, q, n), v_div_fmas = fma(r, y, q), v_div_fixup). The reciprocal refinement depends on d alone
// (for operands that v_div_scale leaves unscaled), so when several quotients share a divisor it is made once
// (rx_recip) and each quotient costs the last four instructions (rx_div): the same operations on the same values, hence
// the same double. v_div_fixup applies the quotient's sign and the special cases (zero, infinite or NaN operands)
// exactly as in the compiler's sequence.
//
// Exactness condition: v_div_scale scales an operand only at the ends of the exponent range — a denormal divisor or
// quotient, |d| > 2^1022, |n| < 2^-969, or |n / d| >= 2^768 — and there the compiler's sequence rescales while this one
// does not (the residual fma(-d, q, n) can go denormal: a 1-ulp difference is possible). The kernels' operands (mass
// and molar fractions, densities, diffusion coefficients, lengths, areas, mechanism constants) stay inside that range
// unless a species is depleted below 2^-969 ~ 1e-292. rx_div<true> (build knob RX_FDIV_GUARD=1 for every
// call site) closes that corner: rx_recip marks a divisor outside [2^-200, 2^52) once (Recip::wide), and rx_div sends
// such divisors and numerators whose exponent field lies outside [2^-969, 2^560) to the compiler's own `n / d`; inside
// both windows the quotient lies in [2^-1021, 2^760] and nothing is scaled, so rx_div<true> is `n / d` for every
// operand pair. It is not the default: the guard splits every division's basic block and the schedulers lose the
// interleaving of independent divisions — same box, C3 (gpurun_out r06b): VISC 1.83 -> 3.35 ms, ASSEMBLE 5.10 ->
// 6.44, PRIMITIVE 1.11 -> 1.73, 25.6 -> 29.1 ms per step. tests/test_gpu_fdiv.py checks rx_div against `/` bitwise
// inside the range and on the special values, and rx_div<true> against `/` over the whole exponent range (denormal and
// tiny numerators, huge and denormal divisors). RX_FDIV=0 at build time turns every rx_div back into `/`.
// Divisors that are compile-time constants keep `/` (the compiler may fold its own reciprocal of a constant).
#pragma once
#include <hip/hip_runtime.h>

#ifndef RX_FDIV
#define RX_FDIV 1
#endif
#ifndef RX_FDIV_GUARD
#define RX_FDIV_GUARD 0  // build knob: 1 = every rx_div guarded (rx_div<true>, above)
#endif

namespace rx {

struct Recip {
  double d, y;  // the divisor and its refined reciprocal (the compiler's y)
  bool wide;    // |d| outside [2^-200, 2^52) (or zero, infinite, NaN): every quotient takes `n / d`
};

// (host passes — the __host__ __device__ helpers of rx_device.h — keep `/`; the divisor's y is then unused)
#if RX_FDIV && defined(__HIP_DEVICE_COMPILE__)
#define RX_FDIV_DEV 1
#else
#define RX_FDIV_DEV 0
#endif

__device__ __host__ __forceinline__ Recip rx_recip(double d) {
#if RX_FDIV_DEV
  double y = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-d, y, 1.0);
  y = __builtin_fma(y, e, y);
  const double ad = __builtin_fabs(d);
  return Recip{d, y, !(ad >= 0x1p-200 && ad < 0x1p52)};
#else
  return Recip{d, 0.0, true};
#endif
}

template <bool Guard = (RX_FDIV_GUARD != 0)>
__device__ __host__ __forceinline__ double rx_div(double n, const Recip& r) {
#if RX_FDIV_DEV
  // the numerator's biased exponent outside [54, 1583) (|n| < 2^-969, denormal, zero, or |n| >= 2^560)
  const unsigned en = (unsigned)__double2hiint(n) & 0x7ff00000u;
  if (Guard && __builtin_expect(r.wide || en - (54u << 20) >= ((1583u - 54u) << 20), 0)) return n / r.d;
  const double q = n * r.y;
  const double e = __builtin_fma(-r.d, q, n);
  return __builtin_amdgcn_div_fixup(__builtin_fma(e, r.y, q), r.d, n);
#else
  return n / r.d;
#endif
}

}  // namespace rx
