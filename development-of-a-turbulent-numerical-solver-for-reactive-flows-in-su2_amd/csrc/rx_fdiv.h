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
// does not. The viscous kernels' operands (mass and molar fractions, densities, diffusion coefficients, lengths, areas,
// mechanism constants) stay far inside that range; tests/test_gpu_fdiv.py checks the two sequences bitwise on random
// operands across it and on the special values. RX_FDIV=0 at build time turns every rx_div back into `/`.
// Divisors that are compile-time constants keep `/` (the compiler may fold its own reciprocal of a constant).
#pragma once
#include <hip/hip_runtime.h>

#ifndef RX_FDIV
#define RX_FDIV 1
#endif

namespace rx {

struct Recip {
  double d, y;  // the divisor and its refined reciprocal (the compiler's y)
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
  return Recip{d, y};
#else
  return Recip{d, 0.0};
#endif
}

__device__ __host__ __forceinline__ double rx_div(double n, const Recip& r) {
#if RX_FDIV_DEV
  const double q = n * r.y;
  const double e = __builtin_fma(-r.d, q, n);
  return __builtin_amdgcn_div_fixup(__builtin_fma(e, r.y, q), r.d, n);
#else
  return n / r.d;
#endif
}

}  // namespace rx
