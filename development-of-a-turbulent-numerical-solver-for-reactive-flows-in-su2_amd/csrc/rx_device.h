// rx_device.h — device-side physics of the reactive-RANS hot path (gfx950, FP64).
//
// Restates, for one edge / one cell, the reference operators cited per function (paths relative to
// the reference root). Compiled with -ffp-contract=off so every expression rounds exactly as the
// x86-64 reference (no FMA contraction); only transcendental calls (exp, pow, log, sqrt, cbrt) may
// differ by an ulp from glibc.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rx_fdiv.h"

namespace rx {

#ifndef RX_SUMM_TILE
#define RX_SUMM_TILE 64  // build knob: edges per tile of the viscous summary scratch (1: edge-major records)
#endif
constexpr int kSummTile = RX_SUMM_TILE;  // edges per tile of the viscous summary scratch (rx_visc.h SummRef)
constexpr double kEPS = 1.0e-16;  // Common/include/option_structure.hpp:134
constexpr double kNA = 6.02214129 * 1.0e23;
constexpr double kKB = 1.3806488 * 1.0e-23;
constexpr double kR = kNA * kKB * 1.0e3;           // physical_chemical_library.hpp:575
constexpr double kRatm = 1.0e-3 * 0.082057338;     // :579
constexpr double kTWO3 = 2.0 / 3.0;
enum { P_CP = 0, P_H = 1, P_S = 2, P_MU = 3, P_KAPPA = 4 };
enum { ERR_NONE = 0, ERR_RANGE = 1, ERR_NAN = 2, ERR_GEOM = 3, ERR_CONV = 4, ERR_NAN_UPWIND = 5 };  // 5: fused AUSM pass

constexpr int kMaxNS = 12;
constexpr int kMaxNR = 8;

// Mechanism + spline tables resident in HBM (~1 MB at Ns = 9: L2 / MALL resident).
struct DevMech {
  int ns, nr, ntab;
  const double *mm;             // [ns]
  const double *sr, *sp;        // [ns][nr]
  const double *er, *ep;        // [nr][ns]
  const double *A, *beta, *Ta, *Ab, *betab, *Tab;
  const int *rev, *hasb;
  const double *tx, *ty, *ty2;  // [5][ns][ntab]
  double mtot;                  // sum of molar masses
  int xshared;                  // 1: every tx row is the same grid (spline_at / spline_k)
  // transport constants of the mechanism, evaluated once on the host with the reference's expressions
  // (ComputeEta / ComputeLambda :634-696, GetDij_SM :751-766 of reacting_model_library.cpp):
  const double *phic;           // [ns][ns] sqrt(8 (1 + M_a / M_b))
  const double *pw25;           // [ns][ns] pow(M_b / M_a, 0.25)
  const double *mij;            // [ns][ns] sqrt(M_a M_b / (M_a + M_b))
  const double *dvs;            // [ns][ns] cbrt(V_a) + cbrt(V_b)
  const double *rmm;            // [ns] rx_recip(mm[s]).y, made on the device (k_recip_table): quotients by M_s
  const double *rphic;          // [ns][ns] rx_recip(phic).y (Wilke's mixing rule, k_set_primitive)
  uint32_t neg_reac[kMaxNR], neg_prod[kMaxNR];  // species masks with negative rate exponents
};

// the divisor M_s with its reciprocal (rx_fdiv.h); host passes divide directly
__device__ __host__ inline Recip mm_recip(const DevMech& m, int s) {
#if RX_FDIV_DEV
  return Recip{m.mm[s], m.rmm[s]};
#else
  return Recip{m.mm[s], 0.0};
#endif
}
__device__ __host__ inline Recip phic_recip(const DevMech& m, int ab) {
#if RX_FDIV_DEV
  return Recip{m.phic[ab], m.rphic[ab]};
#else
  return Recip{m.phic[ab], 0.0};
#endif
}

// MathTools::GetSpline (Common/src/Tools/spline.cpp:62-77). Out of range sets *err (the reference
// throws std::out_of_range).
__device__ __host__ inline double spline(const DevMech& m, int prop, int s, double T, int* err) {
  const size_t off = (size_t)(prop * m.ns + s) * m.ntab;
  const double* x = m.tx + off;
  const double* y = m.ty + off;
  const double* y2 = m.ty2 + off;
  const double x0 = x[0], xn = x[m.ntab - 1];
  if (T < x0 || T > xn) {
    *err = ERR_RANGE;
    return 0.0;
  }
  const double h = x[1] - x0;
  const Recip rh = rx_recip(h);  // three quotients by h (rx_fdiv.h: the same doubles as `/`)
  unsigned long klo = (unsigned long)(rx_div(T - x0, rh) + 1);
  if (klo > (unsigned long)(m.ntab - 1)) klo = m.ntab - 1;  // T == Tmax reads x[n] in the reference
  const double a = rx_div(x[klo] - T, rh);
  const double b = rx_div(T - x[klo - 1], rh);
  return a * y[klo - 1] + b * y[klo] + ((a * a * a - a) * y2[klo - 1] + (b * b * b - b) * y2[klo]) * (h * h) / 6.0;
}

// The same spline with the interval search done once per temperature. Every shipped mechanism tabulates all its
// species and properties on one temperature grid (DevMech::xshared, checked bitwise on the host at upload): then
// klo, a, b and h of spline() are the same for every (prop, s) row at a given T, and spline_k() returns exactly
// spline()'s double from them. Without a shared grid spline_k() falls back to spline() row by row.
struct SplineAt {
  unsigned long klo;
  double a, b, hh;
  bool ok;
};
__device__ __host__ inline SplineAt spline_at(const DevMech& m, double T) {
  SplineAt k{1, 0.0, 0.0, 0.0, false};
  if (!m.xshared) return k;
  const double* x = m.tx;
  const double x0 = x[0], xn = x[m.ntab - 1];
  if (T < x0 || T > xn) return k;
  const double h = x[1] - x0;
  const Recip rh = rx_recip(h);
  unsigned long klo = (unsigned long)(rx_div(T - x0, rh) + 1);
  if (klo > (unsigned long)(m.ntab - 1)) klo = m.ntab - 1;
  k.klo = klo;
  k.a = rx_div(x[klo] - T, rh);
  k.b = rx_div(T - x[klo - 1], rh);
  k.hh = h * h;
  k.ok = true;
  return k;
}
__device__ __host__ inline double spline_k(const DevMech& m, int prop, int s, double T, const SplineAt& k, int* err) {
  if (!m.xshared) return spline(m, prop, s, T, err);
  if (!k.ok) {
    *err = ERR_RANGE;
    return 0.0;
  }
  const size_t off = (size_t)(prop * m.ns + s) * m.ntab;
  const double* y = m.ty + off;
  const double* y2 = m.ty2 + off;
  const double a = k.a, b = k.b;
  return a * y[k.klo - 1] + b * y[k.klo] + ((a * a * a - a) * y2[k.klo - 1] + (b * b * b - b) * y2[k.klo]) * k.hh / 6.0;
}

// ReactingModelLibrary::SetMassFractions + SetMolarFromMass (reacting_model_library.cpp:65-93)
template <int NS>
__device__ __host__ inline void molar_from_mass(const DevMech& m, const double* ys, double* xs) {
  double yc[NS];
  double sy = 0.0, sx = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double y = ys[s];
    if (y < 0.0) y = 1.0e-30;
    yc[s] = y;
    xs[s] = rx_div(y, mm_recip(m, s));
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) sy += yc[s];
#pragma unroll
  for (int s = 0; s < NS; ++s) sx += xs[s];
  const double tot = sy / sx;
#pragma unroll
  for (int s = 0; s < NS; ++s) xs[s] = tot * xs[s];
}

// ------------------------------------------------------------------------------------------------
// AUSM+-up, CUpwReactiveAUSM::ComputeResidual (SU2_CFD/src/numerics_direct_reactive.cpp:53-378).
// The per-edge scalars are computed once; the residual and the Jacobian entries are evaluated
// from them in exactly the reference's operation order.
// ------------------------------------------------------------------------------------------------
// Runtime index into a small register array without dynamic indexing (keeps it out of scratch).
template <int N>
__device__ __host__ inline double pick(const double* a, int idx) {
  double v = a[0];
#pragma unroll
  for (int q = 1; q < N; ++q) {
    double aq = a[q];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(aq));  // a value, not a load: the selects cannot fold back into an indexed load
#endif
    v = (idx == q) ? aq : v;
  }
  return v;
}

struct AusmEdge {
  double Area, UN[3];
  double rho_i, rho_j, p_i, p_j, pv_i, pv_j;
  double mss, mL, mR, mF, mF2, mRef2, fa, alpha, m12, mLF, mRF, M12, pLP, pRM, factor, fpos, sign_m12;
  double pLF;
};

template <int NDIM>
__device__ __host__ inline void ausm_scalars(const double* Vi, const double* Vj, const double* Normal, double mInfty,
                                             AusmEdge& s) {
  constexpr int VX = 1, P_ = NDIM + 1, RHO = NDIM + 2, A_ = NDIM + 4;
  double Area = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) Area += Normal[d] * Normal[d];
  Area = sqrt(Area);
  s.Area = Area;
  {
    const Recip rA = rx_recip(Area);  // (rx_fdiv.h: the same doubles as `/`)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) s.UN[d] = rx_div(Normal[d], rA);
  }
  s.rho_i = Vi[RHO];
  s.rho_j = Vj[RHO];
  s.p_i = Vi[P_];
  s.p_j = Vj[P_];
  double pvi = 0.0, pvj = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    pvi += Vi[VX + d] * s.UN[d];
    pvj += Vj[VX + d] * s.UN[d];
  }
  s.pv_i = pvi;
  s.pv_j = pvj;
  const double mss = 0.5 * (Vi[A_] + Vj[A_]);
  s.mss = mss;
  const Recip rmss = rx_recip(mss);
  const double mL = rx_div(pvi, rmss), mR = rx_div(pvj, rmss);
  s.mL = mL;
  s.mR = mR;
  const double mF2 = 0.5 * (mL * mL + mR * mR);
  const double mRef2 = fmin(1.0, fmax(mF2, mInfty * mInfty));
  s.mF2 = mF2;
  s.mRef2 = mRef2;
  s.mF = sqrt(mF2);
  const double mRef = sqrt(mRef2);
  const double fa = mRef * (2.0 - mRef);
  s.fa = fa;
  const double alpha = 3.0 / 16.0 * (5.0 * fa * fa - 4.0);
  s.alpha = alpha;
  const double beta = 0.125;
  double mLP, mRM, pLP, pRM;
  if (fabs(mL) < 1.0) {
    mLP = 0.25 * (mL + 1.0) * (mL + 1.0) + beta * (mL * mL - 1.0) * (mL * mL - 1.0);
    pLP = 0.25 * (mL + 1.0) * (mL + 1.0) * (2.0 - mL) + alpha * mL * (mL * mL - 1.0) * (mL * mL - 1.0);
  } else {
    mLP = 0.5 * (mL + fabs(mL));
    pLP = 0.5 * (1.0 + rx_div(fabs(mL), rx_recip(mL)));
  }
  if (fabs(mR) < 1.0) {
    mRM = -0.25 * (mR - 1.0) * (mR - 1.0) - beta * (mR * mR - 1.0) * (mR * mR - 1.0);
    pRM = 0.25 * (mR - 1.0) * (mR - 1.0) * (2.0 + mR) - alpha * mR * (mR * mR - 1.0) * (mR * mR - 1.0);
  } else {
    mRM = 0.5 * (mR - fabs(mR));
    pRM = 0.5 * (1.0 - rx_div(fabs(mR), rx_recip(mR)));
  }
  s.pLP = pLP;
  s.pRM = pRM;
  const double kP = 0.25, sigma = 1.0;
  double m12 = mLP + mRM;
  m12 -= rx_div(rx_div(kP, rx_recip(fa)) * fmax(1.0 - sigma * mF2, 0.0) * (s.p_j - s.p_i),
                rx_recip(0.5 * (s.rho_i + s.rho_j) * mss * mss));
  s.m12 = m12;
  s.mLF = 0.5 * (m12 + fabs(m12));
  s.mRF = 0.5 * (m12 - fabs(m12));
  s.M12 = mss * (s.mLF * s.rho_i + s.mRF * s.rho_j);
  const double Ku = 0.75;
  double pLF = pLP * s.p_i + pRM * s.p_j;
  pLF -= Ku * pLP * pRM * (s.rho_i + s.rho_j) * fa * mss * (pvj - pvi);
  s.pLF = pLF;
  s.factor = fmax(1.0 - sigma * mF2, 0.0);
  s.fpos = (s.factor > 0.0) ? 1.0 : 0.0;
  s.sign_m12 = (m12 != 0.0) ? rx_div(fabs(m12), rx_recip(m12)) : 0.0;
}

// Phi (the convected state) for index v of the conservative vector.
template <int NDIM>
__device__ __host__ inline double ausm_phi(const double* V, double h, int v) {
  // RHO: 1, momentum: velocity, RHOE: enthalpy, species: mass fraction
  if (v == 0) return 1.0;
  if (v <= NDIM) return V[v];
  if (v == NDIM + 1) return h;
  return V[NDIM + 5 + (v - NDIM - 2)];
}

// Residual component v (:180-188).
template <int NDIM>
__device__ __host__ inline double ausm_res(const AusmEdge& s, const double* Vi, const double* Vj, int v) {
  constexpr int H_ = NDIM + 3;
  const double pi = ausm_phi<NDIM>(Vi, Vi[H_], v), pj = ausm_phi<NDIM>(Vj, Vj[H_], v);
  double r = 0.5 * (s.M12 * (pi + pj) + fabs(s.M12) * (pi - pj)) * s.Area;
  if (v >= 1 && v <= NDIM) r += s.pLF * s.UN[v - 1] * s.Area;
  return r;
}

// Per-column (b) derivative vectors of the Jacobian (:216-358).
struct AusmCol {
  double PlL, MiL, PlR, MiR, PDL, PDR;
};

template <int NDIM>
__device__ __host__ inline AusmCol ausm_col_impl(const AusmEdge& s, double Sib, double Sjb, int b) {
  const double kP = 0.25, sigma = 1.0, beta = 0.125, Ku = 0.75;
  const double mL = s.mL, mR = s.mR, mss = s.mss, fa = s.fa, alpha = s.alpha;
  const double rho_i = s.rho_i, rho_j = s.rho_j;
  // divisors shared by several quotients, each with its reciprocal (rx_fdiv.h: the same doubles as `/`)
  const Recip rri = rx_recip(rho_i), rrj = rx_recip(rho_j);
  double MLD = 0.0, MRD = 0.0;
  if (b == 0) {
    MLD = rx_div(-mL, rri);
    MRD = rx_div(-mR, rrj);
  } else if (b <= NDIM) {
    const double unb = pick<NDIM>(s.UN, b - 1);
    MLD = rx_div(unb, rx_recip(rho_i * mss));
    MRD = rx_div(unb, rx_recip(rho_j * mss));
  }
  double MPL, MPR;
  if (fabs(mL) < 1.0) MPL = MLD * (0.5 * (mL + 1.0) + 4.0 * beta * mL * (mL * mL - 1.0));
  else MPL = MLD * (0.5 * (1.0 + rx_div(fabs(mL), rx_recip(mL))));
  if (fabs(mR) < 1.0) MPR = MRD * (0.5 * (1.0 - mR) + 4.0 * beta * mR * (1.0 - mR * mR));
  else MPR = MRD * (0.5 * (1.0 - rx_div(fabs(mR), rx_recip(mR))));
  double SL = 0.0, SR = 0.0;
  if (s.mF2 == s.mRef2) {
    const Recip rmF = rx_recip(s.mF);
    SL = rx_div(MLD * mL * (1.0 - s.mF), rmF);
    SR = rx_div(MRD * mR * (1.0 - s.mF), rmF);
  }
  const double MD = 0.5 * (rho_i + rho_j);
  const double dp = s.p_j - s.p_i;
  const Recip rme = rx_recip(mss * mss * fa * fa * MD * MD);
  double MEL = rx_div(-kP, rme) *
               ((s.fpos * sigma * mL * MLD * dp * fa * MD) + (s.factor * Sib * fa * MD) + (s.factor * dp * MD * SL));
  double MER = rx_div(kP, rme) *
               ((s.fpos * sigma * mR * MRD * (s.p_i - s.p_j) * fa * MD) + (s.factor * Sjb * fa * MD) -
                (s.factor * dp * MD * SR));
  if (b == 0) {
    const double kq = rx_div(kP, rx_recip(mss * mss * fa * MD * MD));  // kP / (mss^2 fa MD^2), both rows
    MEL -= kq * 0.5 * s.factor * dp;
    MER -= kq * 0.5 * s.factor * dp;
  }
  AusmCol c;
  c.PlL = 0.5 * (MPL - MEL) * (1.0 + s.sign_m12);
  c.MiL = 0.5 * (MPL - MEL) * (1.0 - s.sign_m12);
  c.PlR = 0.5 * (MPR - MER) * (1.0 + s.sign_m12);
  c.MiR = 0.5 * (MPR - MER) * (1.0 - s.sign_m12);
  double PPL = 0.0, PPR = 0.0;
  if (fabs(mL) < 1.0)
    PPL = 0.25 * (mL + 1.0) * (3.0 * (1.0 - mL) + 4.0 * alpha * (5.0 * mL * mL - 1.0) * (mL - 1.0)) * MLD +
          15.0 / 8.0 * SL * mL * (mL * mL - 1.0) * (mL * mL - 1.0);
  if (fabs(mR) < 1.0)
    PPR = 0.25 * (mR - 1.0) * (3.0 * (1.0 + mR) + 4.0 * alpha * (1.0 - 5.0 * mR * mR) * (mR + 1.0)) * MRD -
          15.0 / 8.0 * SR * mR * (mR * mR - 1.0) * (mR * mR - 1.0);
  const double dvn = s.pv_j - s.pv_i;
  double PEL = Ku * s.pRM * mss * ((PPL * (rho_i + rho_j) * fa * dvn) + (s.pLP * (rho_i + rho_j) * dvn * SL));
  double PER = Ku * s.pLP * mss * ((PPR * (rho_i + rho_j) * fa * dvn) + (s.pRM * (rho_i + rho_j) * dvn * SR));
  if (b == 0) {
    PEL += Ku * s.pRM * mss * s.pLP * fa * (dvn + rx_div((rho_i + rho_j) * s.pv_i, rri));
    PER += Ku * s.pLP * mss * s.pRM * fa * (dvn - rx_div((rho_i + rho_j) * s.pv_j, rrj));
  } else if (b <= NDIM) {
    const double unb = pick<NDIM>(s.UN, b - 1);
    PEL -= rx_div(Ku * s.pRM * mss * s.pLP * fa * (rho_i + rho_j) * unb, rri);
    PER += rx_div(Ku * s.pLP * mss * s.pRM * fa * (rho_i + rho_j) * unb, rrj);
  }
  c.PDL = s.pLP * Sib + s.p_i * PPL - PEL;
  c.PDR = s.pRM * Sjb + s.p_j * PPR - PER;
  return c;
}

template <int NDIM>
__device__ __host__ inline AusmCol ausm_col(const AusmEdge& s, const double* Si, const double* Sj, int b) {
  return ausm_col_impl<NDIM>(s, Si[b], Sj[b], b);
}

// ausm_col for one column b given Si[b], Sj[b] (same arithmetic as ausm_col).
template <int NDIM>
__device__ __host__ inline AusmCol ausm_col_b(const AusmEdge& s, double Sib, double Sjb, int b) {
  return ausm_col_impl<NDIM>(s, Sib, Sjb, b);
}

// Jacobian entry (a, b) of Jac_i (left) and Jac_j (right), accumulation order of :295-374.
template <int NDIM>
__device__ __host__ inline void ausm_jac_entry(const AusmEdge& s, const AusmCol& c, double phia_i, double phia_j,
                                               double Sib, double Sjb, int a, int b, double* ji, double* jj) {
  double vi = 0.0, vj = 0.0;
  vi += s.mss * ((c.PlL * s.rho_i * phia_i) + (c.MiL * s.rho_j * phia_j));
  vj += s.mss * ((c.PlR * s.rho_i * phia_i) + (c.MiR * s.rho_j * phia_j));
  if (a == b) {
    vi += s.mss * s.mLF;
    vj += s.mss * s.mRF;
  }
  if (a == NDIM + 1) {
    vi += s.mss * s.mLF * Sib;
    vj += s.mss * s.mRF * Sjb;
  }
  if (a >= 1 && a <= NDIM) {
    vi += s.UN[a - 1] * c.PDL;
    vj += s.UN[a - 1] * c.PDR;
  }
  *ji = vi * s.Area;
  *jj = vj * s.Area;
}

// The entry of one side only (side 0: Jac_i, 1: Jac_j): the two sides' expressions differ only in the operands
// (PlL / PlR, MiL / MiR, mLF / mRF, Sib / Sjb, PDL / PDR), so they are selected first and the entry is evaluated once
// — the same operations as ausm_jac_entry's vi / vj on the same values. Sb: this side's S[b].
template <int NDIM>
__device__ __host__ inline double ausm_jac_entry_own(const AusmEdge& s, const AusmCol& c, double phia_i, double phia_j,
                                                     double Sb, int a, int b, int side) {
  const double Pl = side ? c.PlR : c.PlL, Mi = side ? c.MiR : c.MiL, mF = side ? s.mRF : s.mLF;
  const double PD = side ? c.PDR : c.PDL;
  double v = 0.0;
  v += s.mss * ((Pl * s.rho_i * phia_i) + (Mi * s.rho_j * phia_j));
  if (a == b) v += s.mss * mF;
  if (a == NDIM + 1) v += s.mss * mF * Sb;
  if (a >= 1 && a <= NDIM) v += s.UN[a - 1] * PD;
  return v * s.Area;
}


// ---- correctly rounded x^1.75 (x > 0, normal), for ReactingModelLibrary::GetDij_SM's pow(T, 1.75)
// (reacting_model_library.cpp:751-766). The host libm's pow is correctly rounded for all but ~0.07 % of the
// temperatures (measured against an 80-digit evaluation), the device's pow is only faithful; both binary
// diffusion coefficients feed the cancelling dJ/drho terms of the viscous Jacobian (Ds ~ 1e21 at pure-species
// points), so the device rounds exactly: starting from pow()'s result r, step to the neighbour while the
// midpoint m between r and it satisfies m^4 < x^7 (resp. >), both sides in double-double (rel. err < 2^-100).
struct DD {
  double hi, lo;
};
__device__ __forceinline__ DD dd_two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
__device__ __forceinline__ DD dd_norm(double s, double e) {
  const double h = s + e;
  return {h, e - (h - s)};
}
__device__ __forceinline__ DD dd_mul(DD a, DD b) {
  DD p = dd_two_prod(a.hi, b.hi);
  const double e = p.lo + (a.hi * b.lo + a.lo * b.hi);
  return dd_norm(p.hi, e);
}
__device__ __forceinline__ DD dd_mul_d(DD a, double b) {
  DD p = dd_two_prod(a.hi, b);
  return dd_norm(p.hi, p.lo + a.lo * b);
}
// sign of a - b for double-doubles
__device__ __forceinline__ int dd_cmp(DD a, DD b) {
  const double d = (a.hi - b.hi) + (a.lo - b.lo);
  return (d > 0.0) - (d < 0.0);
}
__device__ inline double pow175_cr(double x) {
  const DD x2 = dd_two_prod(x, x);
  const DD x4 = dd_mul(x2, x2);
  const DD x7 = dd_mul_d(dd_mul(x4, x2), x);  // x^7
  double r = pow(x, 1.75);
  auto fourth = [](double hi, double lo) {
    const DD m{hi, lo};
    const DD m2 = dd_mul(m, m);
    return dd_mul(m2, m2);
  };
  for (int it = 0; it < 4; ++it) {
    const double up = __longlong_as_double(__double_as_longlong(r) + 1);
    const double dn = __longlong_as_double(__double_as_longlong(r) - 1);
    if (dd_cmp(x7, fourth(r, 0.5 * (up - r))) > 0) {
      r = up;
    } else if (dd_cmp(x7, fourth(r, -0.5 * (r - dn))) < 0) {
      r = dn;
    } else {
      break;
    }
  }
  return r;
}

}  // namespace rx
