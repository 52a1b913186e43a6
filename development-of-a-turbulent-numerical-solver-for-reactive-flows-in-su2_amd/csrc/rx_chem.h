// rx_chem.h — Arrhenius kinetics + PaSR closure for one cell (device).
//
// CSourceReactive::ComputeChemistry   SU2_CFD/src/numerics_direct_reactive.cpp:1728-1879
// ReactingModelLibrary kinetics       Common/src/Framework/reacting_model_library.cpp:
//   SetSourceTerm :99-114, Set_DfrDrhos :122-136, GetMassProductionTerm :143-154 / :196-202,
//   AssemblePaSRConstant :161-190, GetTimeCombustion_r :208-227, Set_BackFor_Contr :233-289,
//   GetTurbSourceJacobian :295-319, GetSourceJacobian :325-350, SetConcentration :701-705,
//   ComputeKeq :803-829, ComputeRateConstants :835-867, SetReactionRates :872-920.
#pragma once

#include "rx_device.h"

namespace rx {

struct SourceParams {
  double C_mu, lb, rho_ref, t_ref, T_ref;
  int rans, implicit;
};

template <int NS>
struct Kin {
  double Ys[NS], F[kMaxNR], B[kMaxNR], Kc[kMaxNR], k[kMaxNR];
};

__device__ inline double delta_gibbs(const DevMech& m, int r, double T, double* dnu, int* err) {
  double dG = 0.0, dn = 0.0;
  const SplineAt k = spline_at(m, T);  // one interval search for every species' H and S rows (rx_device.h)
  for (int s = 0; s < m.ns; ++s) {
    const double dc = m.sp[s * m.nr + r] - m.sr[s * m.nr + r];
    if (dc != 0.0) {
      dG += dc * (spline_k(m, P_H, s, T, k, err) - T * spline_k(m, P_S, s, T, k, err));
      dn += dc;
    }
  }
  *dnu = dn;
  return dG;
}

// Residual (species rows) and, if implicit, the species rows of the cell Jacobian (the other rows are zero and
// not stored): entry (species row s, column j) goes to J[(s * nVar + j) * jstride]. V: primitives, S: dT/dU.
// Returns an error code.
template <int NS, int NDIM>
__device__ inline int source_cell(const DevMech& m, const SourceParams& P, const double* V, const double* S,
                                  double vol, double omega_turb, double* res, double* J, int jstride) {
  constexpr int nVar = NS + NDIM + 2, RHOS_P = NDIM + 5, RHO_P = NDIM + 2, RHOS_S = NDIM + 2;
  const int nr = m.nr;
  int err = ERR_NONE;
  Kin<NS> k;
  const double rho = V[RHO_P];
  const double T = V[0] * P.T_ref;
  const double drho = rho * P.rho_ref;
  double Cs[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double y = V[RHOS_P + s];
    if (y < 0.0) y = 1.0e-30;
    k.Ys[s] = y;
    Cs[s] = 1.0e3 * drho * y / m.mm[s];
  }
  _Pragma("unroll") for (int r = 0; r < kMaxNR; ++r) {
    if (r >= nr) break;
    const double kf = m.A[r] * pow(T, m.beta[r]) * exp(-m.Ta[r] / T);
    double kb;
    if (!m.hasb[r]) {
      double dnu;
      const double dG = delta_gibbs(m, r, T, &dnu, &err);
      const double lnKp = -dG / (kR * T);
      const double lnKc = lnKp - dnu * log(kRatm * T);
      k.Kc[r] = exp(lnKc);
      const bool complete = exp(lnKp) > 1.0e10;
      kb = (!m.rev[r] || complete) ? 0.0 : kf / k.Kc[r];
    } else {
      kb = m.Ab[r] * pow(T, m.betab[r]) * exp(-m.Tab[r] / T);
      k.Kc[r] = kf / kb;
    }
    double fr = 0.0, br = 0.0;
    bool zero = false;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (((m.neg_reac[r] >> s) & 1u) && k.Ys[s] < 1.0e-15) zero = true;
    if (!zero) {
      fr = 1.0;
#pragma unroll
      for (int s = 0; s < NS; ++s) fr *= pow(Cs[s], m.er[r * NS + s]);
      fr *= kf;
    }
    zero = false;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (((m.neg_prod[r] >> s) & 1u) && k.Ys[s] < 1.0e-15) zero = true;
    if (!zero) {
      br = 1.0;
#pragma unroll
      for (int s = 0; s < NS; ++s) br *= pow(Cs[s], m.ep[r * NS + s]);
      br *= kb;
    }
    k.F[r] = fr;
    k.B[r] = br;
  }
  // PaSR constants (Set_DfrDrhos + AssemblePaSRConstant)
  if (P.rans) {
    const double tau_mix = 1 / (P.C_mu * omega_turb);
    _Pragma("unroll") for (int r = 0; r < kMaxNR; ++r) {
    if (r >= nr) break;
      double hd = -1.0;
#pragma unroll
      for (int s = 0; s < NS; ++s)
        if (m.sp[s * nr + r] != 0.0 || m.sr[s * nr + r] != 0.0) {
          double df = 0.0;
          if (k.Ys[s] > 1.0e-10) df = (k.F[r] * m.er[r * NS + s] - k.B[r] * m.ep[r * NS + s]) / (drho * k.Ys[s]);
          const double v = fabs(df * m.mm[s]);
          if (hd < 0.0 || v > hd) hd = v;
        }
      const double tc = 1 / hd;
      double kk;
      if (isinf(tc)) kk = 1.0;
      else if ((tc / (tc + tau_mix)) < P.lb) kk = P.lb;
      else kk = tc / (tc + tau_mix);
      k.k[r] = kk;
    }
  }
#pragma unroll
  for (int v = 0; v < nVar; ++v) res[v] = 0.0;
  const double scale = -vol / (P.rho_ref / P.t_ref);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double o = 0.0;
    _Pragma("unroll") for (int r = 0; r < kMaxNR; ++r) {
    if (r >= nr) break;
      const double wir = 1.0e-3 * m.mm[s] * (m.sp[s * nr + r] - m.sr[s * nr + r]) * (k.F[r] - k.B[r]);
      o += P.rans ? k.k[r] * wir : wir;
    }
    res[RHOS_S + s] = o * scale;
  }
  if (!P.implicit) return err;

  // Set_BackFor_Contr
  double bc[kMaxNR], fc[kMaxNR];
  {
    const double Tp = T + 1.0e-6 * T;
    const double RT = kR * Tp;
    const double lnRT = log(kRatm * Tp);
    _Pragma("unroll") for (int r = 0; r < kMaxNR; ++r) {
    if (r >= nr) break;
      double Kcp;
      if (!m.hasb[r]) {
        if (k.B[r] > 0.0) {
          double dnu;
          const double dG = delta_gibbs(m, r, Tp, &dnu, &err);
          Kcp = exp(-dG / RT - dnu * lnRT);
        } else {
          Kcp = k.Kc[r];
        }
      } else {
        const double kfp = m.A[r] * pow(Tp, m.beta[r]) * exp(-m.Ta[r] / Tp);
        const double kbp = m.Ab[r] * pow(Tp, m.betab[r]) * exp(-m.Tab[r] / Tp);
        Kcp = kfp / kbp;
      }
      const double Kcd = (Kcp - k.Kc[r]) / (Tp - T);
      const double tmp = (m.beta[r] + m.Ta[r] / T) / T;
      fc[r] = k.F[r] * tmp;
      bc[r] = !m.hasb[r] ? k.B[r] * (tmp - Kcd / k.Kc[r]) : k.B[r] * (m.betab[r] + m.Tab[r] / T) / T;
    }
  }
  for (int s = 0; s < NS; ++s) {
    // column 0 (temperature) of the [Ns][Ns+1] source Jacobian, reaction-ordered accumulation
    double sj0 = 0.0;
    _Pragma("unroll") for (int r = 0; r < kMaxNR; ++r) {
    if (r >= nr) break;
      const double fixed = 1.0e-3 * m.mm[s] * (m.sp[s * nr + r] - m.sr[s * nr + r]);
      sj0 += P.rans ? fixed * (fc[r] - bc[r]) * k.k[r] : fixed * (fc[r] - bc[r]);
    }
    const double fx = sj0 * P.t_ref * P.T_ref / P.rho_ref;
    double* row = J + (size_t)s * nVar * jstride;
    row[0] = -fx * S[0] * vol;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) row[(1 + d) * jstride] = -fx * S[1 + d] * vol;
    row[(NDIM + 1) * jstride] = -fx * S[NDIM + 1] * vol;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      double sjj = 0.0;
      _Pragma("unroll") for (int r = 0; r < kMaxNR; ++r) {
    if (r >= nr) break;
        const double fixed = 1.0e-3 * m.mm[s] * (m.sp[s * nr + r] - m.sr[s * nr + r]);
        if (k.Ys[j] > 1.0e-10) {
          const double num = k.F[r] * m.er[r * NS + j] - k.B[r] * m.ep[r * NS + j];
          if (P.rans) sjj += fixed * k.k[r] * (num / (drho * k.Ys[j]));  // Df_rDrho_i stored first
          else sjj += fixed * num / (drho * k.Ys[j]);
        }
      }
      row[(RHOS_S + j) * jstride] = -fx * S[RHOS_S + j] * vol - sjj * P.t_ref * vol;
    }
  }
  return err;
}

}  // namespace rx
