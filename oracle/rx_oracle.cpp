// rx_oracle.cpp — CPU restatement of the reference hot path.
//
// TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg as the checker / CPU baseline. Never linked into, called by, or shipped with the product.
// Parity of this restatement is pinned by tests/golden/*.npz, generated from the compiled
// reference by oracle/make_golden.py (tests/test_oracle_golden.py).
//
// Every function follows the reference file:line it cites (paths relative to the reference root).
// Arithmetic is plain sequential IEEE double (built with -ffp-contract=off: the x86-64 reference
// has no FMA). Layouts (row-major, per node / per edge):
//   V   [N][nPrimVar]   T, u, v, P, rho, h, a, Y_1..Y_Ns        (variable_direct_reactive.cpp:4-17)
//   U   [N][nVar]       rho, rho u, rho v, rho E, rho_1..rho_Ns
//   G   [N][nPrimVarGrad][nDim]  T, u, v, P, X_1..X_Ns
//   Dij [N][Ns][Ns]     Eigen column-major copy (symmetric)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <vector>

#include <omp.h>

namespace {

constexpr double EPS = 1.0e-16;                         // Common/include/option_structure.hpp:134
constexpr double NA = 6.02214129 * 1.0e23;               // physical_chemical_library.hpp:571-579
constexpr double KB = 1.3806488 * 1.0e-23;
constexpr double R_UNGAS = NA * KB * 1.0e3;
constexpr double R_UNGAS_ATM = 1.0e-3 * 0.082057338;
constexpr double TWO3 = 2.0 / 3.0;
enum { P_CP = 0, P_H = 1, P_S = 2, P_MU = 3, P_KAPPA = 4 };

struct Mech {
  int ns, nr, ntab;
  std::vector<double> mm, ri, dv;
  std::vector<double> sr, sp;  // [ns][nr]
  std::vector<double> er, ep;  // [nr][ns]
  std::vector<double> A, beta, Ta, Ab, betab, Tab;
  std::vector<int> rev, hasb;
  std::vector<double> tx, ty, ty2;  // [5][ns][ntab]
  std::vector<std::vector<int>> neg_reac, neg_prod;
  double mtot;
};

// spline.cpp:62-77 (GetSpline). Out of range -> std::out_of_range, as the reference.
double spline(const Mech& m, int prop, int s, double T) {
  const double* x = &m.tx[(prop * m.ns + s) * m.ntab];
  const double* y = &m.ty[(prop * m.ns + s) * m.ntab];
  const double* y2 = &m.ty2[(prop * m.ns + s) * m.ntab];
  if (T < x[0] || T > x[m.ntab - 1]) throw std::out_of_range("temperature out of table range");
  const double h = x[1] - x[0];
  unsigned long klo = (unsigned long)((T - x[0]) / h + 1);
  const double a = (x[klo] - T) / h;
  const double b = (T - x[klo - 1]) / h;
  return a * y[klo - 1] + b * y[klo] + ((a * a * a - a) * y2[klo - 1] + (b * b * b - b) * y2[klo]) * (h * h) / 6.0;
}

// reacting_model_library.cpp:65-93 (SetMassFractions + SetMolarFromMass)
void molar_from_mass(const Mech& m, const double* ys_in, double* ys_clamped, double* xs) {
  double sy = 0.0, sx = 0.0;
  for (int s = 0; s < m.ns; ++s) {
    double y = ys_in[s];
    if (y < 0.0) y = 1.0e-30;
    ys_clamped[s] = y;
    xs[s] = y / m.mm[s];
  }
  for (int s = 0; s < m.ns; ++s) sy += ys_clamped[s];
  for (int s = 0; s < m.ns; ++s) sx += xs[s];
  const double massTot = sy / sx;
  for (int s = 0; s < m.ns; ++s) xs[s] = massTot * xs[s];
}

// ------------------------------------------------------------------------------------------------
// a1: CUpwReactiveAUSM::ComputeResidual  (SU2_CFD/src/numerics_direct_reactive.cpp:53-378)
// ------------------------------------------------------------------------------------------------
void ausm(int nDim, int ns, const double* Vi, const double* Vj, const double* Normal, const double* Si,
          const double* Sj, double mInfty, bool implicit, double* res, double* Ji, double* Jj) {
  const int nVar = ns + nDim + 2;
  const int T_ = 0, VX = 1, P_ = nDim + 1, RHO = nDim + 2, H_ = nDim + 3, A_ = nDim + 4, RHOS = nDim + 5;
  const int RHO_S = 0, RHOVX_S = 1, RHOE_S = nDim + 1, RHOS_S = nDim + 2;
  (void)T_;
  double Area = 0.0;
  for (int d = 0; d < nDim; ++d) Area += Normal[d] * Normal[d];
  Area = std::sqrt(Area);
  double UnitNormal[3];
  for (int d = 0; d < nDim; ++d) UnitNormal[d] = Normal[d] / Area;
  const double Density_i = Vi[RHO], Pressure_i = Vi[P_], Enthalpy_i = Vi[H_], SoundSpeed_i = Vi[A_];
  const double Density_j = Vj[RHO], Pressure_j = Vj[P_], Enthalpy_j = Vj[H_], SoundSpeed_j = Vj[A_];
  double ProjVelocity_i = 0.0, ProjVelocity_j = 0.0;
  for (int d = 0; d < nDim; ++d) {
    ProjVelocity_i += Vi[VX + d] * UnitNormal[d];
    ProjVelocity_j += Vj[VX + d] * UnitNormal[d];
  }
  const double MeanSoundSpeed = 0.5 * (SoundSpeed_i + SoundSpeed_j);
  const double mL = ProjVelocity_i / MeanSoundSpeed;
  const double mR = ProjVelocity_j / MeanSoundSpeed;
  const double mF2 = 0.5 * (mL * mL + mR * mR);
  const double mRef2 = std::min(1.0, std::max(mF2, mInfty * mInfty));
  const double mF = std::sqrt(mF2);
  const double mRef = std::sqrt(mRef2);
  const double fa = mRef * (2.0 - mRef);
  const double alpha = 3.0 / 16.0 * (5.0 * fa * fa - 4.0);
  const double beta = 0.125;
  double mLP, mRM, pLP, pRM;
  if (std::abs(mL) < 1.0) {
    mLP = 0.25 * (mL + 1.0) * (mL + 1.0) + beta * (mL * mL - 1.0) * (mL * mL - 1.0);
    pLP = 0.25 * (mL + 1.0) * (mL + 1.0) * (2.0 - mL) + alpha * mL * (mL * mL - 1.0) * (mL * mL - 1.0);
  } else {
    mLP = 0.5 * (mL + std::abs(mL));
    pLP = 0.5 * (1.0 + std::abs(mL) / mL);
  }
  if (std::abs(mR) < 1.0) {
    mRM = -0.25 * (mR - 1.0) * (mR - 1.0) - beta * (mR * mR - 1.0) * (mR * mR - 1.0);
    pRM = 0.25 * (mR - 1.0) * (mR - 1.0) * (2.0 + mR) - alpha * mR * (mR * mR - 1.0) * (mR * mR - 1.0);
  } else {
    mRM = 0.5 * (mR - std::abs(mR));
    pRM = 0.5 * (1.0 - std::abs(mR) / mR);
  }
  const double kP = 0.25, sigma = 1.0;
  double m12 = mLP + mRM;
  m12 -= kP / fa * std::max(1.0 - sigma * mF2, 0.0) * (Pressure_j - Pressure_i) /
         (0.5 * (Density_i + Density_j) * MeanSoundSpeed * MeanSoundSpeed);
  const double mLF = 0.5 * (m12 + std::abs(m12));
  const double mRF = 0.5 * (m12 - std::abs(m12));
  const double M12 = MeanSoundSpeed * (mLF * Density_i + mRF * Density_j);
  double Phi_i[64], Phi_j[64];
  Phi_i[RHO_S] = 1.0;
  Phi_j[RHO_S] = 1.0;
  for (int d = 0; d < nDim; ++d) {
    Phi_i[RHOVX_S + d] = Vi[VX + d];
    Phi_j[RHOVX_S + d] = Vj[VX + d];
  }
  Phi_i[RHOE_S] = Enthalpy_i;
  Phi_j[RHOE_S] = Enthalpy_j;
  for (int s = 0; s < ns; ++s) {
    Phi_i[RHOS_S + s] = Vi[RHOS + s];
    Phi_j[RHOS_S + s] = Vj[RHOS + s];
  }
  for (int v = 0; v < nVar; ++v)
    res[v] = 0.5 * (M12 * (Phi_i[v] + Phi_j[v]) + std::abs(M12) * (Phi_i[v] - Phi_j[v])) * Area;
  const double Ku = 0.75;
  double pLF = pLP * Pressure_i + pRM * Pressure_j;
  pLF -= Ku * pLP * pRM * (Density_i + Density_j) * fa * MeanSoundSpeed * (ProjVelocity_j - ProjVelocity_i);
  for (int d = 0; d < nDim; ++d) res[RHOVX_S + d] += pLF * UnitNormal[d] * Area;
  if (!implicit) return;

  for (int k = 0; k < nVar * nVar; ++k) Ji[k] = Jj[k] = 0.0;
  double MLD[64] = {0}, MRD[64] = {0};
  MLD[RHO_S] = -mL / Density_i;
  MRD[RHO_S] = -mR / Density_j;
  for (int d = 0; d < nDim; ++d) {
    MLD[RHOVX_S + d] = UnitNormal[d] / (Density_i * MeanSoundSpeed);
    MRD[RHOVX_S + d] = UnitNormal[d] / (Density_j * MeanSoundSpeed);
  }
  double MPL[64], MPR[64];
  if (std::abs(mL) < 1.0)
    for (int v = 0; v < nVar; ++v) MPL[v] = MLD[v] * (0.5 * (mL + 1.0) + 4.0 * beta * mL * (mL * mL - 1.0));
  else
    for (int v = 0; v < nVar; ++v) MPL[v] = MLD[v] * (0.5 * (1.0 + std::abs(mL) / mL));
  if (std::abs(mR) < 1.0)
    for (int v = 0; v < nVar; ++v) MPR[v] = MRD[v] * (0.5 * (1.0 - mR) + 4.0 * beta * mR * (1.0 - mR * mR));
  else
    for (int v = 0; v < nVar; ++v) MPR[v] = MRD[v] * (0.5 * (1.0 - std::abs(mR) / mR));
  double SL[64] = {0}, SR[64] = {0};
  if (mF2 == mRef2) {
    for (int v = 0; v < nVar; ++v) {
      SL[v] = MLD[v] * mL * (1.0 - mF) / mF;
      SR[v] = MRD[v] * mR * (1.0 - mF) / mF;
    }
  }
  double MEL[64], MER[64];
  const double MeanDensity = 0.5 * (Density_i + Density_j);
  const double factor = std::max(1.0 - sigma * mF2, 0.0);
  const double fpos = (factor > 0.0) ? 1.0 : 0.0;
  for (int v = 0; v < nVar; ++v) {
    MEL[v] = -kP / (MeanSoundSpeed * MeanSoundSpeed * fa * fa * MeanDensity * MeanDensity) *
             ((fpos * sigma * mL * MLD[v] * (Pressure_j - Pressure_i) * fa * MeanDensity) +
              (factor * Si[v] * fa * MeanDensity) + (factor * (Pressure_j - Pressure_i) * MeanDensity * SL[v]));
    MER[v] = kP / (MeanSoundSpeed * MeanSoundSpeed * fa * fa * MeanDensity * MeanDensity) *
             ((fpos * sigma * mR * MRD[v] * (Pressure_i - Pressure_j) * fa * MeanDensity) +
              (factor * Sj[v] * fa * MeanDensity) - (factor * (Pressure_j - Pressure_i) * MeanDensity * SR[v]));
  }
  MEL[RHO_S] -= kP / (MeanSoundSpeed * MeanSoundSpeed * fa * MeanDensity * MeanDensity) * 0.5 * factor *
                (Pressure_j - Pressure_i);
  MER[RHO_S] -= kP / (MeanSoundSpeed * MeanSoundSpeed * fa * MeanDensity * MeanDensity) * 0.5 * factor *
                (Pressure_j - Pressure_i);
  double sign_m12 = 0.0;
  if (m12 != 0.0) sign_m12 = std::abs(m12) / m12;
  double MPlL[64], MMiL[64], MPlR[64], MMiR[64];
  for (int v = 0; v < nVar; ++v) {
    MPlL[v] = 0.5 * (MPL[v] - MEL[v]) * (1.0 + sign_m12);
    MMiL[v] = 0.5 * (MPL[v] - MEL[v]) * (1.0 - sign_m12);
    MPlR[v] = 0.5 * (MPR[v] - MER[v]) * (1.0 + sign_m12);
    MMiR[v] = 0.5 * (MPR[v] - MER[v]) * (1.0 - sign_m12);
  }
  for (int a = 0; a < nVar; ++a)
    for (int b = 0; b < nVar; ++b) {
      Ji[a * nVar + b] += MeanSoundSpeed * ((MPlL[b] * Density_i * Phi_i[a]) + (MMiL[b] * Density_j * Phi_j[a]));
      Jj[a * nVar + b] += MeanSoundSpeed * ((MPlR[b] * Density_i * Phi_i[a]) + (MMiR[b] * Density_j * Phi_j[a]));
    }
  for (int v = 0; v < nVar; ++v) {
    Ji[v * nVar + v] += MeanSoundSpeed * mLF;
    Jj[v * nVar + v] += MeanSoundSpeed * mRF;
  }
  for (int v = 0; v < nVar; ++v) {
    Ji[RHOE_S * nVar + v] += MeanSoundSpeed * mLF * Si[v];
    Jj[RHOE_S * nVar + v] += MeanSoundSpeed * mRF * Sj[v];
  }
  double PPL[64] = {0}, PPR[64] = {0};
  if (std::abs(mL) < 1.0)
    for (int v = 0; v < nVar; ++v)
      PPL[v] = 0.25 * (mL + 1.0) * (3.0 * (1.0 - mL) + 4.0 * alpha * (5.0 * mL * mL - 1.0) * (mL - 1.0)) * MLD[v] +
               15.0 / 8.0 * SL[v] * mL * (mL * mL - 1.0) * (mL * mL - 1.0);
  if (std::abs(mR) < 1.0)
    for (int v = 0; v < nVar; ++v)
      PPR[v] = 0.25 * (mR - 1.0) * (3.0 * (1.0 + mR) + 4.0 * alpha * (1.0 - 5.0 * mR * mR) * (mR + 1.0)) * MRD[v] -
               15.0 / 8.0 * SR[v] * mR * (mR * mR - 1.0) * (mR * mR - 1.0);
  double PEL[64], PER[64];
  for (int v = 0; v < nVar; ++v) {
    PEL[v] = Ku * pRM * MeanSoundSpeed *
             ((PPL[v] * (Density_i + Density_j) * fa * (ProjVelocity_j - ProjVelocity_i)) +
              (pLP * (Density_i + Density_j) * (ProjVelocity_j - ProjVelocity_i) * SL[v]));
    PER[v] = Ku * pLP * MeanSoundSpeed *
             ((PPR[v] * (Density_i + Density_j) * fa * (ProjVelocity_j - ProjVelocity_i)) +
              (pRM * (Density_i + Density_j) * (ProjVelocity_j - ProjVelocity_i) * SR[v]));
  }
  PEL[RHO_S] += Ku * pRM * MeanSoundSpeed * pLP * fa *
                ((ProjVelocity_j - ProjVelocity_i) + (Density_i + Density_j) * ProjVelocity_i / Density_i);
  PER[RHO_S] += Ku * pLP * MeanSoundSpeed * pRM * fa *
                ((ProjVelocity_j - ProjVelocity_i) - (Density_i + Density_j) * ProjVelocity_j / Density_j);
  for (int d = 0; d < nDim; ++d) {
    PEL[RHOVX_S + d] -= Ku * pRM * MeanSoundSpeed * pLP * fa * (Density_i + Density_j) * UnitNormal[d] / Density_i;
    PER[RHOVX_S + d] += Ku * pLP * MeanSoundSpeed * pRM * fa * (Density_i + Density_j) * UnitNormal[d] / Density_j;
  }
  double PDL[64], PDR[64];
  for (int v = 0; v < nVar; ++v) {
    PDL[v] = pLP * Si[v] + Pressure_i * PPL[v] - PEL[v];
    PDR[v] = pRM * Sj[v] + Pressure_j * PPR[v] - PER[v];
  }
  for (int d = 0; d < nDim; ++d)
    for (int b = 0; b < nVar; ++b) {
      Ji[(RHOVX_S + d) * nVar + b] += UnitNormal[d] * PDL[b];
      Jj[(RHOVX_S + d) * nVar + b] += UnitNormal[d] * PDR[b];
    }
  for (int k = 0; k < nVar * nVar; ++k) {
    Ji[k] *= Area;
    Jj[k] *= Area;
  }
}

// ------------------------------------------------------------------------------------------------
// a9/a10: kinetics + PaSR source  (numerics_direct_reactive.cpp:1728-1879,
//          reacting_model_library.cpp:99-350, 701-705, 803-920)
// ------------------------------------------------------------------------------------------------
struct KinScratch {
  double Ys[32], Cs[32], F[16], B[16], Kc[16], omega_ir[32 * 16], Df[32 * 16], k_pasr[16], Kcd[16];
};

double delta_gibbs(const Mech& m, int r, double T, double* dnu_out) {
  double dG = 0.0, dnu = 0.0;
  for (int s = 0; s < m.ns; ++s) {
    const double dc = m.sp[s * m.nr + r] - m.sr[s * m.nr + r];
    if (dc != 0.0) {
      dG += dc * (spline(m, P_H, s, T) - T * spline(m, P_S, s, T));
      dnu += dc;
    }
  }
  *dnu_out = dnu;
  return dG;
}

void set_source_term(const Mech& m, double T, double rho, const double* ys, KinScratch& k) {
  for (int s = 0; s < m.ns; ++s) {
    double y = ys[s];
    if (y < 0.0) y = 1.0e-30;
    k.Ys[s] = y;
    k.Cs[s] = 1.0e3 * rho * y / m.mm[s];
  }
  for (int r = 0; r < m.nr; ++r) {
    const double kf = m.A[r] * std::pow(T, m.beta[r]) * std::exp(-m.Ta[r] / T);
    double kb;
    if (!m.hasb[r]) {
      double dnu;
      const double dG = delta_gibbs(m, r, T, &dnu);
      const double RT = R_UNGAS * T;
      const double lnKp = -dG / RT;
      const double lnKc = lnKp - dnu * std::log(R_UNGAS_ATM * T);
      k.Kc[r] = std::exp(lnKc);
      const bool complete = std::exp(lnKp) > 1.0e10;
      if (!m.rev[r]) kb = 0.0;
      else if (complete) kb = 0.0;
      else kb = kf / k.Kc[r];
    } else {
      kb = m.Ab[r] * std::pow(T, m.betab[r]) * std::exp(-m.Tab[r] / T);
      k.Kc[r] = kf / kb;
    }
    double fr = 0.0, br = 0.0;
    bool zero = false;
    for (int s : m.neg_reac[r]) if (k.Ys[s] < 1.0e-15) { zero = true; break; }
    if (!zero) {
      fr = 1.0;
      for (int s = 0; s < m.ns; ++s) fr *= std::pow(k.Cs[s], m.er[r * m.ns + s]);
      fr *= kf;
    }
    zero = false;
    for (int s : m.neg_prod[r]) if (k.Ys[s] < 1.0e-15) { zero = true; break; }
    if (!zero) {
      br = 1.0;
      for (int s = 0; s < m.ns; ++s) br *= std::pow(k.Cs[s], m.ep[r * m.ns + s]);
      br *= kb;
    }
    k.F[r] = fr;
    k.B[r] = br;
  }
  for (int r = 0; r < m.nr; ++r)
    for (int s = 0; s < m.ns; ++s)
      k.omega_ir[s * m.nr + r] = 1.0e-3 * m.mm[s] * (m.sp[s * m.nr + r] - m.sr[s * m.nr + r]) * (k.F[r] - k.B[r]);
}

void set_dfr_drhos(const Mech& m, double rho, KinScratch& k) {
  for (int s = 0; s < m.ns; ++s)
    for (int r = 0; r < m.nr; ++r) {
      k.Df[s * m.nr + r] = 0.0;
      if (k.Ys[s] > 1.0e-10)
        k.Df[s * m.nr + r] = (k.F[r] * m.er[r * m.ns + s] - k.B[r] * m.ep[r * m.ns + s]) / (rho * k.Ys[s]);
    }
}

void assemble_pasr(const Mech& m, double omega_turb, double C_mu, double lb, KinScratch& k) {
  const double tau_mix = 1 / (C_mu * omega_turb);
  for (int r = 0; r < m.nr; ++r) {
    double hd = -1.0;
    for (int s = 0; s < m.ns; ++s)
      if (m.sp[s * m.nr + r] != 0.0 || m.sr[s * m.nr + r] != 0.0) {
        const double v = std::fabs(k.Df[s * m.nr + r] * m.mm[s]);
        if (hd < 0.0 || v > hd) hd = v;
      }
    const double tau_c = 1 / hd;
    double kk;
    if (std::isinf(tau_c)) kk = 1.0;
    else if ((tau_c / (tau_c + tau_mix)) < lb) kk = lb;
    else kk = tau_c / (tau_c + tau_mix);
    k.k_pasr[r] = kk;
  }
}

// Set_BackFor_Contr (:233-289): (back_contr, for_contr) per reaction
void back_for_contr(const Mech& m, double T, KinScratch& k, double* bc, double* fc) {
  const double epsilon = 1.0e-6;
  const double Tp = T + epsilon * T;
  const double RT = R_UNGAS * Tp;
  const double lnRT = std::log(R_UNGAS_ATM * Tp);
  for (int r = 0; r < m.nr; ++r) {
    double Kcp;
    if (!m.hasb[r]) {
      if (k.B[r] > 0.0) {
        double dnu;
        const double dG = delta_gibbs(m, r, Tp, &dnu);
        Kcp = std::exp(-dG / RT - dnu * lnRT);
      } else {
        Kcp = k.Kc[r];
      }
    } else {
      const double kfp = m.A[r] * std::pow(Tp, m.beta[r]) * std::exp(-m.Ta[r] / Tp);
      const double kbp = m.Ab[r] * std::pow(Tp, m.betab[r]) * std::exp(-m.Tab[r] / Tp);
      Kcp = kfp / kbp;
    }
    k.Kcd[r] = (Kcp - k.Kc[r]) / (Tp - T);
  }
  for (int r = 0; r < m.nr; ++r) {
    const double tmp = (m.beta[r] + m.Ta[r] / T) / T;
    fc[r] = k.F[r] * tmp;
    if (!m.hasb[r]) bc[r] = k.B[r] * (tmp - k.Kcd[r] / k.Kc[r]);
    else bc[r] = k.B[r] * (m.betab[r] + m.Tab[r] / T) / T;
  }
}

void source(const Mech& m, int nDim, const double* V, const double* S, double vol, double omega_turb, bool rans,
            bool implicit, double C_mu, double lb, double rho_ref, double t_ref, double T_ref, double* res, double* J) {
  const int ns = m.ns, nr = m.nr, nVar = ns + nDim + 2;
  const int RHOS_P = nDim + 5, RHO_P = nDim + 2, RHOS_S = nDim + 2;
  KinScratch k;
  const double rho = V[RHO_P];
  const double dim_temp = V[0] * T_ref;
  const double dim_rho = rho * rho_ref;
  set_source_term(m, dim_temp, dim_rho, V + RHOS_P, k);
  double omega[32];
  if (rans) {
    set_dfr_drhos(m, dim_rho, k);
    assemble_pasr(m, omega_turb, C_mu, lb, k);
    for (int s = 0; s < ns; ++s) {
      double o = 0.0;
      for (int r = 0; r < nr; ++r) o += k.k_pasr[r] * k.omega_ir[s * nr + r];
      omega[s] = o;
    }
  } else {
    for (int s = 0; s < ns; ++s) {
      double o = 0.0;
      for (int r = 0; r < nr; ++r) o += k.omega_ir[s * nr + r];
      omega[s] = o;
    }
  }
  for (int v = 0; v < nVar; ++v) res[v] = 0.0;
  for (int s = 0; s < ns; ++s) res[RHOS_S + s] = omega[s] * (-vol / (rho_ref / t_ref));
  if (!implicit) return;
  for (int q = 0; q < nVar * nVar; ++q) J[q] = 0.0;
  double bc[16], fc[16];
  back_for_contr(m, dim_temp, k, bc, fc);
  // GetTurbSourceJacobian (:295-319) / GetSourceJacobian (:325-350): [ns][ns+1]
  double sj[32 * 33];
  for (int q = 0; q < ns * (ns + 1); ++q) sj[q] = 0.0;
  for (int r = 0; r < nr; ++r)
    for (int s = 0; s < ns; ++s) {
      const double fixed = 1.0e-3 * m.mm[s] * (m.sp[s * nr + r] - m.sr[s * nr + r]);
      if (rans) {
        sj[s * (ns + 1)] += fixed * (fc[r] - bc[r]) * k.k_pasr[r];
        for (int j = 0; j < ns; ++j)
          if (k.Ys[j] > 1.0e-10) sj[s * (ns + 1) + j + 1] += fixed * k.k_pasr[r] * k.Df[j * nr + r];
      } else {
        sj[s * (ns + 1)] += fixed * (fc[r] - bc[r]);
        for (int j = 0; j < ns; ++j)
          if (k.Ys[j] > 1.0e-10)
            sj[s * (ns + 1) + j + 1] +=
                fixed * (k.F[r] * m.er[r * ns + j] - k.B[r] * m.ep[r * ns + j]) / (dim_rho * k.Ys[j]);
      }
    }
  for (int s = 0; s < ns; ++s) {
    const double fixed = sj[s * (ns + 1)] * t_ref * T_ref / rho_ref;
    double* row = J + (RHOS_S + s) * nVar;
    row[0] = -fixed * S[0] * vol;
    for (int d = 0; d < nDim; ++d) row[1 + d] = -fixed * S[1 + d] * vol;
    row[nDim + 1] = -fixed * S[nDim + 1] * vol;
    for (int j = 0; j < ns; ++j)
      row[RHOS_S + j] = -fixed * S[RHOS_S + j] * vol - sj[s * (ns + 1) + j + 1] * t_ref * vol;
  }
}

// ------------------------------------------------------------------------------------------------
// Eigen 3.3.7 algorithms restated (externals/Eigen, parity dependency of the viscous flux):
//   BiCGSTAB with DiagonalPreconditioner  src/IterativeLinearSolvers/BiCGSTAB.h:28-100
//   ColPivHouseholderQR compute + solve    src/QR/ColPivHouseholderQR.h:480-611
// Matrices here are row-major n x n.
// ------------------------------------------------------------------------------------------------
// Eigen's vectorised reduction order for a contiguous, 16-byte-aligned double vector
// (Core/Redux.h LinearVectorizedTraversal, SSE2 packets of 2, two packet accumulators; no FMA).
double eigen_redux_prod(int n, const double* a, const double* b) {
  auto p = [&](int k) { return a[k] * b[k]; };
  const int as2 = (n / 4) * 4, as = (n / 2) * 2;
  double res;
  if (as) {
    double r0a = p(0), r0b = p(1);
    if (as > 2) {
      double r1a = p(2), r1b = p(3);
      for (int k = 4; k < as2; k += 4) {
        r0a += p(k); r0b += p(k + 1);
        r1a += p(k + 2); r1b += p(k + 3);
      }
      r0a += r1a; r0b += r1b;
      if (as > as2) { r0a += p(as2); r0b += p(as2 + 1); }
    }
    res = r0a + r0b;
    for (int k = as; k < n; ++k) res += p(k);
  } else {
    res = p(0);
    for (int k = 1; k < n; ++k) res += p(k);
  }
  return res;
}
double dot(int n, const double* a, const double* b) { return eigen_redux_prod(n, a, b); }

// Eigen's column-major GEMV order for an n x n heap (16-byte aligned) matrix
// (Core/products/GeneralMatrixVector.h:88-319): 4 columns at once, rows in packets of 2 as
// res + ((a0 x0 + a1 x1) + (a2 x2 + a3 x3)), odd tail row by sequential multiply-adds, then the
// leftover columns one by one. A is given row-major here; y = A x.
void matvec(int n, const double* A, const double* x, double* y) {
  for (int i = 0; i < n; ++i) y[i] = 0.0;
  const int aligned = n & ~1;
  const int bound = (n / 4) * 4;
  for (int c = 0; c < bound; c += 4) {
    for (int r = 0; r < aligned; ++r)
      y[r] = y[r] + ((A[r * n + c] * x[c] + A[r * n + c + 1] * x[c + 1]) +
                     (A[r * n + c + 2] * x[c + 2] + A[r * n + c + 3] * x[c + 3]));
    for (int r = aligned; r < n; ++r) {
      y[r] = A[r * n + c] * x[c] + y[r];
      y[r] = A[r * n + c + 1] * x[c + 1] + y[r];
      y[r] = A[r * n + c + 2] * x[c + 2] + y[r];
      y[r] = A[r * n + c + 3] * x[c + 3] + y[r];
    }
  }
  for (int c = bound; c < n; ++c) {
    for (int r = 0; r < aligned; ++r) y[r] = A[r * n + c] * x[c] + y[r];
    for (int r = aligned; r < n; ++r) y[r] += A[r * n + c] * x[c];
  }
}

void bicgstab(int n, const double* A, const double* rhs, double* x, double tol) {
  const int maxIters = 2 * n;
  double invdiag[32];
  for (int j = 0; j < n; ++j) invdiag[j] = (A[j * n + j] != 0.0) ? 1.0 / A[j * n + j] : 1.0;
  for (int i = 0; i < n; ++i) x[i] = 0.0;
  double r[32], r0[32], tmpv[32];
  matvec(n, A, x, tmpv);
  for (int i = 0; i < n; ++i) r[i] = rhs[i] - tmpv[i];
  for (int i = 0; i < n; ++i) r0[i] = r[i];
  double r0_sqnorm = dot(n, r0, r0);
  const double rhs_sqnorm = dot(n, rhs, rhs);
  if (rhs_sqnorm == 0) {
    for (int i = 0; i < n; ++i) x[i] = 0.0;
    return;
  }
  double rho = 1, alpha = 1, w = 1;
  double v[32] = {0}, p[32] = {0}, y[32], z[32], s[32], t[32];
  const double tol2 = tol * tol * rhs_sqnorm;
  const double eps = std::numeric_limits<double>::epsilon();
  const double eps2 = eps * eps;
  int i = 0, restarts = 0;
  while (dot(n, r, r) > tol2 && i < maxIters) {
    const double rho_old = rho;
    rho = dot(n, r0, r);
    if (std::abs(rho) < eps2 * r0_sqnorm) {
      matvec(n, A, x, tmpv);
      for (int q = 0; q < n; ++q) r[q] = rhs[q] - tmpv[q];
      for (int q = 0; q < n; ++q) r0[q] = r[q];
      rho = r0_sqnorm = dot(n, r, r);
      if (restarts++ == 0) i = 0;
    }
    const double beta = (rho / rho_old) * (alpha / w);
    for (int q = 0; q < n; ++q) p[q] = r[q] + beta * (p[q] - w * v[q]);
    for (int q = 0; q < n; ++q) y[q] = invdiag[q] * p[q];
    matvec(n, A, y, v);
    alpha = rho / dot(n, r0, v);
    for (int q = 0; q < n; ++q) s[q] = r[q] - alpha * v[q];
    for (int q = 0; q < n; ++q) z[q] = invdiag[q] * s[q];
    matvec(n, A, z, t);
    const double tmp = dot(n, t, t);
    w = (tmp > 0.0) ? dot(n, t, s) / tmp : 0.0;
    for (int q = 0; q < n; ++q) x[q] += alpha * y[q] + w * z[q];
    for (int q = 0; q < n; ++q) r[q] = s[q] - w * t[q];
    ++i;
  }
}

struct ColPivQR {
  int n;
  double qr[32 * 32];  // row-major
  double hc[32];
  int perm[32];
  int nonzero;
};

void qr_compute(int n, const double* M, ColPivQR& f) {
  f.n = n;
  std::memcpy(f.qr, M, sizeof(double) * n * n);
  double* Q = f.qr;
  auto at = [&](int i, int j) -> double& { return Q[i * n + j]; };
  double normsU[32], normsD[32];
  int trans[32];
  for (int k = 0; k < n; ++k) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += at(i, k) * at(i, k);
    normsD[k] = std::sqrt(s);
    normsU[k] = normsD[k];
  }
  double mx = normsU[0];
  for (int k = 1; k < n; ++k) mx = std::max(mx, normsU[k]);
  const double epsm = std::numeric_limits<double>::epsilon();
  const double threshold_helper = (mx * epsm) * (mx * epsm) / double(n);
  const double norm_downdate_threshold = std::sqrt(epsm);
  f.nonzero = n;
  for (int k = 0; k < n; ++k) {
    int big = k;
    for (int j = k + 1; j < n; ++j)
      if (normsU[j] > normsU[big]) big = j;
    const double big_sq = normsU[big] * normsU[big];
    if (f.nonzero == n && big_sq < threshold_helper * double(n - k)) f.nonzero = k;
    trans[k] = big;
    if (k != big) {
      for (int i = 0; i < n; ++i) std::swap(at(i, k), at(i, big));
      std::swap(normsU[k], normsU[big]);
      std::swap(normsD[k], normsD[big]);
    }
    // makeHouseholderInPlace on column k rows k..n-1
    double tailSq = 0.0;
    for (int i = k + 1; i < n; ++i) tailSq += at(i, k) * at(i, k);
    const double c0 = at(k, k);
    double tau, beta;
    if (tailSq <= std::numeric_limits<double>::min()) {
      tau = 0.0;
      beta = c0;
      for (int i = k + 1; i < n; ++i) at(i, k) = 0.0;
    } else {
      beta = std::sqrt(c0 * c0 + tailSq);
      if (c0 >= 0.0) beta = -beta;
      for (int i = k + 1; i < n; ++i) at(i, k) = at(i, k) / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    f.hc[k] = tau;
    at(k, k) = beta;
    // applyHouseholderOnTheLeft to bottomRightCorner(n-k, n-k-1)
    if (n - k == 1) {
      for (int j = k + 1; j < n; ++j) at(k, j) *= (1.0 - tau);
    } else if (tau != 0.0) {
      for (int j = k + 1; j < n; ++j) {
        double tmp = 0.0;
        for (int i = k + 1; i < n; ++i) tmp += at(i, k) * at(i, j);
        tmp += at(k, j);
        at(k, j) -= tau * tmp;
        for (int i = k + 1; i < n; ++i) at(i, j) -= tau * at(i, k) * tmp;
      }
    }
    for (int j = k + 1; j < n; ++j) {
      if (normsU[j] != 0.0) {
        double temp = std::abs(at(k, j)) / normsU[j];
        temp = (1.0 + temp) * (1.0 - temp);
        temp = temp < 0.0 ? 0.0 : temp;
        const double rr = normsU[j] / normsD[j];
        const double temp2 = temp * (rr * rr);
        if (temp2 <= norm_downdate_threshold) {
          double s = 0.0;
          for (int i = k + 1; i < n; ++i) s += at(i, j) * at(i, j);
          normsD[j] = std::sqrt(s);
          normsU[j] = normsD[j];
        } else {
          normsU[j] *= std::sqrt(temp);
        }
      }
    }
  }
  for (int k = 0; k < n; ++k) f.perm[k] = k;
  for (int k = 0; k < n; ++k) std::swap(f.perm[k], f.perm[trans[k]]);
}

void qr_solve(const ColPivQR& f, const double* rhs, double* dst) {
  const int n = f.n, np = f.nonzero;
  if (np == 0) {
    for (int i = 0; i < n; ++i) dst[i] = 0.0;
    return;
  }
  double c[32];
  for (int i = 0; i < n; ++i) c[i] = rhs[i];
  for (int k = 0; k < np; ++k) {
    const double tau = f.hc[k];
    if (n - k == 1) {
      c[k] *= (1.0 - tau);
    } else if (tau != 0.0) {
      double tmp = 0.0;
      for (int i = k + 1; i < n; ++i) tmp += f.qr[i * n + k] * c[i];
      tmp += c[k];
      c[k] -= tau * tmp;
      for (int i = k + 1; i < n; ++i) c[i] -= tau * f.qr[i * n + k] * tmp;
    }
  }
  for (int i = np - 1; i >= 0; --i) {  // column-oriented back substitution
    c[i] /= f.qr[i * n + i];
    for (int j = 0; j < i; ++j) c[j] -= c[i] * f.qr[j * n + i];
  }
  for (int i = 0; i < np; ++i) dst[f.perm[i]] = c[i];
  for (int i = np; i < n; ++i) dst[f.perm[i]] = 0.0;
}

// ------------------------------------------------------------------------------------------------
// a3-a6: CAvgGradReactive_Flow::ComputeResidual (numerics_direct_reactive.cpp:1425-1678) with
// SetLaminarTensorFlux (:1099-1190), Solve_SM (:451-470), GetGamma (library :771-798),
// SST_Reactive_ResidualClosure (:656-852), Get_Molar2MassGrad_Operator (:861-880),
// SetLaminarViscousProjJacs (:1200-1401), SST_Reactive_JacobianClosure (:891-1090).
// ------------------------------------------------------------------------------------------------
struct ViscParams {
  double T_ref, E_ref, R_ref, Prandtl_Turb, Lewis_Turb;
  int rans, implicit;
};

void visc_flux(const Mech& m, int nDim, const ViscParams& P, const double* Vi, const double* Vj, const double* Gi,
               const double* Gj, double mu_i, double mu_j, double k_i, double k_j, const double* Dij_i,
               const double* Dij_j, const double* Ci, const double* Cj, const double* Normal, const double* Si,
               const double* Sj, double tke_i, double tke_j, double mut_i, double mut_j, double sigma_k,
               const double* gk_i, const double* gk_j, double* res, double* Ji, double* Jj, bool corrected = true) {
  // corrected = false: CAvgGradReactive_Boundary::ComputeResidual (numerics_direct_reactive.cpp:478-648, a8) —
  // the plain mean gradient, no edge correction and no coincident-point check.
  const int ns = m.ns;
  const int nVar = ns + nDim + 2, nPrimVar = ns + nDim + 5, nGrad = ns + nDim + 2;
  const int T_P = 0, VX_P = 1, RHO_P = nDim + 2, RHOS_P = nDim + 5;
  const int RHO_S = 0, RHOVX_S = 1, RHOE_S = nDim + 1, RHOS_S = nDim + 2;
  const int T_G = 0, VX_G = 1, RHOS_G = nDim + 2;
  const int T_A = 0, VX_A = 1, RHOS_A = 1 + nDim;  // avg-grad rows
  const int nAvg = ns + nDim + 1;

  const double Mean_mu = 2.0 / (1.0 / mu_i + 1.0 / mu_j);
  const double Mean_k = 2.0 / (1.0 / k_i + 1.0 / k_j);
  double Dm[32 * 32];  // [a][b] in the same (column-major) indexing as the input
  double Dmax = -std::numeric_limits<double>::infinity();
  for (int q = 0; q < ns * ns; ++q) {
    Dm[q] = 2.0 / (1.0 / Dij_i[q] + 1.0 / Dij_j[q]);
    Dmax = std::max(Dmax, Dm[q]);
  }
  auto D = [&](const double* d, int a, int b) { return d[b * ns + a]; };  // column-major (a,b)
  double Vm[64];
  for (int v = 0; v < nPrimVar; ++v) Vm[v] = 0.5 * (Vi[v] + Vj[v]);
  double Xs_i[32], Xs_j[32], ytmp[32];
  molar_from_mass(m, Vi + RHOS_P, ytmp, Xs_i);
  molar_from_mass(m, Vj + RHOS_P, ytmp, Xs_j);
  double Edge[3];
  for (int d = 0; d < nDim; ++d) Edge[d] = Cj[d] - Ci[d];
  double G[32][3];  // mean gradient [nAvg][nDim]
  for (int d = 0; d < nDim; ++d) {
    G[T_A][d] = 0.5 * (Gi[T_G * nDim + d] + Gj[T_G * nDim + d]);
    for (int e = 0; e < nDim; ++e) G[VX_A + e][d] = 0.5 * (Gi[(VX_G + e) * nDim + d] + Gj[(VX_G + e) * nDim + d]);
    for (int s = 0; s < ns; ++s) G[RHOS_A + s][d] = 0.5 * (Gi[(RHOS_G + s) * nDim + d] + Gj[(RHOS_G + s) * nDim + d]);
  }
  (void)nGrad;
  double Proj[32];
  for (int r = 0; r < nAvg; ++r) {
    double s = 0.0;
    for (int d = 0; d < nDim; ++d) s += G[r][d] * Edge[d];
    Proj[r] = s;
  }
  double dist2 = 0.0;
  for (int d = 0; d < nDim; ++d) dist2 += Edge[d] * Edge[d];
  if (corrected) {
    if (!(dist2 > EPS)) throw std::runtime_error("Error: You are trying to compute flux between a node and itself");
    double Diff[32];
    Diff[T_A] = Vj[T_P] - Vi[T_P];
    for (int d = 0; d < nDim; ++d) Diff[VX_A + d] = Vj[VX_P + d] - Vi[VX_P + d];
    for (int s = 0; s < ns; ++s) Diff[RHOS_A + s] = Xs_j[s] - Xs_i[s];
    for (int r = 0; r < nAvg; ++r)
      for (int d = 0; d < nDim; ++d) G[r][d] -= (Proj[r] - Diff[r]) * Edge[d] / dist2;
  }

  // --- SetLaminarTensorFlux
  double Flux[32][3], PF[32];
  for (int v = 0; v < nVar; ++v) {
    PF[v] = 0.0;
    for (int d = 0; d < nDim; ++d) Flux[v][d] = 0.0;
  }
  const double rho = Vm[RHO_P], T = Vm[T_P];
  const double dim_temp = T * P.T_ref;
  double hs[32], Ys[32], Xs[32], yc[32];
  for (int s = 0; s < ns; ++s) hs[s] = spline(m, P_H, s, dim_temp) / m.mm[s] / P.E_ref;
  for (int s = 0; s < ns; ++s) Ys[s] = Vm[RHOS_P + s];
  molar_from_mass(m, Ys, yc, Xs);
  double div_vel = 0.0;
  for (int d = 0; d < nDim; ++d) div_vel += G[VX_A + d][d];
  double tau[3][3];
  for (int a = 0; a < nDim; ++a)
    for (int b = 0; b < nDim; ++b) tau[a][b] = 0.0;
  for (int a = 0; a < nDim; ++a) {
    for (int b = 0; b < nDim; ++b) tau[a][b] += Mean_mu * (G[VX_A + b][a] + G[VX_A + a][b]);
    tau[a][a] -= TWO3 * (Mean_mu * div_vel);
  }
  const double alpha = 1.0 / (rho * Dmax);
  double Gxn[32];
  for (int s = 0; s < ns; ++s) Gxn[s] = 0.0;
  for (int a = 0; a < nDim; ++a) {
    for (int b = 0; b < nDim; ++b) {
      Flux[RHOVX_S + b][a] = tau[a][b];
      Flux[RHOE_S][a] += tau[a][b] * Vm[VX_P + b];
    }
    Flux[RHOE_S][a] += Mean_k * G[T_A][a];
    for (int s = 0; s < ns; ++s) Gxn[s] += G[RHOS_A + s][a] * Normal[a];
  }
  // Solve_SM: Gamma (GetGamma) + alpha*Y, BiCGSTAB tol 1e-11
  double Gt[32 * 32];
  {
    double sigma = 0.0, massTot = 0.0;
    for (int s = 0; s < ns; ++s) sigma += Ys[s];
    for (int s = 0; s < ns; ++s) massTot += Ys[s] / m.mm[s];
    massTot = 1.0 / massTot;
    for (int a = 0; a < ns; ++a)
      for (int b = 0; b < ns; ++b) {
        double g;
        if (a != b) {
          g = -sigma * massTot * Xs[a] / (rho * m.mm[b] * D(Dm, a, b));
        } else {
          double tmp = 0.0;
          for (int c = 0; c < ns; ++c)
            if (c != a) tmp += Xs[c] / D(Dm, a, c);
          g = sigma * massTot * tmp / (rho * m.mm[a]);
        }
        Gt[a * ns + b] = g + alpha * Ys[a];
      }
  }
  double nGxn[32], Jd[32];
  for (int s = 0; s < ns; ++s) nGxn[s] = -Gxn[s];
  bicgstab(ns, Gt, nGxn, Jd, 1.0e-11);
  {
    double ones[32];
    for (int s = 0; s < ns; ++s) ones[s] = 1.0;
    PF[RHO_S] = -eigen_redux_prod(ns, Jd, ones);  // Jd.sum(): same packet order
  }
  for (int s = 0; s < ns; ++s) {
    PF[RHOE_S] += -hs[s] * Jd[s];
    PF[RHOS_S + s] = -Jd[s];
  }

  double Mean_mut = 0.0, Mean_tke = 0.0, Cps[32];
  double MassGrads[32][3];
  if (P.rans) {
    Mean_mut = 2.0 / (1.0 / mut_i + 1.0 / mut_j);
    Mean_tke = 0.5 * (tke_i + tke_j);
    double gk[3];
    for (int d = 0; d < nDim; ++d) gk[d] = 0.5 * (gk_i[d] + gk_j[d]);
    for (int s = 0; s < ns; ++s) Cps[s] = spline(m, P_CP, s, dim_temp) / m.mm[s] / P.R_ref;
    double dv = 0.0;
    for (int d = 0; d < nDim; ++d) dv += G[VX_A + d][d];
    double tt[3][3];
    for (int a = 0; a < nDim; ++a)
      for (int b = 0; b < nDim; ++b) tt[a][b] = 0.0;
    for (int a = 0; a < nDim; ++a) {
      for (int b = 0; b < nDim; ++b) tt[a][b] += Mean_mut * (G[VX_A + b][a] + G[VX_A + a][b]);
      tt[a][a] -= TWO3 * (Mean_mut * dv + Mean_tke * rho);
    }
    // Get_Molar2MassGrad_Operator
    double Mt[32 * 32];
    {
      double sig = 0.0;
      for (int s = 0; s < ns; ++s) sig += Xs[s];
      double mt = 0.0;
      for (int s = 0; s < ns; ++s) mt += m.mm[s];
      for (int a = 0; a < ns; ++a)
        for (int b = 0; b < ns; ++b)
          Mt[a * ns + b] = mt / m.mm[a] * (Ys[a] - Xs[a] + sig) * (a == b) +
                           mt * (Ys[a] / m.mm[a] - Xs[a] / m.mm[b]) * (a != b);
    }
    ColPivQR qr;
    qr_compute(ns, Mt, qr);
    for (int d = 0; d < nDim; ++d) {
      double rhs[32], sol[32];
      for (int s = 0; s < ns; ++s) rhs[s] = G[RHOS_A + s][d];
      qr_solve(qr, rhs, sol);
      for (int s = 0; s < ns; ++s) MassGrads[s][d] = sol[s];
    }
    for (int s = 0; s < ns; ++s)
      for (int d = 0; d < nDim; ++d)
        if (std::abs(G[RHOS_A + s][d]) < 1e-8) MassGrads[s][d] = 0.0;
    for (int a = 0; a < nDim; ++a) {
      for (int b = 0; b < nDim; ++b) {
        Flux[RHOVX_S + b][a] += tt[a][b];
        Flux[RHOE_S][a] += tt[a][b] * Vm[VX_P + b];
      }
      for (int s = 0; s < ns; ++s)
        PF[RHOS_S + s] += Mean_mut / (P.Prandtl_Turb * P.Lewis_Turb) * MassGrads[s][a] * Normal[a];
      for (int s = 0; s < ns; ++s)
        Flux[RHOE_S][a] += Mean_mut / (P.Prandtl_Turb * P.Lewis_Turb) * hs[s] * Ys[s] * MassGrads[s][a];
      for (int s = 0; s < ns; ++s) Flux[RHOE_S][a] += Mean_mut / P.Prandtl_Turb * Cps[s] * Ys[s] * G[T_A][a];
      Flux[RHOE_S][a] += (Mean_mu + Mean_mut / sigma_k) * gk[a];
    }
  }
  for (int d = 0; d < nDim; ++d) {
    for (int v = RHOVX_S; v < RHOVX_S + nDim; ++v) PF[v] += Flux[v][d] * Normal[d];
    PF[RHOE_S] += Flux[RHOE_S][d] * Normal[d];
  }
  for (int v = 0; v < nVar; ++v) res[v] = PF[v];
  if (!P.implicit) return;

  // --- implicit part (:1576-1653)
  double Ds_i[32], Ds_j[32], Ds[32];
  for (int a = 0; a < ns; ++a) {
    double di = 0.0, dj = 0.0;
    for (int b = 0; b < ns; ++b)
      if (b != a) {
        di += Xs_i[b] / D(Dij_i, a, b);
        dj += Xs_j[b] / D(Dij_j, a, b);
      }
    Ds_i[a] = (1.0 - Xs_i[a]) / di;
    Ds_j[a] = (1.0 - Xs_j[a]) / dj;
  }
  for (int s = 0; s < ns; ++s) {
    if (std::isnan(Ds_i[s]) || std::isinf(Ds_i[s])) Ds_i[s] = 0.0;
    if (std::isnan(Ds_j[s]) || std::isinf(Ds_j[s])) Ds_j[s] = 0.0;
    Ds[s] = 0.5 * (Ds_i[s] + Ds_j[s]);
  }
  double Area = 0.0;
  for (int d = 0; d < nDim; ++d) Area += Normal[d] * Normal[d];
  Area = std::sqrt(Area);
  double UN[3];
  for (int d = 0; d < nDim; ++d) UN[d] = Normal[d] / Area;
  for (int s = 0; s < ns; ++s) Gxn[s] /= Area;
  const double dij = std::sqrt(dist2), dS = Area;

  static thread_local std::vector<double> buf;
  buf.assign(4 * nVar * nVar, 0.0);
  double* dFdVi = buf.data();
  double* dFdVj = dFdVi + nVar * nVar;
  double* dVdUi = dFdVj + nVar * nVar;
  double* dVdUj = dVdUi + nVar * nVar;
  auto FI = [&](int a, int b) -> double& { return dFdVi[a * nVar + b]; };
  auto FJ = [&](int a, int b) -> double& { return dFdVj[a * nVar + b]; };
  // SetLaminarViscousProjJacs
  {
    double theta = 0.0;
    for (int d = 0; d < nDim; ++d) theta += UN[d] * UN[d];
    const double rho_i = Vi[RHO_P], rho_j = Vj[RHO_P];
    for (int s = 0; s < ns; ++s) Cps[s] = spline(m, P_CP, s, dim_temp) / m.mm[s] / P.R_ref;
    static thread_local std::vector<double> djb;
    djb.assign(2 * ns * (ns + 1), 0.0);
    double* dJdr_j = djb.data();
    double* dJdr_i = dJdr_j + ns * (ns + 1);
    auto DJ = [&](double* a, int r, int c) -> double& { return a[r * (ns + 1) + c]; };
    double totMass = 0.0, totMass_i = 0.0, totMass_j = 0.0, sigma_i = 0.0, sigma_j = 0.0;
    for (int s = 0; s < ns; ++s) totMass += m.mm[s] * Xs[s];
    for (int s = 0; s < ns; ++s) totMass_i += m.mm[s] * Xs_i[s];
    for (int s = 0; s < ns; ++s) totMass_j += m.mm[s] * Xs_j[s];
    for (int s = 0; s < ns; ++s) sigma_i += Xs_i[s];
    for (int s = 0; s < ns; ++s) sigma_j += Xs_j[s];
    for (int a = 0; a < ns; ++a)
      for (int k = 0; k < ns; ++k) {
        DJ(dJdr_j, a, k + 1) = -rho * m.mm[a] * Ds[a] * Xs_j[a] / (totMass * dij * sigma_j * rho_j);
        DJ(dJdr_i, a, k + 1) = rho * m.mm[a] * Ds[a] * Xs_i[a] / (totMass * dij * sigma_i * rho_i);
        for (int b = 0; b < ns; ++b) {
          DJ(dJdr_j, a, k + 1) += rho * Ys[a] * m.mm[b] * Ds[b] * Xs_j[b] / (totMass * dij * sigma_j * rho_j);
          DJ(dJdr_i, a, k + 1) -= rho * Ys[a] * m.mm[b] * Ds[b] * Xs_i[b] / (totMass * dij * sigma_i * rho_i);
        }
        DJ(dJdr_j, a, k + 1) += rho * Ys[a] * Ds[k] * totMass_j * sigma_j / (dij * totMass * rho_j);
        DJ(dJdr_i, a, k + 1) -= rho * Ys[a] * Ds[k] * totMass_i * sigma_i / (dij * totMass * rho_i);
        if (a == k) {
          DJ(dJdr_j, a, k + 1) -= rho * Ds[a] * totMass_j * sigma_j / (dij * totMass * rho_j);
          DJ(dJdr_i, a, k + 1) += rho * Ds[a] * totMass_i * sigma_i / (dij * totMass * rho_i);
        }
      }
    for (int a = 0; a < ns; ++a)
      for (int b = 0; b < ns; ++b) {
        DJ(dJdr_j, a, a + 1) += 0.5 * rho * m.mm[b] * Ds[b] * Gxn[b] / (totMass * rho_j);
        DJ(dJdr_i, a, a + 1) += 0.5 * rho * m.mm[b] * Ds[b] * Gxn[b] / (totMass * rho_i);
      }
    dVdUi[RHO_S * nVar + RHO_S] = 1.0;
    dVdUj[RHO_S * nVar + RHO_S] = 1.0;
    for (int s = 0; s < ns; ++s) {
      dVdUi[(RHOS_S + s) * nVar + RHOS_S + s] = 1.0;
      dVdUj[(RHOS_S + s) * nVar + RHOS_S + s] = 1.0;
    }
    for (int d = 0; d < nDim; ++d) {
      dVdUi[(RHOVX_S + d) * nVar + RHO_S] = -Vi[VX_P + d] / Vi[RHO_P];
      dVdUi[(RHOVX_S + d) * nVar + RHOVX_S + d] = 1.0 / Vi[RHO_P];
      dVdUj[(RHOVX_S + d) * nVar + RHO_S] = -Vj[VX_P + d] / Vj[RHO_P];
      dVdUj[(RHOVX_S + d) * nVar + RHOVX_S + d] = 1.0 / Vj[RHO_P];
    }
    for (int v = 0; v < nVar; ++v) {
      dVdUi[RHOE_S * nVar + v] = Si[v];
      dVdUj[RHOE_S * nVar + v] = Sj[v];
    }
    const double mu = Mean_mu, ktr = Mean_k;
    if (nDim == 2) {
      const double thetax = theta + UN[0] * UN[0] / 3.0, thetay = theta + UN[1] * UN[1] / 3.0;
      const double etaz = UN[0] * UN[1] / 3.0;
      const double pix = Vm[VX_P] * thetax + Vm[VX_P + 1] * etaz;
      const double piy = Vm[VX_P] * etaz + Vm[VX_P + 1] * thetay;
      FJ(RHOVX_S, RHOVX_S) = mu * thetax / dij * dS;
      FJ(RHOVX_S, RHOVX_S + 1) = mu * etaz / dij * dS;
      FJ(RHOVX_S + 1, RHOVX_S) = mu * etaz / dij * dS;
      FJ(RHOVX_S + 1, RHOVX_S + 1) = mu * thetay / dij * dS;
      FJ(RHOE_S, RHOVX_S) = pix * mu / dij * dS;
      FJ(RHOE_S, RHOVX_S + 1) = piy * mu / dij * dS;
      FJ(RHOE_S, RHOE_S) = ktr * theta / dij * dS;
    } else {
      const double thetax = theta + UN[0] * UN[0] / 3.0, thetay = theta + UN[1] * UN[1] / 3.0,
                   thetaz = theta + UN[2] * UN[2] / 3.0;
      const double etax = UN[1] * UN[2] / 3.0, etay = UN[0] * UN[2] / 3.0, etaz = UN[0] * UN[1] / 3.0;
      const double pix = Vm[VX_P] * thetax + Vm[VX_P + 1] * etaz + Vm[VX_P + 2] * etay;
      const double piy = Vm[VX_P] * etaz + Vm[VX_P + 1] * thetay + Vm[VX_P + 2] * etax;
      const double piz = Vm[VX_P] * etay + Vm[VX_P + 1] * etax + Vm[VX_P + 2] * thetaz;
      FJ(RHOVX_S, RHOVX_S) = mu * thetax / dij * dS;
      FJ(RHOVX_S, RHOVX_S + 1) = mu * etaz / dij * dS;
      FJ(RHOVX_S, RHOVX_S + 2) = mu * etay / dij * dS;
      FJ(RHOVX_S + 1, RHOVX_S) = mu * etaz / dij * dS;
      FJ(RHOVX_S + 1, RHOVX_S + 1) = mu * thetay / dij * dS;
      FJ(RHOVX_S + 1, RHOVX_S + 2) = mu * etax / dij * dS;
      FJ(RHOVX_S + 2, RHOVX_S) = mu * etay / dij * dS;
      FJ(RHOVX_S + 2, RHOVX_S + 1) = mu * etax / dij * dS;
      FJ(RHOVX_S + 2, RHOVX_S + 2) = mu * thetaz / dij * dS;
      FJ(RHOE_S, RHOVX_S) = pix * mu / dij * dS;
      FJ(RHOE_S, RHOVX_S + 1) = piy * mu / dij * dS;
      FJ(RHOE_S, RHOVX_S + 2) = piz * mu / dij * dS;
      FJ(RHOE_S, RHOE_S) = ktr * theta / dij * dS;
    }
    for (int a = 0; a < nVar; ++a)
      for (int b = 0; b < nVar; ++b) FI(a, b) = -FJ(a, b);
    for (int s = 0; s < ns; ++s) {
      FI(RHOE_S, RHOE_S) += -0.5 * Jd[s] * Cps[s];
      FJ(RHOE_S, RHOE_S) += -0.5 * Jd[s] * Cps[s];
    }
    for (int a = 0; a < ns; ++a) {
      FJ(RHOS_S + a, RHO_S) = -DJ(dJdr_j, a, 0) * dS;
      FI(RHOS_S + a, RHO_S) = -DJ(dJdr_i, a, 0) * dS;
      FJ(RHO_S, RHO_S) += FJ(RHOS_S + a, RHO_S);
      FI(RHO_S, RHO_S) += FI(RHOS_S + a, RHO_S);
      FJ(RHOE_S, RHO_S) += -DJ(dJdr_j, a, 0) * hs[a] * dS;
      FI(RHOE_S, RHO_S) += -DJ(dJdr_i, a, 0) * hs[a] * dS;
      for (int b = 0; b < ns; ++b) {
        FJ(RHOS_S + a, RHOS_S + b) = -DJ(dJdr_j, a, b + 1) * dS;
        FI(RHOS_S + a, RHOS_S + b) = -DJ(dJdr_i, a, b + 1) * dS;
        FJ(RHO_S, RHOS_S + b) += -DJ(dJdr_j, a, b + 1) * dS;
        FI(RHO_S, RHOS_S + b) += -DJ(dJdr_i, a, b + 1) * dS;
        FJ(RHOE_S, RHOS_S + a) += -DJ(dJdr_j, b, a + 1) * hs[b] * dS;
        FI(RHOE_S, RHOS_S + a) += -DJ(dJdr_i, b, a + 1) * hs[b] * dS;
      }
    }
  }
  // SST_Reactive_JacobianClosure
  if (P.rans) {
    double theta = 0.0;
    for (int d = 0; d < nDim; ++d) theta += UN[d] * UN[d];
    const double sq = std::sqrt(dist2);
    const double rho_i = Vi[RHO_P], rho_j = Vj[RHO_P];
    const double mut = Mean_mut, PrT = P.Prandtl_Turb, LeT = P.Lewis_Turb;
    if (nDim == 2) {
      const double thetax = theta + UN[0] * UN[0] / 3.0, thetay = theta + UN[1] * UN[1] / 3.0;
      const double etaz = UN[0] * UN[1] / 3.0;
      const double pix = Vm[VX_P] * thetax + Vm[VX_P + 1] * etaz;
      const double piy = Vm[VX_P] * etaz + Vm[VX_P + 1] * thetay;
      FJ(RHOVX_S, RHOVX_S) += mut * thetax / sq * Area;
      FJ(RHOVX_S, RHOVX_S + 1) += mut * etaz / sq * Area;
      FI(RHOVX_S, RHOVX_S) -= mut * thetax / sq * Area;
      FI(RHOVX_S, RHOVX_S + 1) -= mut * etaz / sq * Area;
      FJ(RHOVX_S + 1, RHOVX_S) += mut * etaz / sq * Area;
      FJ(RHOVX_S + 1, RHOVX_S + 1) += mut * thetay / sq * Area;
      FI(RHOVX_S + 1, RHOVX_S) -= mut * etaz / sq * Area;
      FI(RHOVX_S + 1, RHOVX_S + 1) -= mut * thetay / sq * Area;
      FJ(RHOE_S, RHOVX_S) += pix * mut / sq * Area;
      FJ(RHOE_S, RHOVX_S + 1) += piy * mut / sq * Area;
      FI(RHOE_S, RHOVX_S) -= pix * mut / sq * Area;
      FI(RHOE_S, RHOVX_S + 1) -= piy * mut / sq * Area;
      for (int s = 0; s < ns; ++s) {
        FJ(RHOE_S, RHOE_S) += mut / PrT * Cps[s] * Ys[s] * theta / sq * Area;
        FI(RHOE_S, RHOE_S) -= mut / PrT * Cps[s] * Ys[s] * theta / sq * Area;
        FJ(RHOE_S, RHOS_S + s) += mut / (PrT * LeT) * hs[s] * Ys[s] / rho_j * theta / sq * Area;
        FI(RHOE_S, RHOS_S + s) -= mut / (PrT * LeT) * hs[s] * Ys[s] / rho_i * theta / sq * Area;
      }
    } else {
      const double thetax = theta + UN[0] * UN[0] / 3.0, thetay = theta + UN[1] * UN[1] / 3.0,
                   thetaz = theta + UN[2] * UN[2] / 3.0;
      const double etax = UN[1] * UN[2] / 3.0, etay = UN[0] * UN[2] / 3.0, etaz = UN[0] * UN[1] / 3.0;
      const double pix = Vm[VX_P] * thetax + Vm[VX_P + 1] * etaz + Vm[VX_P + 2] * etay;
      const double piy = Vm[VX_P] * etaz + Vm[VX_P + 1] * thetay + Vm[VX_P + 2] * etax;
      const double piz = Vm[VX_P] * etay + Vm[VX_P + 1] * etax + Vm[VX_P + 2] * thetaz;
      const double th[3][3] = {{thetax, etaz, etay}, {etaz, thetay, etax}, {etay, etax, thetaz}};
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
          FJ(RHOVX_S + a, RHOVX_S + b) += mut * th[a][b] / sq * Area;
          FI(RHOVX_S + a, RHOVX_S + b) -= mut * th[a][b] / sq * Area;
        }
      const double pi[3] = {pix, piy, piz};
      for (int b = 0; b < 3; ++b) FJ(RHOE_S, RHOVX_S + b) += pi[b] * mut / sq * Area;
      for (int b = 0; b < 3; ++b) FI(RHOE_S, RHOVX_S + b) -= pi[b] * mut / sq * Area;
      for (int s = 0; s < ns; ++s) {
        FJ(RHOE_S, RHOE_S) += mut / PrT * Cps[s] * Ys[s] * theta / sq * Area;
        FI(RHOE_S, RHOE_S) -= mut / PrT * Cps[s] * Ys[s] * theta / sq * Area;
        for (int b = 0; b < ns; ++b) {
          FJ(RHOS_S + s, RHOS_S + b) += (s == b) * mut * Ys[s] / (PrT * LeT) / rho_j * theta / sq * Area;
          FI(RHOS_S + s, RHOS_S + b) -= (s == b) * mut * Ys[s] / (PrT * LeT) / rho_i * theta / sq * Area;
        }
        FJ(RHOE_S, RHOS_S + s) += mut / (PrT * LeT) * hs[s] / rho_j * theta / sq * Area;
        FI(RHOE_S, RHOS_S + s) -= mut / (PrT * LeT) * hs[s] / rho_i * theta / sq * Area;
      }
    }
    // Quirk (numerics_direct_reactive.cpp:1083-1084): inner_product over
    // Mean_Mass_Grads.row(s).data() .. +nDim walks the COLUMN-MAJOR storage, i.e. elements
    // s, s+1, .. of the flattened [col][row] array, not the row. Reproduced, not fixed.
    for (int s = 0; s < ns; ++s) {
      double aux = 0.0;
      for (int d = 0; d < nDim; ++d) {
        const int flat = s + d;
        aux += MassGrads[flat % ns][flat / ns] * UN[d];
      }
      FJ(RHOE_S, RHOE_S) += mut / (PrT * LeT) * Cps[s] * Ys[s] * aux * Area;
      FI(RHOE_S, RHOE_S) += mut / (PrT * LeT) * Cps[s] * Ys[s] * aux * Area;
    }
  }
  for (int d = 0; d < nDim; ++d) {
    FI(RHOE_S, RHOVX_S + d) += 0.5 * PF[RHOVX_S + d];
    FJ(RHOE_S, RHOVX_S + d) += 0.5 * PF[RHOVX_S + d];
  }
  for (int a = 0; a < nVar; ++a)
    for (int b = 0; b < nVar; ++b) {
      double si = 0.0, sj = 0.0;
      for (int k = 0; k < nVar; ++k) {
        si += dFdVi[a * nVar + k] * dVdUi[k * nVar + b];
        sj += dFdVj[a * nVar + k] * dVdUj[k * nVar + b];
      }
      Ji[a * nVar + b] = si;
      Jj[a * nVar + b] = sj;
    }
}

// ------------------------------------------------------------------------------------------------
// a12: CReactiveNSSolver::SetPrimitive_Gradient_LS (solver_direct_reactive.cpp:4887-5050)
// ------------------------------------------------------------------------------------------------
void grad_lsq_node(const Mech& m, int nDim, int i, const double* coord, const double* V, const int64_t* nptr,
                   const int64_t* nbr, double* out) {
  const int ns = m.ns, nPV = ns + nDim + 5, nG = ns + nDim + 2;
  const int P_P = nDim + 1, RHOS_P = nDim + 5, P_G = nDim + 1, RHOS_G = nDim + 2;
  auto prim = [&](int p, double* pv) {
    const double* v = V + (size_t)p * nPV;
    pv[0] = v[0];
    pv[P_G] = v[P_P];
    for (int d = 0; d < nDim; ++d) pv[1 + d] = v[1 + d];
    double yc[32];
    molar_from_mass(m, v + RHOS_P, yc, pv + RHOS_G);
  };
  double pi[32], pj[32], C[32][3];
  prim(i, pi);
  for (int v = 0; v < nG; ++v)
    for (int d = 0; d < nDim; ++d) C[v][d] = 0.0;
  double r11 = 0, r12 = 0, r13 = 0, r22 = 0, r23 = 0, r23_a = 0, r23_b = 0, r33 = 0;
  const double* ci = coord + (size_t)i * nDim;
  for (int64_t k = nptr[i]; k < nptr[i + 1]; ++k) {
    const int64_t j = nbr[k];
    const double* cj = coord + (size_t)j * nDim;
    prim((int)j, pj);
    double cij[3];
    for (int d = 0; d < nDim; ++d) cij[d] = cj[d] - ci[d];
    double w = 0.0;
    for (int d = 0; d < nDim; ++d) w += cij[d] * cij[d];
    if (w > EPS) {
      r11 += cij[0] * cij[0] / w;
      r12 += cij[0] * cij[1] / w;
      r22 += cij[1] * cij[1] / w;
      if (nDim == 3) {
        r13 += cij[0] * cij[2] / w;
        r23_a += cij[1] * cij[2] / w;
        r23_b += cij[0] * cij[2] / w;
        r33 += cij[2] * cij[2] / w;
      }
      for (int v = 0; v < nG; ++v)
        for (int d = 0; d < nDim; ++d) C[v][d] += cij[d] * (pj[v] - pi[v]) / w;
    }
  }
  r11 = (r11 > EPS) ? std::sqrt(r11) : 0.0;
  r12 = (std::abs(r11) > EPS) ? r12 / r11 : 0.0;
  r22 = (r22 - r12 * r12 > EPS) ? std::sqrt(r22 - r12 * r12) : 0.0;
  if (nDim == 3) {
    r13 = (std::abs(r11) > EPS) ? r13 / r11 : 0.0;
    r23 = (std::abs(r22) > EPS && std::abs(r11 * r22) > EPS) ? r23_a / r22 - r23_b * r12 / (r11 * r22) : 0.0;
    r33 = (r33 - r23 * r23 - r13 * r13 > EPS) ? std::sqrt(r33 - r23 * r23 - r13 * r13) : 0.0;
  }
  double detR2 = (nDim == 2) ? (r11 * r22) * (r11 * r22) : (r11 * r22 * r33) * (r11 * r22 * r33);
  bool singular = false;
  if (std::abs(detR2) < EPS) {
    detR2 = 1.0;
    singular = true;
  }
  double S[3][3] = {{0}};
  if (!singular) {
    if (nDim == 2) {
      S[0][0] = (r12 * r12 + r22 * r22) / detR2;
      S[0][1] = -r11 * r12 / detR2;
      S[1][0] = S[0][1];
      S[1][1] = r11 * r11 / detR2;
    } else {
      const double z11 = r22 * r33, z12 = -r12 * r33, z13 = r12 * r23 - r13 * r22;
      const double z22 = r11 * r33, z23 = -r11 * r23, z33 = r11 * r22;
      S[0][0] = (z11 * z11 + z12 * z12 + z13 * z13) / detR2;
      S[0][1] = (z12 * z22 + z13 * z23) / detR2;
      S[0][2] = (z13 * z33) / detR2;
      S[1][0] = S[0][1];
      S[1][1] = (z22 * z22 + z23 * z23) / detR2;
      S[1][2] = (z23 * z33) / detR2;
      S[2][0] = S[0][2];
      S[2][1] = S[1][2];
      S[2][2] = (z33 * z33) / detR2;
    }
  }
  for (int v = 0; v < nG; ++v)
    for (int d = 0; d < nDim; ++d) {
      double r = 0.0;
      for (int e = 0; e < nDim; ++e) r += C[v][e] * S[d][e];
      out[v * nDim + d] = r;
    }
}

// ------------------------------------------------------------------------------------------------
// a2: second-order branch of CReactiveEulerSolver::Upwind_Residual (solver_direct_reactive.cpp:2554-2729):
// MUSCL reconstruction of (T, u, v, P) with the (optional) limiter, then a thermodynamically consistent
// state rebuilt through the library (ComputeDensity :457-460 with SetRgas :26-31, ComputeEnthalpy
// :519-523, ComputeFrozenGamma :398-403 via ComputeCP :612-619, ComputedP_dYs :591-596). Reference
// quirk kept: side j's pressure check reads Prim_Recon_i[P] (:2617).
// refs = {Temperature_Ref, Energy_Ref, Gas_Constant_Ref}.
// ------------------------------------------------------------------------------------------------
void muscl_side(const Mech& m, int nDim, const double* V, const double* dPdU, const double* recon, bool non_phys,
                const double* refs, double* Prim, double* Sec, bool implicit) {
  const int ns = m.ns, nPV = ns + nDim + 5, nVar = ns + nDim + 2;
  const int T_ = 0, VX = 1, P_ = nDim + 1, RHO = nDim + 2, H_ = nDim + 3, A_ = nDim + 4, RHOS = nDim + 5;
  if (non_phys) {
    for (int v = 0; v < nPV; ++v) Prim[v] = V[v];
    if (implicit)
      for (int v = 0; v < nVar; ++v) Sec[v] = dPdU[v];
    return;
  }
  Prim[T_] = recon[0];
  Prim[P_] = recon[nDim + 1];
  for (int d = 0; d < nDim; ++d) Prim[VX + d] = recon[1 + d];
  double Ys[32];
  for (int s = 0; s < ns; ++s) {
    Prim[RHOS + s] = V[RHOS + s];
    Ys[s] = V[RHOS + s] < 0.0 ? 1.0e-30 : V[RHOS + s];  // SetMassFractions clamp
  }
  double Rgas = 0.0;
  for (int s = 0; s < ns; ++s) Rgas += Ys[s] * m.ri[s];
  double rho = Prim[P_] / (Prim[T_] * Rgas);
  rho *= refs[2];
  Prim[RHO] = rho;
  const double dim_temp = Prim[T_] * refs[0];
  double h = 0.0;
  for (int s = 0; s < ns; ++s) h += Ys[s] * (spline(m, P_H, s, dim_temp) / m.mm[s]);
  Prim[H_] = h / refs[1];
  double sq = 0.0;
  for (int d = 0; d < nDim; ++d) sq += Prim[VX + d] * Prim[VX + d];
  Prim[H_] += 0.5 * sq;
  double Cp = 0.0;
  for (int s = 0; s < ns; ++s) Cp += Ys[s] * (spline(m, P_CP, s, dim_temp) / m.mm[s]);
  double Rg2 = 0.0;
  for (int s = 0; s < ns; ++s) Rg2 += Ys[s] * m.ri[s];
  const double Gamma = Cp / (Cp - Rg2);
  Prim[A_] = std::sqrt(Gamma * Prim[P_] / rho);
  if (!implicit) return;
  Sec[0] = (Gamma - 1.0) * 0.5 * sq;
  for (int d = 0; d < nDim; ++d) Sec[1 + d] = (1.0 - Gamma) * Prim[VX + d];
  Sec[nDim + 1] = Gamma - 1.0;
  for (int s = 0; s < ns; ++s) {
    const double e_s = spline(m, P_H, s, dim_temp) / m.mm[s] - m.ri[s] * dim_temp;
    Sec[nDim + 2 + s] = (m.ri[s] * dim_temp - (Gamma - 1.0) * e_s) / refs[1];
  }
}

std::vector<Mech*> g_mechs;

}  // namespace

// =================================================================================================
// C ABI for the Python tests (ctypes).
// =================================================================================================
extern "C" {

// Threads the OpenMP loops of this file use (OMP_NUM_THREADS); 1 = the serial restatement. Every parallel loop
// writes disjoint outputs and keeps the reference's per-item operation order, so results do not depend on it.
int orc_num_threads() { return omp_get_max_threads(); }
void orc_set_num_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

void* orc_mech_create(int ns, int nr, int ntab, const double* mm, const double* dv, const double* sr,
                      const double* sp, const double* er, const double* ep, const double* A, const double* beta,
                      const double* Ta, const double* Ab, const double* betab, const double* Tab,
                      const int64_t* rev, const int64_t* hasb, const double* tx, const double* ty,
                      const double* ty2) {
  Mech* m = new Mech();
  m->ns = ns;
  m->nr = nr;
  m->ntab = ntab;
  m->mm.assign(mm, mm + ns);
  m->dv.assign(dv, dv + ns);
  m->ri.resize(ns);
  for (int s = 0; s < ns; ++s) m->ri[s] = R_UNGAS / mm[s];
  m->mtot = 0.0;
  for (int s = 0; s < ns; ++s) m->mtot += mm[s];
  m->sr.assign(sr, sr + ns * nr);
  m->sp.assign(sp, sp + ns * nr);
  m->er.assign(er, er + ns * nr);
  m->ep.assign(ep, ep + ns * nr);
  m->A.assign(A, A + nr);
  m->beta.assign(beta, beta + nr);
  m->Ta.assign(Ta, Ta + nr);
  m->Ab.assign(Ab, Ab + nr);
  m->betab.assign(betab, betab + nr);
  m->Tab.assign(Tab, Tab + nr);
  m->rev.assign(rev, rev + nr);
  m->hasb.assign(hasb, hasb + nr);
  m->tx.assign(tx, tx + 5 * ns * ntab);
  m->ty.assign(ty, ty + 5 * ns * ntab);
  m->ty2.assign(ty2, ty2 + 5 * ns * ntab);
  m->neg_reac.resize(nr);
  m->neg_prod.resize(nr);
  for (int r = 0; r < nr; ++r)
    for (int s = 0; s < ns; ++s) {
      if (m->er[r * ns + s] < 0.0) m->neg_reac[r].push_back(s);
      if (m->ep[r * ns + s] < 0.0) m->neg_prod[r].push_back(s);
    }
  return m;
}

void orc_mech_destroy(void* h) { delete static_cast<Mech*>(h); }

double orc_spline(void* h, int prop, int s, double T) { return spline(*static_cast<Mech*>(h), prop, s, T); }

// a1 over E edges. Outputs: res[E][nVar], Ji/Jj[E][nVar][nVar] (implicit only).
void orc_ausm_edges(int nDim, int ns, int64_t E, const int64_t* edges, const double* normal, const double* V,
                    const double* dPdU, double mach_inf, int implicit, double* res, double* Ji, double* Jj) {
  const int nVar = ns + nDim + 2, nPV = ns + nDim + 5;
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    ausm(nDim, ns, V + i * nPV, V + j * nPV, normal + e * nDim, implicit ? dPdU + i * nVar : nullptr,
         implicit ? dPdU + j * nVar : nullptr, mach_inf, implicit != 0, res + e * nVar,
         implicit ? Ji + e * nVar * nVar : nullptr, implicit ? Jj + e * nVar * nVar : nullptr);
  }
}

// a2 second-order: reconstruction + AUSM over E edges. grad [N][nG][nDim] (rows T, u, v, P first),
// limiter [N][nDim+2] or null (SECOND_ORDER without limiter). Returns 1 on a table-range error.
int orc_muscl_edges(void* h, int nDim, int64_t E, const int64_t* edges, const double* normal, const double* coord,
                    const double* V, const double* dPdU, const double* grad, const double* limiter,
                    const double* refs, double mach_inf, int implicit, double* res, double* Ji, double* Jj) {
  const Mech& m = *static_cast<Mech*>(h);
  const int ns = m.ns, nVar = ns + nDim + 2, nPV = ns + nDim + 5, nG = ns + nDim + 2, nL = nDim + 2;
  int err = 0;
#pragma omp parallel for schedule(static) reduction(| : err)
  for (int64_t e = 0; e < E; ++e) {
    try {
      const int64_t i = edges[2 * e], j = edges[2 * e + 1];
      const double* Vi = V + i * nPV;
      const double* Vj = V + j * nPV;
      double vec_i[3], vec_j[3];
      for (int d = 0; d < nDim; ++d) {
        vec_i[d] = 0.5 * (coord[j * nDim + d] - coord[i * nDim + d]);
        vec_j[d] = -vec_i[d];
      }
      double ri[8], rj[8];
      ri[0] = Vi[0];
      rj[0] = Vj[0];
      ri[nDim + 1] = Vi[nDim + 1];
      rj[nDim + 1] = Vj[nDim + 1];
      for (int d = 0; d < nDim; ++d) {
        ri[1 + d] = Vi[1 + d];
        rj[1 + d] = Vj[1 + d];
      }
      for (int v = 0; v < nL; ++v) {
        double pgi = 0.0, pgj = 0.0;
        for (int d = 0; d < nDim; ++d) {
          pgi += vec_i[d] * grad[(i * nG + v) * nDim + d];
          pgj += vec_j[d] * grad[(j * nG + v) * nDim + d];
        }
        if (limiter) {
          ri[v] += limiter[i * nL + v] * pgi;
          rj[v] += limiter[j * nL + v] * pgj;
        } else {
          ri[v] += pgi;
          rj[v] += pgj;
        }
      }
      bool npi = !(ri[0] > EPS);
      if (!npi) npi = !(ri[nDim + 1] > EPS);
      bool npj = !(rj[0] > EPS);
      if (!npj) npj = !(ri[nDim + 1] > EPS);  // :2617 checks side i's reconstructed pressure
      double Pi[32], Pj[32], Si[32], Sj[32];
      muscl_side(m, nDim, Vi, implicit ? dPdU + i * nVar : nullptr, ri, npi, refs, Pi, Si, implicit != 0);
      muscl_side(m, nDim, Vj, implicit ? dPdU + j * nVar : nullptr, rj, npj, refs, Pj, Sj, implicit != 0);
      ausm(nDim, ns, Pi, Pj, normal + e * nDim, implicit ? Si : nullptr, implicit ? Sj : nullptr, mach_inf,
           implicit != 0, res + e * nVar, implicit ? Ji + e * nVar * nVar : nullptr,
           implicit ? Jj + e * nVar * nVar : nullptr);
    } catch (const std::out_of_range&) {
      err = 1;
    }
  }
  return err;
}

// a9 over N cells. params = {C_mu, PaSR_lb, rho_ref, t_ref, T_ref}
int orc_source_cells(void* h, int nDim, int64_t N, const double* V, const double* dTdU, const double* vol,
                     const double* omega_turb, int rans, int implicit, const double* params, double* res, double* J) {
  const Mech& m = *static_cast<Mech*>(h);
  const int nVar = m.ns + nDim + 2, nPV = m.ns + nDim + 5;
  int err = 0;
#pragma omp parallel for schedule(static) reduction(| : err)
  for (int64_t i = 0; i < N; ++i) {
    try {
      source(m, nDim, V + i * nPV, implicit ? dTdU + i * nVar : nullptr, vol[i], rans ? omega_turb[i] : 0.0,
             rans != 0, implicit != 0, params[0], params[1], params[2], params[3], params[4], res + i * nVar,
             implicit ? J + i * nVar * nVar : nullptr);
    } catch (const std::exception&) {
      err = 1;
    }
  }
  return err;
}

// a3-a6 over E edges. vparams = {T_ref, E_ref, R_ref, Prandtl_Turb, Lewis_Turb}
int orc_visc_edges(void* h, int nDim, int64_t E, const int64_t* edges, const double* normal, const double* coord,
                   const double* V, const double* grad, const double* mu, const double* kappa, const double* Dij,
                   const double* dTdU, const double* tke, const double* mut, const double* sigma_k,
                   const double* gradk, int rans, int implicit, const double* vparams, double* res, double* Ji,
                   double* Jj) {
  const Mech& m = *static_cast<Mech*>(h);
  const int ns = m.ns, nVar = ns + nDim + 2, nPV = ns + nDim + 5, nG = ns + nDim + 2;
  ViscParams P{vparams[0], vparams[1], vparams[2], vparams[3], vparams[4], rans, implicit};
  int err = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(| : err)
  for (int64_t e = 0; e < E; ++e) {
    try {
      const int64_t i = edges[2 * e], j = edges[2 * e + 1];
      visc_flux(m, nDim, P, V + i * nPV, V + j * nPV, grad + i * nG * nDim, grad + j * nG * nDim, mu[i], mu[j],
                kappa[i], kappa[j], Dij + i * ns * ns, Dij + j * ns * ns, coord + i * nDim, coord + j * nDim,
                normal + e * nDim, implicit ? dTdU + i * nVar : nullptr, implicit ? dTdU + j * nVar : nullptr,
                rans ? tke[i] : 0.0, rans ? tke[j] : 0.0, rans ? mut[i] : 0.0, rans ? mut[j] : 0.0,
                rans ? sigma_k[i] : 1.0, rans ? gradk + i * nDim : nullptr, rans ? gradk + j * nDim : nullptr,
                res + e * nVar, implicit ? Ji + e * nVar * nVar : nullptr, implicit ? Jj + e * nVar * nVar : nullptr);
    } catch (const std::exception&) {
      err = 1;
    }
  }
  return err;
}

// a12 for the listed points (pts), all others untouched.
void orc_grad_lsq(void* h, int nDim, int64_t npts, const int64_t* pts, const double* coord, const double* V,
                  const int64_t* nptr, const int64_t* nbr, double* grad) {
  const Mech& m = *static_cast<Mech*>(h);
  const int nG = m.ns + nDim + 2;
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < npts; ++k) {
    const int64_t i = pts[k];
    grad_lsq_node(m, nDim, (int)i, coord, V, nptr, nbr, grad + i * nG * nDim);
  }
}

// a12, NUM_METHOD_GRAD = GREEN_GAUSS: CReactiveNSSolver::SetPrimitive_Gradient_GG (solver_direct_reactive.cpp:
// 4784-4880) in the reference's loop form: the edge loop (face value 0.5 (P_i + P_j) of (T, u, v(, w), P, X_s) with
// both sides' species taken from node 0, :4812-4813; + to node 0, - to node 1), the boundary vertices in (marker,
// vertex) order (- P_i n), then / Volume. Points [0, Nd) are updated (nPointDomain).
void orc_grad_gg(void* h, int nDim, int64_t Nd, int64_t E, const int64_t* edges, const double* normal, int64_t NB,
                 const int64_t* bpoint, const double* bnormal, const double* vol, const double* V, double* grad) {
  const Mech& m = *static_cast<Mech*>(h);
  const int ns = m.ns, nG = ns + nDim + 2, nPV = ns + nDim + 5, P_P = nDim + 1, RHOS_P = nDim + 5, P_G = nDim + 1,
            RHOS_G = nDim + 2;
  std::vector<double> pi(nG), pj(nG), yc(ns);
  auto prim = [&](int64_t p, int64_t q, double* out) {
    const double* v = V + p * nPV;
    out[0] = v[0];
    out[P_G] = v[P_P];
    for (int d = 0; d < nDim; ++d) out[1 + d] = v[1 + d];
    molar_from_mass(m, V + q * nPV + RHOS_P, yc.data(), out + RHOS_G);
  };
  for (int64_t q = 0; q < Nd * nG * nDim; ++q) grad[q] = 0.0;
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    prim(i, i, pi.data());
    prim(j, i, pj.data());
    for (int v = 0; v < nG; ++v) {
      const double avg = 0.5 * (pi[v] + pj[v]);
      for (int d = 0; d < nDim; ++d) {
        const double pr = avg * normal[e * nDim + d];
        if (i < Nd) grad[(i * nG + v) * nDim + d] += pr;
        if (j < Nd) grad[(j * nG + v) * nDim + d] -= pr;
      }
    }
  }
  for (int64_t b = 0; b < NB; ++b) {
    const int64_t i = bpoint[b];
    if (i >= Nd) continue;
    prim(i, i, pi.data());
    for (int v = 0; v < nG; ++v)
      for (int d = 0; d < nDim; ++d) grad[(i * nG + v) * nDim + d] -= pi[v] * bnormal[b * nDim + d];
  }
  for (int64_t i = 0; i < Nd; ++i)
    for (int q = 0; q < nG * nDim; ++q) grad[i * nG * nDim + q] = grad[i * nG * nDim + q] / vol[i];
}

// CSolver::SetSolution_Gradient_GG (solver_structure.cpp:519-578) of an [N][nVar] solution (the SST's (k, omega)):
// edge loop, boundary vertices of every marker, / (Volume + EPS).
void orc_sol_grad_gg(int nDim, int nVar, int64_t Nd, int64_t E, const int64_t* edges, const double* normal,
                     int64_t NB, const int64_t* bpoint, const double* bnormal, const double* vol, const double* sol,
                     double* grad) {
  for (int64_t q = 0; q < Nd * nVar * nDim; ++q) grad[q] = 0.0;
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    for (int v = 0; v < nVar; ++v) {
      const double avg = 0.5 * (sol[i * nVar + v] + sol[j * nVar + v]);
      for (int d = 0; d < nDim; ++d) {
        const double pr = avg * normal[e * nDim + d];
        if (i < Nd) grad[(i * nVar + v) * nDim + d] += pr;
        if (j < Nd) grad[(j * nVar + v) * nDim + d] -= pr;
      }
    }
  }
  for (int64_t b = 0; b < NB; ++b) {
    const int64_t i = bpoint[b];
    if (i >= Nd) continue;
    for (int v = 0; v < nVar; ++v)
      for (int d = 0; d < nDim; ++d) grad[(i * nVar + v) * nDim + d] -= sol[i * nVar + v] * bnormal[b * nDim + d];
  }
  for (int64_t i = 0; i < Nd; ++i)
    for (int q = 0; q < nVar * nDim; ++q) grad[i * nVar * nDim + q] = grad[i * nVar * nDim + q] / (vol[i] + EPS);
}

// a13: Venkatakrishnan limiter (solver_direct_reactive.cpp:1328-1523), edge-loop form.
void orc_limiter_venkat(int nDim, int ns, int64_t N, int64_t E, const int64_t* edges, const double* coord,
                        const double* V, const double* grad, double ref_len, double lim_coeff, double* lim) {
  const int nL = nDim + 2, nPV = ns + nDim + 5, nG = ns + nDim + 2;
  std::vector<double> mx(N * nL, -EPS), mn(N * nL, EPS);
  for (int64_t q = 0; q < N * nL; ++q) lim[q] = 2.0;
  auto pl = [&](int64_t p, int v) {
    const double* pv = V + p * nPV;
    if (v == 0) return pv[0];
    if (v == nL - 1) return pv[nDim + 1];
    return pv[v];
  };
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    for (int v = 0; v < nL; ++v) {
      const double du = pl(j, v) - pl(i, v);
      mn[i * nL + v] = std::min(mn[i * nL + v], du);
      mx[i * nL + v] = std::max(mx[i * nL + v], du);
      mn[j * nL + v] = std::min(mn[j * nL + v], -du);
      mx[j * nL + v] = std::max(mx[j * nL + v], -du);
    }
  }
  // gradient rows for the limited variables: T, u, v(, w), P are rows 0..nDim+1 of G
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    const double* Gi = grad + i * nG * nDim;
    const double* Gj = grad + j * nG * nDim;
    const double* ci = coord + i * nDim;
    const double* cj = coord + j * nDim;
    for (int v = 0; v < nL; ++v) {
      const double eps1 = lim_coeff * ref_len;
      const double eps2 = eps1 * eps1 * eps1;
      double dm = 0.0;
      for (int d = 0; d < nDim; ++d) dm += 0.5 * (cj[d] - ci[d]) * Gi[v * nDim + d];
      double dp = (dm > 0.0) ? mx[i * nL + v] : mn[i * nL + v];
      double lv = (dp * dp + 2.0 * dp * dm + eps2) / (dp * dp + dp * dm + 2.0 * dm * dm + eps2);
      if (lv < lim[i * nL + v]) lim[i * nL + v] = lv;
      dm = 0.0;
      for (int d = 0; d < nDim; ++d) dm += 0.5 * (ci[d] - cj[d]) * Gj[v * nDim + d];
      dp = (dm > 0.0) ? mx[j * nL + v] : mn[j * nL + v];
      lv = (dp * dp + 2.0 * dp * dm + eps2) / (dp * dp + dp * dm + 2.0 * dm * dm + eps2);
      if (lv < lim[j * nL + v]) lim[j * nL + v] = lv;
    }
  }
}

// a13: Barth-Jespersen branch (solver_direct_reactive.cpp:1383-1440), edge-loop form after the same min/max pass
// (:1346-1379). Reproduced as written: dm < EPS gives 2.0, dp = max only for dm > EPS (min at dm == EPS), and the
// j side tests the bool member `limiter` (true whenever SetPrimitive_Limiter runs, :4739-4742), so node j takes
// the edge's value whenever its current limiter exceeds 1 (:1426-1427). Then y -> (y^2 + 2y) / (y^2 + y + 2).
void orc_limiter_barth(int nDim, int ns, int64_t N, int64_t E, const int64_t* edges, const double* coord,
                       const double* V, const double* grad, double* lim) {
  const int nL = nDim + 2, nPV = ns + nDim + 5, nG = ns + nDim + 2;
  std::vector<double> mx(N * nL, -EPS), mn(N * nL, EPS);
  for (int64_t q = 0; q < N * nL; ++q) lim[q] = 2.0;
  auto pl = [&](int64_t p, int v) {
    const double* pv = V + p * nPV;
    if (v == 0) return pv[0];
    if (v == nL - 1) return pv[nDim + 1];
    return pv[v];
  };
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    for (int v = 0; v < nL; ++v) {
      const double du = pl(j, v) - pl(i, v);
      mn[i * nL + v] = std::min(mn[i * nL + v], du);
      mx[i * nL + v] = std::max(mx[i * nL + v], du);
      mn[j * nL + v] = std::min(mn[j * nL + v], -du);
      mx[j * nL + v] = std::max(mx[j * nL + v], -du);
    }
  }
  const double flag = 1.0;  // (double)limiter
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    const double* Gi = grad + i * nG * nDim;
    const double* Gj = grad + j * nG * nDim;
    const double* ci = coord + i * nDim;
    const double* cj = coord + j * nDim;
    for (int v = 0; v < nL; ++v) {
      double dm = 0.0, lv;
      for (int d = 0; d < nDim; ++d) dm += 0.5 * (cj[d] - ci[d]) * Gi[v * nDim + d];
      if (dm < EPS) {
        lv = 2.0;
      } else {
        const double dp = dm > EPS ? mx[i * nL + v] : mn[i * nL + v];
        lv = dp / dm;
      }
      if (lv < lim[i * nL + v]) lim[i * nL + v] = lv;
      dm = 0.0;
      for (int d = 0; d < nDim; ++d) dm += 0.5 * (ci[d] - cj[d]) * Gj[v * nDim + d];
      if (dm < EPS) {
        lv = 2.0;
      } else {
        const double dp = dm > EPS ? mx[j * nL + v] : mn[j * nL + v];
        lv = dp / dm;
      }
      if (flag < lim[j * nL + v]) lim[j * nL + v] = lv;
    }
  }
  for (int64_t q = 0; q < N * nL; ++q) {
    const double y = lim[q];
    lim[q] = (y * y + 2.0 * y) / (y * y + y + 2.0);
  }
}

// a18: CReactiveNSSolver::SetTime_Step, RANS branch (solver_direct_reactive.cpp:5057-5298).
// bverts[nb][2] = (marker, node) in marker/vertex order, bnormal[nb][nDim]. params = {CFL, Max_DeltaTime,
// Prandtl_Lam, Prandtl_Turb}. Outputs dt, lambda_inv, lambda_visc per node.
void orc_time_step(int nDim, int ns, int64_t N, int64_t E, const int64_t* edges, const double* normal, int64_t NB,
                   const int64_t* bverts, const double* bnormal, const double* V, const double* dPdU,
                   const double* mu, const double* eddy, const double* vol, const int64_t* nptr,
                   const double* params, double* dt, double* li, double* lv) {
  const int nPV = ns + nDim + 5, nVar = ns + nDim + 2;
  const int RHO_P = nDim + 2, A_P = nDim + 4, RHOE_S = nDim + 1;
  const double CFL = params[0], MaxDt = params[1], Pr_l = params[2], Pr_t = params[3];
  const double K_v = 0.25;
  for (int64_t i = 0; i < N; ++i) li[i] = lv[i] = 0.0;
  auto projvel = [&](int64_t p, const double* n) {
    double s = 0.0;
    for (int d = 0; d < nDim; ++d) s += V[p * nPV + 1 + d] * n[d];
    return s;
  };
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    const double* n = normal + e * nDim;
    double Area = 0.0;
    for (int d = 0; d < nDim; ++d) Area += n[d] * n[d];
    Area = std::sqrt(Area);
    const double pv = 0.5 * (projvel(i, n) + projvel(j, n));
    const double a = 0.5 * (V[i * nPV + A_P] + V[j * nPV + A_P]);
    const double rho = 0.5 * (V[i * nPV + RHO_P] + V[j * nPV + RHO_P]);
    const double m = 0.5 * (mu[i] + mu[j]);
    double lam = (std::abs(pv) + a) * Area;
    li[i] += lam;
    li[j] += lam;
    const double mt = 0.5 * (eddy[i] + eddy[j]);
    const double gam = dPdU[i * nVar + RHOE_S] + 1;
    const double l1 = 4.0 / 3.0 * (m + mt);
    const double l2 = (1.0 + (Pr_l / Pr_t) * (mt / m)) * (gam * m / Pr_l);
    lam = (l1 + l2) * Area * Area / rho;
    lv[i] += lam;
    lv[j] += lam;
  }
  for (int64_t b = 0; b < NB; ++b) {
    const int64_t i = bverts[2 * b + 1];
    const double* n = bnormal + b * nDim;
    double Area = 0.0;
    for (int d = 0; d < nDim; ++d) Area += n[d] * n[d];
    Area = std::sqrt(Area);
    const double pv = projvel(i, n);
    const double a = V[i * nPV + A_P];
    const double rho = V[i * nPV + RHO_P];
    const double m = mu[i];
    li[i] += (std::abs(pv) + a) * Area;
    const double mt = eddy[i];
    const double gam = dPdU[i * nVar + RHOE_S] + 1;
    const double l1 = (4.0 / 3.0) * (m + mt);
    const double l2 = (1.0 + (Pr_l / Pr_t) * (mt / m)) * (gam * m / Pr_l);
    lv[i] += (l1 + l2) * Area * Area / rho;
  }
  double minDt = 1.0e6;
  for (int64_t i = 0; i < N; ++i) {
    if (vol[i] > EPS) {
      double d = CFL * vol[i] / li[i];
      const double dv = CFL * K_v * vol[i] * vol[i] / lv[i];
      d = std::min(d, dv);
      minDt = std::min(minDt, d);
      if (d > MaxDt) d = MaxDt;
      dt[i] = d;
    } else {
      dt[i] = 0.0;
    }
  }
  for (int64_t i = 0; i < N; ++i)
    if (nptr[i + 1] - nptr[i] == 1) dt[i] = minDt;
}

// ---- a15-a17: block-sparse linear algebra (Common/src/matrix_structure.cpp, linear_solvers_structure.cpp)
// BSR: row_ptr[N+1], col[nnzb] sorted, blocks[nnzb][nb][nb] row-major. All N rows are domain rows.

// MatrixVectorProduct (:997-1030)
void orc_bsr_spmv(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* x,
                  double* y) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; ++i) {
    for (int a = 0; a < nb; ++a) y[i * nb + a] = 0.0;
    for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
      const double* b = A + k * nb * nb;
      const double* xv = x + col[k] * nb;
      for (int a = 0; a < nb; ++a)
        for (int c = 0; c < nb; ++c) y[i * nb + a] += b[a * nb + c] * xv[c];
    }
  }
}

static void gauss_elim(int nb, const double* Block, double* rhs) {  // Gauss_Elimination (:594-643)
  double blk[32 * 32];
  std::memcpy(blk, Block, sizeof(double) * nb * nb);
  if (nb == 1) {
    rhs[0] /= blk[0];
    return;
  }
  for (int i = 1; i < nb; ++i)
    for (int j = 0; j < i; ++j) {
      const double w = blk[i * nb + j] / blk[j * nb + j];
      for (int k = j; k < nb; ++k) blk[i * nb + k] -= w * blk[j * nb + k];
      rhs[i] -= w * rhs[j];
    }
  rhs[nb - 1] = rhs[nb - 1] / blk[nb * nb - 1];
  for (int i = nb - 2; i >= 0; --i) {
    double aux = 0.0;
    for (int j = i + 1; j < nb; ++j) aux += blk[i * nb + j] * rhs[j];
    rhs[i] = (rhs[i] - aux) / blk[i * nb + i];
  }
}

static int64_t find_diag(const int64_t* rp, const int64_t* col, int64_t i) {
  for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
    if (col[k] == i) return k;
  return -1;
}

// Partitions: rows are grouped in contiguous ranges [part_ptr[p], part_ptr[p+1]) that stand for the
// reference's MPI ranks (each rank's domain points, in the same relative order). A rank's matrix has
// its domain rows with columns on domain AND halo points; the preconditioners see the halo as follows
// (matrix_structure.cpp):
//   ILU(0) build/apply (:1397, :1416, :1472, :1489-1492): halo columns are skipped (block Jacobi);
//   LU-SGS (:1673-1709): LowerProduct only ever meets domain columns (halos are numbered after the
//   domain points), UpperProduct (:743-757) meets every halo column and reads the halo copy of x*
//   exchanged after the forward sweep (SendReceive_Solution :1687). The halo columns of a row come
//   after its domain columns, in increasing global index.
// np = 1, part_ptr = {0, N} is the serial reference.

// Row ranges [b[p], b[p+1]) of the ranks; {0, N} is the serial reference. The ranks are independent in every
// preconditioner sweep below (the halo couplings are block-Jacobi or read the exchanged copy), so they run on
// separate threads with the reference's per-rank arithmetic unchanged.
static std::vector<int64_t> part_bounds(int64_t N, int64_t np, const int64_t* pp) {
  if (!pp || np <= 1) return {0, N};
  return std::vector<int64_t>(pp, pp + np + 1);
}

// ComputeLU_SGSPreconditioner (:1673-1709)
void orc_lusgs_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* b,
                 double* x, int64_t np, const int64_t* part_ptr) {
  const std::vector<int64_t> B = part_bounds(N, np, part_ptr);
  const int64_t nparts = (int64_t)B.size() - 1;
  std::vector<double> xs(N * nb);
#pragma omp parallel
  {
    std::vector<double> aux(nb), prv(nb);
    auto blockprod = [&](int64_t k, const double* xv) {
      const double* blk = A + k * nb * nb;
      for (int a = 0; a < nb; ++a) {
        double pb = 0.0;
        for (int c = 0; c < nb; ++c) pb += blk[a * nb + c] * xv[c];
        prv[a] += pb;
      }
    };
#pragma omp for schedule(dynamic, 1)
    for (int64_t p = 0; p < nparts; ++p)
      for (int64_t i = B[p]; i < B[p + 1]; ++i) {  // (D+L) x* = b, per rank
        for (int a = 0; a < nb; ++a) prv[a] = 0.0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
          if (col[k] < i && col[k] >= B[p]) blockprod(k, x + col[k] * nb);
        for (int a = 0; a < nb; ++a) aux[a] = b[i * nb + a] - prv[a];
        gauss_elim(nb, A + find_diag(rp, col, i) * nb * nb, aux.data());
        for (int a = 0; a < nb; ++a) x[i * nb + a] = aux[a];
      }
#pragma omp for schedule(static)
    for (int64_t q = 0; q < N * nb; ++q) xs[q] = x[q];  // halo copies of x*
#pragma omp for schedule(dynamic, 1)
    for (int64_t p = 0; p < nparts; ++p) {
      const int64_t lo = B[p], hi = B[p + 1];
      for (int64_t i = hi - 1; i >= lo; --i) {  // (D+U) x = D x*
        const double* dblk = A + find_diag(rp, col, i) * nb * nb;
        for (int a = 0; a < nb; ++a) {
          double pb = 0.0;
          for (int c = 0; c < nb; ++c) pb += dblk[a * nb + c] * x[i * nb + c];
          aux[a] = pb;  // DiagonalProduct: prod_row_vector = 0 + block*x
        }
        for (int a = 0; a < nb; ++a) prv[a] = 0.0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
          if (col[k] > i && col[k] < hi) blockprod(k, x + col[k] * nb);
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
          if (col[k] < lo || col[k] >= hi) blockprod(k, xs.data() + col[k] * nb);
        for (int a = 0; a < nb; ++a) aux[a] -= prv[a];
        gauss_elim(nb, dblk, aux.data());
        for (int a = 0; a < nb; ++a) x[i * nb + a] = aux[a];
      }
    }
  }
}

// The forward half of orc_lusgs_p alone: x* of every rank, (D+L) x* = b (:1678-1685) — the values a rank's
// SendReceive_Solution hands its neighbours between the sweeps (:1687). Test infrastructure: the halo preset of the
// reference's own one-rank LU-SGS (oracle/make_golden.py case_rank9).
void orc_lusgs_fwd_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* b,
                     double* x, int64_t np, const int64_t* part_ptr) {
  const std::vector<int64_t> B = part_bounds(N, np, part_ptr);
  std::vector<double> aux(nb), prv(nb);
  for (int64_t p = 0; p + 1 < (int64_t)B.size(); ++p)
    for (int64_t i = B[p]; i < B[p + 1]; ++i) {
      for (int a = 0; a < nb; ++a) prv[a] = 0.0;
      for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
        if (col[k] < i && col[k] >= B[p]) {
          const double* blk = A + k * nb * nb;
          for (int a = 0; a < nb; ++a) {
            double pb = 0.0;
            for (int c = 0; c < nb; ++c) pb += blk[a * nb + c] * x[col[k] * nb + c];
            prv[a] += pb;
          }
        }
      for (int a = 0; a < nb; ++a) aux[a] = b[i * nb + a] - prv[a];
      gauss_elim(nb, A + find_diag(rp, col, i) * nb * nb, aux.data());
      for (int a = 0; a < nb; ++a) x[i * nb + a] = aux[a];
    }
}

void orc_lusgs(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* b,
               double* x) {
  orc_lusgs_p(N, nb, rp, col, A, b, x, 1, nullptr);
}

static void inverse_diag(int nb, const double* D, double* inv) {  // InverseDiagonalBlock_ILUMatrix (:1180-1228)
  double v[32];
  for (int i = 0; i < nb; ++i) {
    for (int j = 0; j < nb; ++j) v[j] = 0.0;
    v[i] = 1.0;
    gauss_elim(nb, D, v);
    for (int j = 0; j < nb; ++j) inv[j * nb + i] = v[j];
  }
}
static void mat_mat(int nb, const double* a, const double* b, double* c) {  // MatrixMatrixProduct
  for (int i = 0; i < nb; ++i)
    for (int j = 0; j < nb; ++j) {
      double s = 0.0;
      for (int k = 0; k < nb; ++k) s += a[i * nb + k] * b[k * nb + j];
      c[i * nb + j] = s;
    }
}
static void mat_vec(int nb, const double* a, const double* x, double* y) {
  for (int i = 0; i < nb; ++i) {
    double s = 0.0;
    for (int k = 0; k < nb; ++k) s += a[i * nb + k] * x[k];
    y[i] = s;
  }
}

// BuildILUPreconditioner (:1368-1451), including the left-multiply quirk at :1432-1436; per rank.
void orc_ilu_build_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, double* F,
                     int64_t np, const int64_t* part_ptr) {
  const std::vector<int64_t> B = part_bounds(N, np, part_ptr);
  const int64_t nparts = (int64_t)B.size() - 1;
  const int64_t nnzb = rp[N];
#pragma omp parallel for schedule(static)
  for (int64_t q = 0; q < nnzb * nb * nb; ++q) F[q] = A[q];
  auto findb = [&](int64_t i, int64_t j) -> double* {
    for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
      if (col[k] == j) return F + k * nb * nb;
    return nullptr;
  };
#pragma omp parallel
  {
    std::vector<double> inv(nb * nb), w(nb * nb), blk(nb * nb);
#pragma omp for schedule(dynamic, 1)
    for (int64_t p = 0; p < nparts; ++p) {
      const int64_t lo = B[p], hi = B[p + 1];
      for (int64_t i = lo + 1; i < hi; ++i) {  // the loop of each rank starts at its second row
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
          const int64_t j = col[k];
          if (j < i && j >= lo) {
            double* Bij = F + k * nb * nb;
            inverse_diag(nb, findb(j, j), inv.data());
            mat_mat(nb, Bij, inv.data(), w.data());
            for (int64_t kk = rp[j]; kk < rp[j + 1]; ++kk) {
              const int64_t kp = col[kk];
              if (kp >= j && kp < hi) {
                const double* Bjk = F + kk * nb * nb;
                mat_mat(nb, Bjk, w.data(), blk.data());
                double* Bik = findb(i, kp);
                if (Bik)  // SubtractBlock_ILUMatrix on a missing block is a no-op of the pattern
                  for (int q = 0; q < nb * nb; ++q) Bik[q] -= blk[q];
              }
            }
            std::memcpy(Bij, w.data(), sizeof(double) * nb * nb);
          }
        }
      }
    }
  }
}

void orc_ilu_build(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, double* F) {
  orc_ilu_build_p(N, nb, rp, col, A, F, 1, nullptr);
}

// ComputeILUPreconditioner (:1453-1515), per rank.
void orc_ilu_apply_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* F, const double* b,
                     double* x, int64_t np, const int64_t* part_ptr) {
  const std::vector<int64_t> B = part_bounds(N, np, part_ptr);
  const int64_t nparts = (int64_t)B.size() - 1;
  auto diag = [&](int64_t i) { return F + find_diag(rp, col, i) * nb * nb; };
#pragma omp parallel
  {
    std::vector<double> aux(nb), sum(nb), inv(nb * nb);
#pragma omp for schedule(dynamic, 1)
    for (int64_t p = 0; p < nparts; ++p) {
      const int64_t lo = B[p], hi = B[p + 1];
      for (int64_t q = lo * nb; q < hi * nb; ++q) x[q] = b[q];
      for (int64_t i = lo + 1; i < hi; ++i)
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
          const int64_t j = col[k];
          if (j < i && j >= lo) {
            mat_vec(nb, F + k * nb * nb, x + j * nb, aux.data());
            for (int a = 0; a < nb; ++a) x[i * nb + a] -= aux[a];
          }
        }
      for (int64_t i = hi - 1; i >= lo; --i) {
        if (i == hi - 1) {  // last row of the rank
          inverse_diag(nb, diag(i), inv.data());
          mat_vec(nb, inv.data(), x + i * nb, aux.data());
          for (int a = 0; a < nb; ++a) x[i * nb + a] = aux[a];
          continue;
        }
        for (int a = 0; a < nb; ++a) sum[a] = 0.0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
          const int64_t j = col[k];
          if (j >= i + 1 && j < hi) {
            mat_vec(nb, F + k * nb * nb, x + j * nb, aux.data());
            for (int a = 0; a < nb; ++a) sum[a] += aux[a];
          }
        }
        for (int a = 0; a < nb; ++a) x[i * nb + a] = x[i * nb + a] - sum[a];
        inverse_diag(nb, diag(i), inv.data());
        mat_vec(nb, inv.data(), x + i * nb, aux.data());
        for (int a = 0; a < nb; ++a) x[i * nb + a] = aux[a];
      }
    }
  }
}

void orc_ilu_apply(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* F, const double* b,
                   double* x) {
  orc_ilu_apply_p(N, nb, rp, col, F, b, x, 1, nullptr);
}

// FGMRES_LinSolver (linear_solvers_structure.cpp:309-463) + ModGramSchmidt (:87-186), Givens (:37-71),
// SolveReduced (:73-85). prec: 0 = LU-SGS on A, 1 = ILU0 with factor F. x in/out (initial guess).
// Returns iterations; *resid = final beta. Returns -1 on divergence (MGS exit, :108-150).
// Inner product used by FGMRES. Mode 0 (default): CSysVector dotProd (vector_structure.cpp:397-419),
// a sequential sum. Mode 1: the summation order of the device kernels (rx_krylov.hip k_dot_part /
// k_dot_fin: 512 x 256 grid-stride partial sums, pairwise tree in each block, then a pairwise tree
// over the 512 partials) — lets tests separate algorithmic parity (bitwise) from reduction order.
// Mode 1 with rank splits (orc_set_dot_ranks): the distributed device solve (rx_comm.hip), one context per rank
// owning the rows [rank_ptr[r], rank_ptr[r+1]): each rank's partial in the device order over its own rows, then
// the rank-ordered sum of the all-reduce (k_sum_ranks / rx_host_comm: ((p_0 + p_1) + p_2) + ...).
static int g_dot_mode = 0;
static std::vector<int64_t> g_dot_ranks;
void orc_set_dot_mode(int mode) { g_dot_mode = mode; }
void orc_set_dot_ranks(int64_t nr, const int64_t* row_ptr) {
  g_dot_ranks.assign(row_ptr ? row_ptr : nullptr, row_ptr ? row_ptr + nr + 1 : nullptr);
}
static double dot_device(int64_t n, const double* a, const double* c);
double orc_dot(int64_t n, const double* a, const double* c) {
  if (g_dot_mode == 0) {
    double s = 0.0;
    for (int64_t q = 0; q < n; ++q) s += a[q] * c[q];
    return s;
  }
  if (g_dot_ranks.size() >= 2 && g_dot_ranks.back() > 0 && n % g_dot_ranks.back() == 0) {
    const int64_t nb = n / g_dot_ranks.back();
    double s = 0.0;
    for (size_t r = 0; r + 1 < g_dot_ranks.size(); ++r) {
      const int64_t q0 = g_dot_ranks[r] * nb, q1 = g_dot_ranks[r + 1] * nb;
      const double p = dot_device(q1 - q0, a + q0, c + q0);
      s = r == 0 ? p : s + p;
    }
    return s;
  }
  return dot_device(n, a, c);
}
static double dot_device(int64_t n, const double* a, const double* c) {
  const int NB = 512, BS = 256;
  std::vector<double> part(NB), sh(BS);
#pragma omp parallel for schedule(static) firstprivate(sh)
  for (int b = 0; b < NB; ++b) {
    for (int t = 0; t < BS; ++t) {
      double s = 0.0;
      for (int64_t q = (int64_t)b * BS + t; q < n; q += (int64_t)NB * BS) s += a[q] * c[q];
      sh[t] = s;
    }
    for (int w = BS / 2; w > 0; w >>= 1)
      for (int t = 0; t < w; ++t) sh[t] += sh[t + w];
    part[b] = sh[0];
  }
  for (int t = 0; t < BS; ++t) sh[t] = part[t] + part[t + BS];
  for (int w = BS / 2; w > 0; w >>= 1)
    for (int t = 0; t < w; ++t) sh[t] += sh[t + w];
  return sh[0];
}

// BuildJacobiPreconditioner (matrix_structure.cpp:1230-1246): invM_i = InverseDiagonalBlock of the diagonal block
// (:1129-1143, the Gauss_Elimination of each unit column)
static std::vector<double> jacobi_build(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A) {
  std::vector<double> inv((size_t)N * nb * nb);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; ++i) inverse_diag(nb, A + find_diag(rp, col, i) * nb * nb, inv.data() + i * nb * nb);
  return inv;
}

// The preconditioner of CSysSolve::Solve (linear_solvers_structure.cpp:633-653) applied to in -> out.
// prec: 0 LU_SGS (ComputeLU_SGSPreconditioner), 1 ILU0 with factor F (ComputeILUPreconditioner), 2 JACOBI with invM
// (ComputeJacobiPreconditioner :1249-1266: prod = 0.0 + invM_i vec_i, c ascending — mat_vec's order).
static void prec_apply(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* F,
                       const std::vector<double>& invM, int prec, const double* in, double* out, int64_t np,
                       const int64_t* part_ptr) {
  if (prec == 0) {
    orc_lusgs_p(N, nb, rp, col, A, in, out, np, part_ptr);
  } else if (prec == 1) {
    orc_ilu_apply_p(N, nb, rp, col, F, in, out, np, part_ptr);
  } else {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) mat_vec(nb, invM.data() + i * nb * nb, in + i * nb, out + i * nb);
  }
}

int orc_fgmres_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* F,
                 int prec, const double* b, double* x, double tol, int m, double* resid, int64_t np,
                 const int64_t* part_ptr) {
  const int64_t n = N * nb;
  auto dotp = [&](const double* a, const double* c) { return orc_dot(n, a, c); };
  auto norm = [&](const double* a) { return std::sqrt(dotp(a, a)); };
  std::vector<double> invM;
  if (prec == 2) invM = jacobi_build(N, nb, rp, col, A);
  auto precond = [&](const double* in, double* out) { prec_apply(N, nb, rp, col, A, F, invM, prec, in, out, np, part_ptr); };
  std::vector<std::vector<double>> w(m + 1, std::vector<double>(n)), z(m + 1, std::vector<double>(n));
  std::vector<double> g(m + 1, 0.0), sn(m + 1, 0.0), cs(m + 1, 0.0), y(m, 0.0);
  std::vector<std::vector<double>> H(m + 1, std::vector<double>(m, 0.0));
  double norm0 = norm(b);
  orc_bsr_spmv(N, nb, rp, col, A, x, w[0].data());
#pragma omp parallel for schedule(static)
  for (int64_t q = 0; q < n; ++q) w[0][q] -= b[q];
  double beta = norm(w[0].data());
  const double epsm = std::numeric_limits<double>::epsilon();
  if ((beta < tol * norm0) || (beta < epsm)) {
    *resid = beta;
    return 0;
  }
#pragma omp parallel for schedule(static)
  for (int64_t q = 0; q < n; ++q) w[0][q] /= -beta;
  g[0] = beta;
  norm0 = beta;
  int i = 0;
  for (i = 0; i < m; ++i) {
    if (beta < tol * norm0) break;
    precond(w[i].data(), z[i].data());
    orc_bsr_spmv(N, nb, rp, col, A, z[i].data(), w[i + 1].data());
    // ModGramSchmidt
    const double reorth = 0.98;
    double nrm = dotp(w[i + 1].data(), w[i + 1].data());
    double thr = nrm * reorth;
    if ((nrm <= 0.0) || (nrm != nrm)) return -1;
    for (int k = 0; k < i + 1; ++k) {
      double prod = dotp(w[i + 1].data(), w[k].data());
      H[k][i] = prod;
#pragma omp parallel for schedule(static)
      for (int64_t q = 0; q < n; ++q) w[i + 1][q] += -prod * w[k][q];
      if (prod * prod > thr) {
        prod = dotp(w[i + 1].data(), w[k].data());
        H[k][i] += prod;
#pragma omp parallel for schedule(static)
        for (int64_t q = 0; q < n; ++q) w[i + 1][q] += -prod * w[k][q];
      }
      nrm -= H[k][i] * H[k][i];
      if (nrm < 0.0) nrm = 0.0;
      thr = nrm * reorth;
    }
    nrm = norm(w[i + 1].data());
    H[i + 1][i] = nrm;
#pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < n; ++q) w[i + 1][q] /= nrm;
    auto applyG = [](double s, double c, double& h1, double& h2) {
      const double t = c * h1 + s * h2;
      h2 = c * h2 - s * h1;
      h1 = t;
    };
    for (int k = 0; k < i; ++k) applyG(sn[k], cs[k], H[k][i], H[k + 1][i]);
    {  // GenerateGivens(H[i][i], H[i+1][i], sn[i], cs[i])
      double& dx = H[i][i];
      double& dy = H[i + 1][i];
      double& s = sn[i];
      double& c = cs[i];
      auto sgn = [](double a, double bb) { return bb == 0.0 ? 0.0 : (bb < 0 ? -std::fabs(a) : std::fabs(a)); };
      if ((dx == 0.0) && (dy == 0.0)) {
        c = 1.0;
        s = 0.0;
      } else if (std::fabs(dy) > std::fabs(dx)) {
        const double tmp = dx / dy;
        dx = std::sqrt(1.0 + tmp * tmp);
        s = sgn(1.0 / dx, dy);
        c = tmp * s;
      } else if (std::fabs(dy) <= std::fabs(dx)) {
        const double tmp = dy / dx;
        dy = std::sqrt(1.0 + tmp * tmp);
        c = sgn(1.0 / dy, dx);
        s = tmp * c;
      } else {
        dx = 0.0;
        dy = 0.0;
        c = 1.0;
        s = 0.0;
      }
      dx = std::fabs(dx * dy);
      dy = 0.0;
    }
    applyG(sn[i], cs[i], g[i], g[i + 1]);
    beta = std::fabs(g[i + 1]);
  }
  // SolveReduced
  for (int k = 0; k < i; ++k) y[k] = g[k];
  for (int k = i - 1; k >= 0; --k) {
    y[k] /= H[k][k];
    for (int j = k - 1; j >= 0; --j) y[j] -= H[j][k] * y[k];
  }
  for (int k = 0; k < i; ++k)
#pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < n; ++q) x[q] += y[k] * z[k][q];
  *resid = beta;
  return i;
}

int orc_fgmres(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* F, int prec,
               const double* b, double* x, double tol, int m, double* resid) {
  return orc_fgmres_p(N, nb, rp, col, A, F, prec, b, x, tol, m, resid, 1, nullptr);
}

// BCGSTAB_LinSolver (linear_solvers_structure.cpp:465-599). prec as orc_fgmres_p. Returns the iteration index of
// the break (or m); *resid = the last |r| (on the initial-guess exit the reference leaves *residual unset).
int orc_bcgstab_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* F,
                  int prec, const double* b, double* x, double tol, int m, double* resid, int64_t np,
                  const int64_t* part_ptr) {
  const int64_t n = N * nb;
  auto dotp = [&](const double* a, const double* c) { return orc_dot(n, a, c); };
  std::vector<double> invM;
  if (prec == 2) invM = jacobi_build(N, nb, rp, col, A);
  auto precond = [&](const double* in, double* out) { prec_apply(N, nb, rp, col, A, F, invM, prec, in, out, np, part_ptr); };
  std::vector<double> r(b, b + n), r0(b, b + n), p(b, b + n), v(b, b + n), sv(b, b + n), t(b, b + n),
      ph(b, b + n), sh(b, b + n), Ax(n);
  orc_bsr_spmv(N, nb, rp, col, A, x, Ax.data());  // mat_vec(x, A_x)
  for (int64_t q = 0; q < n; ++q) r[q] -= Ax[q];  // r -= A_x
  r0 = r;
  double norm_r = std::sqrt(dotp(r.data(), r.data()));
  double norm0 = std::sqrt(dotp(b, b));
  const double epsm = std::numeric_limits<double>::epsilon();
  *resid = norm_r;
  if ((norm_r < tol * norm0) || (norm_r < epsm)) return 0;
  double alpha = 1.0, beta = 1.0, omega = 1.0, rho = 1.0, rho_prime = 1.0;
  norm0 = norm_r;
  int i = 0;
  for (i = 0; i < m; ++i) {
    rho_prime = rho;
    rho = dotp(r.data(), r0.data());
    beta = (rho / rho_prime) * (alpha / omega);
    const double beta_omega = -beta * omega;
    for (int64_t q = 0; q < n; ++q) p[q] = beta * p[q] + beta_omega * v[q];  // Equals_AX_Plus_BY
    for (int64_t q = 0; q < n; ++q) p[q] += 1.0 * r[q];                       // Plus_AX
    precond(p.data(), ph.data());
    orc_bsr_spmv(N, nb, rp, col, A, ph.data(), v.data());
    const double r_0_v = dotp(r0.data(), v.data());
    alpha = rho / r_0_v;
    for (int64_t q = 0; q < n; ++q) sv[q] = 1.0 * r[q] + (-alpha) * v[q];
    precond(sv.data(), sh.data());
    orc_bsr_spmv(N, nb, rp, col, A, sh.data(), t.data());
    omega = dotp(t.data(), sv.data()) / dotp(t.data(), t.data());
    for (int64_t q = 0; q < n; ++q) x[q] += alpha * ph[q];
    for (int64_t q = 0; q < n; ++q) x[q] += omega * sh[q];
    for (int64_t q = 0; q < n; ++q) r[q] = 1.0 * sv[q] + (-omega) * t[q];
    norm_r = std::sqrt(dotp(r.data(), r.data()));
    *resid = norm_r;
    if (norm_r < tol * norm0) break;
  }
  return i;
}

// RESTARTED_FGMRES (CSysSolve::Solve :662-671): FGMRES cycles from the previous cycle's x, MaxIter = iter (the
// remainder once total + restart > iter), the tolerance multiplied by 1 / |b| after each cycle, until iter iterations
// are spent or |b| < tol. Returns the summed iterations (-1 on an FGMRES breakdown); stops after 4096 cycles (the
// reference's loop would not end, see rx_la_restarted_fgmres).
int orc_restarted_fgmres_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A,
                           const double* F, int prec, const double* b, double* x, double tol, int iter, int restart,
                           double* resid, int64_t np, const int64_t* part_ptr) {
  int total = 0, max_iter = iter;
  double stol = tol;
  for (int cycle = 0; total < iter; ++cycle) {
    if (cycle == 4096) return -2;
    if ((int64_t)total + restart > iter) max_iter = iter - total;
    const int it = orc_fgmres_p(N, nb, rp, col, A, F, prec, b, x, stol, max_iter, resid, np, part_ptr);
    if (it < 0) return it;
    total += it;
    const double bn = std::sqrt(orc_dot(N * nb, b, b));  // LinSysRes.norm()
    if (bn < stol) break;
    stol = stol * (1.0 / bn);
  }
  return total;
}

// The smoothers of Solve's non-Krylov branch (:683-701): kind 0 LU_SGS_Smoother (matrix_structure.cpp:1711-1835),
// 1 ILU0_Smoother (:1517-1671, factor F), 2 Jacobi_Smoother (:1268-1366). x += M^-1 r (LU_SGS / ILU0: the
// preconditioner sweeps, whose arithmetic the smoothers repeat, then Plus_AX(omega = 1.0); JACOBI: invM r added into x
// term by term), r = b - A x, |r| < tol |r_0| ends the loop. Returns the iteration index of the break (or m).
int orc_smoother_p(int64_t N, int nb, const int64_t* rp, const int64_t* col, const double* A, const double* F,
                   int kind, const double* b, double* x, double tol, int m, double* resid, int64_t np,
                   const int64_t* part_ptr) {
  const int64_t n = N * nb;
  auto dotp = [&](const double* a, const double* c) { return orc_dot(n, a, c); };
  std::vector<double> invM;
  if (kind == 2) invM = jacobi_build(N, nb, rp, col, A);
  std::vector<double> r(b, b + n), Ax(n), z(n);
  orc_bsr_spmv(N, nb, rp, col, A, x, Ax.data());
  for (int64_t q = 0; q < n; ++q) r[q] -= Ax[q];
  double norm_r = std::sqrt(dotp(r.data(), r.data()));
  double norm0 = std::sqrt(dotp(b, b));
  const double epsm = std::numeric_limits<double>::epsilon();
  *resid = norm_r;
  if ((norm_r < tol * norm0) || (norm_r < epsm)) return 0;
  norm0 = norm_r;
  int i = 0;
  for (i = 0; i < m; ++i) {
    if (kind == 2) {
#pragma omp parallel for schedule(static)
      for (int64_t pt = 0; pt < N; ++pt)
        for (int a = 0; a < nb; ++a)
          for (int c = 0; c < nb; ++c) x[pt * nb + a] += invM[(pt * nb + a) * nb + c] * r[pt * nb + c];
    } else {
      if (kind == 0) orc_lusgs_p(N, nb, rp, col, A, r.data(), z.data(), np, part_ptr);
      else orc_ilu_apply_p(N, nb, rp, col, F, r.data(), z.data(), np, part_ptr);
      for (int64_t q = 0; q < n; ++q) x[q] += 1.0 * z[q];
    }
    orc_bsr_spmv(N, nb, rp, col, A, x, Ax.data());
    for (int64_t q = 0; q < n; ++q) r[q] = b[q] - Ax[q];  // r = b; r -= A_x
    norm_r = std::sqrt(dotp(r.data(), r.data()));
    *resid = norm_r;
    if (norm_r < tol * norm0) break;
  }
  return i;
}

static int64_t blk_of(const int64_t* rp, const int64_t* col, int64_t i, int64_t j) {
  const int64_t* lo = col + rp[i];
  const int64_t* hi = col + rp[i + 1];
  const int64_t* p = std::lower_bound(lo, hi, j);
  return (p != hi && *p == j) ? (p - col) : -1;
}

// Residual + Jacobian assembly in the reference's loop order: Upwind_Residual scatter
// (solver_direct_reactive.cpp:2759-2772: R_i += F, R_j -= F; A_ii += Ji, A_ij += Jj, A_ji -= Ji,
// A_jj -= Jj), Viscous_Residual with the opposite signs (:5374-5381), Source_Residual (R_i += S,
// A_ii += Js), then ImplicitEuler_Iteration (:2336-2380): A_ii += Vol/dt (or A_ii = I, R_i = 0 when
// dt <= EPS), rhs = -(R + 0). Any of the Jacobian pointers may be null (explicit assembly of R only).
void orc_assemble(int64_t N, int64_t E, int nb, const int64_t* edges, const int64_t* rp, const int64_t* col,
                  const double* Fc, const double* Jci, const double* Jcj, const double* Fv, const double* Jvi,
                  const double* Jvj, const double* Rs, const double* Js, const double* vol, const double* dt,
                  double* R, double* A, double* rhs) {
  // The reference scatters edge by edge; every row's residual and blocks receive their contributions in edge
  // order, pass by pass. Gathering per row over its incident edges in increasing edge id (convective pass, then
  // viscous) reproduces each sum's order exactly, so the rows are assembled in parallel.
  const int nb2 = nb * nb;
  std::vector<int64_t> ip(N + 1, 0), ie(2 * E);
  for (int64_t e = 0; e < E; ++e) {
    ++ip[edges[2 * e] + 1];
    ++ip[edges[2 * e + 1] + 1];
  }
  for (int64_t i = 0; i < N; ++i) ip[i + 1] += ip[i];
  {
    std::vector<int64_t> fill(ip.begin(), ip.end() - 1);
    for (int64_t e = 0; e < E; ++e) {
      ie[fill[edges[2 * e]]++] = e;
      ie[fill[edges[2 * e + 1]]++] = e;
    }
  }
  auto add = [&](int64_t b, const double* J, double sgn) {
    double* d = A + b * nb2;
    if (sgn > 0)
      for (int q = 0; q < nb2; ++q) d[q] += J[q];
    else
      for (int q = 0; q < nb2; ++q) d[q] -= J[q];
  };
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t r = 0; r < N; ++r) {
    for (int v = 0; v < nb; ++v) R[r * nb + v] = 0.0;
    if (A)
      for (int64_t q = rp[r] * nb2; q < rp[r + 1] * nb2; ++q) A[q] = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
      const double* F = pass ? Fv : Fc;
      const double* Ji = pass ? Jvi : Jci;
      const double* Jj = pass ? Jvj : Jcj;
      if (!F) continue;
      const double s = pass ? -1.0 : 1.0;
      for (int64_t q = ip[r]; q < ip[r + 1]; ++q) {
        const int64_t e = ie[q];
        const int64_t i = edges[2 * e], j = edges[2 * e + 1];
        if (r == i) {
          for (int v = 0; v < nb; ++v) {
            if (s > 0) R[i * nb + v] += F[e * nb + v];
            else R[i * nb + v] -= F[e * nb + v];
          }
          if (A && Ji) {
            add(blk_of(rp, col, i, i), Ji + e * nb2, s);
            add(blk_of(rp, col, i, j), Jj + e * nb2, s);
          }
        } else {
          for (int v = 0; v < nb; ++v) {
            if (s > 0) R[j * nb + v] -= F[e * nb + v];
            else R[j * nb + v] += F[e * nb + v];
          }
          if (A && Ji) {
            add(blk_of(rp, col, j, i), Ji + e * nb2, -s);
            add(blk_of(rp, col, j, j), Jj + e * nb2, -s);
          }
        }
      }
    }
    if (Rs) {
      for (int v = 0; v < nb; ++v) R[r * nb + v] += Rs[r * nb + v];
      if (A && Js) add(blk_of(rp, col, r, r), Js + r * nb2, 1.0);
    }
    if (!A) continue;
    double* D = A + blk_of(rp, col, r, r) * nb2;
    if (dt[r] > EPS) {
      const double delta = vol[r] / dt[r];
      for (int a = 0; a < nb; ++a) D[a * nb + a] += delta;
    } else {
      for (int a = 0; a < nb; ++a)
        for (int c = 0; c < nb; ++c) D[a * nb + c] = (a == c) ? 1.0 : 0.0;
      for (int a = 0; a < nb; ++a) R[r * nb + a] = 0.0;
    }
    for (int a = 0; a < nb; ++a) rhs[r * nb + a] = -(R[r * nb + a] + 0.0);
  }
}

// CReactiveEulerVariable::AddClippedSolution (variable_reactive.hpp) as called by
// ImplicitEuler_Iteration (:2390-2400, relax * LinSysSol) and ExplicitEuler_Iteration (:2430-2440,
// -Res * dt / Vol). Lower bound 0 for density/species/… and -1/EPS for momentum/energy, upper 1/EPS.
void orc_update(int64_t N, int nb, int nDim, int mode, const double* d, double relax, const double* vol,
                const double* dt, double* U) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; ++i)
    for (int v = 0; v < nb; ++v) {
      double delta;
      if (mode == 0) {
        delta = relax * d[i * nb + v];
      } else {
        double Delta = 0.0;
        if (vol[i] > EPS) Delta = dt[i] / vol[i];
        delta = -(d[i * nb + v] + 0.0) * Delta;
      }
      const double lo = (v >= 1 && v <= nDim + 1) ? -1.0 / EPS : 0.0;
      const double hi = 1.0 / EPS;
      U[i * nb + v] = std::min(std::max(U[i * nb + v] + delta, lo), hi);
    }
}

// CReactiveEulerSolver::ExplicitRK_Iteration (solver_direct_reactive.cpp:2456-2493): one stage,
// U = clip(U_old + (-(Res + 0) * dt / Vol) * alpha) via AddClippedSolution (variable_structure.cpp:207-211).
void orc_update_rk(int64_t N, int nb, int nDim, const double* Res, double alpha, const double* vol, const double* dt,
                   const double* Uold, double* U) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; ++i) {
    double Delta = 0.0;
    if (vol[i] > EPS) Delta = dt[i] / vol[i];
    for (int v = 0; v < nb; ++v) {
      const double r = Res[i * nb + v] + 0.0;
      const double lo = (v >= 1 && v <= nDim + 1) ? -1.0 / EPS : 0.0;
      const double hi = 1.0 / EPS;
      U[i * nb + v] = std::min(std::max(Uold[i * nb + v] + -r * Delta * alpha, lo), hi);
    }
  }
}

// =================================================================================================
// next-1: CReactiveEulerSolver::SetPrimitive_Variables (solver_direct_reactive.cpp:985-1040) per point:
// CReactiveNSVariable::SetPrimVar(eddy, k) (variable_direct_reactive.cpp:1188-1228) ->
// CReactiveEulerVariable::SetPrimVar (:292-330) -> Cons2PrimVar (:550-778), Cp from the sound speed,
// CalcdTdU (:786-823), CalcdPdU (:829-853); transport: ComputeEta (reacting_model_library.cpp:634-656),
// ComputeLambda (:671-696), GetDij_SM (:751-766).
// prm = {Tmin, Tmax, T_ref, E_ref, R_ref, P_ref, Visc_ref, Cond_ref, Vel_ref, Len_ref, ExtIter, clip_temp}.
// U is updated in place (the reference clamps negative partial densities / density in Solution).
// Returns -1 when the bisection fails (std::runtime_error in the reference), else the non-physical count.
// =================================================================================================
namespace {
double mix_enthalpy(const Mech& m, double T, const double* Ys) {  // ComputeEnthalpy :519-523
  double h = 0.0;
  for (int s = 0; s < m.ns; ++s) {
    const double y = Ys[s] < 0.0 ? 1.0e-30 : Ys[s];
    h += y * (spline(m, P_H, s, T) / m.mm[s]);
  }
  return h;
}
double mix_rgas(const Mech& m, const double* Ys) {  // SetRgas :26-31
  double r = 0.0;
  for (int s = 0; s < m.ns; ++s) r += (Ys[s] < 0.0 ? 1.0e-30 : Ys[s]) * m.ri[s];
  return r;
}
// Cons2PrimVar (:550-778); V[T] on entry is the secant's start. Throws std::runtime_error on failure.
bool cons2prim(const Mech& m, int nDim, double* U, double* V, double val_ke, const double* prm) {
  const int ns = m.ns;
  const int T_ = 0, VX = 1, P_ = nDim + 1, RHO = nDim + 2, H_ = nDim + 3, A_ = nDim + 4, RHOS = nDim + 5;
  const int RHO_S = 0, RHOVX_S = 1, RHOE_S = nDim + 1, RHOS_S = nDim + 2;
  bool nonPhys = false;
  for (int s = 0; s < ns; ++s)
    if (U[RHOS_S + s] < 0.0) {
      U[RHOS_S + s] = 1.0e-30;
      nonPhys = true;
    }
  if (U[RHO_S] < EPS) {
    V[RHO] = U[RHO_S] = EPS;
    nonPhys = true;
  } else {
    V[RHO] = U[RHO_S];
  }
  for (int s = 0; s < ns; ++s) V[RHOS + s] = U[RHOS_S + s] / U[RHO_S];
  double Ys[32];
  for (int s = 0; s < ns; ++s) Ys[s] = V[RHOS + s];
  double sy = 0.0;
  for (int s = 0; s < ns; ++s) sy += Ys[s];
  nonPhys = nonPhys || (std::abs(sy - 1.0) > 0.1);
  const double rho = U[RHO_S];
  const double rhoE = U[RHOE_S] - rho * val_ke;
  double sqvel = 0.0;
  for (int d = 0; d < nDim; ++d) {
    V[VX + d] = U[RHOVX_S + d] / rho;
    sqvel += V[VX + d] * V[VX + d];
  }
  const double T_ref = prm[2], E_ref = prm[3], R_ref = prm[4];
  const double Tmin = prm[0] / T_ref, Tmax = prm[1] / T_ref;
  const double NRtol = 1.0e-6, Btol = 1.0e-4;
  const int maxNIter = 7, maxBIter = 32;
  bool NRconvg = false, Bconvg;
  const double Rgas = mix_rgas(m, Ys) / R_ref;
  const double C1 = (-rhoE + 0.5 * rho * sqvel) / (rho * Rgas);
  const double C2 = 1.0 / Rgas;
  const double old_temp = V[T_];
  double T = V[T_], Told = T + 1.0, Tnew, f, df, hs, hs_old;
  for (int iIter = 0; iIter < maxNIter; ++iIter) {
    try {
      const double dim_temp = T * T_ref, dim_temp_old = Told * T_ref;
      hs_old = mix_enthalpy(m, dim_temp_old, Ys) / E_ref;
      hs = mix_enthalpy(m, dim_temp, Ys) / E_ref;
      f = T - C1 - C2 * hs;
      df = T - Told + C2 * (hs_old - hs);
      Tnew = T - f * (T - Told) / df;
      if (std::abs(Tnew - T) < NRtol) {
        NRconvg = true;
        break;
      } else {
        Told = T;
        T = Tnew;
      }
    } catch (const std::out_of_range&) {
      double Ta = Tmin, Tb = Tmax;
      for (int b = 0; b < 10000; ++b) {
        T = (Ta + Tb) / 2.0;
        hs = mix_enthalpy(m, T * T_ref, Ys) / E_ref;
        f = T - C1 - C2 * hs;
        if (std::abs(f) < Btol) {
          NRconvg = true;
          break;
        } else {
          if (f > 0) Ta = T;
          else Tb = T;
        }
      }
      if (NRconvg) break;
      throw std::runtime_error("Convergence not achieved for bisection method after catching out of range");
    }
  }
  if (NRconvg) {
    V[T_] = T;
  } else {
    Bconvg = false;
    double Ta = Tmin, Tb = Tmax;
    for (int b = 0; b < maxBIter; ++b) {
      T = (Ta + Tb) / 2.0;
      hs = mix_enthalpy(m, T * T_ref, Ys) / E_ref;
      f = T - C1 - C2 * hs;
      if (std::abs(f) < Btol) {
        V[T_] = T;
        Bconvg = true;
        break;
      } else {
        if (f > 0) Ta = T;
        else Tb = T;
      }
    }
    if (!Bconvg) throw std::runtime_error("Convergence not achieved for bisection method");
  }
  if (prm[10] > 0 && prm[11] != 0) V[T_] = std::min(std::max(V[T_], 0.95 * old_temp), 1.05 * old_temp);
  if (V[T_] < Tmin) {
    V[T_] = Tmin;
    nonPhys = true;
  } else if (V[T_] > Tmax) {
    V[T_] = Tmax;
    nonPhys = true;
  }
  T = V[T_];
  V[P_] = rho * Rgas * T;
  if (V[P_] < EPS) {
    V[P_] = EPS;
    nonPhys = true;
  }
  const double dim_temp = T * T_ref;
  double Cp = 0.0;  // ComputeFrozenSoundSpeed(T, ys, P, rho) :432-436 via ComputeFrozenGamma :398-403
  for (int s = 0; s < ns; ++s) Cp += (Ys[s] < 0.0 ? 1.0e-30 : Ys[s]) * (spline(m, P_CP, s, dim_temp) / m.mm[s]);
  const double Rg = mix_rgas(m, Ys);
  const double gamma = Cp / (Cp - Rg);
  V[A_] = std::sqrt(gamma * V[P_] / rho);
  if (V[A_] < EPS) {
    V[A_] = EPS;
    nonPhys = true;
  }
  V[H_] = (U[RHOE_S] + V[P_]) / rho;
  return nonPhys;
}
}  // namespace

// prm: [0..9] TEMPERATURE_MIN / MAX and the reference values, [10] ExtIter, [11] CLIPPING_TEMPRATURE, [12..16] ignition
int orc_set_primitive(void* h, int nDim, int64_t N, double* U, double* V, const double* Uold, const double* tke,
                      const double* mut, const double* prm, double* dPdU, double* dTdU, double* mu, double* kappa,
                      double* Dij, double* eddy, double* cp_out, int8_t* fail) {
  const Mech& m = *static_cast<Mech*>(h);
  const int ns = m.ns, nVar = ns + nDim + 2, nPV = ns + nDim + 5;
  const int T_ = 0, VX = 1, P_ = nDim + 1, RHO = nDim + 2, A_ = nDim + 4, RHOS = nDim + 5;
  const double T_ref = prm[2], E_ref = prm[3], R_ref = prm[4], P_ref = prm[5], Visc_ref = prm[6],
               Cond_ref = prm[7], Vel_ref = prm[8], Len_ref = prm[9];
  int64_t count = 0;
  int err = 0;
#pragma omp parallel for schedule(dynamic, 512) reduction(+ : count) reduction(| : err)
  for (int64_t i = 0; i < N; ++i) {
    try {
      double* u = U + i * nVar;
      double* v = V + i * nPV;
      const double ke = tke ? tke[i] : 0.0;
      const double vT0 = v[T_];
      bool nonPhys = cons2prim(m, nDim, u, v, ke, prm);
      if (nonPhys && prm[10] > 0 && Uold) {  // SetPrimVar :297-301: back to Solution_Old
        for (int q = 0; q < nVar; ++q) u[q] = Uold[i * nVar + q];
        (void)vT0;
        const bool np_old = cons2prim(m, nDim, u, v, ke, prm);
        if (np_old) {
          err = 1;
          if (fail) fail[i] = 1;
        }
      }
      // Cp = ComputeCP_FromSoundSpeed(T, a, Ys) / R_ref (:304-311)
      const double dim_temp = v[T_] * T_ref, dim_a = v[A_] * Vel_ref;
      double Ys[32];
      for (int s = 0; s < ns; ++s) Ys[s] = v[RHOS + s];
      const double Rg = mix_rgas(m, Ys);
      const double Cp = (dim_a * dim_a * Rg) / (dim_a * dim_a - Rg * dim_temp) / R_ref;
      if (cp_out) cp_out[i] = Cp;
      // CalcdTdU (:786-823)
      const double rhov = v[RHO], T = v[T_];
      const double dim_cp = Cp * R_ref;
      const double Cv = (dim_cp - mix_rgas(m, Ys)) / R_ref;
      const double rhoCv = rhov * Cv;
      double sq = 0.0;
      for (int d = 0; d < nDim; ++d) sq += v[VX + d] * v[VX + d];
      double dTdYs[32];
      for (int s = 0; s < ns; ++s) dTdYs[s] = (spline(m, P_H, s, dim_temp) / m.mm[s] - m.ri[s] * dim_temp) / E_ref;
      double* dt = dTdU + i * nVar;
      dt[0] = 0.5 * sq / rhoCv;
      for (int d = 0; d < nDim; ++d) dt[1 + d] = -v[VX + d] / rhoCv;
      dt[nDim + 1] = 1.0 / rhoCv;
      for (int s = 0; s < ns; ++s) dt[nDim + 2 + s] = -dTdYs[s] / rhoCv;
      // CalcdPdU (:829-853)
      const double Gamma = dim_cp / (dim_cp - mix_rgas(m, Ys));
      double* dp = dPdU + i * nVar;
      dp[0] = (Gamma - 1.0) * 0.5 * sq;
      for (int d = 0; d < nDim; ++d) dp[1 + d] = (1.0 - Gamma) * v[VX + d];
      dp[nDim + 1] = Gamma - 1.0;
      for (int s = 0; s < ns; ++s) dp[nDim + 2 + s] = m.ri[s] / R_ref * T - (Gamma - 1.0) * dTdYs[s];
      // CReactiveNSVariable::SetPrimVar transport (:1188-1228)
      eddy[i] = mut ? mut[i] : 0.0;
      const double dim_press = v[P_] * P_ref / 101325.0;
      double visc[32], cond[32], yom[32];
      for (int s = 0; s < ns; ++s) {
        visc[s] = spline(m, P_MU, s, dim_temp);
        cond[s] = spline(m, P_KAPPA, s, dim_temp);
      }
      // ComputeEta: clamped mass fractions
      for (int s = 0; s < ns; ++s) yom[s] = (Ys[s] < 0.0 ? 1.0e-30 : Ys[s]) / m.mm[s];
      double eta = 0.0;
      for (int a = 0; a < ns; ++a) {
        double phi = 0.0;
        for (int b = 0; b < ns; ++b)
          phi += yom[b] / std::sqrt(8.0 * (1.0 + m.mm[a] / m.mm[b])) *
                 (1.0 + std::sqrt(visc[a] / visc[b]) * std::pow(m.mm[b] / m.mm[a], 0.25)) *
                 (1.0 + std::sqrt(visc[a] / visc[b]) * std::pow(m.mm[b] / m.mm[a], 0.25));
        eta += visc[a] * yom[a] / phi;
      }
      mu[i] = eta / Visc_ref;
      // ComputeLambda: the argument (unclamped) mass fractions
      for (int s = 0; s < ns; ++s) yom[s] = Ys[s] / m.mm[s];
      double lam = 0.0;
      for (int a = 0; a < ns; ++a) {
        double phi = 0.0;
        for (int b = 0; b < ns; ++b)
          if (b != a)
            phi += 1.065 * yom[b] / std::sqrt(8.0 * (1.0 + m.mm[a] / m.mm[b])) *
                   (1.0 + std::sqrt(visc[a] / visc[b]) * std::pow(m.mm[b] / m.mm[a], 0.25)) *
                   (1.0 + std::sqrt(visc[a] / visc[b]) * std::pow(m.mm[b] / m.mm[a], 0.25));
        phi += yom[a];
        lam += cond[a] * yom[a] / phi;
      }
      kappa[i] = lam / Cond_ref;
      // GetDij_SM / (Vel_ref * Len_ref * 1e4), symmetric
      double* D = Dij + i * ns * ns;
      const double scale = Vel_ref * Len_ref * 1.0e4;
      for (int a = 0; a < ns; ++a) {
        const double mi = m.mm[a], dvi = std::cbrt(m.dv[a]);
        for (int b = a; b < ns; ++b) {
          const double Mij = std::sqrt((mi * m.mm[b]) / (mi + m.mm[b]));
          const double dvj = std::cbrt(m.dv[b]);
          const double d = 1.0e-3 * std::pow(dim_temp, 1.75) / (dim_press * Mij * (dvi + dvj) * (dvi + dvj));
          D[a * ns + b] = d / scale;
          D[b * ns + a] = d / scale;
        }
      }
      // ignition (SetPrimitive_Variables solver_direct_reactive.cpp:1013-1024): prm[12] IGNITION, [13] IGNITION_ITER,
      // [14] IGNITION_TEMPERATURE, [15] FUEL_INDEX, [16] OXIDIZER_INDEX; only the record's T is overwritten
      // (SetTemperature, variable_reactive.hpp:602-607), after the derivatives and transport above
      if (prm[12] != 0.0 && prm[10] < prm[13] && v[RHOS + (int)prm[15]] > 0.4 && v[RHOS + (int)prm[16]] > 0.2 &&
          v[T_] < prm[14])
        v[T_] = prm[14];
      if (nonPhys) ++count;
    } catch (const std::exception&) {
      err = 1;
      if (fail) fail[i] = 1;  // the points whose SetPrimVar throws (error-path parity with the device's index)
    }
  }
  return err ? -1 : (int)count;
}

// =================================================================================================
// a14 + next-2: Menter SST turbulence solver on the flow state (CTurbSSTSolver / CTurbSolver,
// SU2_CFD/src/solver_direct_turbulent.cpp; numerics SU2_CFD/src/numerics_direct_turbulent.cpp;
// node record CTurbSSTVariable SU2_CFD/src/variable_direct_turbulent.cpp). Turbulent solution
// T[N][2] = (k, omega); std::min/std::max are restated as the ternaries they are.
// =================================================================================================
struct SSTConst {
  double sk1, sk2, so1, so2, b1, b2, bs, a1, al1, al2;
};
// CTurbSSTSolver constructor, solver_direct_turbulent.cpp:2716-2725
static SSTConst sst_const() {
  SSTConst c;
  c.sk1 = 0.85;
  c.sk2 = 1.0;
  c.so1 = 0.5;
  c.so2 = 0.856;
  c.b1 = 0.075;
  c.b2 = 0.0828;
  c.bs = 0.09;
  c.a1 = 0.31;
  c.al1 = c.b1 / c.bs - c.so1 * 0.41 * 0.41 / std::sqrt(c.bs);
  c.al2 = c.b2 / c.bs - c.so2 * 0.41 * 0.41 / std::sqrt(c.bs);
  return c;
}
static inline double smin(double a, double b) { return (b < a) ? b : a; }  // std::min
static inline double smax(double a, double b) { return (a < b) ? b : a; }  // std::max

// CSolver::SetSolution_Gradient_LS (Common solver base, SU2_CFD/src/solver_structure.cpp:580-720)
// for an nVar-component solution: weight != 0 test, r11 >= 0 / r11 != 0 guards, |detR2| <= EPS.
void orc_sol_grad_ls(int nDim, int nVar, int64_t N, const double* coord, const double* sol, const int64_t* nptr,
                     const int64_t* nbr, double* grad) {
  double Cv[8][3];
#pragma omp parallel for schedule(static) private(Cv)
  for (int64_t i = 0; i < N; ++i) {
    bool singular = false;
    const double* ci = coord + i * nDim;
    const double* si = sol + i * nVar;
    for (int v = 0; v < nVar; ++v)
      for (int d = 0; d < nDim; ++d) Cv[v][d] = 0.0;
    double r11 = 0, r12 = 0, r13 = 0, r22 = 0, r23 = 0, r23_a = 0, r23_b = 0, r33 = 0;
    for (int64_t k = nptr[i]; k < nptr[i + 1]; ++k) {
      const int64_t j = nbr[k];
      const double* cj = coord + j * nDim;
      const double* sj = sol + j * nVar;
      double w = 0.0;
      for (int d = 0; d < nDim; ++d) w += (cj[d] - ci[d]) * (cj[d] - ci[d]);
      if (w != 0.0) {
        r11 += (cj[0] - ci[0]) * (cj[0] - ci[0]) / w;
        r12 += (cj[0] - ci[0]) * (cj[1] - ci[1]) / w;
        r22 += (cj[1] - ci[1]) * (cj[1] - ci[1]) / w;
        if (nDim == 3) {
          r13 += (cj[0] - ci[0]) * (cj[2] - ci[2]) / w;
          r23_a += (cj[1] - ci[1]) * (cj[2] - ci[2]) / w;
          r23_b += (cj[0] - ci[0]) * (cj[2] - ci[2]) / w;
          r33 += (cj[2] - ci[2]) * (cj[2] - ci[2]) / w;
        }
        for (int v = 0; v < nVar; ++v)
          for (int d = 0; d < nDim; ++d) Cv[v][d] += (cj[d] - ci[d]) * (sj[v] - si[v]) / w;
      }
    }
    if (r11 >= 0.0) r11 = std::sqrt(r11); else r11 = 0.0;
    if (r11 != 0.0) r12 = r12 / r11; else r12 = 0.0;
    if (r22 - r12 * r12 >= 0.0) r22 = std::sqrt(r22 - r12 * r12); else r22 = 0.0;
    if (nDim == 3) {
      if (r11 != 0.0) r13 = r13 / r11; else r13 = 0.0;
      if ((r22 != 0.0) && (r11 * r22 != 0.0)) r23 = r23_a / r22 - r23_b * r12 / (r11 * r22); else r23 = 0.0;
      if (r33 - r23 * r23 - r13 * r13 >= 0.0) r33 = std::sqrt(r33 - r23 * r23 - r13 * r13); else r33 = 0.0;
    }
    double detR2 = (nDim == 2) ? (r11 * r22) * (r11 * r22) : (r11 * r22 * r33) * (r11 * r22 * r33);
    if (std::fabs(detR2) <= EPS) {
      detR2 = 1.0;
      singular = true;
    }
    double S[3][3] = {{0}};
    if (!singular) {
      if (nDim == 2) {
        S[0][0] = (r12 * r12 + r22 * r22) / detR2;
        S[0][1] = -r11 * r12 / detR2;
        S[1][0] = S[0][1];
        S[1][1] = r11 * r11 / detR2;
      } else {
        const double z11 = r22 * r33, z12 = -r12 * r33, z13 = r12 * r23 - r13 * r22;
        const double z22 = r11 * r33, z23 = -r11 * r23, z33 = r11 * r22;
        S[0][0] = (z11 * z11 + z12 * z12 + z13 * z13) / detR2;
        S[0][1] = (z12 * z22 + z13 * z23) / detR2;
        S[0][2] = (z13 * z33) / detR2;
        S[1][0] = S[0][1];
        S[1][1] = (z22 * z22 + z23 * z23) / detR2;
        S[1][2] = (z23 * z33) / detR2;
        S[2][0] = S[0][2];
        S[2][1] = S[1][2];
        S[2][2] = (z33 * z33) / detR2;
      }
    }
    for (int v = 0; v < nVar; ++v)
      for (int d = 0; d < nDim; ++d) {
        double product = 0.0;
        for (int e = 0; e < nDim; ++e) product += S[d][e] * Cv[v][e];
        grad[(i * nVar + v) * nDim + d] = product;
      }
  }
}

// CReactiveNSVariable::SetStrainMag (variable_direct_reactive.cpp:1060-1095) from the flow primitive
// gradient G[N][nG][nDim] (rows 1..nDim = velocity).
void orc_strain_mag(int nDim, int nG, int64_t N, const double* G, double* out) {
  for (int64_t i = 0; i < N; ++i) {
    const double* g = G + i * nG * nDim;
    auto gr = [&](int v, int d) { return g[v * nDim + d]; };
    double Div = 0.0;
    for (int d = 0; d < nDim; ++d) Div += gr(d + 1, d);
    double S = 0.0;
    for (int d = 0; d < nDim; ++d) S += std::pow(gr(d + 1, d) - 1.0 / 3.0 * Div, 2.0);
    S += 2.0 * std::pow(0.5 * (gr(1, 1) + gr(2, 0)), 2.0);
    if (nDim == 3) {
      S += 2.0 * std::pow(0.5 * (gr(1, 2) + gr(3, 0)), 2.0);
      S += 2.0 * std::pow(0.5 * (gr(2, 2) + gr(3, 1)), 2.0);
    }
    out[i] = std::sqrt(2.0 * S);
  }
}

// CTurbSSTSolver::Postprocessing (solver_direct_turbulent.cpp:2953-3000) after its gradient:
// CTurbSSTVariable::SetBlendingFunc (variable_direct_turbulent.cpp:178-203) and mu_t.
// rho, mu: flow density V[nDim+2] and laminar viscosity; strain: flow StrainMag.
void orc_sst_blending(int nDim, int64_t N, const double* T, const double* TG, const double* rho, const double* mu,
                      const double* dist, const double* strain, double* F1, double* F2, double* CDkw, double* muT) {
  const SSTConst c = sst_const();
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; ++i) {
    const double* t = T + 2 * i;
    const double* g = TG + i * 2 * nDim;
    double cd = 0.0;
    for (int d = 0; d < nDim; ++d) cd += g[d] * g[nDim + d];
    cd *= 2.0 * rho[i] * c.so2 / t[1];
    cd = smax(cd, std::pow(10.0, -20.0));
    const double arg2A = std::sqrt(t[0]) / (c.bs * t[1] * dist[i] + EPS * EPS);
    const double arg2B = 500.0 * mu[i] / (rho[i] * dist[i] * dist[i] * t[1] + EPS * EPS);
    double arg2 = smax(arg2A, arg2B);
    const double arg1 = smin(arg2, 4.0 * rho[i] * c.so2 * t[0] / (cd * dist[i] * dist[i] + EPS * EPS));
    F1[i] = std::tanh(std::pow(arg1, 4.0));
    arg2 = smax(2.0 * arg2A, arg2B);
    F2[i] = std::tanh(std::pow(arg2, 2.0));
    CDkw[i] = cd;
    const double zeta = smin(1.0 / t[1], c.a1 / (strain[i] * F2[i]));
    muT[i] = smin(smax(rho[i] * t[0] * zeta, 0.0), 1.0);
  }
}

// CUpwSca_TurbSST::ComputeResidual (numerics_direct_turbulent.cpp:865-922), 1st order, fixed grid.
void orc_sst_upwind(int nDim, int nPV, int64_t E, const int64_t* edges, const double* normal, const double* V,
                    const double* T, double* res, double* Ji, double* Jj) {
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    const double* vi = V + i * nPV;
    const double* vj = V + j * nPV;
    const double* n = normal + e * nDim;
    double q = 0.0;
    for (int d = 0; d < nDim; ++d) q += 0.5 * (vi[d + 1] + vj[d + 1]) * n[d];
    const double a0 = 0.5 * (q + std::fabs(q)), a1 = 0.5 * (q - std::fabs(q));
    const double ri = vi[nDim + 2], rj = vj[nDim + 2];
    res[2 * e] = a0 * ri * T[2 * i] + a1 * rj * T[2 * j];
    res[2 * e + 1] = a0 * ri * T[2 * i + 1] + a1 * rj * T[2 * j + 1];
    if (Ji) {
      double* A = Ji + 4 * e;
      double* B = Jj + 4 * e;
      A[0] = a0; A[1] = 0.0; A[2] = 0.0; A[3] = a0;
      B[0] = a1; B[1] = 0.0; B[2] = 0.0; B[3] = a1;
    }
  }
}

// CSolver::SetSolution_Limiter (solver_structure.cpp:951-1204) on the SST solution (k, omega), called by
// CTurbSSTSolver::Preprocessing when SPATIAL_ORDER_TURB = 2ND_ORDER_LIMITER (solver_direct_turbulent.cpp:2945-2947):
// Solution_Max / _Min from -EPS / EPS over the edges (du = U_j - U_i at i, -du at j), the limiter 2.0 at every
// domain point, then SLOPE_LIMITER_TURB = VENKATAKRISHNAN (kind 0) takes the edge minimum of
// (dp^2 + 2 dp dm + eps2) / (dp^2 + dp dm + 2 dm^2 + eps2), eps2 = (LIMITER_COEFF * REF_ELEM_LENGTH)^3; the function has
// no branch for BARTH_JESPERSEN (kind 1), which leaves 2.0.
void orc_sst_limiter(int nDim, int64_t N, int64_t E, const int64_t* edges, const double* coord, const double* T,
                     const double* TG, double ref_len, double lim_coeff, int kind, double* lim) {
  std::vector<double> mx(N * 2, -EPS), mn(N * 2, EPS);
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    for (int v = 0; v < 2; ++v) {
      const double du = T[2 * j + v] - T[2 * i + v];
      mn[2 * i + v] = std::min(mn[2 * i + v], du);
      mx[2 * i + v] = std::max(mx[2 * i + v], du);
      mn[2 * j + v] = std::min(mn[2 * j + v], -du);
      mx[2 * j + v] = std::max(mx[2 * j + v], -du);
    }
  }
  for (int64_t q = 0; q < N * 2; ++q) lim[q] = 2.0;
  if (kind != 0) return;
  const double eps1 = lim_coeff * ref_len;
  const double eps2 = eps1 * eps1 * eps1;
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    const double* Gi = TG + i * 2 * nDim;
    const double* Gj = TG + j * 2 * nDim;
    const double* ci = coord + i * nDim;
    const double* cj = coord + j * nDim;
    for (int v = 0; v < 2; ++v) {
      double dm = 0.0;
      for (int d = 0; d < nDim; ++d) dm += 0.5 * (cj[d] - ci[d]) * Gi[v * nDim + d];
      double dp = (dm > 0.0) ? mx[2 * i + v] : mn[2 * i + v];
      double lv = (dp * dp + 2.0 * dp * dm + eps2) / (dp * dp + dp * dm + 2.0 * dm * dm + eps2);
      if (lv < lim[2 * i + v]) lim[2 * i + v] = lv;
      dm = 0.0;
      for (int d = 0; d < nDim; ++d) dm += 0.5 * (ci[d] - cj[d]) * Gj[v * nDim + d];
      dp = (dm > 0.0) ? mx[2 * j + v] : mn[2 * j + v];
      lv = (dp * dp + 2.0 * dp * dm + eps2) / (dp * dp + dp * dm + 2.0 * dm * dm + eps2);
      if (lv < lim[2 * j + v]) lim[2 * j + v] = lv;
    }
  }
}

// CTurbSolver::Upwind_Residual's second-order branch (solver_direct_turbulent.cpp:464-510) + CUpwSca_TurbSST, fixed
// grid. order 1 = SPATIAL_ORDER_TURB 2ND_ORDER, 2 = 2ND_ORDER_LIMITER. Vector_i = (x_j - x_i) / 2, Vector_j = (x_i -
// x_j) / 2 (computed as 0.5 * difference). The flow record is reconstructed entry by entry for iVar <
// nPrimVarGrad as FlowPrimVar[iVar] = V[iVar] (+ Limiter_Primitive[iVar] *) sum_d Vector[d] Gradient_Primitive[iVar][d],
// i.e. with the gradient ROW iVar of (T, u, v(, w), P, X_s) against the primitive ENTRY iVar of (T, u, v(, w), P, rho,
// h, a, Y_s): the velocity entries the scalar upwind reads match their rows, its density entry V[nDim+2] is moved
// along the gradient of X_0 (reproduced). With the limiter the flow's Limiter_Primitive (nDim+2 entries: T, u, v(, w),
// P) is read at iVar = nDim+2, one past its end — undefined in the reference; restated as 0.0 (the density is not
// moved), which the flat-plate golden fpit2l pins (tests/test_oracle_bc.py). Lf: the flow limiter [N][nDim+2] or null
// (order 1). The turbulent solution: T (+ TL *) sum_d Vector[d] TG[v][d].
void orc_sst_upwind2(int nDim, int nPV, int nG, int64_t E, const int64_t* edges, const double* normal,
                     const double* coord, const double* V, const double* G, const double* Lf, const double* T,
                     const double* TG, const double* TL, int order, double* res, double* Ji, double* Jj) {
  const bool lim = order == 2;
  const int nL = nDim + 2;
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    double vec_i[3], vec_j[3];
    for (int d = 0; d < nDim; ++d) {
      vec_i[d] = 0.5 * (coord[j * nDim + d] - coord[i * nDim + d]);
      vec_j[d] = 0.5 * (coord[i * nDim + d] - coord[j * nDim + d]);
    }
    auto flow = [&](int64_t p, const double* vec, int v) {  // FlowPrimVar entry v (v = 1..nDim, nDim + 2)
      double pg = 0.0;
      for (int d = 0; d < nDim; ++d) pg += vec[d] * G[(p * nG + v) * nDim + d];
      if (!lim) return V[p * nPV + v] + pg;
      const double l = v < nL ? Lf[p * nL + v] : 0.0;  // v = nDim + 2: past the limiter's end (see above)
      return V[p * nPV + v] + l * pg;
    };
    auto turb = [&](int64_t p, const double* vec, int v) {
      double pg = 0.0;
      for (int d = 0; d < nDim; ++d) pg += vec[d] * TG[(p * 2 + v) * nDim + d];
      return lim ? T[2 * p + v] + TL[2 * p + v] * pg : T[2 * p + v] + pg;
    };
    const double* n = normal + e * nDim;
    double q = 0.0;
    for (int d = 0; d < nDim; ++d) q += 0.5 * (flow(i, vec_i, d + 1) + flow(j, vec_j, d + 1)) * n[d];
    const double a0 = 0.5 * (q + std::fabs(q)), a1 = 0.5 * (q - std::fabs(q));
    const double ri = flow(i, vec_i, nDim + 2), rj = flow(j, vec_j, nDim + 2);
    res[2 * e] = a0 * ri * turb(i, vec_i, 0) + a1 * rj * turb(j, vec_j, 0);
    res[2 * e + 1] = a0 * ri * turb(i, vec_i, 1) + a1 * rj * turb(j, vec_j, 1);
    if (Ji) {
      double* A = Ji + 4 * e;
      double* B = Jj + 4 * e;
      A[0] = a0; A[1] = 0.0; A[2] = 0.0; A[3] = a0;
      B[0] = a1; B[1] = 0.0; B[2] = 0.0; B[3] = a1;
    }
  }
}

// CAvgGradCorrected_TurbSST::ComputeResidual (numerics_direct_turbulent.cpp:1080-1163) with the
// setters of CTurbSolver::Viscous_Residual (solver_direct_turbulent.cpp:545-600): laminar and
// eddy viscosity of the flow nodes, F1 of the turbulent nodes.
void orc_sst_visc(int nDim, int nPV, int64_t E, const int64_t* edges, const double* normal, const double* coord,
                  const double* V, const double* T, const double* TG, const double* F1, const double* mu,
                  const double* eddy, double* res, double* Ji, double* Jj) {
  const SSTConst c = sst_const();
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < E; ++e) {
    const int64_t i = edges[2 * e], j = edges[2 * e + 1];
    const double* n = normal + e * nDim;
    const double ri = V[i * nPV + nDim + 2], rj = V[j * nPV + nDim + 2];
    const double ski = F1[i] * c.sk1 + (1.0 - F1[i]) * c.sk2;
    const double skj = F1[j] * c.sk1 + (1.0 - F1[j]) * c.sk2;
    const double soi = F1[i] * c.so1 + (1.0 - F1[i]) * c.so2;
    const double soj = F1[j] * c.so1 + (1.0 - F1[j]) * c.so2;
    const double dik = mu[i] + ski * eddy[i], djk = mu[j] + skj * eddy[j];
    const double dio = mu[i] + soi * eddy[i], djo = mu[j] + soj * eddy[j];
    const double dk = 0.5 * (dik + djk), dw = 0.5 * (dio + djo);
    double ev[3], dist2 = 0.0, proj = 0.0;
    for (int d = 0; d < nDim; ++d) {
      ev[d] = coord[j * nDim + d] - coord[i * nDim + d];
      dist2 += ev[d] * ev[d];
      proj += ev[d] * n[d];
    }
    if (dist2 == 0.0) proj = 0.0; else proj = proj / dist2;
    double corr[2];
    for (int v = 0; v < 2; ++v) {
      double pn = 0.0, pe = 0.0;
      for (int d = 0; d < nDim; ++d) {
        const double m = 0.5 * (TG[(i * 2 + v) * nDim + d] + TG[(j * 2 + v) * nDim + d]);
        pn += m * n[d];
        pe += m * ev[d];
      }
      corr[v] = pn;
      corr[v] -= pe * proj - (T[2 * j + v] - T[2 * i + v]) * proj;
    }
    res[2 * e] = dk * corr[0];
    res[2 * e + 1] = dw * corr[1];
    if (Ji) {
      double* A = Ji + 4 * e;
      double* B = Jj + 4 * e;
      A[0] = -dk * proj / ri; A[1] = 0.0; A[2] = 0.0; A[3] = -dw * proj / ri;
      B[0] = dk * proj / rj; B[1] = 0.0; B[2] = 0.0; B[3] = dw * proj / rj;
    }
  }
}

// CSourcePieceWise_TurbSST::ComputeResidual (numerics_direct_turbulent.cpp:1183-1256) with the setters
// of CTurbSSTSolver::Source_Residual (solver_direct_turbulent.cpp:3018-3080).
// G: flow primitive gradient [N][nG][nDim].
void orc_sst_source(int nDim, int nPV, int nG, int64_t N, const double* V, const double* G, const double* T,
                    const double* vol, const double* dist, const double* F1, const double* F2, const double* CDkw,
                    const double* strain, const double* eddy, double* res, double* J) {
  const SSTConst c = sst_const();
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; ++i) {
    double* r = res + 2 * i;
    double* A = J ? J + 4 * i : nullptr;
    r[0] = 0.0;
    r[1] = 0.0;
    if (A) A[0] = A[1] = A[2] = A[3] = 0.0;
    const double rho = V[i * nPV + nDim + 2];
    const double k = T[2 * i], w = T[2 * i + 1], S = strain[i], Vol = vol[i];
    const double ab = F1[i] * c.al1 + (1.0 - F1[i]) * c.al2;
    const double bb = F1[i] * c.b1 + (1.0 - F1[i]) * c.b2;
    if (dist[i] > 1e-10) {
      double diverg = 0.0;
      for (int d = 0; d < nDim; ++d) diverg += G[(i * nG + d + 1) * nDim + d];
      double pk = eddy[i] * S * S - 2.0 / 3.0 * rho * k * diverg;
      pk = smin(pk, 20.0 * c.bs * rho * w * k);
      pk = smax(pk, 0.0);
      const double zeta = smax(w, S * F2[i] / c.a1);
      double pw = S * S - 2.0 / 3.0 * zeta * diverg;
      pw = smax(pw, 0.0);
      r[0] += pk * Vol;
      r[1] += ab * rho * pw * Vol;
      r[0] -= c.bs * rho * w * k * Vol;
      r[1] -= bb * rho * w * w * Vol;
      r[1] += (1.0 - F1[i]) * CDkw[i] * Vol;
      if (A) {
        A[0] = -c.bs * w * Vol;
        A[3] = -2.0 * bb * w * Vol;
      }
    }
  }
}

// SST residual / Jacobian assembly in the reference's loop order: CTurbSolver::Upwind_Residual
// (solver_direct_turbulent.cpp:525-538: R_i += F, R_j -= F; A_ii += Ji, A_ij += Jj, A_ji -= Ji, A_jj -= Jj),
// Viscous_Residual (:587-595, opposite signs), CTurbSSTSolver::Source_Residual (:3074-3075: R_i -= S,
// A_ii -= Js); then CTurbSolver::ImplicitEuler_Iteration (:630-655): A_ii += Vol/(CFLRedCoeff_Turb*dt),
// rhs = -R. Jacobian pointers may be null (residual only).
void orc_sst_assemble(int64_t N, int64_t E, const int64_t* edges, const int64_t* rp, const int64_t* col,
                      const double* Fu, const double* Jui, const double* Juj, const double* Fv, const double* Jvi,
                      const double* Jvj, const double* Rs, const double* Js, const double* vol, const double* dt,
                      double cfl_red, double* R, double* A, double* rhs) {
  std::fill(R, R + N * 2, 0.0);
  if (A) std::fill(A, A + rp[N] * 4, 0.0);
  auto add = [&](int64_t b, const double* J, bool plus) {
    double* d = A + b * 4;
    for (int q = 0; q < 4; ++q) {
      if (plus) d[q] += J[q]; else d[q] -= J[q];
    }
  };
  for (int pass = 0; pass < 2; ++pass) {
    const double* F = pass ? Fv : Fu;
    const double* Ji = pass ? Jvi : Jui;
    const double* Jj = pass ? Jvj : Juj;
    if (!F) continue;
    const bool up = pass == 0;
    for (int64_t e = 0; e < E; ++e) {
      const int64_t i = edges[2 * e], j = edges[2 * e + 1];
      for (int v = 0; v < 2; ++v) {
        if (up) {
          R[i * 2 + v] += F[e * 2 + v];
          R[j * 2 + v] -= F[e * 2 + v];
        } else {
          R[i * 2 + v] -= F[e * 2 + v];
          R[j * 2 + v] += F[e * 2 + v];
        }
      }
      if (A && Ji) {
        add(blk_of(rp, col, i, i), Ji + e * 4, up);
        add(blk_of(rp, col, i, j), Jj + e * 4, up);
        add(blk_of(rp, col, j, i), Ji + e * 4, !up);
        add(blk_of(rp, col, j, j), Jj + e * 4, !up);
      }
    }
  }
  if (Rs)
    for (int64_t i = 0; i < N; ++i) {
      for (int v = 0; v < 2; ++v) R[i * 2 + v] -= Rs[i * 2 + v];
      if (A && Js) add(blk_of(rp, col, i, i), Js + i * 4, false);
    }
  if (!A) return;
  for (int64_t i = 0; i < N; ++i) {
    double* D = A + blk_of(rp, col, i, i) * 4;
    const double delta = vol[i] / (cfl_red * dt[i]);
    D[0] += delta;
    D[3] += delta;
    for (int v = 0; v < 2; ++v) rhs[i * 2 + v] = -R[i * 2 + v];
  }
}

// CTurbSolver::ImplicitEuler_Iteration SST branch (solver_direct_turbulent.cpp:698-713) through
// CVariable::AddConservativeSolution (variable_structure.cpp:214-219): limits from the CTurbSSTSolver
// constructor (solver_direct_turbulent.cpp:2731-2735). rho_old = rho (Cons2PrimVar sets V[rho] = U[rho],
// variable_direct_reactive.cpp:579-584, and the flow's Solution_Old is the U the primitives came from).
void orc_sst_update(int64_t N, const double* x, double relax, const double* rho, const double* rho_old, double* T) {
  const double lo[2] = {1.0e-10, 1.0e-4}, hi[2] = {1.0e10, 1.0e15};
  for (int64_t i = 0; i < N; ++i)
    for (int v = 0; v < 2; ++v)
      T[2 * i + v] = smin(smax((T[2 * i + v] * rho_old[i] + relax * x[2 * i + v]) / rho[i], lo[v]), hi[v]);
}

}  // extern "C"

// =================================================================================================
// next-3 + a8: boundary conditions of one Space_Integration (integration_structure.cpp:95-193): the weak
// BCs in marker order, then the strong ones.
//   flow  CReactiveEulerSolver::BC_Inlet    SU2_CFD/src/solver_direct_reactive.cpp:3226-3674
//         CReactiveEulerSolver::BC_Outlet   :3808-4123
//         CReactiveNSSolver::BC_Isothermal_Wall :5393-5711 (no grid motion)
//         boundary viscous numerics CAvgGradReactive_Boundary::ComputeResidual numerics_direct_reactive.cpp:478-648
//   SST   CTurbSSTSolver::BC_Inlet / BC_Outlet / BC_Isothermal_Wall solver_direct_turbulent.cpp:3142-3450
// Library calls restated: ComputeDensity / ComputeTemperature / ComputeRgas (SetRgas on the clamped mass
// fractions), ComputeEnthalpy, ComputeFrozenGamma / ComputeFrozenSoundSpeed, ComputeCV, ComputePartialEnergy,
// ComputedP_dYs, ComputeCps (reacting_model_library.cpp:26-41, 398-470, 519-619, reacting_model_library.hpp:368).
// =================================================================================================
namespace {

struct BCPrm {
  int kind_inlet;             // TOTAL_CONDITIONS / MASS_FLOW / TEMPERATURE_IMPOSE
  double tke_inf, kine_inf, omega_inf, beta1;
  double P_ref, vel_ref, T_ref, E_ref, R_ref, rho_ref;
  int k_inlet, k_outlet, k_iso, k_hf, k_total, k_massflow, k_timpose;  // the reference's enum values
  double mach_inf, Pr_t, Le_t;
  int k_euler;                // EULER_WALL (option_structure.hpp:750)
  int k_sup_in, k_sup_out;    // SUPERSONIC_INLET / SUPERSONIC_OUTLET (-999: not in the dump)
  int implicit, rans;
};

double mix_cp(const Mech& m, double T, const double* Ys) {  // ComputeCP :612-619
  double c = 0.0;
  for (int s = 0; s < m.ns; ++s) c += (Ys[s] < 0.0 ? 1.0e-30 : Ys[s]) * (spline(m, P_CP, s, T) / m.mm[s]);
  return c;
}
double frozen_gamma(const Mech& m, double T, const double* Ys) {  // ComputeFrozenGamma :398-403
  const double Cp = mix_cp(m, T, Ys);
  const double Cv = Cp - mix_rgas(m, Ys);
  return Cp / Cv;
}
double partial_energy(const Mech& m, double T, int s) {  // ComputePartialEnergy(T, s) :583-588
  return spline(m, P_H, s, T) / m.mm[s] - m.ri[s] * T;
}

// Secondary (dP/dU) of a ghost state (BC_Inlet :3510-3533 / BC_Outlet :3941-3962)
void ghost_dpdu(const Mech& m, int nDim, const double* Vg, double Gamma, double vel2, const BCPrm& P, double* S) {
  const int ns = m.ns;
  S[0] = (Gamma - 1.0) * 0.5 * vel2;
  for (int d = 0; d < nDim; ++d) S[1 + d] = (1.0 - Gamma) * Vg[1 + d];
  S[nDim + 1] = Gamma - 1.0;
  const double dim_temp = Vg[0] * P.T_ref;
  for (int s = 0; s < ns; ++s) S[nDim + 2 + s] = (m.ri[s] * dim_temp - (Gamma - 1.0) * partial_energy(m, dim_temp, s)) / P.E_ref;
}
// Secondary (dT/dU) of a ghost state for the boundary viscous numerics (:3573-3595 / :4021-4044)
void ghost_dtdu(const Mech& m, int nDim, const double* Vg, const double* Ys, const BCPrm& P, double* S) {
  const int ns = m.ns;
  const double dim_temp = Vg[0] * P.T_ref;
  const double Cv = (mix_cp(m, dim_temp, Ys) - mix_rgas(m, Ys)) / P.R_ref;
  const double rhoCv = Vg[nDim + 2] * Cv;
  double sq_vel = 0.0;
  for (int d = 0; d < nDim; ++d) sq_vel += Vg[1 + d] * Vg[1 + d];
  S[0] = 0.5 * sq_vel / rhoCv;
  for (int d = 0; d < nDim; ++d) S[1 + d] = -Vg[1 + d] / rhoCv;
  S[nDim + 1] = 1.0 / rhoCv;
  for (int s = 0; s < ns; ++s) S[nDim + 2 + s] = -partial_energy(m, dim_temp, s) / (P.E_ref * rhoCv);
}

struct BCField {
  const double *coord, *U, *V, *dPdU, *dTdU, *G, *mu, *kappa, *Dij, *tke, *mut, *sigk, *gk, *eddy;
  const int64_t *rp, *col;
  double *R, *A, *Uold;
};

// The weak flow BC of one vertex: ghost state, then R += Fc, A_ii += Jc_i, R -= Fv, A_ii -= Jv_i.
void flow_weak_vertex(const Mech& m, int nDim, const BCPrm& P, int kind, const double* md, int64_t i, int64_t pn,
                      const double* bn, BCField& f, double* Vg) {
  const int ns = m.ns, nVar = ns + nDim + 2, nPV = ns + nDim + 5, nG = ns + nDim + 2;
  const int T_ = 0, VX = 1, P_ = nDim + 1, RHO = nDim + 2, H_ = nDim + 3, A_ = nDim + 4, RHOS = nDim + 5;
  double Normal[3], UnitNormal[3];
  double Area = 0.0;
  for (int d = 0; d < nDim; ++d) Area += bn[d] * bn[d];
  Area = std::sqrt(Area);
  for (int d = 0; d < nDim; ++d) {
    Normal[d] = -bn[d];
    UnitNormal[d] = Normal[d] / Area;
  }
  const double* Vd = f.V + i * nPV;
  const double* Sd = f.dPdU + i * nVar;
  double Sc[32], Sv[32], Ys[32];
  bool sup = false;  // supersonic outlet: the node's own secondaries
  if (kind == P.k_sup_in) {
    // CReactiveEulerSolver::BC_Supersonic_Inlet (:3014-3055): the marker's T, P, velocity and the inlet mass fractions;
    // ComputeDensity (P / (T Rgas), :457-460), ComputeEnthalpy and ComputeFrozenSoundSpeed (sqrt(gamma Rgas T),
    // :408-411) at the dimensional temperature, then non-dimensionalised. The reference divides the CONFIG's velocity
    // array by Velocity_Ref in place on every call (:3023, :3045-3046); restated once (identical for dimensional runs)
    for (int s = 0; s < ns; ++s) Ys[s] = md[6 + s];
    const double Temperature = md[1], Pressure = md[2];
    const double Rgas = mix_rgas(m, Ys);
    const double Density = Pressure / (Temperature * Rgas);
    const double Enthalpy = mix_enthalpy(m, Temperature, Ys);
    const double SoundSpeed = std::sqrt(frozen_gamma(m, Temperature, Ys) * Rgas * Temperature);
    double Velocity2 = 0.0;
    for (int d = 0; d < nDim; ++d) {
      Vg[VX + d] = md[3 + d] / P.vel_ref;
      Velocity2 += Vg[VX + d] * Vg[VX + d];
    }
    Vg[T_] = Temperature / P.T_ref;
    Vg[P_] = Pressure / P.P_ref;
    Vg[RHO] = Density / P.rho_ref;
    Vg[H_] = Enthalpy / P.E_ref + 0.5 * Velocity2;
    Vg[A_] = SoundSpeed / P.vel_ref;
    for (int s = 0; s < ns; ++s) Vg[RHOS + s] = Ys[s];
    // the ghost's dP/dU (:3080-3102) enters only Jacobian_j, which the BC discards: the domain's stands in
    for (int v = 0; v < nVar; ++v) Sc[v] = Sd[v];
  } else if (kind == P.k_sup_out) {
    // CReactiveEulerSolver::BC_Supersonic_Outlet (:3708-3717, :3753-3755): ghost = domain state, the node's own
    // secondaries (as the subsonic outlet's supersonic exit)
    for (int v = 0; v < nPV; ++v) Vg[v] = Vd[v];
    sup = true;
  } else if (kind == P.k_inlet) {
    for (int s = 0; s < ns; ++s) Ys[s] = md[6 + s];
    const double* dir = md + 3;
    double Gamma = Sd[nDim + 1] + 1.0, vel_mag = 0.0;
    if (P.kind_inlet == P.k_timpose) {
      const double T = md[1] / P.T_ref;
      vel_mag = md[2] / P.vel_ref;
      Vg[T_] = T;
      for (int d = 0; d < nDim; ++d) Vg[VX + d] = vel_mag * dir[d];
      Vg[P_] = Vd[P_];
      Vg[RHO] = Vg[P_] / (T * mix_rgas(m, Ys)) * P.R_ref;
      const double dim_temp = T * P.T_ref;
      Vg[H_] = mix_enthalpy(m, dim_temp, Ys) / P.E_ref + (P.rans ? 1.0 : 0.0) * P.tke_inf;
      Vg[H_] += 0.5 * vel_mag * vel_mag;
      Vg[A_] = std::sqrt(frozen_gamma(m, dim_temp, Ys) * mix_rgas(m, Ys) * dim_temp) / P.vel_ref;
      // Gamma is left uninitialised by the reference in this branch (:3236, :3515); it only enters the
      // ghost's dP/dU, i.e. Jacobian_j, which the BC discards. The domain value stands in.
    } else if (P.kind_inlet == P.k_massflow) {
      const double Density = md[1] / P.rho_ref;
      vel_mag = md[2] / P.vel_ref;
      double SoundSpeed = Vd[A_];
      const double GM1 = Gamma - 1.0;
      double Vn = 0.0;
      for (int d = 0; d < nDim; ++d) Vn += Vd[VX + d] * UnitNormal[d];
      const double Riemann = Vn + 2.0 * SoundSpeed / GM1;
      double alpha = 0.0;
      for (int d = 0; d < nDim; ++d) alpha += UnitNormal[d] * dir[d];
      SoundSpeed = Riemann - vel_mag * alpha;
      SoundSpeed = std::max(0.0, 0.5 * GM1 * SoundSpeed);
      const double Pressure = SoundSpeed * SoundSpeed * Density / Gamma;
      Vg[T_] = Pressure / (Density * mix_rgas(m, Ys)) * P.R_ref;
      for (int d = 0; d < nDim; ++d) Vg[VX + d] = vel_mag * dir[d];
      Vg[P_] = Pressure;
      Vg[RHO] = Density;
      const double dim_temp = Vg[T_] * P.T_ref;
      double aux = mix_enthalpy(m, dim_temp, Ys) / P.E_ref;
      if (P.rans) aux += P.tke_inf;
      Vg[H_] = aux;
      Vg[H_] += 0.5 * vel_mag * vel_mag;
      Vg[A_] = SoundSpeed;
    } else {  // TOTAL_CONDITIONS :3283-3408
      const double Ttot = md[1] / P.T_ref, Ptot = md[2] / P.P_ref;
      double Velocity2 = 0.0, Vn = 0.0;
      for (int d = 0; d < nDim; ++d) {
        Velocity2 += Vd[VX + d] * Vd[VX + d];
        Vn += Vd[VX + d] * UnitNormal[d];
      }
      const double SoundSpeed = Vd[A_];
      const double dim_temp = Ttot * P.T_ref;
      const double Gamma_Tot = frozen_gamma(m, dim_temp, Ys);
      Gamma = 2.0 / (1.0 / Gamma + 1.0 / Gamma_Tot);
      const double GM1 = Gamma - 1.0;
      const double Riemann = Vn + 2.0 * SoundSpeed / GM1;
      double Tot_Enthalpy = mix_enthalpy(m, dim_temp, Ys);
      double alpha = 0.0;
      for (int d = 0; d < nDim; ++d) alpha += UnitNormal[d] * dir[d];
      const double Rgas = mix_rgas(m, Ys) / P.R_ref;
      auto fT = [&](double T) {
        const double hb = mix_enthalpy(m, T, Ys);
        const double cb = std::sqrt(Gamma * Rgas * T);
        const double Vb = (Riemann - 2.0 * cb / GM1) / alpha;
        return hb + 0.5 * Vb * Vb;
      };
      double Told = Ttot + 1.0, Tcurr = Ttot, Tnew;
      bool conv = false;
      for (int it = 0; it < 15; ++it) {
        const double tmp = fT(Tcurr);
        const double F = tmp - Tot_Enthalpy;
        const double dF = tmp - fT(Told);
        Tnew = Tcurr - F * (Tcurr - Told) / dF;
        if (std::abs(Tnew - Tcurr) < 1.0e-9) {
          conv = true;
          break;
        }
        Told = Tcurr;
        Tcurr = Tnew;
      }
      if (conv) {
        Vg[T_] = Tcurr;
      } else {
        double Ta = 300.0 / P.T_ref, Tb = Ttot;
        bool bconv = false;
        for (int it = 0; it < 100; ++it) {
          Tcurr = (Ta + Tb) / 2.0;
          const double F = fT(Tcurr) - Tot_Enthalpy;
          if (std::abs(F) < 1.0e-6) {
            Vg[T_] = Tcurr;
            bconv = true;
            break;
          }
          if (F > 0.0) Ta = Tcurr; else Tb = Tcurr;
        }
        if (!bconv) throw std::runtime_error("Convergence not achieved for bisection method in inlet boundary condition");
      }
      if (P.rans) Tot_Enthalpy += P.tke_inf;
      Vg[H_] = Tot_Enthalpy;
      const double rho_tot = Ptot / (Rgas * Ttot);
      Vg[RHO] = rho_tot * std::pow(Vg[T_] / Ttot, 1.0 / GM1);
      Vg[P_] = Vg[RHO] * Rgas * Vg[T_];
      Vg[A_] = std::sqrt(Vg[T_] * Gamma * Rgas);
      vel_mag = std::abs((Riemann - 2.0 * Vg[A_] / GM1) / alpha);
      for (int d = 0; d < nDim; ++d) Vg[VX + d] = vel_mag * dir[d];
      (void)Velocity2;
    }
    for (int s = 0; s < ns; ++s) Vg[RHOS + s] = Ys[s];
    if (P.implicit) ghost_dpdu(m, nDim, Vg, Gamma, vel_mag * vel_mag, P, Sc);
  } else {  // OUTLET_FLOW :3826-3930
    const double Density = Vd[RHO];
    double Velocity[3], Velocity2 = 0.0;
    for (int d = 0; d < nDim; ++d) {
      Velocity[d] = Vd[VX + d];
      Velocity2 += Velocity[d] * Velocity[d];
    }
    const double Pressure = Vd[P_];
    const double Gamma = Sd[nDim + 1] + 1.0;
    double SoundSpeed = std::sqrt(Gamma * Pressure / Density);
    const double Mach_Exit = std::sqrt(Velocity2) / SoundSpeed;
    if (Mach_Exit >= 1.0) {
      for (int v = 0; v < nPV; ++v) Vg[v] = Vd[v];
      sup = true;
    } else {
      const double Entropy = Pressure * std::pow(1.0 / Density, Gamma);
      double Vn = 0.0;
      for (int d = 0; d < nDim; ++d) Vn += Velocity[d] * UnitNormal[d];
      const double GM1 = Gamma - 1.0;
      const double Riemann = Vn + 2.0 * SoundSpeed / GM1;
      const double P_Exit = md[1] / P.P_ref;
      Vg[P_] = P_Exit;
      Vg[RHO] = std::pow(P_Exit / Entropy, 1.0 / Gamma);
      SoundSpeed = std::sqrt(Gamma * P_Exit / Vg[RHO]);
      const double Vn_Exit = Riemann - 2.0 * SoundSpeed / GM1;
      Velocity2 = 0.0;
      for (int d = 0; d < nDim; ++d) {
        Velocity[d] += (Vn_Exit - Vn) * UnitNormal[d];
        Velocity2 += Velocity[d] * Velocity[d];
        Vg[VX + d] = Velocity[d];
      }
      for (int s = 0; s < ns; ++s) Ys[s] = Vd[RHOS + s];
      Vg[T_] = P_Exit / (Vg[RHO] * mix_rgas(m, Ys)) * P.R_ref;
      const double dim_temp = Vg[T_] * P.T_ref;
      Vg[H_] = mix_enthalpy(m, dim_temp, Ys) / P.E_ref + (P.rans ? 1.0 : 0.0) * P.tke_inf;
      Vg[H_] += 0.5 * Velocity2;
      Vg[A_] = SoundSpeed;
      for (int s = 0; s < ns; ++s) Vg[RHOS + s] = Ys[s];
      if (P.implicit) ghost_dpdu(m, nDim, Vg, Gamma, Velocity2, P, Sc);
    }
  }
  // convective part (CUpwReactiveAUSM on V_domain | V_ghost)
  double res[32], Ji[32 * 32], Jj[32 * 32];
  ausm(nDim, ns, Vd, Vg, Normal, Sd, sup ? Sd : Sc, P.mach_inf, P.implicit != 0, res, Ji, Jj);
  bool err = false;
  for (int v = 0; v < nVar; ++v) err |= std::isnan(res[v]);
  if (P.implicit && !err)
    for (int q = 0; q < nVar * nVar; ++q) err |= std::isnan(Ji[q]);
  if (err) throw std::runtime_error("NaN found in the convective residual of a boundary condition");
  double* Ri = f.R + i * nVar;
  double* D = P.implicit ? f.A + find_diag(f.rp, f.col, i) * nVar * nVar : nullptr;
  for (int v = 0; v < nVar; ++v) Ri[v] += res[v];
  if (D)
    for (int q = 0; q < nVar * nVar; ++q) D[q] += Ji[q];
  // viscous part (CAvgGradReactive_Boundary: both gradients / transport coefficients of the domain node)
  if (P.implicit) {
    if (sup) {
      for (int v = 0; v < nVar; ++v) Sv[v] = f.dTdU[i * nVar + v];
    } else {
      ghost_dtdu(m, nDim, Vg, Ys, P, Sv);
    }
  }
  ViscParams vp{P.T_ref, P.E_ref, P.R_ref, P.Pr_t, P.Le_t, P.rans, P.implicit};
  const double* Gi = f.G + i * nG * nDim;
  visc_flux(m, nDim, vp, Vd, Vg, Gi, Gi, f.mu[i], f.mu[i], f.kappa[i], f.kappa[i], f.Dij + i * ns * ns,
            f.Dij + i * ns * ns, f.coord + i * nDim, f.coord + pn * nDim, Normal,
            P.implicit ? f.dTdU + i * nVar : nullptr, P.implicit ? Sv : nullptr, P.rans ? f.tke[i] : 0.0,
            P.rans ? f.tke[i] : 0.0, P.rans ? f.mut[i] : 0.0, P.rans ? f.mut[i] : 0.0, P.rans ? f.sigk[i] : 1.0,
            P.rans ? f.gk + i * nDim : nullptr, P.rans ? f.gk + i * nDim : nullptr, res, P.implicit ? Ji : nullptr,
            P.implicit ? Jj : nullptr, false);
  err = false;
  for (int v = 0; v < nVar; ++v) err |= std::isnan(res[v]);
  if (P.implicit && !err)
    for (int q = 0; q < nVar * nVar; ++q) err |= std::isnan(Ji[q]);
  if (err) throw std::runtime_error("NaN found in the viscous residual of a boundary condition");
  for (int v = 0; v < nVar; ++v) Ri[v] -= res[v];
  if (D)
    for (int q = 0; q < nVar * nVar; ++q) D[q] -= Ji[q];
}

// CSysMatrix::DeleteValsRowi (matrix_structure.cpp:483-495) for scalar row r of block row i.
void delete_row(int64_t i, int r, int nb, const int64_t* rp, const int64_t* col, double* A) {
  for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
    for (int c = 0; c < nb; ++c) A[k * nb * nb + r * nb + c] = 0.0;
    if (col[k] == i) A[k * nb * nb + r * nb + r] = 1.0;
  }
}

// CReactiveNSSolver::BC_Isothermal_Wall (:5393-5711), no grid motion.
void flow_wall_vertex(const Mech& m, int nDim, const BCPrm& P, const double* md, int64_t i, int64_t pn,
                      const double* bn, BCField& f) {
  const int ns = m.ns, nVar = ns + nDim + 2, nPV = ns + nDim + 5;
  const double Twall = md[1] / P.T_ref;
  const double dim_temp = Twall * P.T_ref;
  double aux_Cp[32];
  for (int s = 0; s < ns; ++s) aux_Cp[s] = spline(m, P_CP, s, dim_temp) / m.mm[s];
  double Area = 0.0;
  for (int d = 0; d < nDim; ++d) Area += bn[d] * bn[d];
  Area = std::sqrt(Area);
  double dij = 0.0;
  for (int d = 0; d < nDim; ++d) {
    const double x = f.coord[pn * nDim + d] - f.coord[i * nDim + d];
    dij += x * x;
  }
  dij = std::sqrt(dij);
  double Res_Conv[32], Res_Visc[32];
  for (int v = 0; v < nVar; ++v) Res_Conv[v] = Res_Visc[v] = 0.0;
  for (int d = 0; d < nDim; ++d) f.Uold[i * nVar + 1 + d] = 0.0 * f.V[i * nPV + nDim + 2];  // SetVelocity_Old
  double* Ri = f.R + i * nVar;
  for (int d = 0; d < nDim; ++d) Ri[1 + d] = 0.0;  // LinSysRes.SetBlock_Zero(iPoint, RHOVX + iDim)
  const double Tj = f.V[pn * nPV];
  const double ktr = f.kappa[i];
  double turb_closure = 0.0, turb_ktr = 0.0;
  if (P.rans) {
    const double eddy_v = f.eddy[i];
    for (int s = 0; s < ns; ++s) {
      const double aux_ys = f.U[i * nVar + nDim + 2 + s];
      turb_closure += eddy_v / P.Pr_t * aux_Cp[s] * aux_ys * (Twall - Tj) / dij;
    }
    for (int s = 0; s < ns; ++s) {
      const double aux_ys = f.U[i * nVar + nDim + 2 + s];
      turb_ktr += eddy_v / (P.Pr_t) * aux_Cp[s] * aux_ys;
    }
  }
  const double dTdn = +(Twall - Tj) / dij;
  Res_Visc[nDim + 1] = ktr * dTdn * Area + turb_closure * Area;
  if (P.implicit) {
    double J[32 * 32];
    for (int q = 0; q < nVar * nVar; ++q) J[q] = 0.0;
    for (int d = 0; d < nDim; ++d) delete_row(i, 1 + d, nVar, f.rp, f.col, f.A);
    const double* dTdU = f.dTdU + pn * nVar;
    const int E = nDim + 1;
    J[E * nVar + 0] = -ktr * dTdU[0] / dij * Area;
    J[E * nVar + E] = -ktr * dTdU[E] / dij * Area - turb_ktr * dTdU[E] / dij * Area;
    for (int s = 0; s < ns; ++s) J[E * nVar + nDim + 2 + s] = -ktr * dTdU[nDim + 2 + s] / dij * Area;
    double* D = f.A + find_diag(f.rp, f.col, i) * nVar * nVar;
    for (int q = 0; q < nVar * nVar; ++q) D[q] -= J[q];
  }
  for (int v = 0; v < nVar; ++v) Ri[v] += Res_Conv[v];
  for (int v = 0; v < nVar; ++v) Ri[v] -= Res_Visc[v];
  if (P.implicit)
    for (int d = 0; d < nDim; ++d) delete_row(i, 1 + d, nVar, f.rp, f.col, f.A);
}

// CReactiveEulerSolver::BC_Euler_Wall (:2881-2966), no grid motion: momentum residual (p + 2/3 rho k) n A, n = -Normal / A,
// added as a whole block; Jacobian_i's momentum rows dPdU n A, added as a whole block.
void flow_euler_vertex(const Mech& m, int nDim, const BCPrm& P, int64_t i, const double* bn, BCField& f) {
  const int ns = m.ns, nVar = ns + nDim + 2, nPV = ns + nDim + 5;
  double Area = 0.0;
  for (int d = 0; d < nDim; ++d) Area += bn[d] * bn[d];
  Area = std::sqrt(Area);
  double UnitNormal[3];
  for (int d = 0; d < nDim; ++d) UnitNormal[d] = -bn[d] / Area;
  const double Pressure = f.V[i * nPV + nDim + 1], Density = f.V[i * nPV + nDim + 2];
  const double turb_ke = P.rans ? f.tke[i] : 0.0;
  double Residual[32];
  for (int v = 0; v < nVar; ++v) Residual[v] = 0.0;
  for (int d = 0; d < nDim; ++d)
    Residual[1 + d] = Pressure * UnitNormal[d] * Area + 2.0 / 3.0 * Density * turb_ke * UnitNormal[d] * Area;
  double* Ri = f.R + i * nVar;
  for (int v = 0; v < nVar; ++v) Ri[v] += Residual[v];
  if (P.implicit) {
    double J[32 * 32];
    for (int q = 0; q < nVar * nVar; ++q) J[q] = 0.0;
    const double* dPdU = f.dPdU + i * nVar;
    for (int d = 0; d < nDim; ++d)
      for (int v = 0; v < nVar; ++v) J[(1 + d) * nVar + v] = dPdU[v] * UnitNormal[d] * Area;
    double* D = f.A + find_diag(f.rp, f.col, i) * nVar * nVar;
    for (int q = 0; q < nVar * nVar; ++q) D[q] += J[q];
  }
}

// CReactiveNSSolver::BC_HeatFlux_Wall (:5717-5911), no grid motion.
void flow_heatflux_vertex(const Mech& m, int nDim, const BCPrm& P, const double* md, int64_t i, const double* bn,
                          BCField& f) {
  const int ns = m.ns, nVar = ns + nDim + 2, nPV = ns + nDim + 5;
  double Area = 0.0;
  for (int d = 0; d < nDim; ++d) Area += bn[d] * bn[d];
  Area = std::sqrt(Area);
  for (int d = 0; d < nDim; ++d) f.Uold[i * nVar + 1 + d] = 0.0 * f.V[i * nPV + nDim + 2];  // SetVelocity_Old
  double* Ri = f.R + i * nVar;
  for (int d = 0; d < nDim; ++d) Ri[1 + d] = 0.0;  // LinSysRes.SetBlock_Zero(iPoint, RHOVX + iDim)
  double Res_Conv[32], Res_Visc[32];
  for (int v = 0; v < nVar; ++v) Res_Conv[v] = Res_Visc[v] = 0.0;
  Res_Visc[nDim + 1] = md[1] * Area;  // Wall_HeatFlux * Area
  for (int v = 0; v < nVar; ++v) Ri[v] += Res_Conv[v];
  for (int v = 0; v < nVar; ++v) Ri[v] -= Res_Visc[v];
  if (P.implicit)
    for (int d = 0; d < nDim; ++d) delete_row(i, 1 + d, nVar, f.rp, f.col, f.A);
}

BCPrm bc_params(const double* p, int implicit, int rans) {
  BCPrm P;
  P.kind_inlet = (int)p[0];
  P.tke_inf = p[1];
  P.kine_inf = p[2];
  P.omega_inf = p[3];
  P.beta1 = p[4];
  P.P_ref = p[5];
  P.vel_ref = p[6];
  P.T_ref = p[7];
  P.E_ref = p[8];
  P.R_ref = p[9];
  P.rho_ref = p[10];
  P.k_inlet = (int)p[11];
  P.k_outlet = (int)p[12];
  P.k_iso = (int)p[13];
  P.k_hf = (int)p[14];
  P.k_total = (int)p[15];
  P.k_massflow = (int)p[16];
  P.k_timpose = (int)p[17];
  P.mach_inf = p[18];
  P.Pr_t = p[19];
  P.Le_t = p[20];
  P.k_euler = (int)p[21];
  P.k_sup_in = (int)p[22];
  P.k_sup_out = (int)p[23];
  P.implicit = implicit;
  P.rans = rans;
  return P;
}

}  // namespace

extern "C" {

// Flow BCs of one Space_Integration. bvert [NB][3] = (marker, node, kind) in marker / vertex order, pn [NB]
// normal neighbours, mdata [nMarker][W] = (kind, a, b, dir[3], Y[Ns]), prm: bc_params layout (see oracle.py).
// R [N][nVar] and A (BSR, may be null) are updated in place; Uold gets SetVelocity_Old; charac [NB][nPV] the
// ghost states (CharacPrimVar) of the weak BCs. Returns 0, or 1 on a reference exception.
int orc_bc_flow(void* h, int nDim, int64_t NB, const int64_t* bvert, const double* bnormal, const int64_t* pn,
                int nMarker, const double* mdata, int W, const double* prm, int implicit, int rans,
                const double* coord, const double* U, const double* V, const double* dPdU, const double* dTdU,
                const double* G, const double* mu, const double* kappa, const double* Dij, const double* tke,
                const double* mut, const double* sigk, const double* gk, const double* eddy, const int64_t* rp,
                const int64_t* col, double* R, double* A, double* Uold, double* charac) {
  const Mech& m = *static_cast<Mech*>(h);
  const int nPV = m.ns + nDim + 5;
  const BCPrm P = bc_params(prm, implicit, rans);
  BCField f{coord, U, V, dPdU, dTdU, G, mu, kappa, Dij, tke, mut, sigk, gk, eddy, rp, col, R, A, Uold};
  try {
    for (int pass = 0; pass < 2; ++pass)
      for (int mk = 0; mk < nMarker; ++mk) {
        const double* md = mdata + (size_t)mk * W;
        const int kind = (int)md[0];
        const bool weak = kind == P.k_inlet || kind == P.k_outlet || kind == P.k_euler || kind == P.k_sup_in ||
                          kind == P.k_sup_out;
        const bool strong = kind == P.k_iso || kind == P.k_hf;
        if ((pass == 0 && !weak) || (pass == 1 && !strong)) continue;
        for (int64_t b = 0; b < NB; ++b) {
          if (bvert[3 * b] != mk) continue;
          const int64_t i = bvert[3 * b + 1];
          if (kind == P.k_euler)
            flow_euler_vertex(m, nDim, P, i, bnormal + b * nDim, f);
          else if (kind == P.k_hf)
            flow_heatflux_vertex(m, nDim, P, md, i, bnormal + b * nDim, f);
          else if (pass == 0)
            flow_weak_vertex(m, nDim, P, kind, md, i, pn[b], bnormal + b * nDim, f, charac + b * nPV);
          else
            flow_wall_vertex(m, nDim, P, md, i, pn[b], bnormal + b * nDim, f);
        }
      }
  } catch (const std::exception&) {
    return 1;
  }
  return 0;
}

// SST BCs of one Space_Integration (CTurbSSTSolver::BC_Inlet / BC_Outlet :3264-3450, BC_Isothermal_Wall
// :3142-3196; numerics CUpwSca_TurbSST / CAvgGrad_TurbSST) on the flow's V, mu, eddy viscosity and the ghost states charac of the flow BCs. T [N][2] (and
// its Solution_Old: the same array) is set at the walls.
void orc_bc_sst(int nDim, int nPV, int64_t NB, const int64_t* bvert, const double* bnormal, const int64_t* pn,
                int nMarker, const double* mdata, int W, const double* prm, int implicit, const double* coord,
                const double* V, const double* mu, const double* eddy, const double* charac, const double* TG,
                const double* F1, const int64_t* rp, const int64_t* col, double* T, double* R, double* A) {
  const BCPrm P = bc_params(prm, implicit, 1);
  const SSTConst c = sst_const();
  for (int pass = 0; pass < 2; ++pass)
    for (int mk = 0; mk < nMarker; ++mk) {
      const int kind = (int)mdata[(size_t)mk * W];
      const bool weak = kind == P.k_inlet || kind == P.k_outlet;  // CTurbSolver::BC_Euler_Wall: no action
      const bool strong = kind == P.k_iso || kind == P.k_hf;      // BC_HeatFlux_Wall :3087-3140 = the isothermal wall
      if ((pass == 0 && !weak) || (pass == 1 && !strong)) continue;
      for (int64_t b = 0; b < NB; ++b) {
        if (bvert[3 * b] != mk) continue;
        const int64_t i = bvert[3 * b + 1], j = pn[b];
        if (pass == 1) {
          double distance = 0.0;
          for (int d = 0; d < nDim; ++d)
            distance += (coord[i * nDim + d] - coord[j * nDim + d]) * (coord[i * nDim + d] - coord[j * nDim + d]);
          distance = std::sqrt(distance);
          const double density = V[j * nPV + nDim + 2], lam = mu[j];
          T[2 * i] = 0.0;
          T[2 * i + 1] = 60.0 * lam / (density * P.beta1 * distance * distance);
          R[2 * i] = R[2 * i + 1] = 0.0;
          if (implicit)
            for (int v = 0; v < 2; ++v) delete_row(i, v, 2, rp, col, A);
          continue;
        }
        double Normal[3];
        for (int d = 0; d < nDim; ++d) Normal[d] = -bnormal[b * nDim + d];
        const double* Vi = V + i * nPV;
        const double* Vg = charac + b * nPV;
        const double Ti[2] = {T[2 * i], T[2 * i + 1]};
        double Tg[2] = {Ti[0], Ti[1]};
        if (kind == P.k_inlet) {
          Tg[0] = P.kine_inf;
          Tg[1] = P.omega_inf;
        }
        double* D = implicit ? A + find_diag(rp, col, i) * 4 : nullptr;
        // CUpwSca_TurbSST (numerics_direct_turbulent.cpp:865-922)
        double q = 0.0;
        for (int d = 0; d < nDim; ++d) q += 0.5 * (Vi[d + 1] + Vg[d + 1]) * Normal[d];
        const double a0 = 0.5 * (q + std::fabs(q)), a1 = 0.5 * (q - std::fabs(q));
        const double ri = Vi[nDim + 2], rj = Vg[nDim + 2];
        R[2 * i] += a0 * ri * Ti[0] + a1 * rj * Tg[0];
        R[2 * i + 1] += a0 * ri * Ti[1] + a1 * rj * Tg[1];
        if (D) {
          D[0] += a0;
          D[1] += 0.0;
          D[2] += 0.0;
          D[3] += a0;
        }
        // CAvgGrad_TurbSST (numerics_direct_turbulent.cpp:966-1040, the TURB_SOL VISC_BOUND_TERM of
        // driver_structure.cpp:1610): plain mean normal gradient; both gradients, F1, mu, eddy of node i
        const double sk = F1[i] * c.sk1 + (1.0 - F1[i]) * c.sk2;
        const double so = F1[i] * c.so1 + (1.0 - F1[i]) * c.so2;
        const double dik = mu[i] + sk * eddy[i], dio = mu[i] + so * eddy[i];
        const double dk = 0.5 * (dik + dik), dw = 0.5 * (dio + dio);
        double ev[3], dist2 = 0.0, proj = 0.0;
        for (int d = 0; d < nDim; ++d) {
          ev[d] = coord[j * nDim + d] - coord[i * nDim + d];
          dist2 += ev[d] * ev[d];
          proj += ev[d] * Normal[d];
        }
        if (dist2 == 0.0) proj = 0.0; else proj = proj / dist2;
        double corr[2];
        for (int v = 0; v < 2; ++v) {
          double pnv = 0.0;
          for (int d = 0; d < nDim; ++d) pnv += 0.5 * (TG[(i * 2 + v) * nDim + d] + TG[(i * 2 + v) * nDim + d]) * Normal[d];
          corr[v] = pnv;
        }
        R[2 * i] -= dk * corr[0];
        R[2 * i + 1] -= dw * corr[1];
        if (D) {
          D[0] -= -dk * proj / ri;
          D[1] -= 0.0;
          D[2] -= 0.0;
          D[3] -= -dw * proj / ri;
        }
      }
    }
}

}  // extern "C"
