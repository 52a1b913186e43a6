// rx_bc.hip — boundary conditions of the reactive RANS Space_Integration on gfx950 (SURVEY §8 next-3 + a8).
//
// Reference (paths relative to the reference root):
//   CIntegration::Space_Integration — weak BCs in marker order, then strong   SU2_CFD/src/integration_structure.cpp:95-193
//   CReactiveEulerSolver::BC_Inlet (TOTAL_CONDITIONS / MASS_FLOW / TEMPERATURE_IMPOSE)
//                                                                         SU2_CFD/src/solver_direct_reactive.cpp:3226-3674
//   CReactiveEulerSolver::BC_Outlet                                       :3808-4123
//   CReactiveNSSolver::BC_Isothermal_Wall (no grid motion)               :5393-5711
//   boundary numerics CUpwReactiveAUSM (numerics_direct_reactive.cpp:53-378) and
//   CAvgGradReactive_Boundary::ComputeResidual (:478-648, a8: plain mean gradient, no edge correction)
//   CTurbSSTSolver::BC_Inlet / BC_Outlet / BC_Isothermal_Wall            SU2_CFD/src/solver_direct_turbulent.cpp:3142-3450
//   with CUpwSca_TurbSST / CAvgGrad_TurbSST (numerics_direct_turbulent.cpp:865-1040; driver_structure.cpp:1609-1610)
//   library calls ComputeDensity / ComputeTemperature / ComputeRgas / ComputeEnthalpy / ComputeFrozenGamma /
//   ComputeFrozenSoundSpeed / ComputeCV / ComputePartialEnergy / ComputedP_dYs / ComputeCps
//   (Common/src/Framework/reacting_model_library.cpp:26-41, 398-470, 519-619; reacting_model_library.hpp:368)
//
// Work split (boundary vertices are O(sqrt N), so the point is staying on the device, not bandwidth):
//   k_bc_weak       one lane per inlet / outlet vertex: ghost state (CharacPrimVar), AUSM flux + Jacobian_i,
//                   boundary viscous flux + the per-edge summary of the viscous Jacobian;
//   k_bc_visc_jac   16-lane team per vertex: the viscous Jacobian columns (rx_visc.h visc_jac_column);
//   k_bc_apply      one thread per owned boundary point: applies its vertices' contributions in the reference's
//                   order (weak markers then walls; AddBlock / SubtractBlock per vertex), the isothermal wall
//                   (weak energy flux, strong no-slip with DeleteValsRowi on the whole BSR row).
//   k_sst_bc        one thread per owned boundary point, the SST markers in the same order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "rx_ctx.h"
#include "rx_species.h"
#include "rx_visc.h"

using namespace rx;

namespace {

constexpr int kBlock = 256;
inline int blocks(int64_t n, int b = kBlock) { return (int)((n + b - 1) / b); }

__device__ inline void set_err(int* err, int code, int64_t idx) {
  if (atomicCAS(err, 0, code) == 0) err[1] = (int)idx;
}

struct BCDev {
  int inlet_kind, W, implicit, rans;
  double tke_inf, kine_inf, omega_inf;
  double T_ref, E_ref, R_ref, P_ref, vel_ref, rho_ref, mach_inf;
  ViscParams vp;
};

__device__ inline double clampY(double y) { return y < 0.0 ? 1.0e-30 : y; }

// SetRgas: inner_product(Ys (clamped), Ri) (reacting_model_library.cpp:26-31)
template <int NS>
__device__ inline double lib_rgas(const DevMech& m, const double* Y) {
  double r = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) r += clampY(Y[s]) * (kR / m.mm[s]);
  return r;
}
// ComputeEnthalpy (:519-523)
template <int NS>
__device__ inline double lib_enthalpy(const DevMech& m, double T, const double* Y, int* err) {
  double h = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) h += clampY(Y[s]) * (spline(m, P_H, s, T, err) / m.mm[s]);
  return h;
}
// ComputeCP (:612-619)
template <int NS>
__device__ inline double lib_cp(const DevMech& m, double T, const double* Y, int* err) {
  double c = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) c += clampY(Y[s]) * (spline(m, P_CP, s, T, err) / m.mm[s]);
  return c;
}
// ComputeFrozenGamma (:398-403)
template <int NS>
__device__ inline double lib_gamma(const DevMech& m, double T, const double* Y, int* err) {
  const double Cp = lib_cp<NS>(m, T, Y, err);
  const double Cv = Cp - lib_rgas<NS>(m, Y);
  return Cp / Cv;
}
// ComputePartialEnergy(T, s) (:583-588)
__device__ inline double lib_energy_s(const DevMech& m, double T, int s, int* err) {
  return spline(m, P_H, s, T, err) / m.mm[s] - (kR / m.mm[s]) * T;
}

// Ghost secondaries. dP/dU: BC_Inlet :3510-3533 / BC_Outlet :3941-3962 (ComputedP_dYs :591-596).
template <int NS, int NDIM>
__device__ inline void ghost_dpdu(const DevMech& m, const BCDev& B, const double* Vg, double Gamma, double vel2,
                                  double* S, int* err) {
  S[0] = (Gamma - 1.0) * 0.5 * vel2;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) S[1 + d] = (1.0 - Gamma) * Vg[1 + d];
  S[NDIM + 1] = Gamma - 1.0;
  const double dim_temp = Vg[0] * B.T_ref;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    S[NDIM + 2 + s] = ((kR / m.mm[s]) * dim_temp - (Gamma - 1.0) * lib_energy_s(m, dim_temp, s, err)) / B.E_ref;
}
// dT/dU of the ghost for the boundary viscous numerics: :3573-3595 / :4021-4044.
template <int NS, int NDIM>
__device__ inline void ghost_dtdu(const DevMech& m, const BCDev& B, const double* Vg, const double* Ys, double* S,
                                  int* err) {
  const double dim_temp = Vg[0] * B.T_ref;
  const double Cv = (lib_cp<NS>(m, dim_temp, Ys, err) - lib_rgas<NS>(m, Ys)) / B.R_ref;
  const double rhoCv = Vg[NDIM + 2] * Cv;
  double sq_vel = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) sq_vel += Vg[1 + d] * Vg[1 + d];
  S[0] = 0.5 * sq_vel / rhoCv;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) S[1 + d] = -Vg[1 + d] / rhoCv;
  S[NDIM + 1] = 1.0 / rhoCv;
#pragma unroll
  for (int s = 0; s < NS; ++s) S[NDIM + 2 + s] = -lib_energy_s(m, dim_temp, s, err) / (B.E_ref * rhoCv);
}

// The ghost state of one inlet / outlet vertex (BC_Inlet :3253-3502, BC_Outlet :3826-3930). Returns false on the
// reference's bisection failure. sup: supersonic exit (the node's own dP/dU, dT/dU are the ghost's).
template <int NS, int NDIM>
__device__ inline bool ghost_state(const DevMech& m, const BCDev& B, int kind, const double* md, const double* Vd,
                                   const double* Sd, const double* UN, double* Vg, double* Sc, double* Ys, bool* sup,
                                   int* err) {
  constexpr int T_ = 0, VX = 1, P_ = NDIM + 1, RHO = NDIM + 2, H_ = NDIM + 3, A_ = NDIM + 4, RHOS = NDIM + 5;
  constexpr int nPV = NS + NDIM + 5;
  *sup = false;
  if (kind == RX_BC_SUP_INLET) {
    // BC_Supersonic_Inlet (:3014-3055): T, P, velocity and Y from the marker; density from the gas law
    // (ComputeDensity :457-460), enthalpy (ComputeEnthalpy) and frozen sound speed (ComputeFrozenSoundSpeed :408-411:
    // sqrt(gamma Rgas T)) at the dimensional temperature, each then non-dimensionalised; no turbulent kinetic energy
    // in the ghost's enthalpy (the subsonic inlet adds it, :3517)
#pragma unroll
    for (int s = 0; s < NS; ++s) Ys[s] = md[6 + s];
    const double Temperature = md[1], Pressure = md[2];
    const double Rgas = lib_rgas<NS>(m, Ys);
    const double Density = Pressure / (Temperature * Rgas);
    const double Enthalpy = lib_enthalpy<NS>(m, Temperature, Ys, err);
    const double SoundSpeed = sqrt(lib_gamma<NS>(m, Temperature, Ys, err) * Rgas * Temperature);
    double Velocity2 = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      Vg[VX + d] = md[3 + d] / B.vel_ref;
      Velocity2 += Vg[VX + d] * Vg[VX + d];
    }
    Vg[T_] = Temperature / B.T_ref;
    Vg[P_] = Pressure / B.P_ref;
    Vg[RHO] = Density / B.rho_ref;
    Vg[H_] = Enthalpy / B.E_ref + 0.5 * Velocity2;
    Vg[A_] = SoundSpeed / B.vel_ref;
#pragma unroll
    for (int s = 0; s < NS; ++s) Vg[RHOS + s] = Ys[s];
    // the ghost's dP/dU (:3080-3102) enters only Jacobian_j, which the BC discards: the domain's stands in
#pragma unroll
    for (int v = 0; v < NS + NDIM + 2; ++v) Sc[v] = Sd[v];
    return true;
  }
  if (kind == RX_BC_SUP_OUTLET) {  // BC_Supersonic_Outlet (:3708-3717): the ghost is the domain state
#pragma unroll
    for (int v = 0; v < nPV; ++v) Vg[v] = Vd[v];
    *sup = true;
    return true;
  }
  if (kind == RX_BC_INLET) {
#pragma unroll
    for (int s = 0; s < NS; ++s) Ys[s] = md[6 + s];
    const double* dir = md + 3;
    double Gamma = Sd[NDIM + 1] + 1.0, vel_mag = 0.0;
    if (B.inlet_kind == RX_INLET_TEMPERATURE_IMPOSE) {
      const double T = md[1] / B.T_ref;
      vel_mag = md[2] / B.vel_ref;
      Vg[T_] = T;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) Vg[VX + d] = vel_mag * dir[d];
      Vg[P_] = Vd[P_];
      Vg[RHO] = Vg[P_] / (T * lib_rgas<NS>(m, Ys)) * B.R_ref;
      const double dim_temp = T * B.T_ref;
      Vg[H_] = lib_enthalpy<NS>(m, dim_temp, Ys, err) / B.E_ref + (B.rans ? 1.0 : 0.0) * B.tke_inf;
      Vg[H_] += 0.5 * vel_mag * vel_mag;
      Vg[A_] = sqrt(lib_gamma<NS>(m, dim_temp, Ys, err) * lib_rgas<NS>(m, Ys) * dim_temp) / B.vel_ref;
      // the reference leaves Gamma uninitialised in this branch (:3236, :3515); it only enters the ghost's dP/dU,
      // i.e. Jacobian_j, which the BC discards: the domain value stands in
    } else if (B.inlet_kind == RX_INLET_MASS_FLOW) {
      const double Density = md[1] / B.rho_ref;
      vel_mag = md[2] / B.vel_ref;
      double SoundSpeed = Vd[A_];
      const double GM1 = Gamma - 1.0;
      double Vn = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) Vn += Vd[VX + d] * UN[d];
      const double Riemann = Vn + 2.0 * SoundSpeed / GM1;
      double alpha = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) alpha += UN[d] * dir[d];
      SoundSpeed = Riemann - vel_mag * alpha;
      SoundSpeed = (0.0 < 0.5 * GM1 * SoundSpeed) ? 0.5 * GM1 * SoundSpeed : 0.0;  // std::max(0.0, x)
      const double Pressure = SoundSpeed * SoundSpeed * Density / Gamma;
      Vg[T_] = Pressure / (Density * lib_rgas<NS>(m, Ys)) * B.R_ref;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) Vg[VX + d] = vel_mag * dir[d];
      Vg[P_] = Pressure;
      Vg[RHO] = Density;
      const double dim_temp = Vg[T_] * B.T_ref;
      double aux = lib_enthalpy<NS>(m, dim_temp, Ys, err) / B.E_ref;
      if (B.rans) aux += B.tke_inf;
      Vg[H_] = aux;
      Vg[H_] += 0.5 * vel_mag * vel_mag;
      Vg[A_] = SoundSpeed;
    } else {  // TOTAL_CONDITIONS :3283-3408
      const double Ttot = md[1] / B.T_ref, Ptot = md[2] / B.P_ref;
      double Vn = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) Vn += Vd[VX + d] * UN[d];
      const double SoundSpeed = Vd[A_];
      const double dim_temp = Ttot * B.T_ref;
      const double Gamma_Tot = lib_gamma<NS>(m, dim_temp, Ys, err);
      Gamma = 2.0 / (1.0 / Gamma + 1.0 / Gamma_Tot);
      const double GM1 = Gamma - 1.0;
      const double Riemann = Vn + 2.0 * SoundSpeed / GM1;
      double Tot_Enthalpy = lib_enthalpy<NS>(m, dim_temp, Ys, err);
      double alpha = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) alpha += UN[d] * dir[d];
      const double Rgas = lib_rgas<NS>(m, Ys) / B.R_ref;
      auto fT = [&](double T) {
        const double hb = lib_enthalpy<NS>(m, T, Ys, err);
        const double cb = sqrt(Gamma * Rgas * T);
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
        if (fabs(Tnew - Tcurr) < 1.0e-9) {
          conv = true;
          break;
        }
        Told = Tcurr;
        Tcurr = Tnew;
      }
      if (conv) {
        Vg[T_] = Tcurr;
      } else {
        double Ta = 300.0 / B.T_ref, Tb = Ttot;
        bool bconv = false;
        for (int it = 0; it < 100; ++it) {
          Tcurr = (Ta + Tb) / 2.0;
          const double F = fT(Tcurr) - Tot_Enthalpy;
          if (fabs(F) < 1.0e-6) {
            Vg[T_] = Tcurr;
            bconv = true;
            break;
          }
          if (F > 0.0) Ta = Tcurr; else Tb = Tcurr;
        }
        if (!bconv) return false;
      }
      if (B.rans) Tot_Enthalpy += B.tke_inf;
      Vg[H_] = Tot_Enthalpy;
      const double rho_tot = Ptot / (Rgas * Ttot);
      Vg[RHO] = rho_tot * pow(Vg[T_] / Ttot, 1.0 / GM1);
      Vg[P_] = Vg[RHO] * Rgas * Vg[T_];
      Vg[A_] = sqrt(Vg[T_] * Gamma * Rgas);
      vel_mag = fabs((Riemann - 2.0 * Vg[A_] / GM1) / alpha);
#pragma unroll
      for (int d = 0; d < NDIM; ++d) Vg[VX + d] = vel_mag * dir[d];
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) Vg[RHOS + s] = Ys[s];
    if (B.implicit) ghost_dpdu<NS, NDIM>(m, B, Vg, Gamma, vel_mag * vel_mag, Sc, err);
    return true;
  }
  // OUTLET_FLOW :3826-3930
  const double Density = Vd[RHO];
  double Velocity[NDIM], Velocity2 = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    Velocity[d] = Vd[VX + d];
    Velocity2 += Velocity[d] * Velocity[d];
  }
  const double Pressure = Vd[P_];
  const double Gamma = Sd[NDIM + 1] + 1.0;
  double SoundSpeed = sqrt(Gamma * Pressure / Density);
  const double Mach_Exit = sqrt(Velocity2) / SoundSpeed;
  if (Mach_Exit >= 1.0) {
#pragma unroll
    for (int v = 0; v < nPV; ++v) Vg[v] = Vd[v];
    *sup = true;
    return true;
  }
  const double Entropy = Pressure * pow(1.0 / Density, Gamma);
  double Vn = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) Vn += Velocity[d] * UN[d];
  const double GM1 = Gamma - 1.0;
  const double Riemann = Vn + 2.0 * SoundSpeed / GM1;
  const double P_Exit = md[1] / B.P_ref;
  Vg[P_] = P_Exit;
  Vg[RHO] = pow(P_Exit / Entropy, 1.0 / Gamma);
  SoundSpeed = sqrt(Gamma * P_Exit / Vg[RHO]);
  const double Vn_Exit = Riemann - 2.0 * SoundSpeed / GM1;
  Velocity2 = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    Velocity[d] += (Vn_Exit - Vn) * UN[d];
    Velocity2 += Velocity[d] * Velocity[d];
    Vg[VX + d] = Velocity[d];
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) Ys[s] = Vd[RHOS + s];
  Vg[T_] = P_Exit / (Vg[RHO] * lib_rgas<NS>(m, Ys)) * B.R_ref;
  const double dim_temp = Vg[T_] * B.T_ref;
  Vg[H_] = lib_enthalpy<NS>(m, dim_temp, Ys, err) / B.E_ref + (B.rans ? 1.0 : 0.0) * B.tke_inf;
  Vg[H_] += 0.5 * Velocity2;
  Vg[A_] = SoundSpeed;
#pragma unroll
  for (int s = 0; s < NS; ++s) Vg[RHOS + s] = Ys[s];
  if (B.implicit) ghost_dpdu<NS, NDIM>(m, B, Vg, Gamma, Velocity2, Sc, err);
  return true;
}

// One lane per weak vertex: ghost state, AUSM flux (+ Jacobian_i), boundary viscous flux (+ Jacobian summary).
template <int NS, int NDIM>
__global__ __launch_bounds__(64) void k_bc_weak(int NW, const int32_t* __restrict__ weak,
                                                const int32_t* __restrict__ bnode, const int32_t* __restrict__ bpn,
                                                const int32_t* __restrict__ bmark, const double* __restrict__ bnrm,
                                                const int32_t* __restrict__ mkind, const double* __restrict__ mdata,
                                                BCDev B, DevMech m, const double* __restrict__ coord,
                                                const double* __restrict__ V, const double* __restrict__ dPdU,
                                                const double* __restrict__ dTdU, const double* __restrict__ G,
                                                const double* __restrict__ mu, const double* __restrict__ kappa,
                                                const double* __restrict__ Dij, const double* __restrict__ tke,
                                                const double* __restrict__ mut, const double* __restrict__ sigk,
                                                const double* __restrict__ gk, double* __restrict__ charac,
                                                double* __restrict__ resc, double* __restrict__ resv,
                                                double* __restrict__ jacc, double* __restrict__ summ,
                                                double* __restrict__ sv, int* err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5, nG = NS + NDIM + 2, nVar2 = nVar * nVar;
  __shared__ double scr_all[64 * NS * NS];
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= NW) return;
  const int b = weak[q];
  const int i = bnode[b], mk = bmark[b];
  const int kind = mkind[mk];
  const double* md = mdata + (size_t)mk * B.W;
  double Normal[NDIM], UN[NDIM], Area = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) Area += bnrm[(size_t)b * NDIM + d] * bnrm[(size_t)b * NDIM + d];
  Area = sqrt(Area);
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    Normal[d] = -bnrm[(size_t)b * NDIM + d];
    UN[d] = Normal[d] / Area;
  }
  const double* Vd = V + (size_t)i * nPV;
  const double* Sd = dPdU + (size_t)i * nVar;
  double Vg[nPV], Sc[nVar], Ys[NS];
  bool sup = false;
  int e = ERR_NONE;
  if (!ghost_state<NS, NDIM>(m, B, kind, md, Vd, Sd, UN, Vg, Sc, Ys, &sup, &e)) {
    set_err(err, ERR_CONV, i);
    return;
  }
#pragma unroll
  for (int v = 0; v < nPV; ++v) charac[(size_t)b * nPV + v] = Vg[v];
  // CUpwReactiveAUSM on (V_domain, V_ghost)
  double Vi[nPV];
#pragma unroll
  for (int v = 0; v < nPV; ++v) Vi[v] = Vd[v];
  AusmEdge s;
  ausm_scalars<NDIM>(Vi, Vg, Normal, B.mach_inf, s);
  bool bad = false;
#pragma unroll
  for (int v = 0; v < nVar; ++v) {
    const double r = ausm_res<NDIM>(s, Vi, Vg, v);
    bad |= isnan(r);
    resc[(size_t)b * nVar + v] = r;
  }
  if (B.implicit) {
    for (int c = 0; c < nVar; ++c) {
      const double sib = Sd[c], sjb = sup ? Sd[c] : Sc[c];
      const AusmCol col = ausm_col_b<NDIM>(s, sib, sjb, c);
#pragma unroll
      for (int a = 0; a < nVar; ++a) {
        double ji, jj;
        ausm_jac_entry<NDIM>(s, col, ausm_phi<NDIM>(Vi, Vi[NDIM + 3], a), ausm_phi<NDIM>(Vg, Vg[NDIM + 3], a), sib,
                             sjb, a, c, &ji, &jj);
        bad |= isnan(ji);
        jacc[(size_t)b * nVar2 + a * nVar + c] = ji;
      }
    }
  }
  if (bad) set_err(err, ERR_NAN, i);
  // CAvgGradReactive_Boundary: both gradients and transport coefficients of the domain point
  double Sv[nVar];
  if (B.implicit) {
    if (sup) {
#pragma unroll
      for (int v = 0; v < nVar; ++v) Sv[v] = dTdU[(size_t)i * nVar + v];
    } else {
      ghost_dtdu<NS, NDIM>(m, B, Vg, Ys, Sv, &e);
    }
#pragma unroll
    for (int v = 0; v < nVar; ++v) sv[(size_t)b * nVar + v] = Sv[v];
  }
  ViscNode<NS, NDIM> a, g;
  a.V = Vd;
  g.V = Vg;
  a.G = g.G = G + (size_t)i * nG * NDIM;
  a.Dij = g.Dij = Dij + (size_t)i * NS * NS;
  a.S = B.implicit ? dTdU + (size_t)i * nVar : nullptr;
  g.S = B.implicit ? Sv : nullptr;
  a.coord = coord + (size_t)i * NDIM;
  g.coord = coord + (size_t)bpn[b] * NDIM;
  a.mu = g.mu = mu[i];
  a.kappa = g.kappa = kappa[i];
  double sk = 1.0;
  if (B.rans) {
    a.tke = g.tke = tke[i];
    a.mut = g.mut = mut[i];
    a.gk = g.gk = gk + (size_t)i * NDIM;
    sk = sigk[i];
  } else {
    a.tke = g.tke = a.mut = g.mut = 0.0;
    a.gk = g.gk = nullptr;
  }
  double res[nVar];
  double* sm = B.implicit ? summ + (size_t)b * visc_summary_size<NS, NDIM>() : nullptr;
  const int rc = visc_edge<NS, NDIM>(m, B.vp, a, g, sk, Normal, res, SummRef{sm, 1}, Scr{scr_all + threadIdx.x},
                                     false);
  bad = false;
#pragma unroll
  for (int v = 0; v < nVar; ++v) {
    bad |= isnan(res[v]);
    resv[(size_t)b * nVar + v] = res[v];
  }
  if (rc != ERR_NONE || e != ERR_NONE) set_err(err, (rc == ERR_RANGE || e == ERR_RANGE) ? ERR_RANGE : ERR_NAN, i);
  else if (bad) set_err(err, ERR_NAN, i);
}

// Viscous boundary Jacobians, 16-lane team per weak vertex (lane = column), as k_visc_jac.
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) void k_bc_visc_jac(int NW, const int32_t* __restrict__ weak,
                                                        const int32_t* __restrict__ bnode,
                                                        const double* __restrict__ dTdU, const double* __restrict__ sv,
                                                        const double* __restrict__ summ, DevMech m, ViscParams P,
                                                        double* __restrict__ jacv) {
  constexpr int nVar = NS + NDIM + 2, nVar2 = nVar * nVar;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int q = gt / 16, c = gt % 16;
  if (q >= NW) return;  // whole teams exit together (NW * 16 threads)
  const int b = weak[q], i = bnode[b];
  const int cc = c < nVar ? c : 0;
  const double sib = dTdU[(size_t)i * nVar + cc], sjb = sv[(size_t)b * nVar + cc];
  double* Ji = jacv + (size_t)b * 2 * nVar2;
  visc_jac_column<NS, NDIM>(m, P, SummCRef{summ + (size_t)b * visc_summary_size<NS, NDIM>(), 1}, sib, sjb, c, c, Ji,
                            Ji + nVar2);
}

// CSysMatrix::DeleteValsRowi (Common/src/matrix_structure.cpp:483-495) for scalar row r of block row i.
__device__ inline void delete_row(int i, int r, int nb, const int32_t* rp, const int32_t* col, double* A) {
  for (int k = rp[i]; k < rp[i + 1]; ++k) {
    double* blk = A + (size_t)k * nb * nb + r * nb;
    for (int c = 0; c < nb; ++c) blk[c] = 0.0;
    if (col[k] == i) blk[r] = 1.0;
  }
}

// One workgroup per owned boundary point, lane q = entry q of the diagonal block (lanes < nVar also own the
// residual entries): the reference's per-vertex updates in Space_Integration order. Every entry sees its own
// sequence of AddBlock / SubtractBlock operations, so the lanes are independent except around DeleteValsRowi,
// which spans the whole BSR row.
constexpr int kApplyBlock = 256;  // >= nVar^2 (nVar <= 14: Ns = 9 in 3-D)
template <int NS, int NDIM>
__global__ __launch_bounds__(kApplyBlock) void k_bc_apply(const int32_t* __restrict__ bn,
                                                          const int32_t* __restrict__ bn_ptr,
                                                          const int32_t* __restrict__ bn_vtx,
                                                          const int32_t* __restrict__ bmark,
                                                          const int32_t* __restrict__ bpn,
                                                          const double* __restrict__ bnrm,
                                                          const int32_t* __restrict__ mkind,
                                                          const double* __restrict__ mdata, BCDev B, DevMech m,
                                                          const double* __restrict__ coord,
                                                          const double* __restrict__ U, const double* __restrict__ V,
                                                          const double* __restrict__ kappa,
                                                          const double* __restrict__ dTdU,
                                                          const double* __restrict__ eddy,
                                                          const double* __restrict__ dPdU,
                                                          const double* __restrict__ tke,
                                                          const int32_t* __restrict__ rp,
                                                          const int32_t* __restrict__ col,
                                                          const int64_t* __restrict__ diag,
                                                          const double* __restrict__ resc,
                                                          const double* __restrict__ resv,
                                                          const double* __restrict__ jacc,
                                                          const double* __restrict__ jacv, double* __restrict__ R,
                                                          double* __restrict__ A, int* err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5, nVar2 = nVar * nVar, E_ = NDIM + 1;
  static_assert(nVar2 <= kApplyBlock, "one lane per diagonal-block entry");
  const int t = blockIdx.x, q = threadIdx.x;
  const int i = bn[t];
  const int a = q / nVar, c = q - a * nVar;
  const bool ent = q < nVar2;
  double* Ri = R + (size_t)i * nVar;
  double* D = A ? A + diag[i] * nVar2 : nullptr;
  double r = (q < nVar) ? Ri[q] : 0.0;
  double dq = (D && ent) ? D[q] : 0.0;
  // weak markers (inlet, outlet, Euler wall) in marker / vertex order
  for (int k = bn_ptr[t]; k < bn_ptr[t + 1]; ++k) {
    const int b = bn_vtx[k];
    const int kind = mkind[bmark[b]];
    if (kind == RX_BC_EULER) {
      // BC_Euler_Wall (:2881-2966): Residual[RHOVX + d] = P n_d A + 2/3 rho k n_d A with n = -Normal / Area,
      // LinSysRes.AddBlock (every entry, zeros included); Jacobian_i momentum rows dPdU[c] n_d A, AddBlock
      double Area = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) Area += bnrm[(size_t)b * NDIM + d] * bnrm[(size_t)b * NDIM + d];
      Area = sqrt(Area);
      const double Pi = V[(size_t)i * nPV + NDIM + 1], rho = V[(size_t)i * nPV + NDIM + 2];
      const double ke = B.rans ? tke[i] : 0.0;
      if (q < nVar) {
        double res = 0.0;
        if (q >= 1 && q <= NDIM) {
          const double un = -bnrm[(size_t)b * NDIM + q - 1] / Area;
          res = Pi * un * Area + 2.0 / 3.0 * rho * ke * un * Area;
        }
        r += res;
      }
      if (D && ent) {
        double J = 0.0;
        if (a >= 1 && a <= NDIM) J = dPdU[(size_t)i * nVar + c] * (-bnrm[(size_t)b * NDIM + a - 1] / Area) * Area;
        dq += J;
      }
      continue;
    }
    if (kind != RX_BC_INLET && kind != RX_BC_OUTLET && kind != RX_BC_SUP_INLET && kind != RX_BC_SUP_OUTLET) continue;
    if (q < nVar) {
      r += resc[(size_t)b * nVar + q];
      r -= resv[(size_t)b * nVar + q];
    }
    if (D && ent) {
      dq += jacc[(size_t)b * nVar2 + q];
      dq -= jacv[(size_t)b * 2 * nVar2 + q];
    }
  }
  // strong markers: BC_Isothermal_Wall (:5441-5710), BC_HeatFlux_Wall (:5717-5911)
  bool walled = false;
  for (int k = bn_ptr[t]; k < bn_ptr[t + 1]; ++k) {
    const int b = bn_vtx[k];
    const int mk = bmark[b];
    if (mkind[mk] == RX_BC_HEATFLUX) {
      // SetVelocity_Old(0) (in the update, bc_wall), momentum rows of the residual zeroed, Res_Conv = 0 added,
      // Res_Visc[RHOE] = q A subtracted, then DeleteValsRowi on the momentum rows (no Jacobian_i without grid motion)
      walled = true;
      double Area = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) Area += bnrm[(size_t)b * NDIM + d] * bnrm[(size_t)b * NDIM + d];
      Area = sqrt(Area);
      const double resE = mdata[(size_t)mk * B.W + 1] * Area;
      if (q < nVar) {
        if (q >= 1 && q <= NDIM) r = 0.0;
        r += 0.0;
        r -= (q == E_) ? resE : 0.0;
      }
      if (D && ent && a >= 1 && a <= NDIM) dq = (a == c) ? 1.0 : 0.0;
      continue;
    }
    if (mkind[mk] != RX_BC_ISOTHERMAL) continue;
    walled = true;
    const double* md = mdata + (size_t)mk * B.W;
    int e = ERR_NONE;
    const double Twall = md[1] / B.T_ref;
    const double dim_temp = Twall * B.T_ref;
    double Area = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Area += bnrm[(size_t)b * NDIM + d] * bnrm[(size_t)b * NDIM + d];
    Area = sqrt(Area);
    const int pn = bpn[b];
    double dij = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      const double x = coord[(size_t)pn * NDIM + d] - coord[(size_t)i * NDIM + d];
      dij += x * x;
    }
    dij = sqrt(dij);
    const double Tj = V[(size_t)pn * nPV];
    const double ktr = kappa[i];
    double turb_closure = 0.0, turb_ktr = 0.0;
    if (B.rans) {
      const double eddy_v = eddy[i];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double cps = spline(m, P_CP, s, dim_temp, &e) / m.mm[s];
        turb_closure += eddy_v / B.vp.Pr_t * cps * U[(size_t)i * nVar + NDIM + 2 + s] * (Twall - Tj) / dij;
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double cps = spline(m, P_CP, s, dim_temp, &e) / m.mm[s];
        turb_ktr += eddy_v / (B.vp.Pr_t) * cps * U[(size_t)i * nVar + NDIM + 2 + s];
      }
    }
    const double dTdn = +(Twall - Tj) / dij;
    const double resE = ktr * dTdn * Area + turb_closure * Area;
    if (q < nVar) {
      if (q >= 1 && q <= NDIM) r = 0.0;       // LinSysRes.SetBlock_Zero(iPoint, RHOVX + iDim)
      r += 0.0;                                // AddBlock(Res_Conv = 0)
      r -= (q == E_) ? resE : 0.0;             // SubtractBlock(Res_Visc)
    }
    if (D && ent) {
      // Jacobian_i is zero except row RHOE (:5576-5579); momentum rows are deleted below
      const double* S = dTdU + (size_t)pn * nVar;
      double J = 0.0;
      if (a == E_) {
        if (c == 0) J = -ktr * S[0] / dij * Area;
        else if (c == E_) J = -ktr * S[E_] / dij * Area - turb_ktr * S[E_] / dij * Area;
        else if (c >= NDIM + 2) J = -ktr * S[c] / dij * Area;
      }
      if (a >= 1 && a <= NDIM) dq = (a == c) ? 1.0 : 0.0;  // DeleteValsRowi before the SubtractBlock
      dq -= J;
      if (a >= 1 && a <= NDIM) dq = (a == c) ? 1.0 : 0.0;  // and after it (:5703-5708)
    }
    if (e != ERR_NONE && q == 0) set_err(err, ERR_RANGE, i);
  }
  if (q < nVar) Ri[q] = r;
  if (D && ent) D[q] = dq;
  if (D && walled) {
    // DeleteValsRowi on the off-diagonal blocks of the momentum rows (the diagonal block is done above)
    const int k0 = rp[i], nk = rp[i + 1] - k0;
    for (int w = q; w < nk * NDIM * nVar; w += kApplyBlock) {
      const int kb = w / (NDIM * nVar), rem = w - kb * (NDIM * nVar);
      const int rr = 1 + rem / nVar, cc = rem % nVar;
      const int k = k0 + kb;
      if (col[k] != i) A[(size_t)k * nVar2 + rr * nVar + cc] = 0.0;
    }
  }
}

// SST BCs, one thread per owned boundary point: BC_Inlet / BC_Outlet (weak, marker order), then
// BC_Isothermal_Wall (strong).
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_sst_bc(int nbn, const int32_t* __restrict__ bn,
                                                   const int32_t* __restrict__ bn_ptr,
                                                   const int32_t* __restrict__ bn_vtx,
                                                   const int32_t* __restrict__ bmark, const int32_t* __restrict__ bpn,
                                                   const double* __restrict__ bnrm, const int32_t* __restrict__ mkind,
                                                   double kine_inf, double omega_inf, double sk1, double sk2,
                                                   double so1, double so2, double beta1,
                                                   const double* __restrict__ coord, const double* __restrict__ V,
                                                   int nPV, const double* __restrict__ mu,
                                                   const double* __restrict__ eddy, const double* __restrict__ charac,
                                                   const double* __restrict__ TG, const double* __restrict__ F1,
                                                   const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                   const int64_t* __restrict__ diag, double* __restrict__ T,
                                                   double* __restrict__ R, double* __restrict__ A) {
  constexpr int RHO = NDIM + 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nbn) return;
  const int i = bn[t];
  double* D = A ? A + diag[i] * 4 : nullptr;
  for (int k = bn_ptr[t]; k < bn_ptr[t + 1]; ++k) {
    const int b = bn_vtx[k];
    const int kind = mkind[bmark[b]];
    if (kind != RX_BC_INLET && kind != RX_BC_OUTLET) continue;
    double Normal[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Normal[d] = -bnrm[(size_t)b * NDIM + d];
    const double* Vi = V + (size_t)i * nPV;
    const double* Vg = charac + (size_t)b * nPV;
    const double Ti0 = T[2 * (size_t)i], Ti1 = T[2 * (size_t)i + 1];
    const double Tg0 = kind == RX_BC_INLET ? kine_inf : Ti0, Tg1 = kind == RX_BC_INLET ? omega_inf : Ti1;
    // CUpwSca_TurbSST
    double q = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) q += 0.5 * (Vi[d + 1] + Vg[d + 1]) * Normal[d];
    const double a0 = 0.5 * (q + fabs(q)), a1 = 0.5 * (q - fabs(q));
    const double ri = Vi[RHO], rj = Vg[RHO];
    R[2 * (size_t)i] += a0 * ri * Ti0 + a1 * rj * Tg0;
    R[2 * (size_t)i + 1] += a0 * ri * Ti1 + a1 * rj * Tg1;
    if (D) {
      D[0] += a0;
      D[1] += 0.0;
      D[2] += 0.0;
      D[3] += a0;
    }
    // CAvgGrad_TurbSST: node i's gradients, F1, mu, eddy viscosity on both sides
    const double f1 = F1[i];
    const double sk = f1 * sk1 + (1.0 - f1) * sk2, so = f1 * so1 + (1.0 - f1) * so2;
    const double dik = mu[i] + sk * eddy[i], dio = mu[i] + so * eddy[i];
    const double dk = 0.5 * (dik + dik), dw = 0.5 * (dio + dio);
    const int pn = bpn[b];
    double dist2 = 0.0, proj = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      const double ev = coord[(size_t)pn * NDIM + d] - coord[(size_t)i * NDIM + d];
      dist2 += ev * ev;
      proj += ev * Normal[d];
    }
    if (dist2 == 0.0) proj = 0.0; else proj = proj / dist2;
    double c0 = 0.0, c1 = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      const double g0 = TG[((size_t)i * 2) * NDIM + d], g1 = TG[((size_t)i * 2 + 1) * NDIM + d];
      c0 += 0.5 * (g0 + g0) * Normal[d];
      c1 += 0.5 * (g1 + g1) * Normal[d];
    }
    R[2 * (size_t)i] -= dk * c0;
    R[2 * (size_t)i + 1] -= dw * c1;
    if (D) {
      D[0] -= -dk * proj / ri;
      D[1] -= 0.0;
      D[2] -= 0.0;
      D[3] -= -dw * proj / ri;
    }
  }
  for (int k = bn_ptr[t]; k < bn_ptr[t + 1]; ++k) {
    const int b = bn_vtx[k];
    // BC_Isothermal_Wall (:3142-3196) and BC_HeatFlux_Wall (:3087-3140) set the same wall values
    if (mkind[bmark[b]] != RX_BC_ISOTHERMAL && mkind[bmark[b]] != RX_BC_HEATFLUX) continue;
    const int j = bpn[b];
    double distance = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      const double x = coord[(size_t)i * NDIM + d] - coord[(size_t)j * NDIM + d];
      distance += x * x;
    }
    distance = sqrt(distance);
    const double density = V[(size_t)j * nPV + RHO], lam = mu[j];
    T[2 * (size_t)i] = 0.0;
    T[2 * (size_t)i + 1] = 60.0 * lam / (density * beta1 * distance * distance);
    R[2 * (size_t)i] = 0.0;
    R[2 * (size_t)i + 1] = 0.0;
    if (A) {
      delete_row(i, 0, 2, rp, col, A);
      delete_row(i, 1, 2, rp, col, A);
    }
  }
}

#define RX_ND_SWITCH(nd, CALL)                   \
  if ((nd) == 2) {                               \
    constexpr int ND_ = 2;                       \
    CALL;                                        \
  } else if ((nd) == 3) {                        \
    constexpr int ND_ = 3;                       \
    CALL;                                        \
  } else {                                       \
    return RX_ERR_ARG;                           \
  }

template <typename T>
int dup(rx_ctx* ctx, T** d, const T* h, size_t n) {
  if (*d) (void)hipFree(*d);
  *d = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(d), sizeof(T) * std::max<size_t>(n, 1)) != hipSuccess) return RX_ERR_HIP;
  if (n && hipMemcpyAsync(*d, h, sizeof(T) * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return RX_ERR_HIP;
  return RX_OK;
}
template <typename T>
int dzero(rx_ctx* ctx, T** d, size_t n) {
  if (*d) (void)hipFree(*d);
  *d = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(d), sizeof(T) * std::max<size_t>(n, 1)) != hipSuccess) return RX_ERR_HIP;
  if (hipMemsetAsync(*d, 0, sizeof(T) * std::max<size_t>(n, 1), ctx->stream) != hipSuccess) return RX_ERR_HIP;
  return RX_OK;
}

BCDev bc_dev(const rx_ctx* fl) {
  BCDev B;
  B.inlet_kind = fl->bc_inlet_kind;
  B.W = fl->bc_W;
  B.implicit = fl->cfg.implicit;
  B.rans = fl->cfg.rans;
  B.tke_inf = fl->bc_tke_inf;
  B.kine_inf = fl->bc_kine_inf;
  B.omega_inf = fl->bc_omega_inf;
  B.T_ref = fl->cfg.T_ref;
  B.E_ref = fl->cfg.E_ref;
  B.R_ref = fl->cfg.R_ref;
  B.P_ref = fl->cfg.p_ref;
  B.vel_ref = fl->cfg.vel_ref;
  B.rho_ref = fl->cfg.rho_ref;
  B.mach_inf = fl->cfg.mach_inf;
  B.vp = ViscParams{fl->cfg.T_ref, fl->cfg.E_ref, fl->cfg.R_ref, fl->cfg.prandtl_turb, fl->cfg.lewis_turb,
                    fl->cfg.rans, fl->cfg.implicit};
  return B;
}

}  // namespace

#if RX_NS
int RX_NSFN(rx_bc_launch_weak)(rx_ctx* ctx, hipStream_t st) {
  if (ctx->bc_nweak <= 0) return RX_OK;
  const BCDev B = bc_dev(ctx);
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_bc_weak<NS_, ND_><<<blocks(ctx->bc_nweak, 64), 64, 0, st>>>(
                            ctx->bc_nweak, ctx->bc_weak, ctx->bc_node, ctx->bc_pn, ctx->bc_mark, ctx->bc_nrm,
                            ctx->bc_mkind, ctx->bc_mdata, B, ctx->mech, ctx->coord, ctx->f[RX_F_V], ctx->f[RX_F_DPDU],
                            ctx->f[RX_F_DTDU], ctx->f[RX_F_GRAD], ctx->f[RX_F_MU], ctx->f[RX_F_KAPPA],
                            ctx->f[RX_F_DIJ], ctx->f[RX_F_TKE], ctx->f[RX_F_MUT], ctx->f[RX_F_SIGMAK],
                            ctx->f[RX_F_GRADK], ctx->bc_charac, ctx->bc_resc, ctx->bc_resv, ctx->bc_jacc,
                            ctx->bc_summ, ctx->bc_sv, ctx->err)));
  RX_HIP(hipGetLastError());
  if (ctx->cfg.implicit) {
    RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_bc_visc_jac<NS_, ND_><<<blocks((int64_t)ctx->bc_nweak * 16), kBlock, 0, st>>>(
                              ctx->bc_nweak, ctx->bc_weak, ctx->bc_node, ctx->f[RX_F_DTDU], ctx->bc_sv, ctx->bc_summ,
                              ctx->mech, B.vp, ctx->bc_jacv)));
    RX_HIP(hipGetLastError());
  }
  return RX_OK;
}

// the strong conditions and the weak markers' fluxes applied per owned boundary point (k_bc_apply)
int RX_NSFN(rx_bc_apply)(rx_ctx* ctx) {
  const BCDev B = bc_dev(ctx);
  double* A = ctx->cfg.implicit ? ctx->f[RX_F_JAC] : nullptr;
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_bc_apply<NS_, ND_><<<ctx->bc_nbn, kApplyBlock, 0, ctx->stream>>>(
                            ctx->bc_bn, ctx->bc_bn_ptr, ctx->bc_bn_vtx, ctx->bc_mark, ctx->bc_pn,
                            ctx->bc_nrm, ctx->bc_mkind, ctx->bc_mdata, B, ctx->mech, ctx->coord, ctx->f[RX_F_U],
                            ctx->f[RX_F_V], ctx->f[RX_F_KAPPA], ctx->f[RX_F_DTDU], ctx->f[RX_F_EDDY],
                            ctx->f[RX_F_DPDU], ctx->f[RX_F_TKE], ctx->rp,
                            ctx->col, ctx->diag, ctx->bc_resc, ctx->bc_resv, ctx->bc_jacc, ctx->bc_jacv,
                            ctx->f[RX_F_RES], A, ctx->err)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}
#else
RX_NS_DISPATCH(rx_bc_launch_weak, (rx_ctx * ctx, hipStream_t st), (ctx, st))
RX_NS_DISPATCH(rx_bc_apply, (rx_ctx * ctx), (ctx))

void rx_bc_free(rx_ctx* ctx) {
  void* ps[] = {ctx->bc_mkind, ctx->bc_mdata, ctx->bc_node,  ctx->bc_pn,      ctx->bc_mark,  ctx->bc_nrm,
                ctx->bc_weak,  ctx->bc_bn,    ctx->bc_bn_ptr, ctx->bc_bn_vtx, ctx->bc_wall,  ctx->bc_charac,
                ctx->bc_resc,  ctx->bc_resv,  ctx->bc_jacc,  ctx->bc_jacv,    ctx->bc_summ,  ctx->bc_sv};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  ctx->bc_mkind = nullptr;
  ctx->bc_mdata = ctx->bc_nrm = ctx->bc_charac = ctx->bc_resc = ctx->bc_resv = ctx->bc_jacc = ctx->bc_jacv =
      ctx->bc_summ = ctx->bc_sv = nullptr;
  ctx->bc_node = ctx->bc_pn = ctx->bc_mark = ctx->bc_weak = ctx->bc_bn = ctx->bc_bn_ptr = ctx->bc_bn_vtx = nullptr;
  ctx->bc_wall = nullptr;
  if (ctx->bc_stream) {
    (void)hipStreamSynchronize(ctx->bc_stream);
    (void)hipStreamDestroy(ctx->bc_stream);
  }
  if (ctx->bc_fork) (void)hipEventDestroy(ctx->bc_fork);
  if (ctx->bc_join) (void)hipEventDestroy(ctx->bc_join);
  ctx->bc_stream = nullptr;
  ctx->bc_fork = ctx->bc_join = nullptr;
  ctx->bc_pending = false;
  ctx->bc_on = false;
}

extern "C" {

int rx_bc_set(rx_ctx* ctx, const rx_bc_desc* bc) {
  if (!ctx || ctx->kind != RX_KIND_FLOW || !bc || bc->n_marker <= 0 || !bc->kind || !bc->data) return RX_ERR_ARG;
  const int64_t NB = ctx->NB;
  if (NB > 0 && !bc->normal_neighbor) return RX_ERR_ARG;
  if (bc->inlet_kind < RX_INLET_TOTAL_CONDITIONS || bc->inlet_kind > RX_INLET_TEMPERATURE_IMPOSE) return RX_ERR_ARG;
  const int nM = bc->n_marker, W = 6 + ctx->ns, nd = ctx->nDim;
  for (int k = 0; k < nM; ++k) {
    if (bc->kind[k] < RX_BC_NONE || bc->kind[k] > RX_BC_SUP_OUTLET) return RX_ERR_ARG;
    // the reference's supersonic BCs give their viscous numerics no turbulence quantities (BC_Inlet's MANGOTURB
    // add-on, solver_direct_reactive.cpp:3607-3621, has no counterpart at :3131-3203 / :3743-3788): under SST they read
    // whatever the previous boundary call left in that object, so only laminar contexts take them
    if ((bc->kind[k] == RX_BC_SUP_INLET || bc->kind[k] == RX_BC_SUP_OUTLET) && ctx->cfg.rans) return RX_ERR_UNSUPPORTED;
  }
  std::vector<int32_t> node(NB), pn(NB), mark(NB), weak;
  std::vector<uint8_t> wall(ctx->N, 0);
  for (int64_t b = 0; b < NB; ++b) {
    const int64_t mk = ctx->h_bvert[2 * b], p = ctx->h_bvert[2 * b + 1], q = bc->normal_neighbor[b];
    if (mk < 0 || mk >= nM || q < 0 || q >= ctx->N) return RX_ERR_ARG;
    node[b] = (int32_t)p;
    pn[b] = (int32_t)q;
    mark[b] = (int32_t)mk;
    const int kd = bc->kind[mk];
    if ((kd == RX_BC_INLET || kd == RX_BC_OUTLET || kd == RX_BC_SUP_INLET || kd == RX_BC_SUP_OUTLET) && p < ctx->Nd)
      weak.push_back((int32_t)b);
    if ((kd == RX_BC_ISOTHERMAL || kd == RX_BC_HEATFLUX) && p < ctx->Nd) wall[p] = 1;
  }
  // owned boundary points and their vertices in (marker, vertex) = input order; vertices of RX_BC_NONE markers
  // (symmetry planes: the reactive and SST solvers act on them in neither k_bc_apply nor k_sst_bc) are left out,
  // so a point on none but such markers gets no workgroup (C5: the two symmetry planes, 100k points)
  std::vector<int32_t> bn, bn_ptr(1, 0), bn_vtx;
  {
    std::vector<std::vector<int32_t>> per(ctx->N);
    for (int64_t b = 0; b < NB; ++b)
      if (node[b] < ctx->Nd && bc->kind[mark[b]] != RX_BC_NONE) per[node[b]].push_back((int32_t)b);
    for (int64_t p = 0; p < ctx->Nd; ++p)
      if (!per[p].empty()) {
        bn.push_back((int32_t)p);
        bn_vtx.insert(bn_vtx.end(), per[p].begin(), per[p].end());
        bn_ptr.push_back((int32_t)bn_vtx.size());
      }
  }
  rx_bc_free(ctx);
  rx_graph_reset(ctx);  // the captured solve's update reads bc_wall
  ++ctx->bc_epoch;      // and the SST context's graph the flow's markers
  ctx->bc_nmark = nM;
  ctx->bc_W = W;
  ctx->bc_inlet_kind = bc->inlet_kind;
  ctx->bc_tke_inf = bc->tke_inf;
  ctx->bc_kine_inf = bc->kine_inf;
  ctx->bc_omega_inf = bc->omega_inf;
  ctx->bc_nweak = (int)weak.size();
  ctx->bc_nbn = (int)bn.size();
  std::vector<double> md((size_t)nM * W);
  std::copy(bc->data, bc->data + (size_t)nM * W, md.begin());
  const int nv = ctx->nVar, nPV = ctx->nPV;
  const size_t nb1 = (size_t)std::max<int64_t>(NB, 1);
  int rc = RX_OK;
  if (!rc) rc = dup(ctx, &ctx->bc_mkind, bc->kind, nM);
  if (!rc) rc = dup(ctx, &ctx->bc_mdata, md.data(), md.size());
  if (!rc) rc = dup(ctx, &ctx->bc_node, node.data(), NB);
  if (!rc) rc = dup(ctx, &ctx->bc_pn, pn.data(), NB);
  if (!rc) rc = dup(ctx, &ctx->bc_mark, mark.data(), NB);
  if (!rc) rc = dup(ctx, &ctx->bc_nrm, ctx->h_bnormal.data(), (size_t)NB * nd);
  if (!rc) rc = dup(ctx, &ctx->bc_weak, weak.data(), weak.size());
  if (!rc) rc = dup(ctx, &ctx->bc_bn, bn.data(), bn.size());
  if (!rc) rc = dup(ctx, &ctx->bc_bn_ptr, bn_ptr.data(), bn_ptr.size());
  if (!rc) rc = dup(ctx, &ctx->bc_bn_vtx, bn_vtx.data(), bn_vtx.size());
  if (!rc) rc = dup(ctx, &ctx->bc_wall, wall.data(), wall.size());
  if (!rc) rc = dzero(ctx, &ctx->bc_charac, nb1 * nPV);
  if (!rc) rc = dzero(ctx, &ctx->bc_resc, nb1 * nv);
  if (!rc) rc = dzero(ctx, &ctx->bc_resv, nb1 * nv);
  if (!rc && ctx->cfg.implicit) rc = dzero(ctx, &ctx->bc_jacc, nb1 * nv * nv);
  if (!rc && ctx->cfg.implicit) rc = dzero(ctx, &ctx->bc_jacv, nb1 * 2 * nv * nv);
  if (!rc && ctx->cfg.implicit) rc = dzero(ctx, &ctx->bc_summ, nb1 * (24 + 9 * ctx->ns));
  if (!rc && ctx->cfg.implicit) rc = dzero(ctx, &ctx->bc_sv, nb1 * nv);
  if (!rc && hipStreamCreateWithFlags(&ctx->bc_stream, hipStreamNonBlocking) != hipSuccess) rc = RX_ERR_HIP;
  if (!rc && hipEventCreateWithFlags(&ctx->bc_fork, hipEventDisableTiming) != hipSuccess) rc = RX_ERR_HIP;
  if (!rc && hipEventCreateWithFlags(&ctx->bc_join, hipEventDisableTiming) != hipSuccess) rc = RX_ERR_HIP;
  if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = RX_ERR_HIP;
  if (rc) {
    rx_bc_free(ctx);
    return rc;
  }
  ctx->bc_on = true;
  return RX_OK;
}

int rx_bc_flow(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW || !ctx->bc_on) return RX_ERR_ARG;
  int rc = rx_settle_u(ctx);  // the walls write U
  if (!rc && ctx->cfg.implicit) rc = rx_ensure_assembled(ctx);
  if (rc) return rc;
  RxPhase ph(ctx, RX_K_BC);
  if (ctx->bc_pending) {  // boundary fluxes launched by rx_residual_zero on the side stream
    RX_HIP(hipStreamWaitEvent(ctx->stream, ctx->bc_join, 0));
    ctx->bc_pending = false;
  } else if ((rc = rx_bc_launch_weak(ctx, ctx->stream))) {
    return rc;
  }
  if (ctx->bc_nbn > 0) return rx_bc_apply(ctx);
  return RX_OK;
}

int rx_bc_sst(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_SST || !ctx->flow || !ctx->flow->bc_on) return RX_ERR_ARG;
  if (int rc0 = rx_settle_u(ctx)) return rc0;
  const rx_ctx* fl = ctx->flow;
  RxPhase ph(ctx, RX_K_SST_BC);
  if (fl->bc_pending) RX_HIP(hipStreamWaitEvent(ctx->stream, fl->bc_join, 0));  // ghost states of this iteration
  if (fl->bc_nbn > 0) {
    const double sk1 = 0.85, sk2 = 1.0, so1 = 0.5, so2 = 0.856, beta1 = 0.075;  // CTurbSSTSolver constants
    RX_ND_SWITCH(ctx->nDim, (k_sst_bc<ND_><<<blocks(fl->bc_nbn), kBlock, 0, ctx->stream>>>(
        fl->bc_nbn, fl->bc_bn, fl->bc_bn_ptr, fl->bc_bn_vtx, fl->bc_mark, fl->bc_pn, fl->bc_nrm, fl->bc_mkind,
        fl->bc_kine_inf, fl->bc_omega_inf, sk1, sk2, so1, so2, beta1, ctx->coord, fl->f[RX_F_V], fl->nPV,
        fl->f[RX_F_MU], fl->f[RX_F_EDDY], fl->bc_charac, ctx->f[RX_F_GRAD], ctx->f[RX_F_F1], ctx->rp, ctx->col,
        ctx->diag, ctx->f[RX_F_U], ctx->f[RX_F_RES], ctx->cfg.implicit ? ctx->f[RX_F_JAC] : nullptr)));
    RX_HIP(hipGetLastError());
  }
  return RX_OK;
}

}  // extern "C"
#endif  // RX_NS
