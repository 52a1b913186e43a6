// rx_kernels.hip — residual-side kernels of the reactive-RANS hot path for gfx950.
//
// Determinism: every per-node accumulation is a gather over the node's incident edges in
// increasing edge id, which is exactly the order the reference's sequential edge loop applies
// its scatters (LinSysRes.AddBlock(i) / SubtractBlock(j), solver_direct_reactive.cpp:2759-2772,
// 5374-5381). No atomics: results are bitwise reproducible run to run.
#include <hip/hip_runtime.h>

#include <cstdio>

#include <cstdlib>

#include "rx_chem.h"
#include "rx_ctx.h"
#include "rx_species.h"
#include "rx_visc.h"

using namespace rx;

namespace {

constexpr int kBlock = 256;
// waves-per-SIMD targets of register-heavy kernels (build knobs; empty = the compiler's choice). Measured on one
// box at C3: 3 waves per SIMD take SetPrimitive_Variables 1.32 -> 1.22 ms per step (175 -> 157 VGPRs) and the
// source 0.57 -> 0.46 ms (180 -> 168 VGPRs, 12 B spilled); the AUSM edge kernel at 3 spills and slows 1.30 -> 2.06 ms.
#define RX_WPE(n) __attribute__((amdgpu_waves_per_eu(n)))
#ifndef RX_WPE_PRIM
#define RX_WPE_PRIM RX_WPE(3)
#endif
#ifndef RX_WPE_AUSM
#define RX_WPE_AUSM
#endif
#ifndef RX_WPE_SRC
#define RX_WPE_SRC RX_WPE(3)
#endif

__device__ inline void set_err(int* err, int code, int64_t idx) {
  if (atomicCAS(err, 0, code) == 0) err[1] = (int)idx;
}

// ------------------------------------------------------------------------------------------------
// a1/a2 explicit: node-centric AUSM gather. Each node recomputes the flux of its incident edges
// (with the edge's own node order, so both endpoints see bitwise-identical fluxes) and applies
// +F (first node) / -F (second node) in edge order.
// ------------------------------------------------------------------------------------------------
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) void k_ausm_node(int N, const int32_t* __restrict__ adj_ptr,
                                                      const int32_t* __restrict__ adj,
                                                      const int32_t* __restrict__ edges,
                                                      const double* __restrict__ normal, const double* __restrict__ V,
                                                      const double* __restrict__ VR, double mInfty,
                                                      double* __restrict__ R, int* err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double acc[nVar];
#pragma unroll
  for (int v = 0; v < nVar; ++v) acc[v] = R[(size_t)i * nVar + v];
  double Vs[nPV], Vo[nPV];
#pragma unroll
  for (int v = 0; v < nPV; ++v) Vs[v] = V[(size_t)i * nPV + v];
  const int k0 = adj_ptr[i], k1 = adj_ptr[i + 1];
  bool bad = false;
  for (int k = k0; k < k1; ++k) {
    const int a = adj[k];
    const int e = a >> 1;
    const int side = a & 1;
    const int other = edges[2 * e + (side ^ 1)];
    if (VR) {  // second order: the edge's reconstructed states (k_muscl_edge), [2e] node 0, [2e+1] node 1
#pragma unroll
      for (int v = 0; v < nPV; ++v) {
        Vs[v] = VR[(2 * (size_t)e + side) * nPV + v];
        Vo[v] = VR[(2 * (size_t)e + (side ^ 1)) * nPV + v];
      }
    } else {
#pragma unroll
      for (int v = 0; v < nPV; ++v) Vo[v] = V[(size_t)other * nPV + v];
    }
    double nrm[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) nrm[d] = normal[(size_t)e * NDIM + d];
    const double* V0 = side ? Vo : Vs;
    const double* V1 = side ? Vs : Vo;
    AusmEdge s;
    ausm_scalars<NDIM>(V0, V1, nrm, mInfty, s);
#pragma unroll
    for (int v = 0; v < nVar; ++v) {
      const double r = ausm_res<NDIM>(s, V0, V1, v);
      bad |= isnan(r);
      acc[v] = side ? acc[v] - r : acc[v] + r;
    }
  }
#pragma unroll
  for (int v = 0; v < nVar; ++v) R[(size_t)i * nVar + v] = acc[v];
  if (bad) set_err(err, ERR_NAN, i);
}

// next-1: CReactiveEulerSolver::SetPrimitive_Variables (solver_direct_reactive.cpp:985-1040), one thread per
// point: CReactiveNSVariable::SetPrimVar(eddy, k) (variable_direct_reactive.cpp:1188-1228) ->
// CReactiveEulerVariable::SetPrimVar (:292-330): Cons2PrimVar (:550-778; secant from the previous T, then
// the bisection fallbacks), Cp from the sound speed, CalcdTdU (:786-823), CalcdPdU (:829-853); transport
// ComputeEta / ComputeLambda / GetDij_SM (reacting_model_library.cpp:634-766) with the mechanism
// constants of DevMech. std::min/max as ternaries. ERR_CONV: the reference's "Convergence not achieved
// for bisection method" runtime_error.
struct PrimParams {
  double Tmin, Tmax, T_ref, E_ref, R_ref, P_ref, Visc_ref, Cond_ref, Vel_ref, Len_ref;
  int ext_iter, clip_temp, rans;
  int ignite, fuel, oxidizer;  // ignition branch active at this ext_iter (IGNITION and ext_iter < IGNITION_ITER)
  double T_ign;
};

template <int NS>
__device__ inline double mix_h(const DevMech& m, double T, const double* Yc, int* err) {
  const SplineAt k = spline_at(m, T);
  double h = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) h += Yc[s] * rx_div(spline_k(m, P_H, s, T, k, err), mm_recip(m, s));
  return h;
}

// Cons2PrimVar on one point; V[T] holds the secant's start. Returns nonPhys; *fail on bisection failure.
template <int NS, int NDIM>
__device__ inline bool cons2prim_dev(const DevMech& m, const PrimParams& P, double* U, double* V, double val_ke,
                                     bool* fail) {
  constexpr int VX = 1, P_ = NDIM + 1, RHO = NDIM + 2, H_ = NDIM + 3, A_ = NDIM + 4, RHOS = NDIM + 5;
  constexpr int RHOVX_S = 1, RHOE_S = NDIM + 1, RHOS_S = NDIM + 2;
  bool nonPhys = false;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (U[RHOS_S + s] < 0.0) {
      U[RHOS_S + s] = 1.0e-30;
      nonPhys = true;
    }
  if (U[0] < kEPS) {
    V[RHO] = U[0] = kEPS;
    nonPhys = true;
  } else {
    V[RHO] = U[0];
  }
  double Ys[NS], Yc[NS];
  const Recip rrho = rx_recip(U[0]);  // rho's quotients share its reciprocal (rx_fdiv.h: the same doubles as `/`)
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    V[RHOS + s] = rx_div(U[RHOS_S + s], rrho);
    Ys[s] = V[RHOS + s];
    Yc[s] = Ys[s] < 0.0 ? 1.0e-30 : Ys[s];
  }
  double sy = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) sy += Ys[s];
  nonPhys = nonPhys || (fabs(sy - 1.0) > 0.1);
  const double rho = U[0];
  const double rhoE = U[RHOE_S] - rho * val_ke;
  double sqvel = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    V[VX + d] = rx_div(U[RHOVX_S + d], rrho);
    sqvel += V[VX + d] * V[VX + d];
  }
  const double Tmin = P.Tmin / P.T_ref, Tmax = P.Tmax / P.T_ref;
  double Rg = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) Rg += Yc[s] * rx_div(kR, mm_recip(m, s));
  const double Rgas = rx_div(Rg, rx_recip(P.R_ref));
  const double C1 = rx_div(-rhoE + 0.5 * rho * sqvel, rx_recip(rho * Rgas));
  const double C2 = rx_div(1.0, rx_recip(Rgas));
  const Recip rE = rx_recip(P.E_ref);
  const double old_temp = V[0];
  double T = V[0], Told = T + 1.0;
  bool conv = false;
  // h(Told) of an iteration is h(T) of the one before (Told = T there, the same product by T_ref): it is carried
  // instead of evaluated again; its error flag was the previous iteration's, which went to the bisection if set
  double hs_prev = 0.0;
  for (int it = 0; it < 7; ++it) {
    int e1 = ERR_NONE;
    const double hs_old = it == 0 ? rx_div(mix_h<NS>(m, Told * P.T_ref, Yc, &e1), rE) : hs_prev;
    const double hs = rx_div(mix_h<NS>(m, T * P.T_ref, Yc, &e1), rE);
    hs_prev = hs;
    if (e1 != ERR_NONE) {  // std::out_of_range inside the secant: bisection on [Tmin, Tmax], 10000 steps
      double Ta = Tmin, Tb = Tmax;
      for (int b = 0; b < 10000; ++b) {
        T = (Ta + Tb) / 2.0;
        int e2 = ERR_NONE;
        const double h2 = rx_div(mix_h<NS>(m, T * P.T_ref, Yc, &e2), rE);
        const double f = T - C1 - C2 * h2;
        if (fabs(f) < 1.0e-4) {
          conv = true;
          break;
        }
        if (f > 0) Ta = T;
        else Tb = T;
      }
      if (!conv) *fail = true;
      break;
    }
    const double f = T - C1 - C2 * hs;
    const double df = T - Told + C2 * (hs_old - hs);
    const double Tnew = T - rx_div(f * (T - Told), rx_recip(df));
    if (fabs(Tnew - T) < 1.0e-6) {
      conv = true;
      break;
    }
    Told = T;
    T = Tnew;
  }
  if (*fail) return nonPhys;
  if (conv) {
    V[0] = T;
  } else {
    bool bconv = false;
    double Ta = Tmin, Tb = Tmax;
    for (int b = 0; b < 32; ++b) {
      T = (Ta + Tb) / 2.0;
      int e2 = ERR_NONE;
      const double h2 = rx_div(mix_h<NS>(m, T * P.T_ref, Yc, &e2), rE);
      const double f = T - C1 - C2 * h2;
      if (fabs(f) < 1.0e-4) {
        V[0] = T;
        bconv = true;
        break;
      }
      if (f > 0) Ta = T;
      else Tb = T;
    }
    if (!bconv) {
      *fail = true;
      return nonPhys;
    }
  }
  if (P.ext_iter > 0 && P.clip_temp) {
    const double lo = 0.95 * old_temp, hi = 1.05 * old_temp;
    const double mx = (V[0] < lo) ? lo : V[0];
    V[0] = (hi < mx) ? hi : mx;
  }
  if (V[0] < Tmin) {
    V[0] = Tmin;
    nonPhys = true;
  } else if (V[0] > Tmax) {
    V[0] = Tmax;
    nonPhys = true;
  }
  T = V[0];
  V[P_] = rho * Rgas * T;
  if (V[P_] < kEPS) {
    V[P_] = kEPS;
    nonPhys = true;
  }
  const double dim_temp = T * P.T_ref;
  int e3 = ERR_NONE;
  double Cp = 0.0;
  const SplineAt kT = spline_at(m, dim_temp);
#pragma unroll
  for (int s = 0; s < NS; ++s) Cp += Yc[s] * rx_div(spline_k(m, P_CP, s, dim_temp, kT, &e3), mm_recip(m, s));
  const double gamma = rx_div(Cp, rx_recip(Cp - Rg));
  V[A_] = sqrt(rx_div(gamma * V[P_], rrho));
  if (V[A_] < kEPS) {
    V[A_] = kEPS;
    nonPhys = true;
  }
  V[H_] = rx_div(U[RHOE_S] + V[P_], rrho);
  if (e3 != ERR_NONE) *fail = true;
  return nonPhys;
}

#ifndef RX_PRIM_UNROLL
#define RX_PRIM_UNROLL 16  // >= NS: the species-pair loops fully unrolled (rolled: primitives 1.22 -> 1.43 ms at C3)
#endif
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) RX_WPE_PRIM void k_set_primitive(int lo, int N, DevMech m, PrimParams P, double* __restrict__ Ug,
                                                          double* __restrict__ Vg, const double* __restrict__ Uold,
                                                          const double* __restrict__ tke,
                                                          const double* __restrict__ mut, double* __restrict__ dPdU,
                                                          double* __restrict__ dTdU, double* __restrict__ mu,
                                                          double* __restrict__ kappa, double* __restrict__ Dij,
                                                          double* __restrict__ eddy, int* __restrict__ err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5;
  constexpr int VX = 1, P_ = NDIM + 1, RHO = NDIM + 2, A_ = NDIM + 4, RHOS = NDIM + 5;
  const int i = lo + (int)(blockIdx.x * blockDim.x + threadIdx.x);  // points [lo, N)
  if (i >= N) return;
  double U[nVar], V[nPV];
#pragma unroll
  for (int q = 0; q < nVar; ++q) U[q] = Ug[(size_t)i * nVar + q];
  V[0] = Vg[(size_t)i * nPV];
  const double ke = P.rans ? tke[i] : 0.0;
  bool fail = false;
  bool nonPhys = cons2prim_dev<NS, NDIM>(m, P, U, V, ke, &fail);
  if (!fail && nonPhys && P.ext_iter > 0 && Uold) {  // SetPrimVar :297-301: restart from Solution_Old
#pragma unroll
    for (int q = 0; q < nVar; ++q) U[q] = Uold[(size_t)i * nVar + q];
    if (cons2prim_dev<NS, NDIM>(m, P, U, V, ke, &fail)) fail = true;
  }
  if (fail) {
    if (atomicCAS(err, 0, ERR_CONV) == 0) err[1] = i;
    return;
  }
  if (nonPhys) atomicAdd(err + 2, 1);
#pragma unroll
  for (int q = 0; q < nVar; ++q) Ug[(size_t)i * nVar + q] = U[q];
#pragma unroll
  for (int q = 0; q < nPV; ++q) Vg[(size_t)i * nPV + q] = V[q];
  // Cp = ComputeCP_FromSoundSpeed(T, a, Ys) / R_ref
  const double dim_temp = V[0] * P.T_ref, dim_a = V[A_] * P.Vel_ref;
  double Ys[NS], Yc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    Ys[s] = V[RHOS + s];
    Yc[s] = Ys[s] < 0.0 ? 1.0e-30 : Ys[s];
  }
  double Rg = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) Rg += Yc[s] * rx_div(kR, mm_recip(m, s));
  // the divisors shared by several quotients below, each with its reciprocal (rx_fdiv.h: the same doubles as `/`)
  const Recip rR = rx_recip(P.R_ref), rE = rx_recip(P.E_ref);
  const double Cp = rx_div(rx_div(dim_a * dim_a * Rg, rx_recip(dim_a * dim_a - Rg * dim_temp)), rR);
  // CalcdTdU / CalcdPdU
  const double dim_cp = Cp * P.R_ref;
  const double Cv = rx_div(dim_cp - Rg, rR);
  const double rhoCv = V[RHO] * Cv;
  const Recip rcv = rx_recip(rhoCv);
  double sq = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) sq += V[VX + d] * V[VX + d];
  int e4 = ERR_NONE;
  const SplineAt kT = spline_at(m, dim_temp);  // the interval of dim_temp, shared by the H, MU and KAPPA rows below
  double dTdYs[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
    dTdYs[s] = rx_div(rx_div(spline_k(m, P_H, s, dim_temp, kT, &e4), mm_recip(m, s)) - rx_div(kR, mm_recip(m, s)) * dim_temp,
                      rE);
  double* dt = dTdU + (size_t)i * nVar;
  dt[0] = rx_div(0.5 * sq, rcv);
#pragma unroll
  for (int d = 0; d < NDIM; ++d) dt[1 + d] = rx_div(-V[VX + d], rcv);
  dt[NDIM + 1] = rx_div(1.0, rcv);
#pragma unroll
  for (int s = 0; s < NS; ++s) dt[NDIM + 2 + s] = rx_div(-dTdYs[s], rcv);
  const double Gamma = rx_div(dim_cp, rx_recip(dim_cp - Rg));
  double* dp = dPdU + (size_t)i * nVar;
  dp[0] = (Gamma - 1.0) * 0.5 * sq;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) dp[1 + d] = (1.0 - Gamma) * V[VX + d];
  dp[NDIM + 1] = Gamma - 1.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) dp[NDIM + 2 + s] = rx_div(rx_div(kR, mm_recip(m, s)), rR) * V[0] - (Gamma - 1.0) * dTdYs[s];
  // transport (CReactiveNSVariable::SetPrimVar)
  eddy[i] = P.rans ? mut[i] : 0.0;
  const double dim_press = V[P_] * P.P_ref / 101325.0;
  double visc[NS], cond[NS], yom[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    visc[s] = spline_k(m, P_MU, s, dim_temp, kT, &e4);
    cond[s] = spline_k(m, P_KAPPA, s, dim_temp, kT, &e4);
    yom[s] = rx_div(Yc[s], mm_recip(m, s));
  }
  Recip rvisc[NS];  // visc[b] divides visc[a] for every a (rx_fdiv.h)
#pragma unroll
  for (int b = 0; b < NS; ++b) rvisc[b] = rx_recip(visc[b]);
  // ComputeEta and ComputeLambda side by side: Wilke's factor f(a, b) is the same expression in both, so it is
  // evaluated once per pair; each phi still sums over b, and eta / lam over a, in the reference's order
  double yoml[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) yoml[s] = rx_div(Ys[s], mm_recip(m, s));  // ComputeLambda: the unclamped argument
  double eta = 0.0, lam = 0.0;
#pragma unroll RX_PRIM_UNROLL
  for (int a = 0; a < NS; ++a) {
    double phi = 0.0, phl = 0.0;
#pragma unroll
    for (int b = 0; b < NS; ++b) {
      const double f = 1.0 + sqrt(rx_div(visc[a], rvisc[b])) * m.pw25[a * NS + b];
      phi += rx_div(yom[b], phic_recip(m, a * NS + b)) * f * f;
      if (b != a) phl += rx_div(1.065 * yoml[b], phic_recip(m, a * NS + b)) * f * f;
    }
    phl += yoml[a];
    eta += rx_div(visc[a] * yom[a], rx_recip(phi));
    lam += rx_div(cond[a] * yoml[a], rx_recip(phl));
  }
  mu[i] = rx_div(eta, rx_recip(P.Visc_ref));
  kappa[i] = rx_div(lam, rx_recip(P.Cond_ref));
  const double pT = 1.0e-3 * pow175_cr(dim_temp);
  const double scale = P.Vel_ref * P.Len_ref * 1.0e4;
  const Recip rscale = rx_recip(scale);
  double* D = Dij + (size_t)i * NS * NS;
#pragma unroll RX_PRIM_UNROLL
  for (int a = 0; a < NS; ++a)
#pragma unroll
    for (int b = a; b < NS; ++b) {
      const double sv = m.dvs[a * NS + b];
      const double d = rx_div(pT, rx_recip(dim_press * m.mij[a * NS + b] * sv * sv));
      D[a * NS + b] = rx_div(d, rscale);
      D[b * NS + a] = rx_div(d, rscale);
    }
  if (e4 != ERR_NONE) {
    if (atomicCAS(err, 0, ERR_RANGE) == 0) err[1] = i;
  }
  // ignition (SetPrimitive_Variables solver_direct_reactive.cpp:1013-1024): after SetPrimVar only the record's
  // temperature is overwritten (CReactiveEulerVariable::SetTemperature, variable_reactive.hpp:602-607); the
  // derivatives and transport above keep the secant's temperature, as in the reference
  if (P.ignite) {
    double yf = 0.0, yo = 0.0;  // selected by an unrolled compare: a run-time index would put V in scratch
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s == P.fuel) yf = V[RHOS + s];
      if (s == P.oxidizer) yo = V[RHOS + s];
    }
    if (yf > 0.4 && yo > 0.2 && V[0] < P.T_ign) Vg[(size_t)i * nPV] = P.T_ign;
  }
}

// a2 second order: MUSCL reconstruction of (T, u, v, P) per edge side with the optional limiter, and the
// thermodynamically consistent state + pressure derivatives rebuilt through the library
// (CReactiveEulerSolver::Upwind_Residual, solver_direct_reactive.cpp:2554-2729; ComputeDensity :457-460,
// ComputeEnthalpy :519-523, ComputeFrozenGamma :398-403, ComputedP_dYs :591-596 of
// reacting_model_library.cpp). One thread per (edge, side); [2e + side] of VR / SR. Quirk kept: side j's
// pressure check reads side i's reconstructed pressure (:2617). Table range -> ERR_RANGE.
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) void k_muscl_edge(int E, const int32_t* __restrict__ edges,
                                                       const double* __restrict__ coord,
                                                       const double* __restrict__ V, const double* __restrict__ dPdU,
                                                       const double* __restrict__ G, const double* __restrict__ lim,
                                                       DevMech m, double T_ref, double E_ref, double R_ref,
                                                       int implicit, double* __restrict__ VR,
                                                       double* __restrict__ SR, int* err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5, nG = NS + NDIM + 2, nL = NDIM + 2;
  constexpr int VX = 1, P_ = NDIM + 1, RHO = NDIM + 2, H_ = NDIM + 3, A_ = NDIM + 4, RHOS = NDIM + 5;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * E) return;
  const int e = t >> 1, side = t & 1;
  const int n0 = edges[2 * e], n1 = edges[2 * e + 1];
  const int me = side ? n1 : n0;
  // Vector_i = 0.5 (x_j - x_i), Vector_j = -Vector_i
  double vec[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    const double vi = 0.5 * (coord[(size_t)n1 * NDIM + d] - coord[(size_t)n0 * NDIM + d]);
    vec[d] = side ? -vi : vi;
  }
  const double* Vm = V + (size_t)me * nPV;
  double rc[nL];
  rc[0] = Vm[0];
  rc[P_] = Vm[P_];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) rc[VX + d] = Vm[VX + d];
#pragma unroll
  for (int v = 0; v < nL; ++v) {
    double pg = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) pg += vec[d] * G[((size_t)me * nG + v) * NDIM + d];
    if (lim) rc[v] += lim[(size_t)me * nL + v] * pg;
    else rc[v] += pg;
  }
  // side i's reconstructed pressure (the j-side check of :2617 reads it)
  double p_i = rc[P_];
  if (side) {
    double pg = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) pg += -vec[d] * G[((size_t)n0 * nG + P_) * NDIM + d];
    p_i = V[(size_t)n0 * nPV + P_];
    if (lim) p_i += lim[(size_t)n0 * nL + P_] * pg;
    else p_i += pg;
  }
  bool np = !(rc[0] > kEPS);
  if (!np) np = !(p_i > kEPS);
  double* out = VR + (size_t)t * nPV;
  double* sout = SR ? SR + (size_t)t * nVar : nullptr;
  if (np) {
#pragma unroll
    for (int v = 0; v < nPV; ++v) out[v] = Vm[v];
    if (implicit)
#pragma unroll
      for (int v = 0; v < nVar; ++v) sout[v] = dPdU[(size_t)me * nVar + v];
    return;
  }
  double Ys[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const double y = Vm[RHOS + s];
    out[RHOS + s] = y;
    Ys[s] = y < 0.0 ? 1.0e-30 : y;
  }
  const double T = rc[0], P = rc[P_];
  double Rgas = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) Rgas += Ys[s] * (kR / m.mm[s]);
  double rho = P / (T * Rgas);
  rho *= R_ref;
  const double dim_temp = T * T_ref;
  int ierr = ERR_NONE;
  double hs[NS], h = 0.0, Cp = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    hs[s] = spline(m, P_H, s, dim_temp, &ierr) / m.mm[s];
    h += Ys[s] * hs[s];
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) Cp += Ys[s] * (spline(m, P_CP, s, dim_temp, &ierr) / m.mm[s]);
  if (ierr != ERR_NONE) set_err(err, ERR_RANGE, e);
  double sq = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) sq += rc[VX + d] * rc[VX + d];
  const double Gamma = Cp / (Cp - Rgas);
  out[0] = T;
  out[P_] = P;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) out[VX + d] = rc[VX + d];
  out[RHO] = rho;
  double hh = h / E_ref;
  hh += 0.5 * sq;
  out[H_] = hh;
  out[A_] = sqrt(Gamma * P / rho);
  if (!implicit) return;
  sout[0] = (Gamma - 1.0) * 0.5 * sq;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) sout[1 + d] = (1.0 - Gamma) * rc[VX + d];
  sout[NDIM + 1] = Gamma - 1.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const double ri = kR / m.mm[s];
    const double es = hs[s] - ri * dim_temp;
    sout[NDIM + 2 + s] = (ri * dim_temp - (Gamma - 1.0) * es) / E_ref;
  }
}

// a1 implicit: flux + both Jacobians into per-edge scratch. An edge is shared by a team of 4 lanes
// (16 edges per wavefront): every lane evaluates the edge scalars (~15 divisions / square roots) once
// and owns the residual components and Jacobian columns b = t, t + 4, t + 8 (t = lane in team), in the
// reference's operation order per entry. The 16 edges of a wavefront own one contiguous scratch range
// ([e][Ji|Jj], edge-major), so Ji and then Jj of the 16 edges are staged in LDS and stored as whole
// 512-byte rows (full cache lines).
// RX_AUSM_STAGE (build knob): 2 = both Jacobians staged through LDS (Jj held in registers while
// Ji is stored: 201 VGPRs, 2 waves per SIMD); 1 = Ji staged, Jj stored straight from the lane (no register copy);
// 0 = both stored straight from the lanes (no LDS). A team's four lanes write four consecutive doubles of a block row,
// so a direct store instruction writes sixteen 32-byte runs, and every byte of the edge's two blocks is written by
// the same wavefront within a few hundred cycles (the L2 merges the partial lines).
#ifndef RX_AUSM_STAGE
#define RX_AUSM_STAGE 2
#endif
constexpr int kAusmTeam = 4;
constexpr int kAusmBlock = 128;
template <int NS, int NDIM>
__global__ __launch_bounds__(kAusmBlock) RX_WPE_AUSM void k_ausm_edge(int E, const int32_t* __restrict__ edges,
                                                          const double* __restrict__ normal,
                                                          const double* __restrict__ V,
                                                          const double* __restrict__ dPdU,
                                                          const double* __restrict__ VR,
                                                          const double* __restrict__ SR, double mInfty,
                                                          double* __restrict__ F, double* __restrict__ Jac,
                                                          int* err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5, nVar2 = nVar * nVar;
  constexpr int CPL = (nVar + kAusmTeam - 1) / kAusmTeam;
  constexpr int EW = 64 / kAusmTeam;
  constexpr int kStage = RX_AUSM_STAGE;
  __shared__ double stage[kAusmBlock / 64][kStage ? EW * nVar2 : 1];
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, k = lane / kAusmTeam, t = lane % kAusmTeam;
  const int e0 = (gt >> 6) * EW;  // first edge of this wavefront
  if (e0 >= E) return;            // whole wavefronts exit together
  const int e = e0 + k;
  const bool live = e < E;
  const int ee = live ? e : e0;
  double* sj = stage[threadIdx.x >> 6];
  const int n0 = edges[2 * ee], n1 = edges[2 * ee + 1];
  // node states (1st order) or the edge's reconstructed states and pressure derivatives (2nd order)
  const double* Vsi = VR ? VR + 2 * (size_t)ee * nPV : V + (size_t)n0 * nPV;
  const double* Vsj = VR ? VR + (2 * (size_t)ee + 1) * nPV : V + (size_t)n1 * nPV;
  const double* Ssi = VR ? SR + 2 * (size_t)ee * nVar : dPdU + (size_t)n0 * nVar;
  const double* Ssj = VR ? SR + (2 * (size_t)ee + 1) * nVar : dPdU + (size_t)n1 * nVar;
  double Vi[nPV], Vj[nPV];
#pragma unroll
  for (int v = 0; v < nPV; ++v) {
    Vi[v] = Vsi[v];
    Vj[v] = Vsj[v];
  }
  double nrm[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) nrm[d] = normal[(size_t)ee * NDIM + d];
  AusmEdge s;
  ausm_scalars<NDIM>(Vi, Vj, nrm, mInfty, s);
  bool bad = false;
  double jjr[kStage == 2 ? CPL : 1][nVar];
  double* Jd = Jac + (size_t)ee * 2 * nVar2;  // this lane's edge (direct stores)
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int b = t + kAusmTeam * c;
    if (b < nVar) {
      // ausm_res for the runtime component b, with phi read by index (no dynamic register indexing)
      const int pidx = (b <= NDIM) ? b : (b == NDIM + 1 ? NDIM + 3 : b + 3);
      const double pi = b == 0 ? 1.0 : Vsi[pidx];
      const double pj = b == 0 ? 1.0 : Vsj[pidx];
      double r = 0.5 * (s.M12 * (pi + pj) + fabs(s.M12) * (pi - pj)) * s.Area;
      if (b >= 1 && b <= NDIM) r += s.pLF * pick<NDIM>(s.UN, b - 1) * s.Area;
      bad |= isnan(r);
      if (live) F[(size_t)e * nVar + b] = r;
      // dP/dU of both nodes: only column b is needed by this lane's Jacobian column
      const double sib = Ssi[b], sjb = Ssj[b];
      const AusmCol col = ausm_col_b<NDIM>(s, sib, sjb, b);
#pragma unroll
      for (int a = 0; a < nVar; ++a) {
        double ji, jj;
        ausm_jac_entry<NDIM>(s, col, ausm_phi<NDIM>(Vi, Vi[NDIM + 3], a), ausm_phi<NDIM>(Vj, Vj[NDIM + 3], a), sib,
                             sjb, a, b, &ji, &jj);
        bad |= isnan(ji) || isnan(jj);
        if (kStage) sj[k * nVar2 + a * nVar + b] = ji;
        else if (live) Jd[a * nVar + b] = ji;
        if (kStage == 2) jjr[c][a] = jj;
        else if (live) Jd[nVar2 + a * nVar + b] = jj;
      }
    }
  }
  if (kStage == 0) {
    if (live && bad) set_err(err, ERR_NAN, e);
    return;
  }
  const int ne = min(EW, E - e0);
  double* Jo = Jac + (size_t)e0 * 2 * nVar2;
#pragma unroll
  for (int side = 0; side < (kStage == 2 ? 2 : 1); ++side) {
    if (side && kStage == 2) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int b = t + kAusmTeam * c;
        if (b < nVar)
#pragma unroll
          for (int a = 0; a < nVar; ++a) sj[k * nVar2 + a * nVar + b] = jjr[kStage == 2 ? c : 0][a];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    for (int q = lane; q < ne * nVar2; q += 64) {
      const int kk = q / nVar2, r = q - kk * nVar2;
      Jo[(size_t)kk * 2 * nVar2 + side * nVar2 + r] = sj[q];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  if (live && bad) set_err(err, ERR_NAN, e);
}

// a3-a6: viscous flux (+ Jacobians) per edge into scratch.
#ifdef RX_VISC_WPE  // build knob (tools/build_variant.sh): waves per SIMD the viscous edge kernel is compiled for
#define RX_VISC_ATTR __attribute__((amdgpu_waves_per_eu(RX_VISC_WPE)))
#else
#define RX_VISC_ATTR
#endif
template <int NS, int NDIM>
__global__ __launch_bounds__(64) RX_VISC_ATTR void k_visc_edge(int E, const int32_t* __restrict__ edges,
                                                  const double* __restrict__ normal, const double* __restrict__ coord,
                                                  const double* __restrict__ V, const double* __restrict__ G,
                                                  const double* __restrict__ mu, const double* __restrict__ kappa,
                                                  const double* __restrict__ Dij, const double* __restrict__ dTdU,
                                                  const double* __restrict__ tke, const double* __restrict__ mut,
                                                  const double* __restrict__ sigk, const double* __restrict__ gk,
                                                  DevMech m, ViscParams P, double* __restrict__ F,
                                                  double* __restrict__ Summ, int* err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5, nG = NS + NDIM + 2;
  constexpr int SS = visc_summary_size<NS, NDIM>();
  __shared__ double scr_all[64 * NS * NS];  // dense Stefan-Maxwell / QR matrices, one slice per lane
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) {
    const int n0 = edges[2 * e], n1 = edges[2 * e + 1];
    ViscNode<NS, NDIM> a, b;
    a.V = V + (size_t)n0 * nPV;
    b.V = V + (size_t)n1 * nPV;
    a.G = G + (size_t)n0 * nG * NDIM;
    b.G = G + (size_t)n1 * nG * NDIM;
    a.Dij = Dij + (size_t)n0 * NS * NS;
    b.Dij = Dij + (size_t)n1 * NS * NS;
    a.S = P.implicit ? dTdU + (size_t)n0 * nVar : nullptr;
    b.S = P.implicit ? dTdU + (size_t)n1 * nVar : nullptr;
    a.coord = coord + (size_t)n0 * NDIM;
    b.coord = coord + (size_t)n1 * NDIM;
    a.mu = mu[n0];
    b.mu = mu[n1];
    a.kappa = kappa[n0];
    b.kappa = kappa[n1];
    double sk = 1.0;
    if (P.rans) {
      a.tke = tke[n0];
      b.tke = tke[n1];
      a.mut = mut[n0];
      b.mut = mut[n1];
      a.gk = gk + (size_t)n0 * NDIM;
      b.gk = gk + (size_t)n1 * NDIM;
      sk = sigk[n0];  // Set_Sigmak(node i), solver_direct_reactive.cpp:5345
    } else {
      a.tke = b.tke = a.mut = b.mut = 0.0;
      a.gk = b.gk = nullptr;
    }
    double nrm[NDIM];
  #pragma unroll
    for (int d = 0; d < NDIM; ++d) nrm[d] = normal[(size_t)e * NDIM + d];
    double res[nVar];
    // the summary in 64-edge tiles, edge index fastest ([E/64][SS][64]): each store of the wavefront is one
    // contiguous 512-B run (per-edge [SS] rows touched 64 lines per store and amplified the kernel's HBM writes
    // 1.25x, profiles/r02_pmc_c3.json); k_visc_jac stages its 16 edges' records from the tile through LDS
    const SummRef summ{P.implicit ? Summ + (size_t)(e / kSummTile) * SS * kSummTile + e % kSummTile : nullptr,
                       kSummTile};
    const int rc = visc_edge<NS, NDIM>(m, P, a, b, sk, nrm, res, summ, Scr{scr_all + threadIdx.x});
    bool bad = false;
  #pragma unroll
    for (int v = 0; v < nVar; ++v) {
      bad |= isnan(res[v]);
      F[(size_t)e * nVar + v] = res[v];
    }
    if (rc != ERR_NONE) set_err(err, rc == ERR_RANGE ? ERR_RANGE : ERR_NAN, e);
    else if (bad) set_err(err, ERR_NAN, e);
  }
}

// a6: viscous Jacobians from the per-edge summary; a team of 16 lanes per edge, lane b = column b,
// so every row of Ji / Jj is stored as one contiguous segment per team.
// Fused assembly (Jc != nullptr): the same lanes also write the edge's two off-diagonal BSR blocks from its own
// convective scratch, so k_assemble only builds the diagonal blocks and the residual (each Jc / Jv block is read
// by the edge that made it and by its own node's diagonal, instead of by both nodes' teams).
// waves per SIMD: 3 in 2-D (at 2: VISC_JAC 3.86 -> 4.27 ms at C3), 2 in 3-D (at 3 the 12-row columns spill 28
// VGPRs: C5 VISC_JAC 7.54 -> 7.16 ms at 2)
#ifndef RX_WPE_VJAC
#define RX_WPE_VJAC RX_WPE(NDIM == 2 ? 3 : 2)
#endif
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) RX_WPE_VJAC void k_visc_jac(int E, const int32_t* __restrict__ edges,
                                                     const double* __restrict__ dTdU, const double* __restrict__ Summ,
                                                     DevMech m, ViscParams P, double* __restrict__ Jac,
                                                     const double* __restrict__ Jc,
                                                     const int64_t* __restrict__ edge_blk, double* __restrict__ A) {
  constexpr int nVar = NS + NDIM + 2, nVar2 = nVar * nVar, SS = visc_summary_size<NS, NDIM>(), kEB = kBlock / 16;

  // the workgroup's kEB consecutive edge records, staged from their tile: each load is kEB consecutive doubles
  __shared__ double ssm[SS * kEB];
  const int eb = blockIdx.x * kEB;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = gt / 16, b = gt % 16;
  const bool live = e < E;
  const int bc = b < nVar ? b : 0;
  // the team's own inputs (edge, dT/dU of both nodes, this lane's column of both convective blocks) are loaded
  // before the summary staging and its barrier, so that both sets of loads are in flight together (plain loads stay
  // in flight across __syncthreads): C3 VISC_JAC 3.86 -> 3.73 ms; in 3-D, with 2 waves per SIMD (no spills), C5
  // 7.16 -> 6.68 ms (at 3 waves the 12-row columns spilled and it lost 0.27 ms). RX_VJ_LATE3 keeps 3-D's late loads.
#ifdef RX_VJ_LATE3
  constexpr bool kEarlyJc = NDIM == 2;
#else
  constexpr bool kEarlyJc = true;
#endif
  int n0 = 0, n1 = 0;
  double sib = 0.0, sjb = 0.0, jci[nVar], jcj[nVar];
  auto load_jc = [&]() {
    const double* Jci = Jc + (size_t)e * 2 * nVar2;
#pragma unroll
    for (int r = 0; r < nVar; ++r) {
      jci[r] = Jci[r * nVar + bc];
      jcj[r] = Jci[nVar2 + r * nVar + bc];
    }
  };
  if (live) {
    n0 = edges[2 * e];
    n1 = edges[2 * e + 1];
    sib = dTdU[(size_t)n0 * nVar + bc];
    sjb = dTdU[(size_t)n1 * nVar + bc];
    if (kEarlyJc && Jc) load_jc();
  }
  for (int q = threadIdx.x; q < SS * kEB; q += kBlock) {
    const int k = q / kEB, el = q - k * kEB, ee = eb + el;
    if (ee < E) ssm[q] = Summ[(size_t)(ee / kSummTile) * SS * kSummTile + (size_t)k * kSummTile + ee % kSummTile];
  }
  __syncthreads();
  if (!live) return;  // whole teams exit together (E * 16 threads)
  double* Ji = Jac + (size_t)e * 2 * nVar2;
  const SummCRef sm{ssm + (e - eb), kEB};
  if (Jc) {
    if (!kEarlyJc) load_jc();
    visc_jac_column<NS, NDIM>(m, P, sm, sib, sjb, b, b, Ji, Ji + nVar2, jci, jcj, A + edge_blk[2 * e] * nVar2,
                              A + edge_blk[2 * e + 1] * nVar2);
  } else {
    visc_jac_column<NS, NDIM>(m, P, sm, sib, sjb, b, b, Ji, Ji + nVar2);
  }
}

// Generic node gather of an edge flux array: node0 += sign*F, node1 -= sign*F (edge order).
__global__ __launch_bounds__(kBlock) void k_gather_flux(int N, int nVar, const int32_t* __restrict__ adj_ptr,
                                                        const int32_t* __restrict__ adj, const double* __restrict__ F,
                                                        double sign_first, double* __restrict__ R) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * nVar) return;
  const int i = t / nVar, v = t - i * nVar;
  double acc = R[t];
  for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
    const int a = adj[k];
    const double f = F[(size_t)(a >> 1) * nVar + v];
    // node0: acc (+/-) f ; node1: the opposite sign (R[j] -= F for conv, += F for visc)
    const bool plus = ((a & 1) == 0) == (sign_first > 0.0);
    acc = plus ? acc + f : acc - f;
  }
  R[t] = acc;
}

// a9: PaSR source per cell: R[i] += S; implicit: the species rows of the cell Jacobian into scratch, in
// 64-cell tiles with the cell index fastest ([N/64][NS*nVar][64], kSrcTile): every store of a wavefront is one
// contiguous 512-B segment (the [N][nVar^2] thread-per-cell layout wrote 64 lines per store and amplified the
// kernel's HBM writes 2.8x, profiles/r02_pmc_c3.json).
template <int NS, int NDIM>
__global__ __launch_bounds__(128) RX_WPE_SRC void k_source(int N, const double* __restrict__ V, const double* __restrict__ dTdU,
                                                const double* __restrict__ vol, const double* __restrict__ omega,
                                                DevMech m, SourceParams P, double* __restrict__ R, int add,
                                                double* __restrict__ Js, int* err) {
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double Vl[nPV];
#pragma unroll
  for (int v = 0; v < nPV; ++v) Vl[v] = V[(size_t)i * nPV + v];
  double res[nVar];
  const int rc = source_cell<NS, NDIM>(
      m, P, Vl, P.implicit ? dTdU + (size_t)i * nVar : nullptr, vol[i], P.rans ? omega[i] : 0.0, res,
      P.implicit ? Js + (size_t)(i / kSrcTile) * NS * nVar * kSrcTile + (i % kSrcTile) : nullptr, kSrcTile);
  bool bad = false;
#pragma unroll
  for (int v = 0; v < nVar; ++v) {
    bad |= isnan(res[v]);
    if (add) R[(size_t)i * nVar + v] += res[v];
    else R[(size_t)i * nVar + v] = res[v];
  }
  if (rc != ERR_NONE) set_err(err, ERR_RANGE, i);
  else if (bad) set_err(err, ERR_NAN, i);
}

// Implicit assembly: a team of 128 lanes per node, lane t < nVar^2 owns entry t of every block of
// the node's BSR row (coalesced block reads and writes), lane t < nVar also owns residual component
// t. Reference accumulation order:
//   R  = 0 + conv(edge order) - visc(edge order) + source
//   Aii = 0 + conv(edge order) + visc(edge order) + source     (AddVal2Diag comes later)
//   A(n0,n1) = (0 + Jc_j) - Jv_j ;  A(n1,n0) = (0 - Jc_i) + Jv_i
// Team = one or two whole wavefronts up to nVar = 11; above, exactly nVar^2 lanes (no intra-team synchronisation:
// teams may straddle wavefronts), so nVar = 12 / 13 / 14 do not idle 112 / 87 / 60 of 256 lanes (C5 assembly
// 10.0 -> 7.9 ms).
template <int NVAR>
constexpr int asm_team() {
  return NVAR * NVAR <= 64 ? 64 : (NVAR * NVAR <= 128 ? 128 : NVAR * NVAR);
}
// XCD-aware block order: the hardware deals consecutive workgroups round-robin to the 8 XCDs; this remaps them
// so that XCD x assembles one contiguous range of nodes, and the 64 teams reading one source tile (and the
// neighbouring nodes sharing edge blocks) run under the same L2.
__device__ inline int xcd_block(int b, int nb) {
  constexpr int kXcd = 8;
  const int x = b % kXcd, idx = b / kXcd, q = nb / kXcd, r = nb % kXcd;
  return x < r ? x * (q + 1) + idx : r * (q + 1) + (x - r) * q + idx;
}

// DEG: incident edges of a node assembled from registers (larger degrees take the loop); the launcher picks the
// smallest of 4 / 8 that covers the mesh's maximum degree (2-D quads: 4, so fewer registers and more waves)
template <int NVAR, int kAsmDeg>
__global__ __launch_bounds__(kBlock) void k_assemble(int N, int rhos, const int32_t* __restrict__ adj_ptr,
                                                     const int32_t* __restrict__ adj,
                                                     const int64_t* __restrict__ adj_blk,
                                                     const int64_t* __restrict__ diag, const double* __restrict__ Fc,
                                                     const double* __restrict__ Fv, const double* __restrict__ Jc,
                                                     const double* __restrict__ Jv, const double* __restrict__ Js,
                                                     const double* __restrict__ Rsrc, double* __restrict__ R,
                                                     double* __restrict__ A, int visc, int src, int write_off) {
  constexpr int nVar2 = NVAR * NVAR, kTeam = asm_team<NVAR>();
  const int gt = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int i = gt / kTeam, t = gt % kTeam;
  if (i >= N || t >= nVar2) return;
  const bool res = t < NVAR;
  double r = 0.0, D = 0.0;
  const int k0 = adj_ptr[i], k1 = adj_ptr[i + 1];
  double rs = 0.0, js = 0.0;  // source residual / Jacobian entry, loaded up front
  if (src) {
    if (res) rs = Rsrc[(size_t)i * NVAR + t];
    // species rows from the tiled scratch of k_source; the other rows of the reference's block are zeros
    const int a = t / NVAR;
    const int nsv = (NVAR - rhos) * NVAR;
    js = a >= rhos ? Js[(size_t)(i / kSrcTile) * nsv * kSrcTile + (size_t)((a - rhos) * NVAR + t % NVAR) * kSrcTile +
                        i % kSrcTile]
                   : 0.0;
  }
  if (!write_off && k1 - k0 <= kAsmDeg) {
    // fused path (k_visc_jac wrote the off-diagonals), degree <= kAsmDeg: every load of the node is issued
    // before the first sum, so a team waits for one round trip instead of one per incident edge and pass;
    // the sums then run in the reference's order (conv over edges, then visc over edges)
    int ad[kAsmDeg];
    double jc[kAsmDeg], jv[kAsmDeg], fc[kAsmDeg], fv[kAsmDeg];
#pragma unroll
    for (int q = 0; q < kAsmDeg; ++q) ad[q] = k0 + q < k1 ? adj[k0 + q] : 0;
#pragma unroll
    for (int q = 0; q < kAsmDeg; ++q) {
      if (k0 + q < k1) {
        const size_t e = (size_t)(ad[q] >> 1);
        const int side = ad[q] & 1;
        jc[q] = Jc[(e * 2 + side) * nVar2 + t];
        jv[q] = visc ? Jv[(e * 2 + side) * nVar2 + t] : 0.0;
        fc[q] = res ? Fc[e * NVAR + t] : 0.0;
        fv[q] = res && visc ? Fv[e * NVAR + t] : 0.0;
      }
    }
#pragma unroll
    for (int q = 0; q < kAsmDeg; ++q)
      if (k0 + q < k1) {
        const int side = ad[q] & 1;
        r = side ? r - fc[q] : r + fc[q];
        D = side ? D - jc[q] : D + jc[q];
      }
    if (visc) {
#pragma unroll
      for (int q = 0; q < kAsmDeg; ++q)
        if (k0 + q < k1) {
          const int side = ad[q] & 1;
          r = side ? r + fv[q] : r - fv[q];
          D = side ? D + jv[q] : D - jv[q];
        }
    }
  } else {
    // convective pass: residual and diagonal (own-side blocks)
    for (int k = k0; k < k1; ++k) {
      const int ad = adj[k];
      const size_t e = (size_t)(ad >> 1);
      const int side = ad & 1;
      if (res) {
        const double f = Fc[e * NVAR + t];
        r = side ? r - f : r + f;
      }
      const double jd = Jc[(e * 2 + side) * nVar2 + t];  // own side: Ji for n0, Jj for n1
      D = side ? D - jd : D + jd;
    }
    // viscous pass: residual, diagonal, and (unless k_visc_jac wrote them) each off-diagonal block written once
    // as (0 +- Jc) -+ Jv
    for (int k = k0; k < k1; ++k) {
      const int ad = adj[k];
      const size_t e = (size_t)(ad >> 1);
      const int side = ad & 1;
      if (visc) {
        if (res) {
          const double f = Fv[e * NVAR + t];
          r = side ? r + f : r - f;
        }
        const double jd = Jv[(e * 2 + side) * nVar2 + t];
        D = side ? D + jd : D - jd;
      }
      if (write_off) {
        const double joc = Jc[(e * 2 + (side ^ 1)) * nVar2 + t];  // other side
        double off = side ? 0.0 - joc : 0.0 + joc;
        if (visc) {
          const double jov = Jv[(e * 2 + (side ^ 1)) * nVar2 + t];
          off = side ? off + jov : off - jov;
        }
        A[adj_blk[k] * nVar2 + t] = off;
      }
    }
  }
  if (src) {
    if (res) r += rs;
    D += js;
  }
  if (res) R[(size_t)i * NVAR + t] = r;
  A[diag[i] * nVar2 + t] = D;
}

// Node-centric viscous Jacobians + assembly (round 4): one 16-lane team per node, lane b =
// column b. The team walks the node's edges in adjacency (= edge) order twice, as k_assemble does: the convective
// pass adds its own-side convective blocks to the diagonal and the convective fluxes to the residual; the viscous pass
// stages each edge's summary record in the team's LDS slot, evaluates the edge's viscous Jacobian columns
// (visc_jac_column_f, the same arithmetic as k_visc_jac), folds its own side into the diagonal and writes the
// edge's off-diagonal block of the neighbour's row from its own side, A(n1,n0) = (0 - Jc_i) + Jv_i or
// A(n0,n1) = (0 + Jc_j) - Jv_j. Only the own side's columns are evaluated (visc_jac_column_own), so each side of
// each edge is still evaluated once. Every diagonal entry, residual component and off-diagonal entry is the same
// sum in the same order as k_visc_jac + k_assemble make it, so the system is bitwise theirs; the per-edge viscous
// blocks (2 x 968 B per edge, written once and read once) and the second read of the convective blocks are gone.
// inputs of k_asm_visc's fused AUSM pass (V == nullptr: the convective blocks and fluxes come from k_ausm_edge)
struct AusmIn {
  const double *V, *dPdU, *VR, *SR, *normal;
  double mInfty;
  int* err;
};
// the system build's diagonal folded into k_asm_visc (vol == nullptr: not folded; rx_ctx::fold_req)
struct SysFold {
  const double *vol, *dt;
  const int32_t* skip;
  int Nd;
};
#ifndef RX_ASMV_SHS
#define RX_ASMV_SHS 1  // build knob: the fused AUSM pass makes each edge's scalars once per team (LDS-shared)
#endif
#ifndef RX_ASMV_FUSE
#define RX_ASMV_FUSE 1  // build knob: 0 compiles k_asm_visc without its fused AUSM pass
#endif
#ifndef RX_ASMV_PARK
// build knob: 0 (default since round 5's cycle r) = each off-diagonal block written once, the own-side AUSM column
// evaluated again in the viscous pass; 1 = the fused pass parks 0 -+ Jc in the off-diagonal block for
// the viscous pass to finish (each off-diagonal block written twice, read back once). Same-box A/B at C3, two runs
// each: first (r05c) ASSEMBLE 6.16 / 6.15 ms parked against 6.92 / 6.93 single-write; once the column evaluates only
// its own side's entries and the teams are nVar lanes wide (r05r): 5.77 / 5.78 parked against 5.56 / 5.58, C5 9.15
// against 8.79 ms
#define RX_ASMV_PARK 0
#endif
#ifndef RX_ASMV_CDEG
#define RX_ASMV_CDEG -1  // build knob: node degree up to which k_asm_visc's convective pass loads everything first
#endif                   // (-1: the quad / hex stencils' 4 in 2-D, 6 in 3-D; 0: never)
#ifndef RX_WPE_ASMV
#define RX_WPE_ASMV RX_WPE(NDIM == 2 ? 3 : 2)
#endif
#ifndef RX_ASMV_NARROW
// build knob: 1 (default) = teams of nVar lanes, floor(64 / nVar) nodes per wavefront (5 at nVar 11 / 12, lanes 55..63
// or 60..63 idle); 0 = 16-lane teams, 4 nodes per wavefront with 5 / 4 of every 16 lanes idle
#define RX_ASMV_NARROW 1
#endif
// a k_asm_visc team's width and the nodes one 256-thread workgroup assembles
__host__ __device__ constexpr int asmv_team_width(int nVar) { return RX_ASMV_NARROW ? nVar : 16; }
__host__ __device__ constexpr int asmv_nodes_per_block(int nVar) { return (kBlock / 64) * (64 / asmv_team_width(nVar)); }
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) RX_WPE_ASMV void k_asm_visc(
    int N, const int32_t* __restrict__ adj_ptr, const int32_t* __restrict__ adj, const int32_t* __restrict__ edges,
    const int64_t* __restrict__ edge_blk, const int64_t* __restrict__ diag, const double* __restrict__ Fc,
    const double* __restrict__ Fv, const double* __restrict__ Jc, const double* __restrict__ dTdU,
    const double* __restrict__ Summ, const double* __restrict__ Js, const double* __restrict__ Rsrc, DevMech m,
    ViscParams P, double* __restrict__ R, double* __restrict__ A, int src, AusmIn cv, SysFold fd) {
  constexpr int nVar = NS + NDIM + 2, nVar2 = nVar * nVar, SS = visc_summary_size<NS, NDIM>();
  constexpr int TW = asmv_team_width(nVar), TPW = 64 / TW, kTeams = asmv_nodes_per_block(nVar);
  static_assert(TW >= nVar && TW <= 64, "a team holds one lane per column");
  constexpr int nPV = NS + NDIM + 5;
  constexpr int rhos = NDIM + 2, nsv = NS * nVar;
  constexpr int CD = RX_ASMV_CDEG < 0 ? (NDIM == 2 ? 4 : 6) : (RX_ASMV_CDEG > 0 ? RX_ASMV_CDEG : 1);
  constexpr int kES = sizeof(AusmEdge) / sizeof(double);  // one edge's AUSM scalars
  // a team's LDS slot: the viscous summary record of the edge being folded at [0, SS); the shared edge scalars of
  // the node's first CD edges at [SCO, SCO + CD kES) — after the summary, so that the viscous pass still reads them
  // (RX_ASMV_PARK: at 0, reused by the summary)
  constexpr int SCO = RX_ASMV_PARK ? 0 : SS;
  constexpr int TS = !RX_ASMV_SHS ? SS : (RX_ASMV_PARK ? (CD * kES > SS ? CD * kES : SS) : SS + CD * kES);
  static_assert(CD <= TW, "the shared edge scalars of the first CD edges are made by team lanes 0..CD-1");
  __shared__ double ssm[kTeams * TS];
  const int lane = threadIdx.x % 64, wv = threadIdx.x / 64, tw = lane / TW;
  if (tw >= TPW) return;  // the wavefront's lanes past its last whole team
  const int team = wv * TPW + tw, b = lane - tw * TW, sbase = tw * TW;
  const int i = xcd_block(blockIdx.x, gridDim.x) * kTeams + team;
  if (i >= N) return;  // whole teams
  const bool col = b < nVar;
  const int bc = col ? b : 0;
  double* slot = ssm + team * TS;
  const int k0 = adj_ptr[i], k1 = adj_ptr[i + 1];
  double r = 0.0, D[nVar];
#pragma unroll
  for (int a = 0; a < nVar; ++a) D[a] = 0.0;
  const bool fused = RX_ASMV_FUSE && cv.V != nullptr;
  // fused AUSM (cv.V set, k_ausm_edge skipped): the edge scalars (from the team's LDS slot for the node's first CD
  // edges, else made here) and this lane's column of the own side's convective Jacobian, with k_ausm_edge's
  // arithmetic (the other side's column is the neighbour team's own side): jd[a] = J_own[a][bc]
  auto edge_scalars = [&](size_t e, int n0, int n1, AusmEdge& s) {
    const double* Vsi = cv.VR ? cv.VR + 2 * e * nPV : cv.V + (size_t)n0 * nPV;
    const double* Vsj = cv.VR ? cv.VR + (2 * e + 1) * nPV : cv.V + (size_t)n1 * nPV;
    double Vi[nPV], Vj[nPV], nrm[NDIM];  // the entries ausm_scalars reads
#pragma unroll
    for (int v = 0; v < nPV; ++v) {
      Vi[v] = v <= NDIM + 2 || v == NDIM + 4 ? Vsi[v] : 0.0;
      Vj[v] = v <= NDIM + 2 || v == NDIM + 4 ? Vsj[v] : 0.0;
    }
#pragma unroll
    for (int d = 0; d < NDIM; ++d) nrm[d] = cv.normal[e * NDIM + d];
    ausm_scalars<NDIM>(Vi, Vj, nrm, cv.mInfty, s);
  };
  auto own_column = [&](size_t e, int side, int n0, int n1, const AusmEdge& s, double* jd) {
    const double* Vsi = cv.VR ? cv.VR + 2 * e * nPV : cv.V + (size_t)n0 * nPV;
    const double* Vsj = cv.VR ? cv.VR + (2 * e + 1) * nPV : cv.V + (size_t)n1 * nPV;
    const double* Ssi = cv.VR ? cv.SR + 2 * e * nVar : cv.dPdU + (size_t)n0 * nVar;
    const double* Ssj = cv.VR ? cv.SR + (2 * e + 1) * nVar : cv.dPdU + (size_t)n1 * nVar;
    const double sib = Ssi[bc], sjb = Ssj[bc];
    const AusmCol cc = ausm_col_b<NDIM>(s, sib, sjb, bc);
    bool bad = false;
#pragma unroll
    for (int a = 0; a < nVar; ++a) {
      // (k_ausm_edge's NaN check sees both sides' entries; the other side's is the neighbour team's own entry, checked
      // there, so every entry of the edge is still checked once)
      const double v = ausm_jac_entry_own<NDIM>(s, cc, ausm_phi<NDIM>(Vsi, Vsi[NDIM + 3], a),
                                                ausm_phi<NDIM>(Vsj, Vsj[NDIM + 3], a), side ? sjb : sib, a, bc, side);
      bad |= isnan(v);
      jd[a] = v;
    }
    return bad;
  };
  auto load_scalars = [&](const double* from, AusmEdge& s) {
    double* sp = reinterpret_cast<double*>(&s);
#pragma unroll
    for (int f = 0; f < kES; ++f) sp[f] = from[f];
  };
  int nq = 0;  // the node's first nq edges have their scalars in the team's slot
  // convective pass; for degrees up to RX_ASMV_CDEG every load of the pass is issued before the first sum (one round
  // trip instead of one per edge), then the sums run in edge order
  if (fused) {
    // the edge's flux and its own-side Jacobian column, folded into the residual and diagonal in edge order
    auto fused_edge = [&](int ad, int n0, int n1, const double* shared_s) {
      const size_t e = (size_t)(ad >> 1);
      const int side = ad & 1;
      AusmEdge s;
      if (RX_ASMV_SHS && shared_s) load_scalars(shared_s, s);
      else edge_scalars(e, n0, n1, s);
      bool bad = false;
      if (col) {
        const double* Vsi = cv.VR ? cv.VR + 2 * e * nPV : cv.V + (size_t)n0 * nPV;
        const double* Vsj = cv.VR ? cv.VR + (2 * e + 1) * nPV : cv.V + (size_t)n1 * nPV;
        const int pidx = (b <= NDIM) ? b : (b == NDIM + 1 ? NDIM + 3 : b + 3);
        const double pi = b == 0 ? 1.0 : Vsi[pidx];
        const double pj = b == 0 ? 1.0 : Vsj[pidx];
        double f = 0.5 * (s.M12 * (pi + pj) + fabs(s.M12) * (pi - pj)) * s.Area;
        if (b >= 1 && b <= NDIM) f += s.pLF * pick<NDIM>(s.UN, b - 1) * s.Area;
        bad |= isnan(f);
        r = side ? r - f : r + f;
      }
      double jd[nVar];
      bad |= own_column(e, side, n0, n1, s, jd);
      double* Ao = A + edge_blk[2 * e + (side ? 0 : 1)] * nVar2;
#pragma unroll
      for (int a = 0; a < nVar; ++a) {
        D[a] = side ? D[a] - jd[a] : D[a] + jd[a];
        if (RX_ASMV_PARK && col) Ao[a * nVar + b] = side ? 0.0 + jd[a] : 0.0 - jd[a];
      }
      if (col && bad) set_err(cv.err, ERR_NAN_UPWIND, (int64_t)e);
    };
    int kq = k0;
    if (RX_ASMV_SHS && k1 > k0) {
      // the edge scalars of the node's first CD edges are made once, lane q of the team making edge k0 + q's (the
      // same function on the same inputs, so the same values), and read back from the team's LDS slot
      nq = k1 - k0 < CD ? k1 - k0 : CD;
      {
        const int ad = adj[k0 + (b < nq ? b : 0)];
        const size_t e = (size_t)(ad >> 1);
        AusmEdge s;
        edge_scalars(e, edges[2 * e], edges[2 * e + 1], s);
        const double* sp = reinterpret_cast<const double*>(&s);
        if (b < nq)
#pragma unroll
          for (int f = 0; f < kES; ++f) slot[SCO + b * kES + f] = sp[f];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      for (int q = 0; q < nq; ++q) {
        const int ad = adj[k0 + q];
        fused_edge(ad, edges[2 * (ad >> 1)], edges[2 * (ad >> 1) + 1], slot + SCO + q * kES);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();  // (RX_ASMV_PARK) the viscous pass reuses the slot
      kq = k0 + nq;
      if (RX_ASMV_PARK) nq = 0;
    }
    for (int k = kq; k < k1; ++k) {
      const int ad = adj[k];
      fused_edge(ad, edges[2 * (ad >> 1)], edges[2 * (ad >> 1) + 1], nullptr);
    }
  } else if (RX_ASMV_CDEG != 0 && k1 - k0 <= CD) {
    int sd[CD];
    double fc[CD], jc[CD][nVar];
#pragma unroll
    for (int q = 0; q < CD; ++q) {
      const int k = k0 + q < k1 ? k0 + q : k0;  // clamped: always a valid address
      const int ad = adj[k];
      const size_t e = (size_t)(ad >> 1);
      sd[q] = ad & 1;
      fc[q] = Fc[e * nVar + bc];
      const double* J = Jc + (e * 2 + sd[q]) * nVar2 + bc;
#pragma unroll
      for (int a = 0; a < nVar; ++a) jc[q][a] = J[a * nVar];
    }
#pragma unroll
    for (int q = 0; q < CD; ++q)
      if (k0 + q < k1) {
        if (col) r = sd[q] ? r - fc[q] : r + fc[q];
#pragma unroll
        for (int a = 0; a < nVar; ++a) D[a] = sd[q] ? D[a] - jc[q][a] : D[a] + jc[q][a];
      }
  } else {
    for (int k = k0; k < k1; ++k) {
      const int ad = adj[k];
      const size_t e = (size_t)(ad >> 1);
      const int side = ad & 1;
      if (col) {
        const double f = Fc[e * nVar + b];
        r = side ? r - f : r + f;
      }
      const double* J = Jc + (e * 2 + side) * nVar2 + bc;
#pragma unroll
      for (int a = 0; a < nVar; ++a) {
        const double jd = J[a * nVar];
        D[a] = side ? D[a] - jd : D[a] + jd;
      }
    }
  }
  // viscous pass: each edge's off-diagonal block of the neighbour's row is written once, (0 -+ Jc) +- Jv
  for (int k = k0; k < k1; ++k) {
    const int ad = adj[k];
    const int e = ad >> 1;
    const int side = ad & 1;
    const int n0 = edges[2 * e], n1 = edges[2 * e + 1];
    {
      const double* tile = Summ + (size_t)(e / kSummTile) * SS * kSummTile + e % kSummTile;
      for (int q = b; q < SS; q += TW) slot[q] = tile[(size_t)q * kSummTile];
    }
    const double sob = dTdU[(size_t)(side ? n1 : n0) * nVar + bc];  // the own node's dT/dU
    double* Ao = A + edge_blk[2 * e + (side ? 0 : 1)] * nVar2;
    double jco[nVar];  // 0 -+ this lane's column of the own-side convective block
    if (fused && !RX_ASMV_PARK) {
      // the column the convective pass folded into the diagonal, evaluated again (same function, same inputs: the
      // same doubles) instead of parked in the off-diagonal block and read back
      AusmEdge s;
      if (RX_ASMV_SHS && k - k0 < nq) load_scalars(slot + SCO + (k - k0) * kES, s);
      else edge_scalars((size_t)e, n0, n1, s);
      double jd[nVar];
      (void)own_column((size_t)e, side, n0, n1, s, jd);
#pragma unroll
      for (int a = 0; a < nVar; ++a) jco[a] = side ? 0.0 + jd[a] : 0.0 - jd[a];
    } else if (fused) {
#pragma unroll
      for (int a = 0; a < nVar; ++a) jco[a] = col ? Ao[a * nVar + b] : 0.0;
    } else {
      const double* J = Jc + ((size_t)e * 2 + side) * nVar2 + bc;
#pragma unroll
      for (int a = 0; a < nVar; ++a) jco[a] = side ? 0.0 + J[a * nVar] : 0.0 - J[a * nVar];
    }
    if (col) {
      const double f = Fv[(size_t)e * nVar + b];
      r = side ? r + f : r - f;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    visc_jac_column_own<NS, NDIM>(m, P, SummCRef{slot, 1}, sob, side, b, b, sbase, [&](int rr, double jv) {
      D[rr] = side ? D[rr] + jv : D[rr] - jv;
      Ao[rr * nVar + b] = side ? jco[rr] - jv : jco[rr] + jv;
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  if (!col) return;
  if (src) {
    r += Rsrc[(size_t)i * nVar + b];
#pragma unroll
    for (int a = 0; a < nVar; ++a) {
      const double js = a >= rhos ? Js[(size_t)(i / kSrcTile) * nsv * kSrcTile +
                                       (size_t)((a - rhos) * nVar + b) * kSrcTile + i % kSrcTile]
                                  : 0.0;
      D[a] += js;
    }
  }
  if (fd.vol && i < fd.Nd && !fd.skip[i]) {
    // ImplicitEuler_Iteration's AddVal2Diag (k_build_system_elem's operations on this lane's column: the same
    // quotient added to the diagonal entry, or the identity row with the residual zeroed)
    if (fd.dt[i] > rx::kEPS) {
      const double delta = fd.vol[i] / fd.dt[i];
#pragma unroll
      for (int a = 0; a < nVar; ++a)
        if (a == b) D[a] += delta;
    } else {
#pragma unroll
      for (int a = 0; a < nVar; ++a) D[a] = (a == b) ? 1.0 : 0.0;
      r = 0.0;
    }
  }
  R[(size_t)i * nVar + b] = r;
  double* Ad = A + diag[i] * nVar2 + b;
#pragma unroll
  for (int a = 0; a < nVar; ++a) Ad[a * nVar] = D[a];
}

// The same assembly with a node's edges evaluated side by side (round 6). k_asm_visc's team walks its
// node's edges one after another: per edge a gather of the summary record, a wave barrier, the own-side AUSM column
// (evaluated twice: once for the diagonal, once more for the off-diagonal block), the viscous column, a second barrier
// — four dependent rounds per wavefront. Here a team of nVar lanes (lane b = column b) owns one edge side, i.e. one
// adjacency entry (node i, edge e): a 256-thread workgroup takes a run of consecutive nodes whose adjacency entries fit
// its 4 * floor(64 / nVar) teams (rx_ctx::asmes_wg, planned on the host), and
//  - phase A: every team stages its edge's summary record, evaluates the AUSM flux and the own-side Jacobian column
//    once, the viscous flux and column, writes the neighbour row's off-diagonal block (0 -+ Jc) +- Jv straight from
//    its lanes, and parks its signed contributions (flux, Jc column, viscous flux, Jv column) in its LDS slot;
//  - phase B (after one workgroup barrier): the team of the run's j-th node adds its edges' parked contributions in
//    k_asm_visc's order (the convective ones in edge order, then the viscous ones in edge order; r -+ f is r + (-+f)
//    exactly), then the source and the folded V / dt, and stores the residual and the diagonal block.
// Every value and every sum is k_asm_visc's, so the system is bitwise the same (tests/test_gpu_assembly.py).
// Reference: Upwind_Residual / Viscous_Residual's AddBlock / SubtractBlock (solver_direct_reactive.cpp:2759-2772,
// :5365-5381), CUpwReactiveAUSM::ComputeResidual (numerics_direct_reactive.cpp:53-378), the viscous Jacobian closure
// (:1200-1401, :1637-1653).
#ifndef RX_WPE_ASMES
#define RX_WPE_ASMES RX_WPE(NDIM == 2 ? 3 : 2)
#endif
#ifndef RX_ASMES_WAVES
#define RX_ASMES_WAVES 4  // build knob: wavefronts per k_asm_es workgroup
#endif
#ifndef RX_ASMES_STAGE
#define RX_ASMES_STAGE 1  // build knob: 0 = phase A gathers its node records per entry and stages the summary first
#endif
#ifndef RX_ASMES_PROBE
// build knob (tools/asm_probe.py, timing only, results wrong): 1 = no summary gather (constant records), 2 = no viscous
// column, 3 = no AUSM evaluation, 4 = no phase-B sums, 5 = neither column, 6 = no off-diagonal stores, 7 = no source
// loads in phase B
#define RX_ASMES_PROBE 0
#endif
__host__ __device__ constexpr int asmes_teams(int nVar) { return RX_ASMES_WAVES * (64 / nVar); }
__host__ __device__ constexpr int asmes_out(int nVar) { return 2 * nVar + 2; }  // parked doubles per lane
template <int NS, int NDIM>
__global__ __launch_bounds__(RX_ASMES_WAVES * 64) RX_WPE_ASMES void k_asm_es(
    const int2* __restrict__ wg_plan, const int4* __restrict__ side_rec, const int32_t* __restrict__ adj_ptr,
    const int64_t* __restrict__ diag,
    const double* __restrict__ Fc, const double* __restrict__ Fv, const double* __restrict__ Jc,
    const double* __restrict__ dTdU, const double* __restrict__ Summ, const double* __restrict__ Js,
    const double* __restrict__ Rsrc, DevMech m, ViscParams P, double* __restrict__ R, double* __restrict__ A, int src,
    AusmIn cv, SysFold fd) {
  constexpr int nVar = NS + NDIM + 2, nVar2 = nVar * nVar, SS = visc_summary_size<NS, NDIM>();
  constexpr int TPW = 64 / nVar, kTeams = asmes_teams(nVar), OW = asmes_out(nVar);
  constexpr int TS = SS > nVar * OW ? SS : nVar * OW;  // a team's slot: the summary record, then its parked outputs
  constexpr int nPV = NS + NDIM + 5;
  constexpr int rhos = NDIM + 2, nsv = NS * nVar;
  __shared__ double ssm[kTeams * TS];
  const int lane = threadIdx.x % 64, wv = threadIdx.x / 64, tw = lane / nVar;
  const bool live = tw < TPW;  // lanes past the wavefront's last whole team take no part
  const int team = wv * TPW + (live ? tw : 0), b = live ? lane - tw * nVar : 0, sbase = tw * nVar;
  const int g = xcd_block(blockIdx.x, gridDim.x);
  const int2 w0 = wg_plan[g], w1 = wg_plan[g + 1];  // {first node, its first adjacency entry}
  const int n_lo = w0.x, n_hi = w1.x, kb = w0.y, ke = w1.y;
  double* slot = ssm + team * TS;
  const bool fused = RX_ASMV_FUSE && cv.V != nullptr;
  // ---- phase A: edge side kb + team
  if (live && kb + team < ke) {
    const int4 sr = side_rec[kb + team];  // {edge | side << 31, n0, n1, BSR block of the neighbour row's entry}
    const int e = sr.x & 0x7fffffff, side = (int)((unsigned)sr.x >> 31);
    const int n0 = sr.y, n1 = sr.z;
    const double* tile = Summ + (size_t)(e / kSummTile) * SS * kSummTile + e % kSummTile;
    double fc, jd[nVar];
    double sob, fv;
    double* Ao;
    if (RX_ASMES_STAGE && fused && RX_ASMES_PROBE != 3 && RX_ASMES_PROBE != 5) {
      // loads in two groups, in this issue order (vmcnt retires in order): (1) the node records the AUSM pass reads,
      // one entry per lane, and the per-edge indices; (2) the summary record, into registers. The AUSM pass waits
      // only for group 1 (through the team's LDS slot: one global load per lane and record instead of one per entry
      // and lane); the summary lands while it computes, and goes to the slot after it.
      const double* Vsi = cv.VR ? cv.VR + 2 * (size_t)e * nPV : cv.V + (size_t)n0 * nPV;
      const double* Vsj = cv.VR ? cv.VR + (2 * (size_t)e + 1) * nPV : cv.V + (size_t)n1 * nPV;
      const double* Ssi = cv.VR ? cv.SR + 2 * (size_t)e * nVar : cv.dPdU + (size_t)n0 * nVar;
      const double* Ssj = cv.VR ? cv.SR + (2 * (size_t)e + 1) * nVar : cv.dPdU + (size_t)n1 * nVar;
      constexpr int kVX = nPV - nVar;  // record entries past the team's width (3 in every instantiation)
      static_assert(kVX >= 0 && kVX <= nVar, "a record is at most two loads per lane");
      static_assert(SS + 2 * nPV + 2 * nVar <= TS, "the staged records fit the team's slot beside the summary");
      const double gvi = Vsi[b], gvj = Vsj[b], gsi = Ssi[b], gsj = Ssj[b];
      const double gxi = b < kVX ? Vsi[nVar + b] : 0.0, gxj = b < kVX ? Vsj[nVar + b] : 0.0;
      double nrm[NDIM];
#pragma unroll
      for (int d = 0; d < NDIM; ++d) nrm[d] = cv.normal[(size_t)e * NDIM + d];
      sob = dTdU[(size_t)(side ? n1 : n0) * nVar + b];
      fv = Fv[(size_t)e * nVar + b];
      Ao = A + (int64_t)sr.w * nVar2;
      __builtin_amdgcn_sched_barrier(0);
      constexpr int kSR = (SS + nVar - 1) / nVar;
      double sreg[kSR];
#pragma unroll
      for (int q = 0; q < kSR; ++q)
        sreg[q] = RX_ASMES_PROBE == 1 ? 0.25 + q : b + q * nVar < SS ? tile[(size_t)(b + q * nVar) * kSummTile] : 0.0;
      __builtin_amdgcn_sched_barrier(0);
      double* vs = slot + SS;  // V_i, V_j, dP/dU_i, dP/dU_j
      vs[b] = gvi;
      vs[nPV + b] = gvj;
      if (b < kVX) {
        vs[nVar + b] = gxi;
        vs[nPV + nVar + b] = gxj;
      }
      vs[2 * nPV + b] = gsi;
      vs[2 * nPV + nVar + b] = gsj;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const double* Li = vs;
      const double* Lj = vs + nPV;
      AusmEdge s;
      {
        double Vi[nPV], Vj[nPV];  // the entries ausm_scalars reads
#pragma unroll
        for (int v = 0; v < nPV; ++v) {
          Vi[v] = v <= NDIM + 2 || v == NDIM + 4 ? Li[v] : 0.0;
          Vj[v] = v <= NDIM + 2 || v == NDIM + 4 ? Lj[v] : 0.0;
        }
        ausm_scalars<NDIM>(Vi, Vj, nrm, cv.mInfty, s);
      }
      bool bad = false;
      {
        const int pidx = (b <= NDIM) ? b : (b == NDIM + 1 ? NDIM + 3 : b + 3);
        const double pi = b == 0 ? 1.0 : Li[pidx];
        const double pj = b == 0 ? 1.0 : Lj[pidx];
        double f = 0.5 * (s.M12 * (pi + pj) + fabs(s.M12) * (pi - pj)) * s.Area;
        if (b >= 1 && b <= NDIM) f += s.pLF * pick<NDIM>(s.UN, b - 1) * s.Area;
        bad |= isnan(f);
        fc = f;
      }
      const AusmCol cc = ausm_col_b<NDIM>(s, gsi, gsj, b);
#pragma unroll
      for (int a = 0; a < nVar; ++a) {
        const double v = ausm_jac_entry_own<NDIM>(s, cc, ausm_phi<NDIM>(Li, Li[NDIM + 3], a),
                                                  ausm_phi<NDIM>(Lj, Lj[NDIM + 3], a), side ? gsj : gsi, a, b, side);
        bad |= isnan(v);
        jd[a] = v;
      }
      if (bad) set_err(cv.err, ERR_NAN_UPWIND, (int64_t)e);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < kSR; ++q)
        if (b + q * nVar < SS) slot[b + q * nVar] = sreg[q];
    } else {
      for (int q = b; q < SS; q += nVar) slot[q] = RX_ASMES_PROBE == 1 ? 0.25 + q : tile[(size_t)q * kSummTile];
      sob = dTdU[(size_t)(side ? n1 : n0) * nVar + b];  // the own node's dT/dU
      fv = Fv[(size_t)e * nVar + b];
      Ao = A + (int64_t)sr.w * nVar2;
    if (RX_ASMES_PROBE == 3 || RX_ASMES_PROBE == 5) {
      const double* Vsi = cv.V + (size_t)n0 * nPV;
      fc = Vsi[b];
#pragma unroll
      for (int a = 0; a < nVar; ++a) jd[a] = cv.dPdU[(size_t)n1 * nVar + a];
    } else if (fused) {
      // k_asm_visc's fused pass: the edge scalars (every lane of the team makes the same ones: one pass of the
      // wavefront for its five edges), this lane's flux component and the own side's Jacobian column
      const double* Vsi = cv.VR ? cv.VR + 2 * (size_t)e * nPV : cv.V + (size_t)n0 * nPV;
      const double* Vsj = cv.VR ? cv.VR + (2 * (size_t)e + 1) * nPV : cv.V + (size_t)n1 * nPV;
      const double* Ssi = cv.VR ? cv.SR + 2 * (size_t)e * nVar : cv.dPdU + (size_t)n0 * nVar;
      const double* Ssj = cv.VR ? cv.SR + (2 * (size_t)e + 1) * nVar : cv.dPdU + (size_t)n1 * nVar;
      AusmEdge s;
      {
        double Vi[nPV], Vj[nPV], nrm[NDIM];  // the entries ausm_scalars reads
#pragma unroll
        for (int v = 0; v < nPV; ++v) {
          Vi[v] = v <= NDIM + 2 || v == NDIM + 4 ? Vsi[v] : 0.0;
          Vj[v] = v <= NDIM + 2 || v == NDIM + 4 ? Vsj[v] : 0.0;
        }
#pragma unroll
        for (int d = 0; d < NDIM; ++d) nrm[d] = cv.normal[(size_t)e * NDIM + d];
        ausm_scalars<NDIM>(Vi, Vj, nrm, cv.mInfty, s);
      }
      bool bad = false;
      {
        const int pidx = (b <= NDIM) ? b : (b == NDIM + 1 ? NDIM + 3 : b + 3);
        const double pi = b == 0 ? 1.0 : Vsi[pidx];
        const double pj = b == 0 ? 1.0 : Vsj[pidx];
        double f = 0.5 * (s.M12 * (pi + pj) + fabs(s.M12) * (pi - pj)) * s.Area;
        if (b >= 1 && b <= NDIM) f += s.pLF * pick<NDIM>(s.UN, b - 1) * s.Area;
        bad |= isnan(f);
        fc = f;
      }
      const double sib = Ssi[b], sjb = Ssj[b];
      const AusmCol cc = ausm_col_b<NDIM>(s, sib, sjb, b);
#pragma unroll
      for (int a = 0; a < nVar; ++a) {
        const double v = ausm_jac_entry_own<NDIM>(s, cc, ausm_phi<NDIM>(Vsi, Vsi[NDIM + 3], a),
                                                  ausm_phi<NDIM>(Vsj, Vsj[NDIM + 3], a), side ? sjb : sib, a, b, side);
        bad |= isnan(v);
        jd[a] = v;
      }
      if (bad) set_err(cv.err, ERR_NAN_UPWIND, (int64_t)e);
    } else {
      fc = Fc[(size_t)e * nVar + b];
      const double* J = Jc + ((size_t)e * 2 + side) * nVar2 + b;
#pragma unroll
      for (int a = 0; a < nVar; ++a) jd[a] = J[a * nVar];
    }
    }
    double jco[nVar];  // 0 -+ this lane's column of the own-side convective block
#pragma unroll
    for (int a = 0; a < nVar; ++a) jco[a] = side ? 0.0 + jd[a] : 0.0 - jd[a];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    double jv[nVar];
    if (RX_ASMES_PROBE == 2 || RX_ASMES_PROBE == 5) {
#pragma unroll
      for (int rr = 0; rr < nVar; ++rr) {
        jv[rr] = sob * slot[rr];
        Ao[rr * nVar + b] = side ? jco[rr] - jv[rr] : jco[rr] + jv[rr];
      }
    } else {
      visc_jac_column_own<NS, NDIM>(m, P, SummCRef{slot, 1}, sob, side, b, b, sbase, [&](int rr, double v) {
        jv[rr] = v;
        if (RX_ASMES_PROBE != 6) Ao[rr * nVar + b] = side ? jco[rr] - v : jco[rr] + v;
      });
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // the team has read its summary record: the slot takes the parked outputs
    double* o = slot + b * OW;
#pragma unroll
    for (int a = 0; a < nVar; ++a) {
      o[a] = side ? -jd[a] : jd[a];
      o[nVar + 1 + a] = side ? jv[a] : -jv[a];
    }
    o[nVar] = side ? -fc : fc;
    o[2 * nVar + 1] = side ? fv : -fv;
  }
  // ---- phase B: node n_lo + team. Its loads are issued before the barrier (phase A's registers are dead here), so
  // they are in flight while the other teams finish
  const int i = n_lo + team;
  const bool node = live && i < n_hi;
  int k0 = 0, k1 = 0, fold = 0;
  double rs = 0.0, js[NS], delta = 0.0;
  int64_t dblk = 0;
  if (node) {
    k0 = adj_ptr[i];
    k1 = adj_ptr[i + 1];
    dblk = diag[i];
    if (src && RX_ASMES_PROBE != 7) {
      rs = Rsrc[(size_t)i * nVar + b];
#pragma unroll
      for (int a = 0; a < NS; ++a)
        js[a] = Js[(size_t)(i / kSrcTile) * nsv * kSrcTile + (size_t)(a * nVar + b) * kSrcTile + i % kSrcTile];
    }
    if (fd.vol && i < fd.Nd && !fd.skip[i]) {
      // ImplicitEuler_Iteration's AddVal2Diag (k_build_system_elem's operations on this lane's column)
      const double dt = fd.dt[i];
      fold = dt > rx::kEPS ? 1 : 2;
      if (fold == 1) delta = fd.vol[i] / dt;
    }
  }
  __syncthreads();
  if (!node) return;
  double r = 0.0, D[nVar];
#pragma unroll
  for (int a = 0; a < nVar; ++a) D[a] = 0.0;
  for (int k = k0; k < (RX_ASMES_PROBE == 4 ? k0 + 1 : k1); ++k) {
    const double* o = ssm + (k - kb) * TS + b * OW;
    r += o[nVar];
#pragma unroll
    for (int a = 0; a < nVar; ++a) D[a] += o[a];
  }
  for (int k = k0; k < (RX_ASMES_PROBE == 4 ? k0 : k1); ++k) {
    const double* o = ssm + (k - kb) * TS + b * OW;
    r += o[2 * nVar + 1];
#pragma unroll
    for (int a = 0; a < nVar; ++a) D[a] += o[nVar + 1 + a];
  }
  if (src) {
    r += rs;
#pragma unroll
    for (int a = 0; a < nVar; ++a) D[a] += a >= rhos ? js[a - rhos] : 0.0;
  }
  if (fold == 1) {
#pragma unroll
    for (int a = 0; a < nVar; ++a)
      if (a == b) D[a] += delta;
  } else if (fold == 2) {
#pragma unroll
    for (int a = 0; a < nVar; ++a) D[a] = (a == b) ? 1.0 : 0.0;
    r = 0.0;
  }
  R[(size_t)i * nVar + b] = r;
  double* Ad = A + dblk * nVar2 + b;
#pragma unroll
  for (int a = 0; a < nVar; ++a) Ad[a * nVar] = D[a];
}

// a12: weighted least-squares gradient of (T, u, v, P, X_s) per node.
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) void k_grad_lsq(int N, const int32_t* __restrict__ nptr,
                                                     const int32_t* __restrict__ nbr, const double* __restrict__ coord,
                                                     const double* __restrict__ V, DevMech m, double* __restrict__ Gout,
                                                     const int32_t* __restrict__ list) {
  constexpr int nPV = NS + NDIM + 5, nG = NS + NDIM + 2, P_P = NDIM + 1, RHOS_P = NDIM + 5, P_G = NDIM + 1,
                RHOS_G = NDIM + 2;
#ifndef RX_GRAD_XCD
#define RX_GRAD_XCD 1  // round 6: workgroups in XCD order (xcd_block), the neighbour records under one L2
#endif
  const int t = (RX_GRAD_XCD ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= N) return;
  const int i = list ? list[t] : t;  // list: the points of one half of the distributed split (rx_grad_lsq)
  double pi[nG], pj[nG], C[nG][NDIM];
  {
    const double* v = V + (size_t)i * nPV;
    pi[0] = v[0];
    pi[P_G] = v[P_P];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) pi[1 + d] = v[1 + d];
    double ys[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) ys[s] = v[RHOS_P + s];
    molar_from_mass<NS>(m, ys, pi + RHOS_G);
  }
#pragma unroll
  for (int g = 0; g < nG; ++g)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) C[g][d] = 0.0;
  double r11 = 0, r12 = 0, r13 = 0, r22 = 0, r23 = 0, r23_a = 0, r23_b = 0, r33 = 0;
  double ci[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) ci[d] = coord[(size_t)i * NDIM + d];
  auto neighbour = [&](int j) {
    const double* v = V + (size_t)j * nPV;
    pj[0] = v[0];
    pj[P_G] = v[P_P];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) pj[1 + d] = v[1 + d];
    double ys[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) ys[s] = v[RHOS_P + s];
    molar_from_mass<NS>(m, ys, pj + RHOS_G);
    double cij[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int d = 0; d < NDIM; ++d) cij[d] = coord[(size_t)j * NDIM + d] - ci[d];
    double w = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) w += cij[d] * cij[d];
    if (w > kEPS) {
      r11 += cij[0] * cij[0] / w;
      r12 += cij[0] * cij[1] / w;
      r22 += cij[1] * cij[1] / w;
      if (NDIM == 3) {
        r13 += cij[0] * cij[2] / w;
        r23_a += cij[1] * cij[2] / w;
        r23_b += cij[0] * cij[2] / w;
        r33 += cij[2] * cij[2] / w;
      }
#pragma unroll
      for (int g = 0; g < nG; ++g)
#pragma unroll
        for (int d = 0; d < NDIM; ++d) C[g][d] += cij[d] * (pj[g] - pi[g]) / w;
    }
  };
  // neighbours in the reference's order; the first 2 NDIM indices are loaded together first, so the neighbours'
  // record loads do not each wait on their index load
  {
    const int k0 = nptr[i], k1 = nptr[i + 1];
    constexpr int PF = 2 * NDIM;
    int jp[PF];
#pragma unroll
    for (int t = 0; t < PF; ++t) jp[t] = nbr[k0 + t < k1 ? k0 + t : k0];
#pragma unroll
    for (int t = 0; t < PF; ++t)
      if (k0 + t < k1) neighbour(jp[t]);
    for (int k = k0 + PF; k < k1; ++k) neighbour(nbr[k]);
  }
  r11 = (r11 > kEPS) ? sqrt(r11) : 0.0;
  r12 = (fabs(r11) > kEPS) ? r12 / r11 : 0.0;
  r22 = (r22 - r12 * r12 > kEPS) ? sqrt(r22 - r12 * r12) : 0.0;
  if (NDIM == 3) {
    r13 = (fabs(r11) > kEPS) ? r13 / r11 : 0.0;
    r23 = (fabs(r22) > kEPS && fabs(r11 * r22) > kEPS) ? r23_a / r22 - r23_b * r12 / (r11 * r22) : 0.0;
    r33 = (r33 - r23 * r23 - r13 * r13 > kEPS) ? sqrt(r33 - r23 * r23 - r13 * r13) : 0.0;
  }
  double detR2 = (NDIM == 2) ? (r11 * r22) * (r11 * r22) : (r11 * r22 * r33) * (r11 * r22 * r33);
  bool singular = false;
  if (fabs(detR2) < kEPS) {
    detR2 = 1.0;
    singular = true;
  }
  double S[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
  if (!singular) {
    if (NDIM == 2) {
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
#pragma unroll
  for (int g = 0; g < nG; ++g)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      double r = 0.0;
#pragma unroll
      for (int e = 0; e < NDIM; ++e) r += C[g][e] * S[d][e];
      Gout[((size_t)i * nG + g) * NDIM + d] = r;
    }
}

// a13: Venkatakrishnan limiter, node-centric (min over incident edges is order independent).
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_limiter_minmax(int N, int nPV, const int32_t* __restrict__ adj_ptr,
                                                           const int32_t* __restrict__ adj,
                                                           const int32_t* __restrict__ edges,
                                                           const double* __restrict__ V, double* __restrict__ mn,
                                                           double* __restrict__ mx) {
  constexpr int nL = NDIM + 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double lo[nL], hi[nL];
#pragma unroll
  for (int v = 0; v < nL; ++v) {
    lo[v] = kEPS;
    hi[v] = -kEPS;
  }
  auto pl = [&](int p, int v) {
    const double* pv = V + (size_t)p * nPV;
    return v == 0 ? pv[0] : (v == nL - 1 ? pv[NDIM + 1] : pv[v]);
  };
  for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
    const int a = adj[k];
    const int e = a >> 1, side = a & 1;
    const int n0 = edges[2 * e], n1 = edges[2 * e + 1];
#pragma unroll
    for (int v = 0; v < nL; ++v) {
      const double du = pl(n1, v) - pl(n0, v);
      const double d = side ? -du : du;
      lo[v] = fmin(lo[v], d);
      hi[v] = fmax(hi[v], d);
    }
  }
#pragma unroll
  for (int v = 0; v < nL; ++v) {
    mn[(size_t)i * nL + v] = lo[v];
    mx[(size_t)i * nL + v] = hi[v];
  }
}

template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_limiter_venkat(int N, int nG, const int32_t* __restrict__ adj_ptr,
                                                           const int32_t* __restrict__ adj,
                                                           const int32_t* __restrict__ edges,
                                                           const double* __restrict__ coord,
                                                           const double* __restrict__ G, const double* __restrict__ mn,
                                                           const double* __restrict__ mx, double eps2,
                                                           double* __restrict__ lim) {
  constexpr int nL = NDIM + 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double l[nL];
#pragma unroll
  for (int v = 0; v < nL; ++v) l[v] = 2.0;
  double ci[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) ci[d] = coord[(size_t)i * NDIM + d];
  const double* Gi = G + (size_t)i * nG * NDIM;
  for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
    const int a = adj[k];
    const int e = a >> 1, side = a & 1;
    const int other = edges[2 * e + (side ^ 1)];
#pragma unroll
    for (int v = 0; v < nL; ++v) {
      double dm = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) dm += 0.5 * (coord[(size_t)other * NDIM + d] - ci[d]) * Gi[v * NDIM + d];
      const double dp = (dm > 0.0) ? mx[(size_t)i * nL + v] : mn[(size_t)i * nL + v];
      const double lv = (dp * dp + 2.0 * dp * dm + eps2) / (dp * dp + dp * dm + 2.0 * dm * dm + eps2);
      if (lv < l[v]) l[v] = lv;
    }
  }
#pragma unroll
  for (int v = 0; v < nL; ++v) lim[(size_t)i * nL + v] = l[v];
}

// a13: Barth-Jespersen branch (solver_direct_reactive.cpp:1383-1440), node-centric. Unlike Venkatakrishnan's min,
// the j side's update (:1426-1427: `if (limiter < L_j) L_j = value`, the bool member, 1 whenever the limiter runs)
// is an overwrite, so the order matters: a node walks its incident edges in ascending edge index (adj is built
// edge-ordered), i.e. the reference's edge loop restricted to that node. dm < EPS gives 2.0; dp is the max for
// dm > EPS, the min for dm == EPS. Then y -> (y^2 + 2y) / (y^2 + y + 2) (:1433-1439).
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_limiter_barth(int N, int nG, const int32_t* __restrict__ adj_ptr,
                                                          const int32_t* __restrict__ adj,
                                                          const int32_t* __restrict__ edges,
                                                          const double* __restrict__ coord,
                                                          const double* __restrict__ G, const double* __restrict__ mn,
                                                          const double* __restrict__ mx, double* __restrict__ lim) {
  constexpr int nL = NDIM + 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double l[nL], lo[nL], hi[nL];
#pragma unroll
  for (int v = 0; v < nL; ++v) {
    l[v] = 2.0;
    lo[v] = mn[(size_t)i * nL + v];
    hi[v] = mx[(size_t)i * nL + v];
  }
  double ci[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) ci[d] = coord[(size_t)i * NDIM + d];
  const double* Gi = G + (size_t)i * nG * NDIM;
  for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
    const int a = adj[k];
    const int e = a >> 1, side = a & 1;
    const int other = edges[2 * e + (side ^ 1)];
#pragma unroll
    for (int v = 0; v < nL; ++v) {
      double dm = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) dm += 0.5 * (coord[(size_t)other * NDIM + d] - ci[d]) * Gi[v * NDIM + d];
      const double lv = dm < kEPS ? 2.0 : (dm > kEPS ? hi[v] : lo[v]) / dm;
      if (side ? 1.0 < l[v] : lv < l[v]) l[v] = lv;
    }
  }
#pragma unroll
  for (int v = 0; v < nL; ++v) {
    const double y = l[v];
    lim[(size_t)i * nL + v] = (y * y + 2.0 * y) / (y * y + y + 2.0);
  }
}

// a18: SetTime_Step (RANS branch), node-centric over incident edges then boundary vertices.
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_time_step(int N, int nPV, int nVar, const int32_t* __restrict__ adj_ptr,
                                                      const int32_t* __restrict__ adj,
                                                      const int32_t* __restrict__ edges,
                                                      const double* __restrict__ normal,
                                                      const int32_t* __restrict__ bv_ptr,
                                                      const double* __restrict__ bv_normal,
                                                      const double* __restrict__ V, const double* __restrict__ dPdU,
                                                      const double* __restrict__ mu, const double* __restrict__ eddy,
                                                      const double* __restrict__ vol,
                                                      const int32_t* __restrict__ nptr, double CFL, double maxdt,
                                                      double Pr_l, double Pr_t, double* __restrict__ dt,
                                                      double* __restrict__ li_out, double* __restrict__ lv_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int RHO_P = NDIM + 2, A_P = NDIM + 4, RHOE_S = NDIM + 1;
  double li = 0.0, lv = 0.0;
  auto pvel = [&](int p, const double* n) {
    double s = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) s += V[(size_t)p * nPV + 1 + d] * n[d];
    return s;
  };
  auto edge = [&](int e, int n0, int n1) {
    double n[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) n[d] = normal[(size_t)e * NDIM + d];
    double Area = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Area += n[d] * n[d];
    Area = sqrt(Area);
    const double pv = 0.5 * (pvel(n0, n) + pvel(n1, n));
    const double a = 0.5 * (V[(size_t)n0 * nPV + A_P] + V[(size_t)n1 * nPV + A_P]);
    const double rho = 0.5 * (V[(size_t)n0 * nPV + RHO_P] + V[(size_t)n1 * nPV + RHO_P]);
    const double m = 0.5 * (mu[n0] + mu[n1]);
    li += (fabs(pv) + a) * Area;
    const double mt = 0.5 * (eddy[n0] + eddy[n1]);
    const double gam = dPdU[(size_t)n0 * nVar + RHOE_S] + 1;
    const double l1 = 4.0 / 3.0 * (m + mt);
    const double l2 = (1.0 + (Pr_l / Pr_t) * (mt / m)) * (gam * m / Pr_l);
    lv += (l1 + l2) * Area * Area / rho;
  };
  // incident edges in edge order; the index chains of the first 2 NDIM edges are loaded together first, so the
  // edges' data loads do not wait on one another (DT 0.18 ms at C3 with the serial adj -> edges -> data chain)
  const int k0 = adj_ptr[i], k1 = adj_ptr[i + 1];
  constexpr int PF = 2 * NDIM;
  int ep[PF], e0p[PF], e1p[PF];
#pragma unroll
  for (int t = 0; t < PF; ++t) ep[t] = adj[k0 + t < k1 ? k0 + t : k0] >> 1;
#pragma unroll
  for (int t = 0; t < PF; ++t) {
    e0p[t] = edges[2 * ep[t]];
    e1p[t] = edges[2 * ep[t] + 1];
  }
#pragma unroll
  for (int t = 0; t < PF; ++t)
    if (k0 + t < k1) edge(ep[t], e0p[t], e1p[t]);
  for (int k = k0 + PF; k < k1; ++k) {
    const int e = adj[k] >> 1;
    edge(e, edges[2 * e], edges[2 * e + 1]);
  }
  for (int b = bv_ptr[i]; b < bv_ptr[i + 1]; ++b) {
    double n[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) n[d] = bv_normal[(size_t)b * NDIM + d];
    double Area = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Area += n[d] * n[d];
    Area = sqrt(Area);
    const double pv = pvel(i, n);
    li += (fabs(pv) + V[(size_t)i * nPV + A_P]) * Area;
    const double m = mu[i], mt = eddy[i];
    const double gam = dPdU[(size_t)i * nVar + RHOE_S] + 1;
    const double l1 = (4.0 / 3.0) * (m + mt);
    const double l2 = (1.0 + (Pr_l / Pr_t) * (mt / m)) * (gam * m / Pr_l);
    lv += (l1 + l2) * Area * Area / V[(size_t)i * nPV + RHO_P];
  }
  li_out[i] = li;
  lv_out[i] = lv;
  double d = 0.0;
  if (vol[i] > kEPS) {
    d = CFL * vol[i] / li;
    const double dv = CFL * 0.25 * vol[i] * vol[i] / lv;
    d = fmin(d, dv);
    if (d > maxdt) d = maxdt;
  }
  dt[i] = d;
  // points with a single neighbour take the global minimum (rare; fixed up on the host path)
  (void)nptr;
}

inline int blocks(int64_t n, int b = kBlock) { return (int)((n + b - 1) / b); }

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

}  // namespace

#if !RX_NS
int rx_fail_hip(rx_ctx* ctx, hipError_t e) {
  (void)ctx;
  fprintf(stderr, "rx: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
  return RX_ERR_HIP;
}

int rx_check_error(rx_ctx* ctx) {
  int h[2] = {0, 0};
  RX_HIP(hipMemcpyAsync(h, ctx->err, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  RX_HIP(hipStreamSynchronize(ctx->stream));
  if (h[0] != 0) {
    ctx->last_err_index = h[1];
    ctx->last_err_phase = h[0] == ERR_NAN_UPWIND ? 1 : 0;
    RX_HIP(hipMemsetAsync(ctx->err, 0, 2 * sizeof(int), ctx->stream));
    return h[0] == ERR_RANGE ? RX_ERR_RANGE : (h[0] == ERR_CONV ? RX_ERR_NONPHYS : RX_ERR_NAN);
  }
  return RX_OK;
}

#endif  // !RX_NS

#if RX_NS
int RX_NSFN(rx_launch_set_primitive)(rx_ctx* ctx, int ext_iter, int64_t lo, int64_t hi) {  // points [lo, hi)
  if (hi <= lo) return RX_OK;
  const rx_cfg& c = ctx->cfg;
  const int ignite = c.ignition && (int64_t)ext_iter < c.ignition_iter ? 1 : 0;
  if (ignite && (c.fuel_index < 0 || c.fuel_index >= ctx->ns || c.oxidizer_index < 0 || c.oxidizer_index >= ctx->ns))
    return RX_ERR_ARG;
  PrimParams P{c.t_min, c.t_max, c.T_ref, c.E_ref, c.R_ref, c.p_ref, c.visc_ref, c.cond_ref, c.vel_ref, c.len_ref,
               ext_iter, c.clip_temp, c.rans, ignite, c.fuel_index, c.oxidizer_index, c.ignition_temp};
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_set_primitive<NS_, ND_><<<blocks(hi - lo), kBlock, 0, ctx->stream>>>(
                            (int)lo, (int)hi, ctx->mech, P, ctx->f[RX_F_U], ctx->f[RX_F_V], ext_iter > 0 ? ctx->uold : nullptr,
                            ctx->f[RX_F_TKE], ctx->f[RX_F_MUT], ctx->f[RX_F_DPDU], ctx->f[RX_F_DTDU], ctx->f[RX_F_MU],
                            ctx->f[RX_F_KAPPA], ctx->f[RX_F_DIJ], ctx->f[RX_F_EDDY], ctx->err)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int RX_NSFN(rx_launch_muscl)(rx_ctx* ctx) {
  if (!ctx->recon) return RX_ERR_ARG;
  const double* lim = ctx->cfg.spatial_order == 2 ? ctx->f[RX_F_LIMITER] : nullptr;
  double* SR = ctx->cfg.implicit ? ctx->recon + 2 * ctx->E * (int64_t)ctx->nPV : nullptr;
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_muscl_edge<NS_, ND_><<<blocks(2 * ctx->E), kBlock, 0, ctx->stream>>>(
                            (int)ctx->E, ctx->edges, ctx->coord, ctx->f[RX_F_V], ctx->f[RX_F_DPDU], ctx->f[RX_F_GRAD],
                            lim, ctx->mech, ctx->cfg.T_ref, ctx->cfg.E_ref, ctx->cfg.R_ref, ctx->cfg.implicit,
                            ctx->recon, SR, ctx->err)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int RX_NSFN(rx_launch_ausm_node)(rx_ctx* ctx) {
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_ausm_node<NS_, ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>(
                            (int)ctx->N, ctx->adj_ptr, ctx->adj, ctx->edges, ctx->normal, ctx->f[RX_F_V],
                            ctx->cfg.spatial_order ? ctx->recon : nullptr, ctx->cfg.mach_inf, ctx->f[RX_F_RES],
                            ctx->err)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

#endif  // RX_NS

#if !RX_NS
// the implicit convective fluxes and Jacobians are made by the node-centric assembly (k_asm_visc's fused AUSM pass)
// instead of k_ausm_edge whenever the assembly also makes the viscous Jacobians. 2-D since round 4: C3 (same box) CONV
// 1.31 + ASSEMBLE 4.89 -> ASSEMBLE 6.79 ms then, 5.75 ms now. 3-D since round 5: with only the own side's entries
// evaluated and nVar-lane teams (5 nodes per wavefront), C5 (same box, gpurun_out r05q) CONV 2.01 + ASSEMBLE 7.53 ->
// ASSEMBLE 9.13 ms, 39.91 -> 39.55 ms per step (round 4: 2.29 + 8.71 -> 11.76 ms, so 3-D kept the edge kernel).
// RX_ASM_CONV=0 never fuses (A/B, tests/test_gpu_assembly.py); RX_ASM_VISC=0 never fuses
int rx_asmes_teams(int nVar) { return asmes_teams(nVar); }

bool rx_fuse_conv(int nDim) {
  (void)nDim;
  static const int mode = [] {
    const char* v = getenv("RX_ASM_CONV");
    const char* w = getenv("RX_ASM_VISC");
    if (w && w[0] == '0') return 0;
    return v && v[0] == '0' ? 0 : 1;
  }();
  return mode == 1;
}
#endif  // !RX_NS

#if RX_NS
int RX_NSFN(rx_launch_ausm_edge)(rx_ctx* ctx) {
  if (!ctx->jconv) {  // allocated at first use: the 2-D fused assembly never needs the per-edge blocks
    if (ctx->capturing) return RX_ERR_STATE;
    // both or neither (a failed jconv used to leave fconv allocated, and the next call allocated it again)
    if (!ctx->fconv) RX_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->fconv), sizeof(double) * ctx->E * ctx->nVar));
    const hipError_t e =
        hipMalloc(reinterpret_cast<void**>(&ctx->jconv), sizeof(double) * ctx->E * 2 * ctx->nVar * ctx->nVar);
    if (e != hipSuccess) {
      (void)hipFree(ctx->fconv);
      ctx->fconv = nullptr;
      ctx->jconv = nullptr;
      return rx_fail_hip(ctx, e);
    }
  }
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_ausm_edge<NS_, ND_><<<blocks(ctx->E * kAusmTeam, kAusmBlock), kAusmBlock, 0, ctx->stream>>>(
                            (int)ctx->E, ctx->edges, ctx->normal, ctx->f[RX_F_V], ctx->f[RX_F_DPDU],
                            ctx->cfg.spatial_order ? ctx->recon : nullptr,
                            ctx->cfg.spatial_order ? ctx->recon + 2 * ctx->E * (int64_t)ctx->nPV : nullptr,
                            ctx->cfg.mach_inf, ctx->fconv, ctx->jconv, ctx->err)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int RX_NSFN(rx_launch_visc_edge)(rx_ctx* ctx) {
  ViscParams P{ctx->cfg.T_ref, ctx->cfg.E_ref, ctx->cfg.R_ref, ctx->cfg.prandtl_turb, ctx->cfg.lewis_turb,
               ctx->cfg.rans, ctx->cfg.implicit};
  {
    RxPhase ph(ctx, RX_K_VISC);
    RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_visc_edge<NS_, ND_><<<blocks(ctx->E, 64), 64, 0, ctx->stream>>>(
                              (int)ctx->E, ctx->edges, ctx->normal, ctx->coord, ctx->f[RX_F_V], ctx->f[RX_F_GRAD],
                              ctx->f[RX_F_MU], ctx->f[RX_F_KAPPA], ctx->f[RX_F_DIJ], ctx->f[RX_F_DTDU],
                              ctx->f[RX_F_TKE], ctx->f[RX_F_MUT], ctx->f[RX_F_SIGMAK], ctx->f[RX_F_GRADK],
                              ctx->mech, P, ctx->fvisc, ctx->vsumm, ctx->err)));
    RX_HIP(hipGetLastError());
  }
  // the node-centric viscous Jacobians + assembly (k_asm_visc, launched by rx_launch_assemble) replace k_visc_jac
  // and k_assemble's viscous pass (C3: 3.57 + 2.17 -> 5.13 ms, 128/128 GPU tests bitwise); RX_ASM_VISC=0 restores
  // the edge kernel + node assembly (A/B, diagnosis)
  static const bool asm_visc = [] {
    const char* v = getenv("RX_ASM_VISC");
    return !(v && v[0] == '0');
  }();
  ctx->asm_visc = ctx->cfg.implicit && asm_visc ? 1 : 0;
  if (ctx->cfg.implicit && ctx->asm_visc) return RX_OK;
  if (ctx->cfg.implicit) {
    RxPhase ph(ctx, RX_K_VISC_JAC);
    // fused off-diagonal assembly needs this residual's convective blocks (rx_edge_flux_conv ran first)
    static const bool no_fuse = getenv("RX_NO_FUSED_ASM") != nullptr;  // diagnostic: the unfused assembly
    const int fuse = ctx->phase_conv && !no_fuse ? 1 : 0;
    RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_visc_jac<NS_, ND_><<<blocks(ctx->E * 16), kBlock, 0, ctx->stream>>>(
                              (int)ctx->E, ctx->edges, ctx->f[RX_F_DTDU], ctx->vsumm, ctx->mech, P, ctx->jvisc,
                              fuse ? ctx->jconv : nullptr, ctx->edge_blk, ctx->f[RX_F_JAC])));
    RX_HIP(hipGetLastError());
    ctx->offdiag_done = fuse;
  }
  return RX_OK;
}

#endif  // RX_NS

#if !RX_NS
int rx_launch_gather_edge_flux(rx_ctx* ctx, const double* flux, double sign_first) {
  k_gather_flux<<<blocks(ctx->N * ctx->nVar), kBlock, 0, ctx->stream>>>(
      (int)ctx->N, ctx->nVar, ctx->adj_ptr, ctx->adj, flux, sign_first, ctx->f[RX_F_RES]);
  RX_HIP(hipGetLastError());
  return RX_OK;
}

#endif  // !RX_NS

#if RX_NS
int RX_NSFN(rx_launch_source)(rx_ctx* ctx) {
  SourceParams P{ctx->cfg.c_mu, ctx->cfg.pasr_lb, ctx->cfg.rho_ref, ctx->cfg.t_ref, ctx->cfg.T_ref, ctx->cfg.rans,
                 ctx->cfg.implicit};
  // explicit: R += S directly; implicit: S and its Jacobian go to scratch, folded in by k_assemble
  double* Rdst = ctx->cfg.implicit ? ctx->rsrc : ctx->f[RX_F_RES];
  const int add = ctx->cfg.implicit ? 0 : 1;
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_source<NS_, ND_><<<blocks(ctx->N, 128), 128, 0, ctx->stream>>>(
                            (int)ctx->N, ctx->f[RX_F_V], ctx->f[RX_F_DTDU], ctx->vol, ctx->f[RX_F_OMEGA], ctx->mech,
                            P, Rdst, add, ctx->jsrc, ctx->err)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// the node-centric viscous Jacobians + assembly (k_asm_visc), with the AUSM pass fused when fused_conv
int RX_NSFN(rx_launch_asm_visc)(rx_ctx* ctx, int with_src, int fused_conv) {
  ViscParams P{ctx->cfg.T_ref, ctx->cfg.E_ref, ctx->cfg.R_ref, ctx->cfg.prandtl_turb, ctx->cfg.lewis_turb,
               ctx->cfg.rans, ctx->cfg.implicit};
  AusmIn cv{nullptr, nullptr, nullptr, nullptr, nullptr, ctx->cfg.mach_inf, ctx->err};
  if (fused_conv) {
    cv.V = ctx->f[RX_F_V];
    cv.dPdU = ctx->f[RX_F_DPDU];
    cv.VR = ctx->cfg.spatial_order ? ctx->recon : nullptr;
    cv.SR = ctx->cfg.spatial_order ? ctx->recon + 2 * ctx->E * (int64_t)ctx->nPV : nullptr;
    cv.normal = ctx->normal;
  }
  SysFold fd{nullptr, nullptr, nullptr, (int)ctx->Nd};
  if (ctx->fold_req && ctx->fold_skip && with_src) {  // (the whole residual: the build follows)
    fd.vol = ctx->vol;
    fd.dt = ctx->f[RX_F_DT];
    fd.skip = ctx->fold_skip;
  }
  // edge-side teams (k_asm_es, round 6) unless a node has more edges than a workgroup has teams, or RX_ASMV_ES=0 (the
  // node-serial k_asm_visc, for A/B and tests/test_gpu_assembly.py)
  static const bool es = [] {
    const char* v = getenv("RX_ASMV_ES");
    return !(v && v[0] == '0');
  }();
  if (es && !RX_ASMV_PARK && ctx->asmes_wg && ctx->asmes_nwg > 0) {
    RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_asm_es<NS_, ND_><<<ctx->asmes_nwg, RX_ASMES_WAVES * 64, 0, ctx->stream>>>(
                              reinterpret_cast<const int2*>(ctx->asmes_wg),
                              reinterpret_cast<const int4*>(ctx->asmes_side), ctx->adj_ptr, ctx->diag, ctx->fconv,
                              ctx->fvisc, ctx->jconv, ctx->f[RX_F_DTDU], ctx->vsumm, ctx->jsrc, ctx->rsrc, ctx->mech, P,
                              ctx->f[RX_F_RES], ctx->f[RX_F_JAC], with_src, cv, fd)));
    RX_HIP(hipGetLastError());
    ctx->sys_folded = fd.vol ? 1 : 0;
    return RX_OK;
  }
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_asm_visc<NS_, ND_><<<(ctx->N + asmv_nodes_per_block(NS_ + ND_ + 2) - 1) /
                                                                     asmv_nodes_per_block(NS_ + ND_ + 2),
                                                                 kBlock, 0, ctx->stream>>>(
                            (int)ctx->N, ctx->adj_ptr, ctx->adj, ctx->edges, ctx->edge_blk, ctx->diag, ctx->fconv,
                            ctx->fvisc, ctx->jconv, ctx->f[RX_F_DTDU], ctx->vsumm, ctx->jsrc, ctx->rsrc, ctx->mech,
                            P, ctx->f[RX_F_RES], ctx->f[RX_F_JAC], with_src, cv, fd)));
  RX_HIP(hipGetLastError());
  ctx->sys_folded = fd.vol ? 1 : 0;
  return RX_OK;
}
#endif  // RX_NS

#if !RX_NS
RX_NS_DISPATCH(rx_launch_set_primitive, (rx_ctx * ctx, int ext_iter, int64_t lo, int64_t hi), (ctx, ext_iter, lo, hi))
RX_NS_DISPATCH(rx_launch_muscl, (rx_ctx * ctx), (ctx))
RX_NS_DISPATCH(rx_launch_ausm_node, (rx_ctx * ctx), (ctx))
RX_NS_DISPATCH(rx_launch_ausm_edge, (rx_ctx * ctx), (ctx))
RX_NS_DISPATCH(rx_launch_visc_edge, (rx_ctx * ctx), (ctx))
RX_NS_DISPATCH(rx_launch_source, (rx_ctx * ctx), (ctx))
RX_NS_DISPATCH(rx_launch_asm_visc, (rx_ctx * ctx, int with_src, int fused_conv), (ctx, with_src, fused_conv))
RX_NS_DISPATCH(rx_launch_grad_gg, (rx_ctx * ctx), (ctx))
RX_NS_DISPATCH(rx_launch_grad, (rx_ctx * ctx, const int32_t* list, int64_t n), (ctx, list, n))

int rx_launch_assemble(rx_ctx* ctx, int with_visc, int with_src) {
  const int nv = ctx->nVar;
  ctx->sys_folded = 0;  // (set again by a folding k_asm_visc launch)
  const bool fused_conv = ctx->conv_deferred && with_visc && ctx->asm_visc;
  if (ctx->conv_deferred && !fused_conv) {  // deferred, but no viscous pass to fuse it into: the edge kernel now
    const int rc = rx_launch_ausm_edge(ctx);
    if (rc) return rc;
    ctx->conv_deferred = 0;  // this residual's per-edge convective blocks now exist; later assemblies read them
  }
  // fused: conv_deferred stays set (only rx_residual_zero / rx_edge_flux_conv change it), so a re-assembly of the
  // same residual (e.g. a RES download after the viscous loop, then Source_Residual) fuses the AUSM pass again: it
  // rewrites the residual, the diagonal and the off-diagonal blocks, and no per-edge convective block ever exists
  if (with_visc && ctx->asm_visc)  // k_visc_jac was skipped: the node-centric viscous Jacobians + assembly
    return rx_launch_asm_visc(ctx, with_src, fused_conv ? 1 : 0);
  switch (nv) {
#define RX_ASM_DEG(NV, DEG)                                                                                       \
  k_assemble<NV, DEG><<<blocks(ctx->N * asm_team<NV>()), kBlock, 0, ctx->stream>>>(                              \
      (int)ctx->N, NV - ctx->ns, ctx->adj_ptr, ctx->adj, ctx->adj_blk, ctx->diag, ctx->fconv, ctx->fvisc, ctx->jconv, \
      ctx->jvisc, ctx->jsrc, ctx->rsrc, ctx->f[RX_F_RES], ctx->f[RX_F_JAC], with_visc, with_src,                   \
      with_visc && ctx->offdiag_done ? 0 : 1)
#define RX_ASM(NV)                      \
  case NV:                              \
    if (ctx->max_degree <= 4)           \
      RX_ASM_DEG(NV, 4);                \
    else                                \
      RX_ASM_DEG(NV, 8);                \
    break;
    RX_ASM(7)
    RX_ASM(8)
    RX_ASM(9)
    RX_ASM(10)
    RX_ASM(11)
    RX_ASM(12)
    RX_ASM(13)
    RX_ASM(14)
#undef RX_ASM
#undef RX_ASM_DEG
    default:
      return RX_ERR_ARG;
  }
  RX_HIP(hipGetLastError());
  return RX_OK;
}
#endif  // !RX_NS

namespace {
// NUM_METHOD_GRAD = GREEN_GAUSS: CReactiveNSSolver::SetPrimitive_Gradient_GG (solver_direct_reactive.cpp:4784-4880),
// one thread per owned point gathering its incident edges in edge order (the reference's edge loop restricted to the
// point: + at node 0, - at node 1), then its boundary vertices in (marker, vertex) order, then / Volume. Edge face
// value 0.5 (P_i + P_j) of (T, u, v(, w), P, X_s), with the reference's quirk (:4812-4813): both sides' species are
// node 0's, so X_j = X_i. Boundary vertex value: the point's own record.
template <int NS, int NDIM>
__global__ __launch_bounds__(kBlock) void k_grad_gg(int Nd, const int32_t* __restrict__ adj_ptr,
                                                    const int32_t* __restrict__ adj, const int32_t* __restrict__ edges,
                                                    const double* __restrict__ normal, const int32_t* __restrict__ bv_ptr,
                                                    const double* __restrict__ bv_normal,
                                                    const double* __restrict__ vol, const double* __restrict__ V,
                                                    DevMech m, double* __restrict__ Gout) {
  constexpr int nPV = NS + NDIM + 5, nG = NS + NDIM + 2, P_P = NDIM + 1, RHOS_P = NDIM + 5, P_G = NDIM + 1,
                RHOS_G = NDIM + 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Nd) return;
  // (T, u, v(, w), P) of point p into out[0 .. P_G]; X_s of point q into out[RHOS_G ..]
  auto prim = [&](int p, int q, double* out) {
    const double* v = V + (size_t)p * nPV;
    out[0] = v[0];
    out[P_G] = v[P_P];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) out[1 + d] = v[1 + d];
    const double* w = V + (size_t)q * nPV;
    double ys[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) ys[s] = w[RHOS_P + s];
    molar_from_mass<NS>(m, ys, out + RHOS_G);
  };
  double g[nG][NDIM];
#pragma unroll
  for (int v = 0; v < nG; ++v)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) g[v][d] = 0.0;
  for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
    const int a = adj[k], e = a >> 1, side = a & 1;
    const int n0 = edges[2 * e], n1 = edges[2 * e + 1];
    double pi[nG], pj[nG], nrm[NDIM];
    prim(n0, n0, pi);
    prim(n1, n0, pj);  // :4812-4813: node 0's species on both sides
#pragma unroll
    for (int d = 0; d < NDIM; ++d) nrm[d] = normal[(size_t)e * NDIM + d];
#pragma unroll
    for (int v = 0; v < nG; ++v) {
      const double avg = 0.5 * (pi[v] + pj[v]);
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        const double pr = avg * nrm[d];
        if (side == 0) g[v][d] += pr;
        else g[v][d] -= pr;
      }
    }
  }
  if (bv_ptr[i] < bv_ptr[i + 1]) {
    double pv[nG];
    prim(i, i, pv);
    for (int b = bv_ptr[i]; b < bv_ptr[i + 1]; ++b)
#pragma unroll
      for (int v = 0; v < nG; ++v)
#pragma unroll
        for (int d = 0; d < NDIM; ++d) g[v][d] -= pv[v] * bv_normal[(size_t)b * NDIM + d];
  }
  const double V_i = vol[i];
#pragma unroll
  for (int v = 0; v < nG; ++v)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Gout[((size_t)i * nG + v) * NDIM + d] = g[v][d] / V_i;
}
}  // namespace

#if RX_NS
int RX_NSFN(rx_launch_grad_gg)(rx_ctx* ctx) {
  if (ctx->Nd <= 0) return RX_OK;
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_grad_gg<NS_, ND_><<<blocks(ctx->Nd), kBlock, 0, ctx->stream>>>(
                            (int)ctx->Nd, ctx->adj_ptr, ctx->adj, ctx->edges, ctx->normal, ctx->bv_ptr, ctx->bv_normal,
                            ctx->vol, ctx->f[RX_F_V], ctx->mech, ctx->f[RX_F_GRAD])));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int RX_NSFN(rx_launch_grad)(rx_ctx* ctx, const int32_t* list, int64_t n) {
  if (n <= 0) return RX_OK;
  RX_DNS_SWITCH(ctx->nDim, ctx->ns, (k_grad_lsq<NS_, ND_><<<blocks(n), kBlock, 0, ctx->stream>>>(
                            (int)n, ctx->nbr_ptr, ctx->nbr, ctx->coord, ctx->f[RX_F_V], ctx->mech,
                            ctx->f[RX_F_GRAD], list)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

#endif  // RX_NS

#if !RX_NS
int rx_launch_limiter(rx_ctx* ctx) {
  RX_ND_SWITCH(ctx->nDim, (k_limiter_minmax<ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>((int)ctx->N, ctx->nPV, ctx->adj_ptr, ctx->adj,
                                                                  ctx->edges, ctx->f[RX_F_V], ctx->lim_mn,
                                                                  ctx->lim_mx)));
  RX_HIP(hipGetLastError());
  if (ctx->cfg.slope_limiter == RX_LIMITER_BARTH_JESPERSEN) {
    RX_ND_SWITCH(ctx->nDim, (k_limiter_barth<ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>((int)ctx->N, ctx->nG, ctx->adj_ptr,
                                                                   ctx->adj, ctx->edges, ctx->coord,
                                                                   ctx->f[RX_F_GRAD], ctx->lim_mn, ctx->lim_mx,
                                                                   ctx->f[RX_F_LIMITER])));
    RX_HIP(hipGetLastError());
    return RX_OK;
  }
  const double eps1 = ctx->cfg.limiter_coeff * ctx->cfg.ref_elem_length;
  const double eps2 = eps1 * eps1 * eps1;
  RX_ND_SWITCH(ctx->nDim, (k_limiter_venkat<ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>((int)ctx->N, ctx->nG, ctx->adj_ptr, ctx->adj,
                                                                  ctx->edges, ctx->coord, ctx->f[RX_F_GRAD],
                                                                  ctx->lim_mn, ctx->lim_mx, eps2,
                                                                  ctx->f[RX_F_LIMITER])));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_launch_time_step(rx_ctx* ctx) {
  RX_ND_SWITCH(ctx->nDim, (k_time_step<ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>(
      (int)ctx->N, ctx->nPV, ctx->nVar, ctx->adj_ptr, ctx->adj, ctx->edges, ctx->normal, ctx->bv_ptr, ctx->bv_normal,
      ctx->f[RX_F_V], ctx->f[RX_F_DPDU], ctx->f[RX_F_MU], ctx->f[RX_F_EDDY], ctx->vol, ctx->nbr_ptr, ctx->cfg.cfl,
      ctx->cfg.max_delta_time, ctx->cfg.prandtl_lam, ctx->cfg.prandtl_turb, ctx->f[RX_F_DT], ctx->f[RX_F_LAMBDA_INV],
      ctx->f[RX_F_LAMBDA_VISC])));
  RX_HIP(hipGetLastError());
  return RX_OK;
}
#endif  // !RX_NS
