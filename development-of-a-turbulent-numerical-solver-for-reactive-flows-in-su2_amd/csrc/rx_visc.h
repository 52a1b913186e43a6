// rx_visc.h — reactive laminar + SST viscous flux of one edge (device).
//
// CAvgGradReactive_Flow::ComputeResidual  SU2_CFD/src/numerics_direct_reactive.cpp:1425-1678
//   SetLaminarTensorFlux :1099-1190, Solve_SM :451-470 (library GetGamma reacting_model_library.cpp:771-798),
//   SST_Reactive_ResidualClosure :656-852, Get_Molar2MassGrad_Operator :861-880,
//   SetLaminarViscousProjJacs :1200-1401, SST_Reactive_JacobianClosure :891-1090.
// The two dense solves inside are restated from Eigen 3.3.7 (vendored in the reference,
// externals/Eigen): BiCGSTAB + DiagonalPreconditioner (IterativeLinearSolvers/BiCGSTAB.h:28-100)
// with Eigen's SSE2 reduction / GEMV summation order (Core/Redux.h, products/GeneralMatrixVector.h),
// and ColPivHouseholderQR (QR/ColPivHouseholderQR.h:480-611).
#pragma once

#include "rx_device.h"

namespace rx {

struct ViscParams {
  double T_ref, E_ref, R_ref, Pr_t, Le_t;
  int rans, implicit;
};

// Eigen redux order for a[k]*b[k] over a 16-byte aligned vector of length n (2-wide packets,
// two packet accumulators).
template <int N>
__device__ inline double eig_dot(const double* a, const double* b) {
  constexpr int as2 = (N / 4) * 4, as = (N / 2) * 2;
  double res;
  if (as) {
    double r0a = a[0] * b[0], r0b = a[1] * b[1];
    if (as > 2) {
      double r1a = a[2] * b[2], r1b = a[3] * b[3];
#pragma unroll
      for (int k = 4; k < as2; k += 4) {
        r0a += a[k] * b[k];
        r0b += a[k + 1] * b[k + 1];
        r1a += a[k + 2] * b[k + 2];
        r1b += a[k + 3] * b[k + 3];
      }
      r0a += r1a;
      r0b += r1b;
      if (as > as2) {
        r0a += a[as2] * b[as2];
        r0b += a[as2 + 1] * b[as2 + 1];
      }
    }
    res = r0a + r0b;
#pragma unroll
    for (int k = as; k < N; ++k) res += a[k] * b[k];
  } else {
    res = a[0] * b[0];
#pragma unroll
    for (int k = 1; k < N; ++k) res += a[k] * b[k];
  }
  return res;
}

// Eigen col-major GEMV order (4 columns at once, packet rows, odd tail row sequential), A row-major.
template <int N>
__device__ inline void eig_gemv(const double* A, const double* x, double* y) {
  constexpr int aligned = N & ~1, bound = (N / 4) * 4;
#pragma unroll
  for (int i = 0; i < N; ++i) y[i] = 0.0;
#pragma unroll
  for (int c = 0; c < bound; c += 4) {
#pragma unroll
    for (int r = 0; r < aligned; ++r)
      y[r] = y[r] + ((A[r * N + c] * x[c] + A[r * N + c + 1] * x[c + 1]) +
                     (A[r * N + c + 2] * x[c + 2] + A[r * N + c + 3] * x[c + 3]));
#pragma unroll
    for (int r = aligned; r < N; ++r) {
      y[r] = A[r * N + c] * x[c] + y[r];
      y[r] = A[r * N + c + 1] * x[c + 1] + y[r];
      y[r] = A[r * N + c + 2] * x[c + 2] + y[r];
      y[r] = A[r * N + c + 3] * x[c + 3] + y[r];
    }
  }
#pragma unroll
  for (int c = bound; c < N; ++c) {
#pragma unroll
    for (int r = 0; r < aligned; ++r) y[r] = A[r * N + c] * x[c] + y[r];
#pragma unroll
    for (int r = aligned; r < N; ++r) y[r] += A[r * N + c] * x[c];
  }
}

template <int N>
__device__ inline void bicgstab(const double* A, const double* rhs, double* x, double tol) {
  const int maxIters = 2 * N;
  double invdiag[N];
#pragma unroll
  for (int j = 0; j < N; ++j) invdiag[j] = (A[j * N + j] != 0.0) ? 1.0 / A[j * N + j] : 1.0;
  double r[N], r0[N], tmp[N];
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = 0.0;
  // r = rhs - A*0
  eig_gemv<N>(A, x, tmp);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    r[i] = rhs[i] - tmp[i];
    r0[i] = r[i];
  }
  double r0_sqnorm = eig_dot<N>(r0, r0);
  const double rhs_sqnorm = eig_dot<N>(rhs, rhs);
  if (rhs_sqnorm == 0) return;
  double rho = 1, alpha = 1, w = 1;
  double v[N], p[N], y[N], z[N], s[N], t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = p[i] = 0.0;
  const double tol2 = tol * tol * rhs_sqnorm;
  const double eps = 2.220446049250313e-16;
  const double eps2 = eps * eps;
  int i = 0, restarts = 0;
  while (eig_dot<N>(r, r) > tol2 && i < maxIters) {
    const double rho_old = rho;
    rho = eig_dot<N>(r0, r);
    if (fabs(rho) < eps2 * r0_sqnorm) {
      eig_gemv<N>(A, x, tmp);
#pragma unroll
      for (int q = 0; q < N; ++q) {
        r[q] = rhs[q] - tmp[q];
        r0[q] = r[q];
      }
      rho = r0_sqnorm = eig_dot<N>(r, r);
      if (restarts++ == 0) i = 0;
    }
    const double beta = (rho / rho_old) * (alpha / w);
#pragma unroll
    for (int q = 0; q < N; ++q) p[q] = r[q] + beta * (p[q] - w * v[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) y[q] = invdiag[q] * p[q];
    eig_gemv<N>(A, y, v);
    alpha = rho / eig_dot<N>(r0, v);
#pragma unroll
    for (int q = 0; q < N; ++q) s[q] = r[q] - alpha * v[q];
#pragma unroll
    for (int q = 0; q < N; ++q) z[q] = invdiag[q] * s[q];
    eig_gemv<N>(A, z, t);
    const double tt = eig_dot<N>(t, t);
    w = (tt > 0.0) ? eig_dot<N>(t, s) / tt : 0.0;
#pragma unroll
    for (int q = 0; q < N; ++q) x[q] += alpha * y[q] + w * z[q];
#pragma unroll
    for (int q = 0; q < N; ++q) r[q] = s[q] - w * t[q];
    ++i;
  }
}

// ColPivHouseholderQR: factor M (row-major NxN, overwritten) and solve for NDIM right-hand sides.
template <int N, int NDIM>
__device__ inline void colpiv_qr_solve(double* Q, const double (*rhs)[NDIM], double (*sol)[NDIM]) {
  double hc[N], normsU[N], normsD[N];
  int trans[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i) s += Q[i * N + k] * Q[i * N + k];
    normsD[k] = sqrt(s);
    normsU[k] = normsD[k];
  }
  double mx = normsU[0];
#pragma unroll
  for (int k = 1; k < N; ++k) mx = fmax(mx, normsU[k]);
  const double epsm = 2.220446049250313e-16;
  const double threshold_helper = (mx * epsm) * (mx * epsm) / double(N);
  const double ndt = sqrt(epsm);
  int nonzero = N;
  for (int k = 0; k < N; ++k) {
    int big = k;
    for (int j = k + 1; j < N; ++j)
      if (normsU[j] > normsU[big]) big = j;
    const double big_sq = normsU[big] * normsU[big];
    if (nonzero == N && big_sq < threshold_helper * double(N - k)) nonzero = k;
    trans[k] = big;
    if (k != big) {
      for (int i = 0; i < N; ++i) {
        const double t = Q[i * N + k];
        Q[i * N + k] = Q[i * N + big];
        Q[i * N + big] = t;
      }
      double t = normsU[k]; normsU[k] = normsU[big]; normsU[big] = t;
      t = normsD[k]; normsD[k] = normsD[big]; normsD[big] = t;
    }
    double tailSq = 0.0;
    for (int i = k + 1; i < N; ++i) tailSq += Q[i * N + k] * Q[i * N + k];
    const double c0 = Q[k * N + k];
    double tau, beta;
    if (tailSq <= 2.2250738585072014e-308) {
      tau = 0.0;
      beta = c0;
      for (int i = k + 1; i < N; ++i) Q[i * N + k] = 0.0;
    } else {
      beta = sqrt(c0 * c0 + tailSq);
      if (c0 >= 0.0) beta = -beta;
      for (int i = k + 1; i < N; ++i) Q[i * N + k] = Q[i * N + k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    hc[k] = tau;
    Q[k * N + k] = beta;
    if (N - k == 1) {
      for (int j = k + 1; j < N; ++j) Q[k * N + j] *= (1.0 - tau);
    } else if (tau != 0.0) {
      for (int j = k + 1; j < N; ++j) {
        double tmp = 0.0;
        for (int i = k + 1; i < N; ++i) tmp += Q[i * N + k] * Q[i * N + j];
        tmp += Q[k * N + j];
        Q[k * N + j] -= tau * tmp;
        for (int i = k + 1; i < N; ++i) Q[i * N + j] -= tau * Q[i * N + k] * tmp;
      }
    }
    for (int j = k + 1; j < N; ++j) {
      if (normsU[j] != 0.0) {
        double temp = fabs(Q[k * N + j]) / normsU[j];
        temp = (1.0 + temp) * (1.0 - temp);
        temp = temp < 0.0 ? 0.0 : temp;
        const double rr = normsU[j] / normsD[j];
        const double temp2 = temp * (rr * rr);
        if (temp2 <= ndt) {
          double s = 0.0;
          for (int i = k + 1; i < N; ++i) s += Q[i * N + j] * Q[i * N + j];
          normsD[j] = sqrt(s);
          normsU[j] = normsD[j];
        } else {
          normsU[j] *= sqrt(temp);
        }
      }
    }
  }
  int perm[N];
#pragma unroll
  for (int k = 0; k < N; ++k) perm[k] = k;
  for (int k = 0; k < N; ++k) {
    const int t = perm[k];
    perm[k] = perm[trans[k]];
    perm[trans[k]] = t;
  }
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    double c[N];
#pragma unroll
    for (int i = 0; i < N; ++i) c[i] = rhs[i][d];
    if (nonzero == 0) {
#pragma unroll
      for (int i = 0; i < N; ++i) sol[i][d] = 0.0;
      continue;
    }
    for (int k = 0; k < nonzero; ++k) {
      const double tau = hc[k];
      if (N - k == 1) {
        c[k] *= (1.0 - tau);
      } else if (tau != 0.0) {
        double tmp = 0.0;
        for (int i = k + 1; i < N; ++i) tmp += Q[i * N + k] * c[i];
        tmp += c[k];
        c[k] -= tau * tmp;
        for (int i = k + 1; i < N; ++i) c[i] -= tau * Q[i * N + k] * tmp;
      }
    }
    for (int i = nonzero - 1; i >= 0; --i) {
      c[i] /= Q[i * N + i];
      for (int j = 0; j < i; ++j) c[j] -= c[i] * Q[j * N + i];
    }
    double out[N];
    for (int i = 0; i < N; ++i) out[i] = 0.0;
    for (int i = 0; i < nonzero; ++i) out[perm[i]] = c[i];
#pragma unroll
    for (int i = 0; i < N; ++i) sol[i][d] = out[i];
  }
}

// Per-edge summary written by visc_edge (implicit) for the Jacobian kernel: scalars, then nine
// species arrays (Xs_i, Xs_j, Ys, hs, Cps, Jd, Gxn/|n|, Ds, quirk aux).
enum {
  VS_MU = 0, VS_K, VS_MUT, VS_RHO, VS_VM, VS_RHOI = 6, VS_RHOJ, VS_VI, VS_VJ = 10, VS_THETA = 12, VS_DIJ, VS_DS,
  VS_UN, VS_PF = 17, VS_TM = 19, VS_TMI, VS_TMJ, VS_SGI, VS_SGJ, VS_ARR
};
template <int NS>
constexpr int visc_summary_size() { return VS_ARR + 9 * NS; }

// Per-edge inputs gathered from the two node records.
template <int NS, int NDIM>
struct ViscNode {
  const double *V, *G, *Dij, *S, *gk, *coord;
  double mu, kappa, tke, mut;
};

// Computes the projected viscous flux res[nVar] and, if implicit, Ji/Jj (row-major nVar x nVar).
template <int NS, int NDIM>
__device__ inline int visc_edge(const DevMech& m, const ViscParams& P, const ViscNode<NS, NDIM>& ni,
                                const ViscNode<NS, NDIM>& nj, double sigma_k, const double* Normal, double* res,
                                double* summ, double* scr, bool corrected = true) {
  // corrected = false: CAvgGradReactive_Boundary::ComputeResidual (numerics_direct_reactive.cpp:478-648, a8):
  // the plain mean gradient — no edge correction, no coincident-point check.
  constexpr int nVar = NS + NDIM + 2, nPV = NS + NDIM + 5;
  constexpr int T_P = 0, VX_P = 1, RHO_P = NDIM + 2, RHOS_P = NDIM + 5;
  constexpr int RHO_S = 0, RHOVX_S = 1, RHOE_S = NDIM + 1, RHOS_S = NDIM + 2;
  constexpr int T_G = 0, VX_G = 1, RHOS_G = NDIM + 2;
  constexpr int T_A = 0, VX_A = 1, RHOS_A = 1 + NDIM, nAvg = NS + NDIM + 1;
  int err = ERR_NONE;
  const double* Vi = ni.V;
  const double* Vj = nj.V;
  const double Mean_mu = 2.0 / (1.0 / ni.mu + 1.0 / nj.mu);
  const double Mean_k = 2.0 / (1.0 / ni.kappa + 1.0 / nj.kappa);
  // harmonic means of the binary diffusion coefficients (recomputed where used: same arithmetic)
  auto Dm = [&](int q) { return 2.0 / (1.0 / ni.Dij[q] + 1.0 / nj.Dij[q]); };
  double Dmax = -INFINITY;
#pragma unroll
  for (int q = 0; q < NS * NS; ++q) Dmax = fmax(Dmax, Dm(q));
  double Vm[nPV];
#pragma unroll
  for (int v = 0; v < nPV; ++v) Vm[v] = 0.5 * (Vi[v] + Vj[v]);
  double Xs_i[NS], Xs_j[NS];
  molar_from_mass<NS>(m, Vi + RHOS_P, Xs_i);
  molar_from_mass<NS>(m, Vj + RHOS_P, Xs_j);
  double Edge[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) Edge[d] = nj.coord[d] - ni.coord[d];
  double G[nAvg][NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    G[T_A][d] = 0.5 * (ni.G[T_G * NDIM + d] + nj.G[T_G * NDIM + d]);
#pragma unroll
    for (int e = 0; e < NDIM; ++e) G[VX_A + e][d] = 0.5 * (ni.G[(VX_G + e) * NDIM + d] + nj.G[(VX_G + e) * NDIM + d]);
#pragma unroll
    for (int s = 0; s < NS; ++s)
      G[RHOS_A + s][d] = 0.5 * (ni.G[(RHOS_G + s) * NDIM + d] + nj.G[(RHOS_G + s) * NDIM + d]);
  }
  double dist2 = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) dist2 += Edge[d] * Edge[d];
  if (corrected && !(dist2 > kEPS)) return ERR_GEOM;
  if (corrected) {
    double Diff[nAvg], Proj[nAvg];
#pragma unroll
    for (int r = 0; r < nAvg; ++r) {
      double s = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) s += G[r][d] * Edge[d];
      Proj[r] = s;
    }
    Diff[T_A] = Vj[T_P] - Vi[T_P];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Diff[VX_A + d] = Vj[VX_P + d] - Vi[VX_P + d];
#pragma unroll
    for (int s = 0; s < NS; ++s) Diff[RHOS_A + s] = Xs_j[s] - Xs_i[s];
#pragma unroll
    for (int r = 0; r < nAvg; ++r)
#pragma unroll
      for (int d = 0; d < NDIM; ++d) G[r][d] -= (Proj[r] - Diff[r]) * Edge[d] / dist2;
  }
  // ---- SetLaminarTensorFlux
  double Flux[nVar][NDIM], PF[nVar];
#pragma unroll
  for (int v = 0; v < nVar; ++v) {
    PF[v] = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Flux[v][d] = 0.0;
  }
  const double rho = Vm[RHO_P];
  const double dim_temp = Vm[T_P] * P.T_ref;
  double hs[NS], Ys[NS], Xs[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) hs[s] = spline(m, P_H, s, dim_temp, &err) / m.mm[s] / P.E_ref;
#pragma unroll
  for (int s = 0; s < NS; ++s) Ys[s] = Vm[RHOS_P + s];
  molar_from_mass<NS>(m, Ys, Xs);
  double div_vel = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) div_vel += G[VX_A + d][d];
  double tau[NDIM][NDIM];
#pragma unroll
  for (int a = 0; a < NDIM; ++a) {
#pragma unroll
    for (int b = 0; b < NDIM; ++b) tau[a][b] = 0.0 + Mean_mu * (G[VX_A + b][a] + G[VX_A + a][b]);
    tau[a][a] -= kTWO3 * (Mean_mu * div_vel);
  }
  const double alpha = 1.0 / (rho * Dmax);
  double Gxn[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) Gxn[s] = 0.0;
#pragma unroll
  for (int a = 0; a < NDIM; ++a) {
#pragma unroll
    for (int b = 0; b < NDIM; ++b) {
      Flux[RHOVX_S + b][a] = tau[a][b];
      Flux[RHOE_S][a] += tau[a][b] * Vm[VX_P + b];
    }
    Flux[RHOE_S][a] += Mean_k * G[T_A][a];
#pragma unroll
    for (int s = 0; s < NS; ++s) Gxn[s] += G[RHOS_A + s][a] * Normal[a];
  }
  double Jd[NS];
  {
    double* Gt = scr;  // LDS scratch of this lane (NS*NS)
    double sigma = 0.0, massTot = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) sigma += Ys[s];
#pragma unroll
    for (int s = 0; s < NS; ++s) massTot += Ys[s] / m.mm[s];
    massTot = 1.0 / massTot;
#pragma unroll
    for (int a = 0; a < NS; ++a)
#pragma unroll
      for (int b = 0; b < NS; ++b) {
        double g;
        if (a != b) {
          g = -sigma * massTot * Xs[a] / (rho * m.mm[b] * Dm(b * NS + a));
        } else {
          double tmp = 0.0;
#pragma unroll
          for (int c = 0; c < NS; ++c)
            if (c != a) tmp += Xs[c] / Dm(c * NS + a);
          g = sigma * massTot * tmp / (rho * m.mm[a]);
        }
        Gt[a * NS + b] = g + alpha * Ys[a];
      }
    double nG[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) nG[s] = -Gxn[s];
    bicgstab<NS>(Gt, nG, Jd, 1.0e-11);
  }
  {
    double ones[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) ones[s] = 1.0;
    PF[RHO_S] = -eig_dot<NS>(Jd, ones);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    PF[RHOE_S] += -hs[s] * Jd[s];
    PF[RHOS_S + s] = -Jd[s];
  }
  double Mean_mut = 0.0, Mean_tke = 0.0, Cps[NS];
  double MG[NS][NDIM];
  if (P.rans) {
    Mean_mut = 2.0 / (1.0 / ni.mut + 1.0 / nj.mut);
    Mean_tke = 0.5 * (ni.tke + nj.tke);
    double gk[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) gk[d] = 0.5 * (ni.gk[d] + nj.gk[d]);
#pragma unroll
    for (int s = 0; s < NS; ++s) Cps[s] = spline(m, P_CP, s, dim_temp, &err) / m.mm[s] / P.R_ref;
    double dv = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) dv += G[VX_A + d][d];
    double tt[NDIM][NDIM];
#pragma unroll
    for (int a = 0; a < NDIM; ++a) {
#pragma unroll
      for (int b = 0; b < NDIM; ++b) tt[a][b] = 0.0 + Mean_mut * (G[VX_A + b][a] + G[VX_A + a][b]);
      tt[a][a] -= kTWO3 * (Mean_mut * dv + Mean_tke * rho);
    }
    {
      double* Mt = scr;  // LDS scratch of this lane (NS*NS), Gt is dead here
      double sig = 0.0;
#pragma unroll
      for (int s = 0; s < NS; ++s) sig += Xs[s];
#pragma unroll
      for (int a = 0; a < NS; ++a)
#pragma unroll
        for (int b = 0; b < NS; ++b)
          Mt[a * NS + b] = m.mtot / m.mm[a] * (Ys[a] - Xs[a] + sig) * (double)(a == b) +
                           m.mtot * (Ys[a] / m.mm[a] - Xs[a] / m.mm[b]) * (double)(a != b);
      double rhs[NS][NDIM];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int d = 0; d < NDIM; ++d) rhs[s][d] = G[RHOS_A + s][d];
      colpiv_qr_solve<NS, NDIM>(Mt, rhs, MG);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int d = 0; d < NDIM; ++d)
        if (fabs(G[RHOS_A + s][d]) < 1e-8) MG[s][d] = 0.0;
#pragma unroll
    for (int a = 0; a < NDIM; ++a) {
#pragma unroll
      for (int b = 0; b < NDIM; ++b) {
        Flux[RHOVX_S + b][a] += tt[a][b];
        Flux[RHOE_S][a] += tt[a][b] * Vm[VX_P + b];
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) PF[RHOS_S + s] += Mean_mut / (P.Pr_t * P.Le_t) * MG[s][a] * Normal[a];
#pragma unroll
      for (int s = 0; s < NS; ++s) Flux[RHOE_S][a] += Mean_mut / (P.Pr_t * P.Le_t) * hs[s] * Ys[s] * MG[s][a];
#pragma unroll
      for (int s = 0; s < NS; ++s) Flux[RHOE_S][a] += Mean_mut / P.Pr_t * Cps[s] * Ys[s] * G[T_A][a];
      Flux[RHOE_S][a] += (Mean_mu + Mean_mut / sigma_k) * gk[a];
    }
  }
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
#pragma unroll
    for (int v = RHOVX_S; v < RHOVX_S + NDIM; ++v) PF[v] += Flux[v][d] * Normal[d];
    PF[RHOE_S] += Flux[RHOE_S][d] * Normal[d];
  }
#pragma unroll
  for (int v = 0; v < nVar; ++v) res[v] = PF[v];
  if (!P.implicit) return err;

  // ---- implicit part: the per-edge summary the Jacobian kernel (visc_jac_column) needs
  double Ds[NS];
  {
    double Ds_i[NS], Ds_j[NS];
#pragma unroll
    for (int a = 0; a < NS; ++a) {
      double di = 0.0, dj = 0.0;
#pragma unroll
      for (int b = 0; b < NS; ++b)
        if (b != a) {
          di += Xs_i[b] / ni.Dij[b * NS + a];
          dj += Xs_j[b] / nj.Dij[b * NS + a];
        }
      Ds_i[a] = (1.0 - Xs_i[a]) / di;
      Ds_j[a] = (1.0 - Xs_j[a]) / dj;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (isnan(Ds_i[s]) || isinf(Ds_i[s])) Ds_i[s] = 0.0;
      if (isnan(Ds_j[s]) || isinf(Ds_j[s])) Ds_j[s] = 0.0;
      Ds[s] = 0.5 * (Ds_i[s] + Ds_j[s]);
    }
  }
  double Area = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) Area += Normal[d] * Normal[d];
  Area = sqrt(Area);
  double UN[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) UN[d] = Normal[d] / Area;
#pragma unroll
  for (int s = 0; s < NS; ++s) Gxn[s] /= Area;
  double theta = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) theta += UN[d] * UN[d];
  if (!P.rans) {
#pragma unroll
    for (int s = 0; s < NS; ++s) Cps[s] = spline(m, P_CP, s, dim_temp, &err) / m.mm[s] / P.R_ref;
  }
  double totMass = 0.0, totMass_i = 0.0, totMass_j = 0.0, sigma_i = 0.0, sigma_j = 0.0;
#pragma unroll
  for (int s = 0; s < NS; ++s) totMass += m.mm[s] * Xs[s];
#pragma unroll
  for (int s = 0; s < NS; ++s) totMass_i += m.mm[s] * Xs_i[s];
#pragma unroll
  for (int s = 0; s < NS; ++s) totMass_j += m.mm[s] * Xs_j[s];
#pragma unroll
  for (int s = 0; s < NS; ++s) sigma_i += Xs_i[s];
#pragma unroll
  for (int s = 0; s < NS; ++s) sigma_j += Xs_j[s];
  // quirk :1083-1084 — row(s).data() walks the column-major storage of Mean_Mass_Grads
  double qaux[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double aux = 0.0;
    if (P.rans) {
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        const int flat = s + d;
        aux += MG[flat % NS][flat / NS] * UN[d];
      }
    }
    qaux[s] = aux;
  }
  double* o = summ;
  o[VS_MU] = Mean_mu;
  o[VS_K] = Mean_k;
  o[VS_MUT] = Mean_mut;
  o[VS_RHO] = rho;
  o[VS_VM] = Vm[VX_P];
  o[VS_VM + 1] = Vm[VX_P + 1];
  o[VS_RHOI] = Vi[RHO_P];
  o[VS_RHOJ] = Vj[RHO_P];
  o[VS_VI] = Vi[VX_P];
  o[VS_VI + 1] = Vi[VX_P + 1];
  o[VS_VJ] = Vj[VX_P];
  o[VS_VJ + 1] = Vj[VX_P + 1];
  o[VS_THETA] = theta;
  o[VS_DIJ] = sqrt(dist2);
  o[VS_DS] = Area;
  o[VS_UN] = UN[0];
  o[VS_UN + 1] = UN[NDIM - 1];
  o[VS_PF] = PF[RHOVX_S];
  o[VS_PF + 1] = PF[RHOVX_S + 1];
  o[VS_TM] = totMass;
  o[VS_TMI] = totMass_i;
  o[VS_TMJ] = totMass_j;
  o[VS_SGI] = sigma_i;
  o[VS_SGJ] = sigma_j;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    o[VS_ARR + 0 * NS + s] = Xs_i[s];
    o[VS_ARR + 1 * NS + s] = Xs_j[s];
    o[VS_ARR + 2 * NS + s] = Ys[s];
    o[VS_ARR + 3 * NS + s] = hs[s];
    o[VS_ARR + 4 * NS + s] = Cps[s];
    o[VS_ARR + 5 * NS + s] = Jd[s];
    o[VS_ARR + 6 * NS + s] = Gxn[s];
    o[VS_ARR + 7 * NS + s] = Ds[s];
    o[VS_ARR + 8 * NS + s] = qaux[s];
  }
  return err;
}

// Jacobian column b (0 <= b < nVar) of Jac_i and Jac_j for one edge, from the visc_edge summary:
// SetLaminarViscousProjJacs (:1200-1401) + SST_Reactive_JacobianClosure (:891-1090, 2-D branch)
// build dF/dV (FI for node i, FJ for node j); J = dF/dV * dV/dU (:1637-1653). A team of lanes owns
// the columns of one edge; every dF/dV entry is accumulated in the reference's order, and J's sum over
// k keeps the reference's order (the F*0 terms of dV/dU's zero entries are dropped: they can only
// change the sign of an exact zero). base_i/base_j: the column-independent part of row a of dJ/drho
// (this lane's a = lane index in the team), shared through shuffles. Only 2-D.
template <int NS, int NDIM>
__device__ inline void visc_jac_column(const DevMech& m, const ViscParams& P, const double* __restrict__ sm,
                                       double Sib, double Sjb, int b, int tl, double* __restrict__ Ji,
                                       double* __restrict__ Jj) {
  constexpr int nVar = NS + NDIM + 2;
  constexpr int RHOE_S = NDIM + 1, RHOS_S = NDIM + 2;
  const double mu = sm[VS_MU], ktr = sm[VS_K], mut = sm[VS_MUT], rho = sm[VS_RHO];
  const double rho_i = sm[VS_RHOI], rho_j = sm[VS_RHOJ];
  const double theta = sm[VS_THETA], dij = sm[VS_DIJ], dS = sm[VS_DS], sq = sm[VS_DIJ], Area = sm[VS_DS];
  const double totMass = sm[VS_TM], totMass_i = sm[VS_TMI], totMass_j = sm[VS_TMJ];
  const double sigma_i = sm[VS_SGI], sigma_j = sm[VS_SGJ];
  const double* Xs_i = sm + VS_ARR;
  const double* Xs_j = Xs_i + NS;
  const double* Ys = Xs_j + NS;
  const double* hs = Ys + NS;
  const double* Cps = hs + NS;
  const double* Jd = Cps + NS;
  const double* Gxn = Jd + NS;
  const double* Ds = Gxn + NS;
  const double* qaux = Ds + NS;
  const double PrT = P.Pr_t, LeT = P.Le_t;
  // ---- column-independent part of dJ/drho rows (lane tl < NS owns row a = tl)
  double bj = 0.0, bi = 0.0;
  if (tl < NS) {
    const int a = tl;
    double vj = -rho * m.mm[a] * Ds[a] * Xs_j[a] / (totMass * dij * sigma_j * rho_j);
    double vi = rho * m.mm[a] * Ds[a] * Xs_i[a] / (totMass * dij * sigma_i * rho_i);
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      vj += rho * Ys[a] * m.mm[q] * Ds[q] * Xs_j[q] / (totMass * dij * sigma_j * rho_j);
      vi -= rho * Ys[a] * m.mm[q] * Ds[q] * Xs_i[q] / (totMass * dij * sigma_i * rho_i);
    }
    bj = vj;
    bi = vi;
  }
  double colj[NS], coli[NS];  // dJ/drho column k = b - RHOS_S (species columns only)
  const int k = b - RHOS_S;
  const int kk = (k >= 0 && k < NS) ? k : 0;
  // the a == k term of :1352-1357, evaluated once for this lane's column (no divergent divisions)
  const double dkj = rho * Ds[kk] * totMass_j * sigma_j / (dij * totMass * rho_j);
  const double dki = rho * Ds[kk] * totMass_i * sigma_i / (dij * totMass * rho_i);
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    const double baj = __shfl(bj, a, 16), bai = __shfl(bi, a, 16);
    double vj = baj, vi = bai;
    if (k >= 0) {
      vj += rho * Ys[a] * Ds[kk] * totMass_j * sigma_j / (dij * totMass * rho_j);
      vi -= rho * Ys[a] * Ds[kk] * totMass_i * sigma_i / (dij * totMass * rho_i);
      if (a == k) {
        vj -= dkj;
        vi += dki;
      }
    }
    colj[a] = vj;
    coli[a] = vi;
  }
  if (b >= nVar) return;
  if (k >= 0) {  // diagonal increments of dJ/drho (:1369-1374): the same sequence for every diagonal entry
    double tj[NS], ti[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      tj[q] = 0.5 * rho * m.mm[q] * Ds[q] * Gxn[q] / (totMass * rho_j);
      ti[q] = 0.5 * rho * m.mm[q] * Ds[q] * Gxn[q] / (totMass * rho_i);
    }
#pragma unroll
    for (int a = 0; a < NS; ++a)
      if (a == k) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
          colj[a] += tj[q];
          coli[a] += ti[q];
        }
      }
  }
  // ---- dF/dV flow block rows 0..3, columns 0..3 (index [row][col]); zero-initialised
  double FJ[4][4], FI[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) FJ[r][c] = FI[r][c] = 0.0;
  const double UN0 = sm[VS_UN], UN1 = sm[VS_UN + 1];
  const double thetax = theta + UN0 * UN0 / 3.0, thetay = theta + UN1 * UN1 / 3.0;
  const double etaz = UN0 * UN1 / 3.0;
  const double pix = sm[VS_VM] * thetax + sm[VS_VM + 1] * etaz;
  const double piy = sm[VS_VM] * etaz + sm[VS_VM + 1] * thetay;
  FJ[1][1] = mu * thetax / dij * dS;
  FJ[1][2] = mu * etaz / dij * dS;
  FJ[2][1] = mu * etaz / dij * dS;
  FJ[2][2] = mu * thetay / dij * dS;
  FJ[3][1] = pix * mu / dij * dS;
  FJ[3][2] = piy * mu / dij * dS;
  FJ[3][3] = ktr * theta / dij * dS;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) FI[r][c] = -FJ[r][c];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    FI[3][3] += -0.5 * Jd[q] * Cps[q];
    FJ[3][3] += -0.5 * Jd[q] * Cps[q];
  }
  // species column of rows 0 (rho) and 3 (rho E), accumulated over the species rows in order
  double FJ0k = 0.0, FI0k = 0.0, FJ3k = 0.0, FI3k = 0.0;
  if (k >= 0) {
#pragma unroll
    for (int a = 0; a < NS; ++a) {
      FJ0k += -colj[a] * dS;
      FI0k += -coli[a] * dS;
      FJ3k += -colj[a] * hs[a] * dS;
      FI3k += -coli[a] * hs[a] * dS;
    }
  }
  if (P.rans) {
    FJ[1][1] += mut * thetax / sq * Area;
    FJ[1][2] += mut * etaz / sq * Area;
    FI[1][1] -= mut * thetax / sq * Area;
    FI[1][2] -= mut * etaz / sq * Area;
    FJ[2][1] += mut * etaz / sq * Area;
    FJ[2][2] += mut * thetay / sq * Area;
    FI[2][1] -= mut * etaz / sq * Area;
    FI[2][2] -= mut * thetay / sq * Area;
    FJ[3][1] += pix * mut / sq * Area;
    FJ[3][2] += piy * mut / sq * Area;
    FI[3][1] -= pix * mut / sq * Area;
    FI[3][2] -= piy * mut / sq * Area;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      FJ[3][3] += mut / PrT * Cps[q] * Ys[q] * theta / sq * Area;
      FI[3][3] -= mut / PrT * Cps[q] * Ys[q] * theta / sq * Area;
    }
    if (k >= 0) {
      FJ3k += mut / (PrT * LeT) * hs[kk] * Ys[kk] / rho_j * theta / sq * Area;
      FI3k -= mut / (PrT * LeT) * hs[kk] * Ys[kk] / rho_i * theta / sq * Area;
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      FJ[3][3] += mut / (PrT * LeT) * Cps[q] * Ys[q] * qaux[q] * Area;
      FI[3][3] += mut / (PrT * LeT) * Cps[q] * Ys[q] * qaux[q] * Area;
    }
  }
  FI[3][1] += 0.5 * sm[VS_PF];
  FJ[3][1] += 0.5 * sm[VS_PF];
  FI[3][2] += 0.5 * sm[VS_PF + 1];
  FJ[3][2] += 0.5 * sm[VS_PF + 1];
  // ---- J[a][b] = sum_k F[a][k] dV/dU[k][b]
  const double ui = sm[VS_VI], vvi = sm[VS_VI + 1], uj = sm[VS_VJ], vvj = sm[VS_VJ + 1];
  double ci1, ci2, cj1, cj2;  // dV/dU velocity rows, column b
  if (b == 0) {
    ci1 = -ui / rho_i;
    ci2 = -vvi / rho_i;
    cj1 = -uj / rho_j;
    cj2 = -vvj / rho_j;
  } else {
    ci1 = (b == 1) ? 1.0 / rho_i : 0.0;
    ci2 = (b == 2) ? 1.0 / rho_i : 0.0;
    cj1 = (b == 1) ? 1.0 / rho_j : 0.0;
    cj2 = (b == 2) ? 1.0 / rho_j : 0.0;
  }
  const double d0 = (b == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double si = 0.0, sj = 0.0;
    si += FI[r][0] * d0;
    sj += FJ[r][0] * d0;
    si += FI[r][1] * ci1;
    sj += FJ[r][1] * cj1;
    si += FI[r][2] * ci2;
    sj += FJ[r][2] * cj2;
    si += FI[r][RHOE_S] * Sib;
    sj += FJ[r][RHOE_S] * Sjb;
    if (k >= 0) {
      if (r == 0) {
        si += FI0k;
        sj += FJ0k;
      } else if (r == RHOE_S) {
        si += FI3k;
        sj += FJ3k;
      }
    }
    Ji[r * nVar + b] = si;
    Jj[r * nVar + b] = sj;
  }
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    double si = 0.0, sj = 0.0;
    if (k >= 0) {
      si = -coli[a] * dS;
      sj = -colj[a] * dS;
    }
    Ji[(RHOS_S + a) * nVar + b] = si;
    Jj[(RHOS_S + a) * nVar + b] = sj;
  }
}

}  // namespace rx
