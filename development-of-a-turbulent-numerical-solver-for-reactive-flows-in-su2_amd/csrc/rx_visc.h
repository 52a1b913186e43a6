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

#ifndef RX_VISC_PROBE
#define RX_VISC_PROBE 0
#endif

namespace rx {

// 2 / (1 / a + 1 / b) with the device's division sequence (rx_fdiv.h): the same double
__device__ __forceinline__ double hmean2(double a, double b) {
  return rx_div(2.0, rx_recip(rx_div(1.0, rx_recip(a)) + rx_div(1.0, rx_recip(b))));
}

// The lane's dense NS x NS matrix (Gamma, then the closure matrix) in its workgroup's LDS scratch, entry q at
// p[q * kScrLanes]: the 64 lanes' matrices interleaved, so that a wavefront's access to one entry touches 64
// consecutive 8-byte words (no bank conflicts; a lane-contiguous [NS*NS] slice per lane put lanes 16 apart on the
// same bank).
constexpr int kScrLanes = 64;
struct Scr {
  double* p;
  __device__ double& operator[](int q) const { return p[q * kScrLanes]; }
};

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
__device__ inline void eig_gemv(const Scr A, const double* x, double* y) {
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
__device__ inline void bicgstab(const Scr A, const double* rhs, double* x, double tol) {
  const int maxIters = 2 * N;
  double invdiag[N];
#pragma unroll
  for (int j = 0; j < N; ++j) invdiag[j] = (A[j * N + j] != 0.0) ? rx_div(1.0, rx_recip(A[j * N + j])) : 1.0;
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
    const double beta = rx_div(rho, rx_recip(rho_old)) * rx_div(alpha, rx_recip(w));
#pragma unroll
    for (int q = 0; q < N; ++q) p[q] = r[q] + beta * (p[q] - w * v[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) y[q] = invdiag[q] * p[q];
    eig_gemv<N>(A, y, v);
    alpha = rx_div(rho, rx_recip(eig_dot<N>(r0, v)));
#pragma unroll
    for (int q = 0; q < N; ++q) s[q] = r[q] - alpha * v[q];
#pragma unroll
    for (int q = 0; q < N; ++q) z[q] = invdiag[q] * s[q];
    eig_gemv<N>(A, z, t);
    const double tt = eig_dot<N>(t, t);
    w = (tt > 0.0) ? rx_div(eig_dot<N>(t, s), rx_recip(tt)) : 0.0;
#pragma unroll
    for (int q = 0; q < N; ++q) x[q] += alpha * y[q] + w * z[q];
#pragma unroll
    for (int q = 0; q < N; ++q) r[q] = s[q] - w * t[q];
    ++i;
  }
}

// ColPivHouseholderQR: factor M (row-major NxN, overwritten) and solve for NDIM right-hand sides. Every loop has a
// compile-time trip count (fully unrolled: static LDS offsets, register arrays); the data-dependent parts — the pivot
// column, the rank `nonzero`, the permutation — are predicated, in Eigen's order.
template <int N, int NDIM>
__device__ inline void colpiv_qr_solve(const Scr Q, const double (*rhs)[NDIM], double (*sol)[NDIM]) {
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
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int big = k;
    double bigU = normsU[k];
#pragma unroll
    for (int j = k + 1; j < N; ++j)
      if (normsU[j] > bigU) {
        big = j;
        bigU = normsU[j];
      }
    const double big_sq = bigU * bigU;
    if (nonzero == N && big_sq < threshold_helper * double(N - k)) nonzero = k;
    trans[k] = big;
    if (k != big) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const double t = Q[i * N + k];
        Q[i * N + k] = Q[i * N + big];
        Q[i * N + big] = t;
      }
#pragma unroll
      for (int j = k + 1; j < N; ++j)
        if (j == big) {
          double t = normsU[k]; normsU[k] = normsU[j]; normsU[j] = t;
          t = normsD[k]; normsD[k] = normsD[j]; normsD[j] = t;
        }
    }
    double tailSq = 0.0;
#pragma unroll
    for (int i = k + 1; i < N; ++i) tailSq += Q[i * N + k] * Q[i * N + k];
    const double c0 = Q[k * N + k];
    double tau, beta;
    if (tailSq <= 2.2250738585072014e-308) {
      tau = 0.0;
      beta = c0;
#pragma unroll
      for (int i = k + 1; i < N; ++i) Q[i * N + k] = 0.0;
    } else {
      beta = sqrt(c0 * c0 + tailSq);
      if (c0 >= 0.0) beta = -beta;
      const Recip rcb = rx_recip(c0 - beta);  // one divisor for the column (rx_fdiv.h)
#pragma unroll
      for (int i = k + 1; i < N; ++i) Q[i * N + k] = rx_div(Q[i * N + k], rcb);
      tau = rx_div(beta - c0, rx_recip(beta));
    }
    hc[k] = tau;
    Q[k * N + k] = beta;
    if (N - k == 1) {
      // (no trailing columns: Eigen's `*= (1 - tau)` loop over j > k is empty)
    } else if (tau != 0.0) {
      double v[N];  // the Householder vector below the diagonal, read once
#pragma unroll
      for (int i = k + 1; i < N; ++i) v[i] = Q[i * N + k];
#pragma unroll
      for (int j = k + 1; j < N; ++j) {
        double tmp = 0.0;
#pragma unroll
        for (int i = k + 1; i < N; ++i) tmp += v[i] * Q[i * N + j];
        tmp += Q[k * N + j];
        Q[k * N + j] -= tau * tmp;
#pragma unroll
        for (int i = k + 1; i < N; ++i) Q[i * N + j] -= tau * v[i] * tmp;
      }
    }
#pragma unroll
    for (int j = k + 1; j < N; ++j) {
      if (normsU[j] != 0.0) {
        double temp = rx_div(fabs(Q[k * N + j]), rx_recip(normsU[j]));
        temp = (1.0 + temp) * (1.0 - temp);
        temp = temp < 0.0 ? 0.0 : temp;
        const double rr = rx_div(normsU[j], rx_recip(normsD[j]));
        const double temp2 = temp * (rr * rr);
        if (temp2 <= ndt) {
          double s = 0.0;
#pragma unroll
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
#pragma unroll
  for (int k = 0; k < N; ++k) {
    // swap perm[k] and perm[trans[k]] (trans[k] >= k)
    int pt = perm[k];
#pragma unroll
    for (int j = k + 1; j < N; ++j)
      if (trans[k] == j) pt = perm[j];
    const int pk = perm[k];
#pragma unroll
    for (int j = k + 1; j < N; ++j)
      if (trans[k] == j) perm[j] = pk;
    perm[k] = pt;
  }
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    double c[N];
#pragma unroll
    for (int i = 0; i < N; ++i) c[i] = rhs[i][d];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (k < nonzero) {
        const double tau = hc[k];
        if (N - k == 1) {
          c[k] *= (1.0 - tau);
        } else if (tau != 0.0) {
          double tmp = 0.0;
#pragma unroll
          for (int i = k + 1; i < N; ++i) tmp += Q[i * N + k] * c[i];
          tmp += c[k];
          c[k] -= tau * tmp;
#pragma unroll
          for (int i = k + 1; i < N; ++i) c[i] -= tau * Q[i * N + k] * tmp;
        }
      }
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
      if (i < nonzero) {
        c[i] = rx_div(c[i], rx_recip(Q[i * N + i]));
#pragma unroll
        for (int j = 0; j < i; ++j) c[j] -= c[i] * Q[j * N + i];
      }
    }
#pragma unroll
    for (int p = 0; p < N; ++p) {
      double o = 0.0;
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (i < nonzero && perm[i] == p) o = c[i];
      sol[p][d] = o;
    }
  }
}

// Per-edge summary written by visc_edge (implicit) for the Jacobian kernel: scalars and NDIM-vectors (mean
// velocity, both velocities, unit normal, projected flux momentum rows), then nine species arrays (Xs_i, Xs_j, Ys,
// hs, Cps, Jd, Gxn/|n|, Ds, quirk aux).
template <int NDIM>
struct VSL {
  static constexpr int MU = 0, K = 1, MUT = 2, RHO = 3, VM = 4, RHOI = VM + NDIM, RHOJ = RHOI + 1, VI = RHOJ + 1,
                       VJ = VI + NDIM, THETA = VJ + NDIM, DIJ = THETA + 1, DS = DIJ + 1, UN = DS + 1, PF = UN + NDIM,
                       TM = PF + NDIM, TMI = TM + 1, TMJ = TMI + 1, SGI = TMJ + 1, SGJ = SGI + 1, ARR = SGJ + 1;
};
template <int NS, int NDIM>
constexpr int visc_summary_size() { return VSL<NDIM>::ARR + 9 * NS; }

// A summary record seen through its layout: entry q at p[q * s]. Interior edges: kSummTile-edge tiles with the
// edge index fastest ([E/kSummTile][size][kSummTile], s = kSummTile, written by k_visc_edge) and the LDS copy
// of a k_visc_jac workgroup's edges (s = edges per workgroup); boundary vertices: [size] rows (s = 1).
struct SummRef {
  double* p;
  int s;
  __device__ double& operator[](int q) const { return p[(size_t)q * s]; }
  __device__ SummRef operator+(int q) const { return SummRef{p + (size_t)q * s, s}; }
};
struct SummCRef {
  const double* p;
  int s;
  __device__ double operator[](int q) const { return p[(size_t)q * s]; }
  __device__ SummCRef operator+(int q) const { return SummCRef{p + (size_t)q * s, s}; }
};

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
                                SummRef summ, Scr scr, bool corrected = true) {
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
  const double Mean_mu = hmean2(ni.mu, nj.mu);
  const double Mean_k = hmean2(ni.kappa, nj.kappa);
  // harmonic means of the binary diffusion coefficients
  auto Dm = [&](int q) { return hmean2(ni.Dij[q], nj.Dij[q]); };
  double Vm[nPV];
#pragma unroll
  for (int v = 0; v < nPV; ++v) Vm[v] = 0.5 * (Vi[v] + Vj[v]);
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
    const Recip rd2 = rx_recip(dist2);
    double Xs_i[NS], Xs_j[NS];  // recomputed for the summary below: not live across the two solves
    molar_from_mass<NS>(m, Vi + RHOS_P, Xs_i);
    molar_from_mass<NS>(m, Vj + RHOS_P, Xs_j);
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
      for (int d = 0; d < NDIM; ++d) G[r][d] -= rx_div((Proj[r] - Diff[r]) * Edge[d], rd2);
  }
  // ---- SetLaminarTensorFlux, in an order that keeps few values live across the two dense solves: the
  // Stefan-Maxwell solve first, then the SST closure solve, then the tensors and the flux rows. Every
  // accumulator keeps the reference's operation order (each Flux / PF entry sums its terms in the same sequence).
  const double rho = Vm[RHO_P];
  const double dim_temp = Vm[T_P] * P.T_ref;
  double Ys[NS], Xs[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) Ys[s] = Vm[RHOS_P + s];
  molar_from_mass<NS>(m, Ys, Xs);
  double Gxn[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) Gxn[s] = 0.0;
#pragma unroll
  for (int a = 0; a < NDIM; ++a)
#pragma unroll
    for (int s = 0; s < NS; ++s) Gxn[s] += G[RHOS_A + s][a] * Normal[a];
  double Jd[NS];
  {
    // The harmonic means go to the lane's LDS scratch as they are made, transposed (row a = Dm(. * NS + a), what
    // row a of Gamma reads), and Gamma is built over them in place row by row: the 2 NS^2 Dij loads are consumed
    // at once instead of being held in registers from the top of the kernel. Dmax is an exact max (order-free).
    const Scr Gt = scr;  // LDS scratch of this lane (NS*NS)
    // Dij is symmetric at every point (GetDij_SM sets Dij(j, i) = Dij(i, j), reacting_model_library.cpp:761-762;
    // k_set_primitive stores the one quotient in both places), so the harmonic mean of pair (a, b) is the same double
    // as that of (b, a): each is made once. Dmax is an exact max (order-free).
    double Dmax = -INFINITY;
#pragma unroll
    for (int b = 0; b < NS; ++b)
#pragma unroll
      for (int a = 0; a <= b; ++a) {
        const double dm = Dm(b * NS + a);
        Dmax = fmax(Dmax, dm);
        Gt[a * NS + b] = dm;
        if (a != b) Gt[b * NS + a] = dm;
      }
    const double alpha = rx_div(1.0, rx_recip(rho * Dmax));
    double sigma = 0.0, massTot = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) sigma += Ys[s];
#pragma unroll
    for (int s = 0; s < NS; ++s) massTot += rx_div(Ys[s], mm_recip(m, s));
    massTot = rx_div(1.0, rx_recip(massTot));
#pragma unroll
    for (int a = 0; a < NS; ++a) {
      double dr[NS];  // Dm(b * NS + a), b = 0 .. NS-1
#pragma unroll
      for (int b = 0; b < NS; ++b) dr[b] = Gt[a * NS + b];
#pragma unroll
      for (int b = 0; b < NS; ++b) {
        double g;
        if (a != b) {
          g = rx_div(-sigma * massTot * Xs[a], rx_recip(rho * m.mm[b] * dr[b]));
        } else {
          double tmp = 0.0;
#pragma unroll
          for (int c = 0; c < NS; ++c)
            if (c != a) tmp += rx_div(Xs[c], rx_recip(dr[c]));
          g = rx_div(sigma * massTot * tmp, rx_recip(rho * m.mm[a]));
        }
        Gt[a * NS + b] = g + alpha * Ys[a];
      }
    }
    double nG[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) nG[s] = -Gxn[s];
#if RX_VISC_PROBE & 1  // timing probe (build variant only): no Stefan-Maxwell solve
#pragma unroll
    for (int s = 0; s < NS; ++s) Jd[s] = nG[s] * Gt[s * NS + s];
#else
    bicgstab<NS>(Gt, nG, Jd, 1.0e-11);
#endif
  }
  double hs[NS];
  {
    const Recip rE = rx_recip(P.E_ref);
    const SplineAt kT = spline_at(m, dim_temp);
#pragma unroll
    for (int s = 0; s < NS; ++s) hs[s] = rx_div(rx_div(spline_k(m, P_H, s, dim_temp, kT, &err), mm_recip(m, s)), rE);
  }
  double PF[nVar];
#pragma unroll
  for (int v = 0; v < nVar; ++v) PF[v] = 0.0;
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
    Mean_mut = hmean2(ni.mut, nj.mut);
    Mean_tke = 0.5 * (ni.tke + nj.tke);
    {
      const Recip rR = rx_recip(P.R_ref);
      const SplineAt kT = spline_at(m, dim_temp);
#pragma unroll
      for (int s = 0; s < NS; ++s) Cps[s] = rx_div(rx_div(spline_k(m, P_CP, s, dim_temp, kT, &err), mm_recip(m, s)), rR);
    }
    {
      const Scr Mt = scr;  // LDS scratch of this lane (NS*NS), Gt is dead here
      double sig = 0.0;
#pragma unroll
      for (int s = 0; s < NS; ++s) sig += Xs[s];
#pragma unroll
      for (int a = 0; a < NS; ++a)
#pragma unroll
        for (int b = 0; b < NS; ++b)
          Mt[a * NS + b] = rx_div(m.mtot, mm_recip(m, a)) * (Ys[a] - Xs[a] + sig) * (double)(a == b) +
                           m.mtot * (rx_div(Ys[a], mm_recip(m, a)) - rx_div(Xs[a], mm_recip(m, b))) * (double)(a != b);
      double rhs[NS][NDIM];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int d = 0; d < NDIM; ++d) rhs[s][d] = G[RHOS_A + s][d];
#if RX_VISC_PROBE & 2  // timing probe (build variant only): no closure QR solve
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int d = 0; d < NDIM; ++d) MG[s][d] = rhs[s][d] * Mt[s * NS + s];
#else
      colpiv_qr_solve<NS, NDIM>(Mt, rhs, MG);
#endif
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int d = 0; d < NDIM; ++d)
        if (fabs(G[RHOS_A + s][d]) < 1e-8) MG[s][d] = 0.0;
  }
  double Flux[nVar][NDIM];
#pragma unroll
  for (int v = 0; v < nVar; ++v)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Flux[v][d] = 0.0;
  {
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
#pragma unroll
    for (int a = 0; a < NDIM; ++a) {
#pragma unroll
      for (int b = 0; b < NDIM; ++b) {
        Flux[RHOVX_S + b][a] = tau[a][b];
        Flux[RHOE_S][a] += tau[a][b] * Vm[VX_P + b];
      }
      Flux[RHOE_S][a] += Mean_k * G[T_A][a];
    }
  }
  if (P.rans) {
    double gk[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) gk[d] = 0.5 * (ni.gk[d] + nj.gk[d]);
    double dv = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) dv += G[VX_A + d][d];
    // Mean_mut / (Pr_t Le_t), Mean_mut / Pr_t, Mean_mut / sigma_k: the same quotients in every term that uses them
    const double mut_prle = rx_div(Mean_mut, rx_recip(P.Pr_t * P.Le_t));
    const double mut_pr = rx_div(Mean_mut, rx_recip(P.Pr_t));
    const double mut_sk = rx_div(Mean_mut, rx_recip(sigma_k));
    double tt[NDIM][NDIM];
#pragma unroll
    for (int a = 0; a < NDIM; ++a) {
#pragma unroll
      for (int b = 0; b < NDIM; ++b) tt[a][b] = 0.0 + Mean_mut * (G[VX_A + b][a] + G[VX_A + a][b]);
      tt[a][a] -= kTWO3 * (Mean_mut * dv + Mean_tke * rho);
    }
#pragma unroll
    for (int a = 0; a < NDIM; ++a) {
#pragma unroll
      for (int b = 0; b < NDIM; ++b) {
        Flux[RHOVX_S + b][a] += tt[a][b];
        Flux[RHOE_S][a] += tt[a][b] * Vm[VX_P + b];
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) PF[RHOS_S + s] += mut_prle * MG[s][a] * Normal[a];
#pragma unroll
      for (int s = 0; s < NS; ++s) Flux[RHOE_S][a] += mut_prle * hs[s] * Ys[s] * MG[s][a];
#pragma unroll
      for (int s = 0; s < NS; ++s) Flux[RHOE_S][a] += mut_pr * Cps[s] * Ys[s] * G[T_A][a];
      Flux[RHOE_S][a] += (Mean_mu + mut_sk) * gk[a];
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

  double Xs_i[NS], Xs_j[NS];
  molar_from_mass<NS>(m, Vi + RHOS_P, Xs_i);
  molar_from_mass<NS>(m, Vj + RHOS_P, Xs_j);
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
          di += rx_div(Xs_i[b], rx_recip(ni.Dij[b * NS + a]));
          dj += rx_div(Xs_j[b], rx_recip(nj.Dij[b * NS + a]));
        }
      Ds_i[a] = rx_div(1.0 - Xs_i[a], rx_recip(di));
      Ds_j[a] = rx_div(1.0 - Xs_j[a], rx_recip(dj));
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
  const Recip rA = rx_recip(Area);
#pragma unroll
  for (int d = 0; d < NDIM; ++d) UN[d] = rx_div(Normal[d], rA);
#pragma unroll
  for (int s = 0; s < NS; ++s) Gxn[s] = rx_div(Gxn[s], rA);
  double theta = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) theta += UN[d] * UN[d];
  if (!P.rans) {
    const Recip rR = rx_recip(P.R_ref);
    const SplineAt kT = spline_at(m, dim_temp);
#pragma unroll
    for (int s = 0; s < NS; ++s) Cps[s] = rx_div(rx_div(spline_k(m, P_CP, s, dim_temp, kT, &err), mm_recip(m, s)), rR);
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
  using L = VSL<NDIM>;
  const SummRef o = summ;
  o[L::MU] = Mean_mu;
  o[L::K] = Mean_k;
  o[L::MUT] = Mean_mut;
  o[L::RHO] = rho;
  o[L::RHOI] = Vi[RHO_P];
  o[L::RHOJ] = Vj[RHO_P];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    o[L::VM + d] = Vm[VX_P + d];
    o[L::VI + d] = Vi[VX_P + d];
    o[L::VJ + d] = Vj[VX_P + d];
    o[L::UN + d] = UN[d];
    o[L::PF + d] = PF[RHOVX_S + d];
  }
  o[L::THETA] = theta;
  o[L::DIJ] = sqrt(dist2);
  o[L::DS] = Area;
  o[L::TM] = totMass;
  o[L::TMI] = totMass_i;
  o[L::TMJ] = totMass_j;
  o[L::SGI] = sigma_i;
  o[L::SGJ] = sigma_j;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    o[L::ARR + 0 * NS + s] = Xs_i[s];
    o[L::ARR + 1 * NS + s] = Xs_j[s];
    o[L::ARR + 2 * NS + s] = Ys[s];
    o[L::ARR + 3 * NS + s] = hs[s];
    o[L::ARR + 4 * NS + s] = Cps[s];
    o[L::ARR + 5 * NS + s] = Jd[s];
    o[L::ARR + 6 * NS + s] = Gxn[s];
    o[L::ARR + 7 * NS + s] = Ds[s];
    o[L::ARR + 8 * NS + s] = qaux[s];
  }
  return err;
}

// Jacobian column b (0 <= b < nVar) of Jac_i and Jac_j for one edge, from the visc_edge summary:
// SetLaminarViscousProjJacs (:1200-1401) + SST_Reactive_JacobianClosure (:891-1090; the 2-D branch :891-1000, the
// 3-D branch :1001-1090 with its species-species diagonal term and hs/rho instead of hs*Ys/rho in the energy row)
// build dF/dV (FI for node i, FJ for node j); J = dF/dV * dV/dU (:1637-1653). A team of lanes owns
// the columns of one edge; every dF/dV entry is accumulated in the reference's order, and J's sum over
// k keeps the reference's order (the F*0 terms of dV/dU's zero entries are dropped: they can only
// change the sign of an exact zero). base_i/base_j: the column-independent part of row a of dJ/drho
// (this lane's a = lane index in the team), shared through shuffles.
template <int NS, int NDIM>
__device__ inline void visc_jac_column(const DevMech& m, const ViscParams& P, const SummCRef sm,
                                       double Sib, double Sjb, int b, int tl, double* __restrict__ Ji,
                                       double* __restrict__ Jj, const double* jci = nullptr,
                                       const double* jcj = nullptr, double* __restrict__ Aij = nullptr,
                                       double* __restrict__ Aji = nullptr);

// The column computation with the entries handed to put(r, Ji[r][b], Jj[r][b]) row by row (r = 0 .. nVar-1, in
// order) instead of stored: visc_jac_column is this with put = the stores; the node-centric assembly
// (k_asm_visc) folds them into the node's diagonal and off-diagonal blocks.
template <int NS, int NDIM, typename Put>
__device__ inline void visc_jac_column_f(const DevMech& m, const ViscParams& P, const SummCRef sm, double Sib,
                                         double Sjb, int b, int tl, Put put) {
  using L = VSL<NDIM>;
  constexpr int nVar = NS + NDIM + 2, NF = NDIM + 2;
  constexpr int RHOE_S = NDIM + 1, RHOS_S = NDIM + 2;
  const double mu = sm[L::MU], ktr = sm[L::K], mut = sm[L::MUT], rho = sm[L::RHO];
  const double rho_i = sm[L::RHOI], rho_j = sm[L::RHOJ];
  const double theta = sm[L::THETA], dij = sm[L::DIJ], dS = sm[L::DS], sq = sm[L::DIJ], Area = sm[L::DS];
  const double totMass = sm[L::TM], totMass_i = sm[L::TMI], totMass_j = sm[L::TMJ];
  const double sigma_i = sm[L::SGI], sigma_j = sm[L::SGJ];
  const SummCRef Xs_i = sm + L::ARR;
  const SummCRef Xs_j = Xs_i + NS;
  const SummCRef Ys = Xs_j + NS;
  const SummCRef hs = Ys + NS;
  const SummCRef Cps = hs + NS;
  const SummCRef Jd = Cps + NS;
  const SummCRef Gxn = Jd + NS;
  const SummCRef Ds = Gxn + NS;
  const SummCRef qaux = Ds + NS;
  const double PrT = P.Pr_t, LeT = P.Le_t;
  // the divisors shared by many quotients below, each with its reciprocal (rx_fdiv.h: the same doubles as `/`)
  const Recip rdij = rx_recip(dij), rri = rx_recip(rho_i), rrj = rx_recip(rho_j);
  // ---- column-independent part of dJ/drho rows (lane tl < NS owns row a = tl)
  double bj = 0.0, bi = 0.0;
  if (tl < NS) {
    const int a = tl;
    const Recip r1j = rx_recip(totMass * dij * sigma_j * rho_j), r1i = rx_recip(totMass * dij * sigma_i * rho_i);
    double vj = rx_div(-rho * m.mm[a] * Ds[a] * Xs_j[a], r1j);
    double vi = rx_div(rho * m.mm[a] * Ds[a] * Xs_i[a], r1i);
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      vj += rx_div(rho * Ys[a] * m.mm[q] * Ds[q] * Xs_j[q], r1j);
      vi -= rx_div(rho * Ys[a] * m.mm[q] * Ds[q] * Xs_i[q], r1i);
    }
    bj = vj;
    bi = vi;
  }
  double colj[NS], coli[NS];  // dJ/drho column k = b - RHOS_S (species columns only)
  const int k = b - RHOS_S;
  const int kk = (k >= 0 && k < NS) ? k : 0;
  // the a == k term of :1352-1357, evaluated once for this lane's column (no divergent divisions)
  const Recip r2j = rx_recip(dij * totMass * rho_j), r2i = rx_recip(dij * totMass * rho_i);
  const double dkj = rx_div(rho * Ds[kk] * totMass_j * sigma_j, r2j);
  const double dki = rx_div(rho * Ds[kk] * totMass_i * sigma_i, r2i);
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    const double baj = __shfl(bj, a, 16), bai = __shfl(bi, a, 16);
    double vj = baj, vi = bai;
    if (k >= 0) {
      vj += rx_div(rho * Ys[a] * Ds[kk] * totMass_j * sigma_j, r2j);
      vi -= rx_div(rho * Ys[a] * Ds[kk] * totMass_i * sigma_i, r2i);
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
    const Recip r3j = rx_recip(totMass * rho_j), r3i = rx_recip(totMass * rho_i);
    double tj[NS], ti[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      tj[q] = rx_div(0.5 * rho * m.mm[q] * Ds[q] * Gxn[q], r3j);
      ti[q] = rx_div(0.5 * rho * m.mm[q] * Ds[q] * Gxn[q], r3i);
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
  // ---- dF/dV flow block rows / columns 0..RHOE (index [row][col]); zero-initialised
  double FJ[NF][NF], FI[NF][NF];
#pragma unroll
  for (int r = 0; r < NF; ++r)
#pragma unroll
    for (int c = 0; c < NF; ++c) FJ[r][c] = FI[r][c] = 0.0;
  double UN[NDIM], th[NDIM][NDIM], pi[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) UN[d] = sm[L::UN + d];
  // theta_x = theta + n_x^2/3 on the diagonal, eta = n_a n_b / 3 off it (:1265-1275 / :1300-1320)
#pragma unroll
  for (int a = 0; a < NDIM; ++a)
#pragma unroll
    for (int c = 0; c < NDIM; ++c) th[a][c] = (a == c) ? theta + UN[a] * UN[a] / 3.0 : UN[a] * UN[c] / 3.0;
#pragma unroll
  for (int c = 0; c < NDIM; ++c) {
    double p = sm[L::VM] * th[0][c];
#pragma unroll
    for (int a = 1; a < NDIM; ++a) p += sm[L::VM + a] * th[a][c];
    pi[c] = p;
  }
#pragma unroll
  for (int a = 0; a < NDIM; ++a)
#pragma unroll
    for (int c = 0; c < NDIM; ++c) FJ[1 + a][1 + c] = rx_div(mu * th[a][c], rdij) * dS;
#pragma unroll
  for (int c = 0; c < NDIM; ++c) FJ[RHOE_S][1 + c] = rx_div(pi[c] * mu, rdij) * dS;
  FJ[RHOE_S][RHOE_S] = rx_div(ktr * theta, rdij) * dS;
#pragma unroll
  for (int r = 0; r < NF; ++r)
#pragma unroll
    for (int c = 0; c < NF; ++c) FI[r][c] = -FJ[r][c];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    FI[RHOE_S][RHOE_S] += -0.5 * Jd[q] * Cps[q];
    FJ[RHOE_S][RHOE_S] += -0.5 * Jd[q] * Cps[q];
  }
  // species column of rows 0 (rho) and RHOE (rho E), accumulated over the species rows in order
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
  double dsj = 0.0, dsi = 0.0;  // 3-D species-species diagonal closure term of this lane's column (:1053-1060)
  if (P.rans) {
    const Recip rprle = rx_recip(PrT * LeT);
    const double mut_pr = rx_div(mut, rx_recip(PrT)), mut_prle = rx_div(mut, rprle);  // mut / PrT, mut / (PrT LeT)
#pragma unroll
    for (int a = 0; a < NDIM; ++a)
#pragma unroll
      for (int c = 0; c < NDIM; ++c) {
        FJ[1 + a][1 + c] += rx_div(mut * th[a][c], rdij) * Area;
        FI[1 + a][1 + c] -= rx_div(mut * th[a][c], rdij) * Area;
      }
#pragma unroll
    for (int c = 0; c < NDIM; ++c) {
      FJ[RHOE_S][1 + c] += rx_div(pi[c] * mut, rdij) * Area;
      FI[RHOE_S][1 + c] -= rx_div(pi[c] * mut, rdij) * Area;
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      FJ[RHOE_S][RHOE_S] += rx_div(mut_pr * Cps[q] * Ys[q] * theta, rdij) * Area;
      FI[RHOE_S][RHOE_S] -= rx_div(mut_pr * Cps[q] * Ys[q] * theta, rdij) * Area;
    }
    if (k >= 0) {
      if constexpr (NDIM == 2) {
        FJ3k += rx_div(rx_div(mut_prle * hs[kk] * Ys[kk], rrj) * theta, rdij) * Area;
        FI3k -= rx_div(rx_div(mut_prle * hs[kk] * Ys[kk], rri) * theta, rdij) * Area;
      } else {
        dsj = rx_div(rx_div(rx_div(mut * Ys[kk], rprle), rrj) * theta, rdij) * Area;
        dsi = rx_div(rx_div(rx_div(mut * Ys[kk], rprle), rri) * theta, rdij) * Area;
        FJ3k += rx_div(rx_div(mut_prle * hs[kk], rrj) * theta, rdij) * Area;
        FI3k -= rx_div(rx_div(mut_prle * hs[kk], rri) * theta, rdij) * Area;
      }
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      FJ[RHOE_S][RHOE_S] += mut_prle * Cps[q] * Ys[q] * qaux[q] * Area;
      FI[RHOE_S][RHOE_S] += mut_prle * Cps[q] * Ys[q] * qaux[q] * Area;
    }
  }
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    FI[RHOE_S][1 + d] += 0.5 * sm[L::PF + d];
    FJ[RHOE_S][1 + d] += 0.5 * sm[L::PF + d];
  }
  // ---- J[a][b] = sum_k F[a][k] dV/dU[k][b]; with Aij/Aji the fused assembly also writes the edge's two
  // off-diagonal blocks in the reference order A(i,j) = (0 + Jc_j) - Jv_j, A(j,i) = (0 - Jc_i) + Jv_i
  // (AddBlock / SubtractBlock of Upwind_Residual then Viscous_Residual, solver_direct_reactive.cpp:2240-2246,
  // :5365-5371); jci / jcj: column b of the convective blocks, row r at [r] (registers, loaded up front)
  double ci[NDIM], cj[NDIM];  // dV/dU velocity rows, column b
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    if (b == 0) {
      ci[d] = rx_div(-sm[L::VI + d], rri);
      cj[d] = rx_div(-sm[L::VJ + d], rrj);
    } else {
      ci[d] = (b == 1 + d) ? rx_div(1.0, rri) : 0.0;
      cj[d] = (b == 1 + d) ? rx_div(1.0, rrj) : 0.0;
    }
  }
  const double d0 = (b == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int r = 0; r < NF; ++r) {
    double si = 0.0, sj = 0.0;
    si += FI[r][0] * d0;
    sj += FJ[r][0] * d0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      si += FI[r][1 + d] * ci[d];
      sj += FJ[r][1 + d] * cj[d];
    }
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
    put(r, si, sj);
  }
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    double si = 0.0, sj = 0.0;
    if (k >= 0) {
      si = -coli[a] * dS;
      sj = -colj[a] * dS;
      if (NDIM == 3 && a == k) {
        si -= dsi;
        sj += dsj;
      }
    }
    put(RHOS_S + a, si, sj);
  }
}

// One side's column only (side 0: Jac_i, side 1: Jac_j), for the node-centric assembly, which needs at each end of
// an edge only that end's block. The two sides' expressions differ only in the node data they read (rho, X_s,
// sigma, sum M_s X_s, dT/dU, velocity) and in signs: every j-side quantity is the i-side expression evaluated on the
// j data with the sign flipped at the same points (-(a - t) = (-a) + t exactly in round-to-nearest), so each entry
// here is, bitwise, the one visc_jac_column_f hands to put for that side. Sob: dT/dU[b] of the own node.
// sbase: the wave lane of the team's lane 0 (teams of TW lanes, not necessarily a power of two)
template <int NS, int NDIM, typename Put>
__device__ inline void visc_jac_column_own(const DevMech& m, const ViscParams& P, const SummCRef sm, double Sob,
                                           int side, int b, int tl, int sbase, Put put) {
  using L = VSL<NDIM>;
  constexpr int nVar = NS + NDIM + 2, NF = NDIM + 2;
  constexpr int RHOE_S = NDIM + 1, RHOS_S = NDIM + 2;
  const bool J = side != 0;
  const double mu = sm[L::MU], ktr = sm[L::K], mut = sm[L::MUT], rho = sm[L::RHO];
  const double rho_o = J ? sm[L::RHOJ] : sm[L::RHOI];
  const double theta = sm[L::THETA], dij = sm[L::DIJ], dS = sm[L::DS], sq = sm[L::DIJ], Area = sm[L::DS];
  const double totMass = sm[L::TM], totMass_o = J ? sm[L::TMJ] : sm[L::TMI];
  const double sigma_o = J ? sm[L::SGJ] : sm[L::SGI];
  const SummCRef Xs_o = sm + L::ARR + (J ? NS : 0);
  const SummCRef Ys = sm + L::ARR + 2 * NS;
  const SummCRef hs = Ys + NS;
  const SummCRef Cps = hs + NS;
  const SummCRef Jd = Cps + NS;
  const SummCRef Gxn = Jd + NS;
  const SummCRef Ds = Gxn + NS;
  const SummCRef qaux = Ds + NS;
  const double PrT = P.Pr_t, LeT = P.Le_t;
  // the divisors shared by many quotients below, each with its reciprocal (rx_fdiv.h: the same doubles as `/`)
  const Recip rdij = rx_recip(dij), rro = rx_recip(rho_o);
  // column-independent part of dJ/drho row a = tl, i-side form on the own data (the j side is its negative)
  double bo = 0.0;
  if (tl < NS) {
    const int a = tl;
    const Recip r1 = rx_recip(totMass * dij * sigma_o * rho_o);
    double v = rx_div(rho * m.mm[a] * Ds[a] * Xs_o[a], r1);
#pragma unroll
    for (int q = 0; q < NS; ++q) v -= rx_div(rho * Ys[a] * m.mm[q] * Ds[q] * Xs_o[q], r1);
    bo = v;
  }
  double col[NS];  // dJ/drho column k = b - RHOS_S, own side (signed)
  const int k = b - RHOS_S;
  const int kk = (k >= 0 && k < NS) ? k : 0;
  const Recip r2 = rx_recip(dij * totMass * rho_o);
  const double dko = rx_div(rho * Ds[kk] * totMass_o * sigma_o, r2);
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    double v = __shfl(bo, sbase + a);
    if (k >= 0) {
      v -= rx_div(rho * Ys[a] * Ds[kk] * totMass_o * sigma_o, r2);
      if (a == k) v += dko;
    }
    col[a] = J ? -v : v;
  }
  if (b >= nVar) return;
  if (k >= 0) {
    double to[NS];
    const Recip r3 = rx_recip(totMass * rho_o);
#pragma unroll
    for (int q = 0; q < NS; ++q) to[q] = rx_div(0.5 * rho * m.mm[q] * Ds[q] * Gxn[q], r3);
#pragma unroll
    for (int a = 0; a < NS; ++a)
      if (a == k) {
#pragma unroll
        for (int q = 0; q < NS; ++q) col[a] += to[q];
      }
  }
  // dF/dV flow block of the own side: F_j = the i-side base, F_i = its negative (zeros included: -0.0)
  double F[NF][NF];
#pragma unroll
  for (int r = 0; r < NF; ++r)
#pragma unroll
    for (int c = 0; c < NF; ++c) F[r][c] = 0.0;
  double UN[NDIM], th[NDIM][NDIM], pi[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) UN[d] = sm[L::UN + d];
#pragma unroll
  for (int a = 0; a < NDIM; ++a)
#pragma unroll
    for (int c = 0; c < NDIM; ++c) th[a][c] = (a == c) ? theta + UN[a] * UN[a] / 3.0 : UN[a] * UN[c] / 3.0;
#pragma unroll
  for (int c = 0; c < NDIM; ++c) {
    double p = sm[L::VM] * th[0][c];
#pragma unroll
    for (int a = 1; a < NDIM; ++a) p += sm[L::VM + a] * th[a][c];
    pi[c] = p;
  }
#pragma unroll
  for (int a = 0; a < NDIM; ++a)
#pragma unroll
    for (int c = 0; c < NDIM; ++c) F[1 + a][1 + c] = rx_div(mu * th[a][c], rdij) * dS;
#pragma unroll
  for (int c = 0; c < NDIM; ++c) F[RHOE_S][1 + c] = rx_div(pi[c] * mu, rdij) * dS;
  F[RHOE_S][RHOE_S] = rx_div(ktr * theta, rdij) * dS;
  if (!J) {
#pragma unroll
    for (int r = 0; r < NF; ++r)
#pragma unroll
      for (int c = 0; c < NF; ++c) F[r][c] = -F[r][c];
  }
#pragma unroll
  for (int q = 0; q < NS; ++q) F[RHOE_S][RHOE_S] += -0.5 * Jd[q] * Cps[q];
  double F0k = 0.0, F3k = 0.0;
  if (k >= 0) {
#pragma unroll
    for (int a = 0; a < NS; ++a) {
      F0k += -col[a] * dS;
      F3k += -col[a] * hs[a] * dS;
    }
  }
  double dso = 0.0;  // 3-D species-species diagonal closure term (own side)
  auto pm = [&](double f, double x) { return J ? f + x : f - x; };  // FJ += x / FI -= x
  if (P.rans) {
    const Recip rprle = rx_recip(PrT * LeT);
    const double mut_pr = rx_div(mut, rx_recip(PrT)), mut_prle = rx_div(mut, rprle);  // mut / PrT, mut / (PrT LeT)
#pragma unroll
    for (int a = 0; a < NDIM; ++a)
#pragma unroll
      for (int c = 0; c < NDIM; ++c) F[1 + a][1 + c] = pm(F[1 + a][1 + c], rx_div(mut * th[a][c], rdij) * Area);
#pragma unroll
    for (int c = 0; c < NDIM; ++c) F[RHOE_S][1 + c] = pm(F[RHOE_S][1 + c], rx_div(pi[c] * mut, rdij) * Area);
#pragma unroll
    for (int q = 0; q < NS; ++q)
      F[RHOE_S][RHOE_S] = pm(F[RHOE_S][RHOE_S], rx_div(mut_pr * Cps[q] * Ys[q] * theta, rdij) * Area);
    if (k >= 0) {
      if constexpr (NDIM == 2) {
        F3k = pm(F3k, rx_div(rx_div(mut_prle * hs[kk] * Ys[kk], rro) * theta, rdij) * Area);
      } else {
        dso = rx_div(rx_div(rx_div(mut * Ys[kk], rprle), rro) * theta, rdij) * Area;
        F3k = pm(F3k, rx_div(rx_div(mut_prle * hs[kk], rro) * theta, rdij) * Area);
      }
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) F[RHOE_S][RHOE_S] += mut_prle * Cps[q] * Ys[q] * qaux[q] * Area;
  }
#pragma unroll
  for (int d = 0; d < NDIM; ++d) F[RHOE_S][1 + d] += 0.5 * sm[L::PF + d];
  double co[NDIM];  // dV/dU velocity rows, column b, own node
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    if (b == 0) co[d] = rx_div(-sm[(J ? L::VJ : L::VI) + d], rro);
    else co[d] = (b == 1 + d) ? rx_div(1.0, rro) : 0.0;
  }
  const double d0 = (b == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int r = 0; r < NF; ++r) {
    double so = 0.0;
    so += F[r][0] * d0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) so += F[r][1 + d] * co[d];
    so += F[r][RHOE_S] * Sob;
    if (k >= 0) {
      if (r == 0) so += F0k;
      else if (r == RHOE_S) so += F3k;
    }
    put(r, so);
  }
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    double so = 0.0;
    if (k >= 0) {
      so = -col[a] * dS;
      if (NDIM == 3 && a == k) so = pm(so, dso);
    }
    put(RHOS_S + a, so);
  }
}

template <int NS, int NDIM>
__device__ inline void visc_jac_column(const DevMech& m, const ViscParams& P, const SummCRef sm,
                                       double Sib, double Sjb, int b, int tl, double* __restrict__ Ji,
                                       double* __restrict__ Jj, const double* jci, const double* jcj,
                                       double* __restrict__ Aij, double* __restrict__ Aji) {
  constexpr int nVar = NS + NDIM + 2;
  visc_jac_column_f<NS, NDIM>(m, P, sm, Sib, Sjb, b, tl, [&](int r, double si, double sj) {
    const int idx = r * nVar + b;
    Ji[idx] = si;
    Jj[idx] = sj;
    if (Aij) {
      Aij[idx] = (0.0 + jcj[r]) - sj;
      Aji[idx] = (0.0 - jci[r]) + si;
    }
  });
}

}  // namespace rx
