// rx_sst.hip — Menter SST turbulence solver of the reactive RANS iteration on gfx950 (SURVEY §8 a14 +
// next-2), and the flow-side StrainMag it reads.
//
// Reference (paths relative to the reference root):
//   CTurbSSTSolver::Preprocessing / Postprocessing / Source_Residual   SU2_CFD/src/solver_direct_turbulent.cpp:2923-3080
//   CTurbSolver::Upwind_Residual / Viscous_Residual / ImplicitEuler     solver_direct_turbulent.cpp:429-728
//   CUpwSca_TurbSST / CAvgGradCorrected_TurbSST / CSourcePieceWise_TurbSST
//                                                  SU2_CFD/src/numerics_direct_turbulent.cpp:865-922, 1080-1256
//   CSolver::SetSolution_Gradient_LS               SU2_CFD/src/solver_structure.cpp:580-720
//   CTurbSSTVariable::SetBlendingFunc              SU2_CFD/src/variable_direct_turbulent.cpp:178-203
//   CReactiveNSVariable::SetStrainMag              SU2_CFD/src/variable_direct_reactive.cpp:1060-1095
//
// The SST context is a second rx_ctx (nVar = 2) on the flow context's stream: its linear system reuses
// the BSR / ILU(0) / LU-SGS / FGMRES kernels with 2x2 blocks. Residual loops are node-centric gathers:
// each node recomputes the flux of its incident edges in increasing edge id (the reference's scatter
// order) and applies the row's own residual and Jacobian-block updates, so every block of row i is
// written by one thread only and the accumulation order is the reference's. The per-edge operators are
// cheap (tens of flops), so recomputing each edge from both ends costs less than a scratch round trip.
// std::min / std::max are restated as their ternaries (NaN / signed-zero behaviour included).
#include <hip/hip_runtime.h>

#include <cmath>

#include "rx_ctx.h"

namespace {

constexpr int kBlock = 256;
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

inline int blocks(int64_t n, int b = kBlock) { return (int)((n + b - 1) / b); }

struct SSTC {
  double sk1, sk2, so1, so2, b1, b2, bs, a1, al1, al2;
};
// CTurbSSTSolver constructor (solver_direct_turbulent.cpp:2716-2725), evaluated on the host as there.
SSTC sst_constants() {
  SSTC c;
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

__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }

// CSolver::SetSolution_Gradient_LS for the two turbulent variables, one thread per owned point.
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_sol_grad_ls(int Nd, const double* __restrict__ coord,
                                                        const int32_t* __restrict__ nptr,
                                                        const int32_t* __restrict__ nbr,
                                                        const double* __restrict__ sol, double* __restrict__ grad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Nd) return;
  double ci[NDIM];
#pragma unroll
  for (int d = 0; d < NDIM; ++d) ci[d] = coord[(size_t)i * NDIM + d];
  const double s0 = sol[2 * (size_t)i], s1 = sol[2 * (size_t)i + 1];
  double Cv[2][NDIM];
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Cv[v][d] = 0.0;
  double r11 = 0, r12 = 0, r13 = 0, r22 = 0, r23 = 0, r23_a = 0, r23_b = 0, r33 = 0;
  for (int k = nptr[i]; k < nptr[i + 1]; ++k) {
    const int j = nbr[k];
    double dx[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) dx[d] = coord[(size_t)j * NDIM + d] - ci[d];
    double w = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) w += dx[d] * dx[d];
    if (w != 0.0) {
      r11 += dx[0] * dx[0] / w;
      r12 += dx[0] * dx[1] / w;
      r22 += dx[1] * dx[1] / w;
      if constexpr (NDIM == 3) {
        r13 += dx[0] * dx[NDIM - 1] / w;
        r23_a += dx[1] * dx[NDIM - 1] / w;
        r23_b += dx[0] * dx[NDIM - 1] / w;
        r33 += dx[NDIM - 1] * dx[NDIM - 1] / w;
      }
      const double d0 = sol[2 * (size_t)j] - s0, d1 = sol[2 * (size_t)j + 1] - s1;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        Cv[0][d] += dx[d] * d0 / w;
        Cv[1][d] += dx[d] * d1 / w;
      }
    }
  }
  if (r11 >= 0.0) r11 = sqrt(r11); else r11 = 0.0;
  if (r11 != 0.0) r12 = r12 / r11; else r12 = 0.0;
  if (r22 - r12 * r12 >= 0.0) r22 = sqrt(r22 - r12 * r12); else r22 = 0.0;
  if constexpr (NDIM == 3) {
    if (r11 != 0.0) r13 = r13 / r11; else r13 = 0.0;
    if ((r22 != 0.0) && (r11 * r22 != 0.0)) r23 = r23_a / r22 - r23_b * r12 / (r11 * r22); else r23 = 0.0;
    if (r33 - r23 * r23 - r13 * r13 >= 0.0) r33 = sqrt(r33 - r23 * r23 - r13 * r13); else r33 = 0.0;
  }
  double detR2 = (NDIM == 2) ? (r11 * r22) * (r11 * r22) : (r11 * r22 * r33) * (r11 * r22 * r33);
  bool singular = false;
  if (fabs(detR2) <= rx::kEPS) {
    detR2 = 1.0;
    singular = true;
  }
  double S[NDIM][NDIM];
#pragma unroll
  for (int a = 0; a < NDIM; ++a)
#pragma unroll
    for (int b = 0; b < NDIM; ++b) S[a][b] = 0.0;
  if (!singular) {
    if constexpr (NDIM == 2) {
      S[0][0] = (r12 * r12 + r22 * r22) / detR2;
      S[0][1] = -r11 * r12 / detR2;
      S[1][0] = S[0][1];
      S[1][1] = r11 * r11 / detR2;
    } else {
      const double z11 = r22 * r33, z12 = -r12 * r33, z13 = r12 * r23 - r13 * r22;
      const double z22 = r11 * r33, z23 = -r11 * r23, z33 = r11 * r22;
      double* s = &S[0][0];
      s[0] = (z11 * z11 + z12 * z12 + z13 * z13) / detR2;
      s[1] = (z12 * z22 + z13 * z23) / detR2;
      s[NDIM - 1] = (z13 * z33) / detR2;
      s[NDIM] = s[1];
      s[NDIM + 1] = (z22 * z22 + z23 * z23) / detR2;
      s[2 * NDIM - 1] = (z23 * z33) / detR2;
      s[2 * NDIM] = s[NDIM - 1];
      s[2 * NDIM + 1] = s[2 * NDIM - 1];
      s[NDIM * NDIM - 1] = (z33 * z33) / detR2;
    }
  }
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      double product = 0.0;
#pragma unroll
      for (int e = 0; e < NDIM; ++e) product += S[d][e] * Cv[v][e];
      grad[((size_t)i * 2 + v) * NDIM + d] = product;
    }
}

// NUM_METHOD_GRAD = GREEN_GAUSS: CSolver::SetSolution_Gradient_GG (SU2_CFD/src/solver_structure.cpp:519-578) of the
// turbulent solution, called from CTurbSSTSolver::Preprocessing / Postprocessing (solver_direct_turbulent.cpp:2944,
// 2963): edges in edge order (+ at node 0, - at node 1, face value 0.5 (S_i + S_j)), then the point's boundary
// vertices (every marker: no INTERNAL_BOUNDARY here), then / (Volume + EPS).
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_sol_grad_gg(int Nd, const int32_t* __restrict__ adj_ptr,
                                                        const int32_t* __restrict__ adj,
                                                        const int32_t* __restrict__ edges,
                                                        const double* __restrict__ normal,
                                                        const int32_t* __restrict__ bv_ptr,
                                                        const double* __restrict__ bv_normal,
                                                        const double* __restrict__ vol, const double* __restrict__ U,
                                                        double* __restrict__ grad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Nd) return;
  double g[2][NDIM];
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) g[v][d] = 0.0;
  for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
    const int a = adj[k], e = a >> 1, side = a & 1;
    const int n0 = edges[2 * e], n1 = edges[2 * e + 1];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const double avg = 0.5 * (U[2 * (size_t)n0 + v] + U[2 * (size_t)n1 + v]);
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        const double pr = avg * normal[(size_t)e * NDIM + d];
        if (side == 0) g[v][d] += pr;
        else g[v][d] -= pr;
      }
    }
  }
  for (int b = bv_ptr[i]; b < bv_ptr[i + 1]; ++b)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int d = 0; d < NDIM; ++d) g[v][d] -= U[2 * (size_t)i + v] * bv_normal[(size_t)b * NDIM + d];
  const double da = vol[i] + rx::kEPS;
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int d = 0; d < NDIM; ++d) grad[((size_t)i * 2 + v) * NDIM + d] = g[v][d] / da;
}

// SetStrainMag from the flow primitive gradient (rows 1..NDIM = velocity); pow(x, 2.0) -> x * x.
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_strain(int N, int nG, const double* __restrict__ G,
                                                   double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const double* g = G + (size_t)i * nG * NDIM;
  double Div = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) Div += g[(d + 1) * NDIM + d];
  double S = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) {
    const double x = g[(d + 1) * NDIM + d] - 1.0 / 3.0 * Div;
    S += x * x;
  }
  {
    const double x = 0.5 * (g[1 * NDIM + 1] + g[2 * NDIM + 0]);
    S += 2.0 * (x * x);
  }
  if constexpr (NDIM == 3) {
    const double x = 0.5 * (g[1 * NDIM + NDIM - 1] + g[3 * NDIM + 0]);
    S += 2.0 * (x * x);
    const double y = 0.5 * (g[2 * NDIM + NDIM - 1] + g[3 * NDIM + 1]);
    S += 2.0 * (y * y);
  }
  out[i] = sqrt(2.0 * S);
}

// A node's incident edges in increasing edge id (the reference's scatter order): the adjacency entries, edge ends
// and off-diagonal block indices of the first kSstPF edges are loaded together first, so the edges' data loads do
// not wait on one another's index chain (one thread per node walked adj -> edges -> data serially, edge after edge:
// 0.31 / 0.33 ms at C3 for the upwind / viscous loops); degrees above kSstPF continue in the loop. f(e, side, n0, n1,
// block) is called in edge order.
template <int NDIM>
constexpr int sst_pf() { return 2 * NDIM; }
// Round 6: the node loops' workgroups in XCD order (as rx_kernels.hip's xcd_block): the hardware deals consecutive
// workgroups round-robin to the 8 XCDs, so a node's neighbours in the previous / next grid line were gathered by
// other XCDs, each filling its own L2 with the same record lines; remapped, XCD x walks one contiguous node range.
#ifndef RX_SST_XCD
#define RX_SST_XCD 1
#endif
__device__ inline int sst_node_block(int b, int nb) {
  if (!RX_SST_XCD) return b;
  constexpr int kXcd = 8;
  const int x = b % kXcd, idx = b / kXcd, q = nb / kXcd, r = nb % kXcd;
  return x < r ? x * (q + 1) + idx : r * (q + 1) + (x - r) * q + idx;
}
template <int NDIM, typename Fn>
__device__ __forceinline__ void sst_edges(int i, const int32_t* __restrict__ adj_ptr, const int32_t* __restrict__ adj,
                                          const int64_t* __restrict__ adj_blk, const int32_t* __restrict__ edges,
                                          Fn f) {
  constexpr int PF = sst_pf<NDIM>();
  const int k0 = adj_ptr[i], k1 = adj_ptr[i + 1];
  int ae[PF], n0[PF], n1[PF];
  int64_t ob[PF];
#pragma unroll
  for (int t = 0; t < PF; ++t) {
    const int k = k0 + t < k1 ? k0 + t : k0;
    ae[t] = adj[k];
    ob[t] = adj_blk[k];
  }
#pragma unroll
  for (int t = 0; t < PF; ++t) {
    const int e = ae[t] >> 1;
    n0[t] = edges[2 * e];
    n1[t] = edges[2 * e + 1];
  }
#pragma unroll
  for (int t = 0; t < PF; ++t)
    if (k0 + t < k1) f(ae[t] >> 1, ae[t] & 1, n0[t], n1[t], ob[t]);
  for (int k = k0 + PF; k < k1; ++k) {
    const int a = adj[k];
    const int e = a >> 1;
    f(e, a & 1, edges[2 * e], edges[2 * e + 1], adj_blk[k]);
  }
}

// Residual loops: each node updates its residual, its diagonal block and the off-diagonal block of
// (i, other) per incident edge. Blocks are 2x2 row-major; the reference adds/subtracts whole blocks,
// zeros included (CSysMatrix::AddBlock / SubtractBlock, matrix_structure.cpp:327-357).
// CTurbSolver::Upwind_Residual (solver_direct_turbulent.cpp:429-543) + CUpwSca_TurbSST (:865-922):
// R_i += F, R_j -= F; A_ii += Ji, A_ij += Jj, A_ji -= Ji, A_jj -= Jj.
// Second-order inputs of the SST upwind (SPATIAL_ORDER_TURB, CTurbSolver::Upwind_Residual :464-510): the coordinates,
// the flow's primitive gradient (rows T, u, v(, w), P, X_s) and limiter (T, u, v(, w), P), the SST gradient and
// limiter of (k, omega).
struct SstRecon {
  const double *coord, *G, *Lf, *TG, *TL;
  int nG;
};
// ORDER 0: first order; 1: 2ND_ORDER, 2: 2ND_ORDER_LIMITER. The flow record entry iVar is reconstructed with the
// gradient ROW iVar (:481-493): the velocity entries with their own rows, the density entry V[nDim+2] with the row of
// X_0 (reproduced); with the limiter the flow's Limiter_Primitive is read at iVar = nDim+2, one past its nDim+2
// entries — undefined in the reference — restated as 0.0 (the oracle's orc_sst_upwind2, pinned by the goldens fpit2 /
// fpit2l / it4t).
template <int NDIM, int ORDER>
__global__ __launch_bounds__(kBlock) void k_sst_upwind(int N, const int32_t* __restrict__ adj_ptr,
                                                       const int32_t* __restrict__ adj,
                                                       const int64_t* __restrict__ adj_blk,
                                                       const int64_t* __restrict__ diag,
                                                       const int32_t* __restrict__ edges,
                                                       const double* __restrict__ normal,
                                                       const double* __restrict__ V, int nPV,
                                                       const double* __restrict__ T, double* __restrict__ R,
                                                       double* __restrict__ A, SstRecon rc) {
  const int i = sst_node_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (i >= N) return;
  constexpr int RHO = NDIM + 2, nL = NDIM + 2;
  double r0 = R[2 * (size_t)i], r1 = R[2 * (size_t)i + 1];
  double* Dp = A ? A + diag[i] * 4 : nullptr;
  double D[4] = {0, 0, 0, 0};
  if (Dp)
#pragma unroll
    for (int q = 0; q < 4; ++q) D[q] = Dp[q];
  // first order (round 6): the node's own velocity, density and (k, omega) read once; per edge only the other end's
  // record is gathered (the same values as the two-sided gather, so the same arithmetic)
  double uo[NDIM], rhoo = 0.0, ko = 0.0, wo = 0.0;
  if (ORDER == 0) {
#pragma unroll
    for (int d = 0; d < NDIM; ++d) uo[d] = V[(size_t)i * nPV + d + 1];
    rhoo = V[(size_t)i * nPV + RHO];
    ko = T[2 * (size_t)i];
    wo = T[2 * (size_t)i + 1];
  }
  auto edge = [&](int e, int side, int n0, int n1, int64_t ob) {
    const double* v0 = V + (size_t)n0 * nPV;
    const double* v1 = V + (size_t)n1 * nPV;
    double u0[NDIM], u1[NDIM], rho0, rho1, k0, w0, k1, w1;
    if (ORDER == 0) {
      const int other = side ? n0 : n1;
      const double* vx = V + (size_t)other * nPV;
      double ux[NDIM];
#pragma unroll
      for (int d = 0; d < NDIM; ++d) ux[d] = vx[d + 1];
      const double rhox = vx[RHO], kx = T[2 * (size_t)other], wx = T[2 * (size_t)other + 1];
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        u0[d] = side ? ux[d] : uo[d];
        u1[d] = side ? uo[d] : ux[d];
      }
      rho0 = side ? rhox : rhoo;
      rho1 = side ? rhoo : rhox;
      k0 = side ? kx : ko;
      w0 = side ? wx : wo;
      k1 = side ? ko : kx;
      w1 = side ? wo : wx;
    } else {
      double vec0[NDIM], vec1[NDIM];
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        const double c0 = rc.coord[(size_t)n0 * NDIM + d], c1 = rc.coord[(size_t)n1 * NDIM + d];
        vec0[d] = 0.5 * (c1 - c0);
        vec1[d] = 0.5 * (c0 - c1);
      }
      auto flow = [&](int p, const double* vp, const double* vec, int v) {
        const double* g = rc.G + ((size_t)p * rc.nG + v) * NDIM;
        double pg = 0.0;
#pragma unroll
        for (int d = 0; d < NDIM; ++d) pg += vec[d] * g[d];
        if (ORDER == 1) return vp[v] + pg;
        const double l = v < nL ? rc.Lf[(size_t)p * nL + v] : 0.0;
        return vp[v] + l * pg;
      };
      auto turb = [&](int p, const double* vec, int v) {
        const double* g = rc.TG + ((size_t)p * 2 + v) * NDIM;
        double pg = 0.0;
#pragma unroll
        for (int d = 0; d < NDIM; ++d) pg += vec[d] * g[d];
        return ORDER == 2 ? T[2 * (size_t)p + v] + rc.TL[2 * (size_t)p + v] * pg : T[2 * (size_t)p + v] + pg;
      };
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        u0[d] = flow(n0, v0, vec0, d + 1);
        u1[d] = flow(n1, v1, vec1, d + 1);
      }
      rho0 = flow(n0, v0, vec0, RHO);
      rho1 = flow(n1, v1, vec1, RHO);
      k0 = turb(n0, vec0, 0);
      w0 = turb(n0, vec0, 1);
      k1 = turb(n1, vec1, 0);
      w1 = turb(n1, vec1, 1);
    }
    double q = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) q += 0.5 * (u0[d] + u1[d]) * normal[(size_t)e * NDIM + d];
    const double a0 = 0.5 * (q + fabs(q)), a1 = 0.5 * (q - fabs(q));
    const double f0 = a0 * rho0 * k0 + a1 * rho1 * k1;
    const double f1 = a0 * rho0 * w0 + a1 * rho1 * w1;
    // Ji = diag(a0), Jj = diag(a1) with explicit zeros
    const double Ji[4] = {a0, 0.0, 0.0, a0}, Jj[4] = {a1, 0.0, 0.0, a1};
    if (side == 0) {
      r0 += f0;
      r1 += f1;
      if (Dp) {
        double* O = A + ob * 4;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          D[t] += Ji[t];
          O[t] += Jj[t];
        }
      }
    } else {
      r0 -= f0;
      r1 -= f1;
      if (Dp) {
        double* O = A + ob * 4;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          O[t] -= Ji[t];
          D[t] -= Jj[t];
        }
      }
    }
  };
  sst_edges<NDIM>(i, adj_ptr, adj, adj_blk, edges, edge);
  R[2 * (size_t)i] = r0;
  R[2 * (size_t)i + 1] = r1;
  if (Dp)
#pragma unroll
    for (int q = 0; q < 4; ++q) Dp[q] = D[q];
}

// CSolver::SetSolution_Limiter (solver_structure.cpp:951-1204) on (k, omega), SLOPE_LIMITER_TURB = VENKATAKRISHNAN
// (venkat = 1) or BARTH_JESPERSEN (0: the function has no branch for it, the limiter stays 2.0), node-centric: a
// domain point's Solution_Min / _Max over its incident edges (du = U_j - U_i at node i of the edge, -du at node j;
// order-free), then the edge minimum of the Venkatakrishnan function with its own dm. Halo rows: the exchange.
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_sst_limiter(int Nd, const int32_t* __restrict__ adj_ptr,
                                                        const int32_t* __restrict__ adj,
                                                        const int32_t* __restrict__ edges,
                                                        const double* __restrict__ coord, const double* __restrict__ T,
                                                        const double* __restrict__ TG, double eps2, int venkat,
                                                        double* __restrict__ L) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Nd) return;
  double lo[2] = {rx::kEPS, rx::kEPS}, hi[2] = {-rx::kEPS, -rx::kEPS};
  const int k0 = adj_ptr[i], k1 = adj_ptr[i + 1];
  for (int k = k0; k < k1; ++k) {
    const int a = adj[k];
    const int e = a >> 1, side = a & 1;
    const int n0 = edges[2 * e], n1 = edges[2 * e + 1];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const double du = T[2 * (size_t)n1 + v] - T[2 * (size_t)n0 + v];
      const double d = side ? -du : du;
      lo[v] = fmin(lo[v], d);
      hi[v] = fmax(hi[v], d);
    }
  }
  double l[2] = {2.0, 2.0};
  if (venkat) {
    double ci[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) ci[d] = coord[(size_t)i * NDIM + d];
    const double* Gi = TG + (size_t)i * 2 * NDIM;
    for (int k = k0; k < k1; ++k) {
      const int a = adj[k];
      const int e = a >> 1, side = a & 1;
      const int other = edges[2 * e + (side ^ 1)];
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        double dm = 0.0;
#pragma unroll
        for (int d = 0; d < NDIM; ++d) dm += 0.5 * (coord[(size_t)other * NDIM + d] - ci[d]) * Gi[v * NDIM + d];
        const double dp = (dm > 0.0) ? hi[v] : lo[v];
        const double lv = (dp * dp + 2.0 * dp * dm + eps2) / (dp * dp + dp * dm + 2.0 * dm * dm + eps2);
        if (lv < l[v]) l[v] = lv;
      }
    }
  }
  L[2 * (size_t)i] = l[0];
  L[2 * (size_t)i + 1] = l[1];
}

// CTurbSolver::Viscous_Residual (:545-600) + CAvgGradCorrected_TurbSST (:1080-1163):
// R_i -= F, R_j += F; A_ii -= Ji, A_ij -= Jj, A_ji += Ji, A_jj += Jj.
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_sst_visc(int N, SSTC c, const int32_t* __restrict__ adj_ptr,
                                                     const int32_t* __restrict__ adj,
                                                     const int64_t* __restrict__ adj_blk,
                                                     const int64_t* __restrict__ diag,
                                                     const int32_t* __restrict__ edges,
                                                     const double* __restrict__ normal,
                                                     const double* __restrict__ coord, const double* __restrict__ V,
                                                     int nPV, const double* __restrict__ mu,
                                                     const double* __restrict__ eddy, const double* __restrict__ T,
                                                     const double* __restrict__ TG, const double* __restrict__ F1,
                                                     double* __restrict__ R, double* __restrict__ A) {
  const int i = sst_node_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (i >= N) return;
  constexpr int RHO = NDIM + 2;
  double r0 = R[2 * (size_t)i], r1 = R[2 * (size_t)i + 1];
  double* Dp = A ? A + diag[i] * 4 : nullptr;
  double D[4] = {0, 0, 0, 0};
  if (Dp)
#pragma unroll
    for (int q = 0; q < 4; ++q) D[q] = Dp[q];
  // round 6: the node's own F1, mu, eddy viscosity, coordinates, (k, omega), their gradient and density read once; per
  // edge only the other end's are gathered and each operand is selected into its n0 / n1 place (the same values in
  // the same expressions as the two-sided gather)
  double TGo[2 * NDIM], cdo[NDIM];
  const double F1o = F1[i], muo = mu[i], eto = eddy[i], To0 = T[2 * (size_t)i], To1 = T[2 * (size_t)i + 1];
  const double rhoo = Dp ? V[(size_t)i * nPV + RHO] : 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) cdo[d] = coord[(size_t)i * NDIM + d];
#pragma unroll
  for (int q = 0; q < 2 * NDIM; ++q) TGo[q] = TG[(size_t)i * 2 * NDIM + q];
  auto edge = [&](int e, int side, int n0, int n1, int64_t ob) {
    const int x = side ? n0 : n1;  // the other end
    auto pick0 = [&](double own, double oth) { return side ? oth : own; };  // the n0 operand
    auto pick1 = [&](double own, double oth) { return side ? own : oth; };  // the n1 operand
    const double F1x = F1[x], mux = mu[x], etx = eddy[x];
    const double F1i = pick0(F1o, F1x), F1j = pick1(F1o, F1x);
    const double ski = F1i * c.sk1 + (1.0 - F1i) * c.sk2;
    const double skj = F1j * c.sk1 + (1.0 - F1j) * c.sk2;
    const double soi = F1i * c.so1 + (1.0 - F1i) * c.so2;
    const double soj = F1j * c.so1 + (1.0 - F1j) * c.so2;
    const double mui = pick0(muo, mux), muj = pick1(muo, mux), eti = pick0(eto, etx), etj = pick1(eto, etx);
    const double dik = mui + ski * eti, djk = muj + skj * etj;
    const double dio = mui + soi * eti, djo = muj + soj * etj;
    const double dk = 0.5 * (dik + djk), dw = 0.5 * (dio + djo);
    double ev[NDIM], nrm[NDIM], dist2 = 0.0, proj = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
      const double cx = coord[(size_t)x * NDIM + d];
      nrm[d] = normal[(size_t)e * NDIM + d];
      ev[d] = pick1(cdo[d], cx) - pick0(cdo[d], cx);
      dist2 += ev[d] * ev[d];
      proj += ev[d] * nrm[d];
    }
    if (dist2 == 0.0) proj = 0.0; else proj = proj / dist2;
    const double Tx[2] = {T[2 * (size_t)x], T[2 * (size_t)x + 1]}, To[2] = {To0, To1};
    double corr[2];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      double pn = 0.0, pe = 0.0;
#pragma unroll
      for (int d = 0; d < NDIM; ++d) {
        const double gx = TG[((size_t)x * 2 + v) * NDIM + d], go = TGo[v * NDIM + d];
        const double m = 0.5 * (pick0(go, gx) + pick1(go, gx));
        pn += m * nrm[d];
        pe += m * ev[d];
      }
      corr[v] = pn;
      corr[v] -= pe * proj - (pick1(To[v], Tx[v]) - pick0(To[v], Tx[v])) * proj;
    }
    const double f0 = dk * corr[0], f1 = dw * corr[1];
    if (side == 0) {
      r0 -= f0;
      r1 -= f1;
    } else {
      r0 += f0;
      r1 += f1;
    }
    if (Dp) {
      const double rx = V[(size_t)(side ? n0 : n1) * nPV + RHO];
      const double ri = side ? rx : rhoo, rj = side ? rhoo : rx;
      const double Ji[4] = {-dk * proj / ri, 0.0, 0.0, -dw * proj / ri};
      const double Jj[4] = {dk * proj / rj, 0.0, 0.0, dw * proj / rj};
      double* O = A + ob * 4;
      if (side == 0) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          D[t] -= Ji[t];
          O[t] -= Jj[t];
        }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          O[t] += Ji[t];
          D[t] += Jj[t];
        }
      }
    }
  };
  sst_edges<NDIM>(i, adj_ptr, adj, adj_blk, edges, edge);
  R[2 * (size_t)i] = r0;
  R[2 * (size_t)i + 1] = r1;
  if (Dp)
#pragma unroll
    for (int q = 0; q < 4; ++q) Dp[q] = D[q];
}

// CTurbSSTSolver::Source_Residual (:3018-3080) + CSourcePieceWise_TurbSST (:1183-1256) over the owned
// points: R_i -= S, A_ii -= Js.
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_sst_source(int Nd, SSTC c, const int64_t* __restrict__ diag,
                                                       const double* __restrict__ V, int nPV,
                                                       const double* __restrict__ G, int nG,
                                                       const double* __restrict__ eddy,
                                                       const double* __restrict__ strain,
                                                       const double* __restrict__ T, const double* __restrict__ vol,
                                                       const double* __restrict__ dist,
                                                       const double* __restrict__ F1, const double* __restrict__ F2,
                                                       const double* __restrict__ CDkw, double* __restrict__ R,
                                                       double* __restrict__ A) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Nd) return;
  const double rho = V[(size_t)i * nPV + NDIM + 2];
  const double k = T[2 * (size_t)i], w = T[2 * (size_t)i + 1], S = strain[i], Vol = vol[i], f1 = F1[i];
  const double ab = f1 * c.al1 + (1.0 - f1) * c.al2;
  const double bb = f1 * c.b1 + (1.0 - f1) * c.b2;
  double s0 = 0.0, s1 = 0.0, j00 = 0.0, j11 = 0.0;
  if (dist[i] > 1e-10) {
    double diverg = 0.0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) diverg += G[((size_t)i * nG + d + 1) * NDIM + d];
    double pk = eddy[i] * S * S - 2.0 / 3.0 * rho * k * diverg;
    pk = smin(pk, 20.0 * c.bs * rho * w * k);
    pk = smax(pk, 0.0);
    const double zeta = smax(w, S * F2[i] / c.a1);
    double pw = S * S - 2.0 / 3.0 * zeta * diverg;
    pw = smax(pw, 0.0);
    s0 += pk * Vol;
    s1 += ab * rho * pw * Vol;
    s0 -= c.bs * rho * w * k * Vol;
    s1 -= bb * rho * w * w * Vol;
    s1 += (1.0 - f1) * CDkw[i] * Vol;
    j00 = -c.bs * w * Vol;
    j11 = -2.0 * bb * w * Vol;
  }
  R[2 * (size_t)i] -= s0;
  R[2 * (size_t)i + 1] -= s1;
  if (A) {
    double* D = A + diag[i] * 4;
    D[0] -= j00;
    D[1] -= 0.0;
    D[2] -= 0.0;
    D[3] -= j11;
  }
}

// CTurbSolver::ImplicitEuler_Iteration system build (:630-668): owned rows A_ii += Vol/(CFLRed*dt_flow),
// rhs = -R, x = 0; ghost rows rhs = x = 0.
__global__ __launch_bounds__(kBlock) void k_sst_build_system(int Nd, int N, const int64_t* __restrict__ diag,
                                                             const double* __restrict__ vol,
                                                             const double* __restrict__ dt, double cfl_red,
                                                             double* __restrict__ A, const double* __restrict__ R,
                                                             double* __restrict__ rhs, double* __restrict__ x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if (i >= Nd) {
    rhs[2 * (size_t)i] = rhs[2 * (size_t)i + 1] = 0.0;
    x[2 * (size_t)i] = x[2 * (size_t)i + 1] = 0.0;
    return;
  }
  const double delta = vol[i] / (cfl_red * dt[i]);
  double* D = A + diag[i] * 4;
  D[0] += delta;
  D[3] += delta;
  rhs[2 * (size_t)i] = -R[2 * (size_t)i];
  rhs[2 * (size_t)i + 1] = -R[2 * (size_t)i + 1];
  x[2 * (size_t)i] = x[2 * (size_t)i + 1] = 0.0;
}

// SST branch of the update (:698-713): AddConservativeSolution (variable_structure.cpp:214-219) with
// density = the flow primitive density and density_old = the flow's Solution_Old(0) (the U before the flow
// update, kept by its update kernel). Limits: constructor :2731-2735.
__global__ __launch_bounds__(kBlock) void k_sst_update(int Nd, const double* __restrict__ x, double relax,
                                                       const double* __restrict__ V, int nPV, int rho_idx,
                                                       const double* __restrict__ Uold, int nVarF,
                                                       double* __restrict__ T) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * Nd) return;
  const int i = t >> 1, v = t & 1;
  const double rho = V[(size_t)i * nPV + rho_idx];
  const double rho_old = Uold[(size_t)i * nVarF];
  const double lo = v ? 1.0e-4 : 1.0e-10, hi = v ? 1.0e15 : 1.0e10;
  T[t] = smin(smax((T[t] * rho_old + relax * x[t]) / rho, lo), hi);
}

// CTurbSSTSolver::Postprocessing after its gradient (:2966-3000): SetBlendingFunc, mu_t, over every
// point; then the MANGOTURB coupling the flow reads (turb node k, omega, mu_t, grad k, sigma_k, and the
// flow eddy viscosity SetPrimVar copies from mu_t, variable_direct_reactive.cpp:1188-1193).
template <int NDIM>
__global__ __launch_bounds__(kBlock) void k_sst_post(int N, SSTC c, const double* __restrict__ T,
                                                     const double* __restrict__ TG, const double* __restrict__ V,
                                                     int nPV, const double* __restrict__ mu,
                                                     const double* __restrict__ dist,
                                                     const double* __restrict__ strain, double* __restrict__ F1,
                                                     double* __restrict__ F2, double* __restrict__ CDkw,
                                                     double* __restrict__ muT, double* __restrict__ fl_tke,
                                                     double* __restrict__ fl_omega, double* __restrict__ fl_mut,
                                                     double* __restrict__ fl_eddy, double* __restrict__ fl_sigmak,
                                                     double* __restrict__ fl_gradk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const double k = T[2 * (size_t)i], w = T[2 * (size_t)i + 1];
  const double rho = V[(size_t)i * nPV + NDIM + 2], m = mu[i], ds = dist[i];
  const double* g = TG + (size_t)i * 2 * NDIM;
  double cd = 0.0;
#pragma unroll
  for (int d = 0; d < NDIM; ++d) cd += g[d] * g[NDIM + d];
  cd *= 2.0 * rho * c.so2 / w;
  cd = smax(cd, 1.0e-20);  // pow(10.0, -20.0): glibc's correctly rounded result is the literal
  const double eps2 = rx::kEPS * rx::kEPS;
  const double arg2A = sqrt(k) / (c.bs * w * ds + eps2);
  const double arg2B = 500.0 * m / (rho * ds * ds * w + eps2);
  double arg2 = smax(arg2A, arg2B);
  const double arg1 = smin(arg2, 4.0 * rho * c.so2 * k / (cd * ds * ds + eps2));
  const double f1 = tanh(pow(arg1, 4.0));
  arg2 = smax(2.0 * arg2A, arg2B);
  const double f2 = tanh(pow(arg2, 2.0));
  const double zeta = smin(1.0 / w, c.a1 / (strain[i] * f2));
  const double mt = smin(smax(rho * k * zeta, 0.0), 1.0);
  F1[i] = f1;
  F2[i] = f2;
  CDkw[i] = cd;
  muT[i] = mt;
  fl_tke[i] = k;
  fl_omega[i] = w;
  fl_mut[i] = mt;
  fl_eddy[i] = mt;
  fl_sigmak[i] = c.sk1;  // CTurbSSTVariable::Get_Sigmak = constants[0] (variable_direct_turbulent.cpp:151)
#pragma unroll
  for (int d = 0; d < NDIM; ++d) fl_gradk[(size_t)i * NDIM + d] = g[d];
}

bool is_sst(const rx_ctx* ctx) { return ctx && ctx->kind == RX_KIND_SST && ctx->flow; }

int sst_gradient(rx_ctx* ctx) {
  if (ctx->Nd > 0 && ctx->cfg.grad_method == RX_GRAD_GREEN_GAUSS) {
    RX_ND_SWITCH(ctx->nDim, (k_sol_grad_gg<ND_><<<blocks(ctx->Nd), kBlock, 0, ctx->stream>>>(
                                 (int)ctx->Nd, ctx->adj_ptr, ctx->adj, ctx->edges, ctx->normal, ctx->bv_ptr,
                                 ctx->bv_normal, ctx->vol, ctx->f[RX_F_U], ctx->f[RX_F_GRAD])));
  } else if (ctx->Nd > 0) {
    RX_ND_SWITCH(ctx->nDim, (k_sol_grad_ls<ND_><<<blocks(ctx->Nd), kBlock, 0, ctx->stream>>>((int)ctx->Nd, ctx->coord, ctx->nbr_ptr, ctx->nbr,
                                                                   ctx->f[RX_F_U], ctx->f[RX_F_GRAD])));
  }
  RX_HIP(hipGetLastError());
  return rx_la_exchange(ctx, ctx->f[RX_F_GRAD], 2 * ctx->nDim);  // Set_MPI_Solution_Gradient
}

}  // namespace

int rx_sst_build_system(rx_ctx* ctx) {
  k_sst_build_system<<<blocks(ctx->N), kBlock, 0, ctx->stream>>>((int)ctx->Nd, (int)ctx->N, ctx->diag, ctx->vol,
                                                                 ctx->flow->f[RX_F_DT], ctx->cfg.cfl,
                                                                 ctx->f[RX_F_JAC], ctx->f[RX_F_RES], ctx->f[RX_F_RHS],
                                                                 ctx->f[RX_F_SOL]);
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_sst_update(rx_ctx* ctx) {
  const rx_ctx* fl = ctx->flow;
  if (ctx->Nd > 0)
    k_sst_update<<<blocks(2 * ctx->Nd), kBlock, 0, ctx->stream>>>((int)ctx->Nd, ctx->f[RX_F_SOL], ctx->cfg.relaxation,
                                                                  fl->f[RX_F_V], fl->nPV, fl->nDim + 2, fl->uold,
                                                                  fl->nVar, ctx->f[RX_F_U]);
  RX_HIP(hipGetLastError());
  return rx_la_exchange(ctx, ctx->f[RX_F_U], 2);  // Set_MPI_Solution (:718)
}

extern "C" {

int rx_strain_mag(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_STRAIN);
  RX_ND_SWITCH(ctx->nDim, (k_strain<ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>((int)ctx->N, ctx->nG, ctx->f[RX_F_GRAD],
                                                          ctx->f[RX_F_STRAIN])));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// CTurbSSTSolver::Preprocessing (solver_direct_turbulent.cpp:2923-2951): residual and Jacobian zero, the gradient of
// (k, omega), SetSolution_Limiter when SPATIAL_ORDER_TURB = 2ND_ORDER_LIMITER (this context's cfg.spatial_order = 2),
// and the flow's SetPrimitive_Limiter again when SPATIAL_ORDER_FLOW = 2ND_ORDER_LIMITER (ExtIter <= LIMITER_ITER, whose
// default 999999 is taken): the flow limiter the SST upwind then reads is that of the post-update records.
int rx_sst_preprocessing(rx_ctx* ctx) {
  if (!is_sst(ctx)) return RX_ERR_ARG;
  {
    RxPhase ph(ctx, RX_K_SST_GRAD);
    RX_HIP(hipMemsetAsync(ctx->f[RX_F_RES], 0, sizeof(double) * ctx->fcount[RX_F_RES], ctx->stream));
    if (ctx->cfg.implicit)
      RX_HIP(hipMemsetAsync(ctx->f[RX_F_JAC], 0, sizeof(double) * ctx->fcount[RX_F_JAC], ctx->stream));
    ctx->assembled = 1;
    const int rc = sst_gradient(ctx);
    if (rc) return rc;
    if (ctx->cfg.spatial_order == 2 && ctx->Nd > 0) {
      const double eps1 = ctx->cfg.limiter_coeff * ctx->cfg.ref_elem_length;
      const double eps2 = eps1 * eps1 * eps1;
      RX_ND_SWITCH(ctx->nDim, (k_sst_limiter<ND_><<<blocks(ctx->Nd), kBlock, 0, ctx->stream>>>(
                                   (int)ctx->Nd, ctx->adj_ptr, ctx->adj, ctx->edges, ctx->coord, ctx->f[RX_F_U],
                                   ctx->f[RX_F_GRAD], eps2,
                                   ctx->cfg.slope_limiter == RX_LIMITER_VENKATAKRISHNAN ? 1 : 0,
                                   ctx->f[RX_F_LIMITER])));
      RX_HIP(hipGetLastError());
      const int rc2 = rx_la_exchange(ctx, ctx->f[RX_F_LIMITER], 2);  // Set_MPI_Solution_Limiter (:1202)
      if (rc2) return rc2;
    }
  }
  if (ctx->flow->cfg.spatial_order == 2) return rx_limiter_venkat(ctx->flow);
  return RX_OK;
}

int rx_sst_upwind(rx_ctx* ctx) {
  if (!is_sst(ctx)) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_SST_UPW);
  const rx_ctx* fl = ctx->flow;
  // SPATIAL_ORDER_TURB: 0 1ST_ORDER, 1 2ND_ORDER, 2 2ND_ORDER_LIMITER (the SST context's cfg.spatial_order)
  const SstRecon rc{ctx->coord, fl->f[RX_F_GRAD], fl->f[RX_F_LIMITER], ctx->f[RX_F_GRAD], ctx->f[RX_F_LIMITER], fl->nG};
  switch (ctx->cfg.spatial_order) {
#define RX_SST_UPW(ORD)                                                                                           \
  RX_ND_SWITCH(ctx->nDim, (k_sst_upwind<ND_, ORD><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>(                      \
      (int)ctx->N, ctx->adj_ptr, ctx->adj, ctx->adj_blk, ctx->diag, ctx->edges, ctx->normal, fl->f[RX_F_V], fl->nPV, \
      ctx->f[RX_F_U], ctx->f[RX_F_RES], ctx->cfg.implicit ? ctx->f[RX_F_JAC] : nullptr, rc)))
    case 0: RX_SST_UPW(0); break;
    case 1: RX_SST_UPW(1); break;
    case 2: RX_SST_UPW(2); break;
    default: return RX_ERR_ARG;
#undef RX_SST_UPW
  }
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_sst_viscous(rx_ctx* ctx) {
  if (!is_sst(ctx)) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_SST_VISC);
  const rx_ctx* fl = ctx->flow;
  RX_ND_SWITCH(ctx->nDim, (k_sst_visc<ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>(
      (int)ctx->N, sst_constants(), ctx->adj_ptr, ctx->adj, ctx->adj_blk, ctx->diag, ctx->edges, ctx->normal,
      ctx->coord, fl->f[RX_F_V], fl->nPV, fl->f[RX_F_MU], fl->f[RX_F_EDDY], ctx->f[RX_F_U], ctx->f[RX_F_GRAD],
      ctx->f[RX_F_F1], ctx->f[RX_F_RES], ctx->cfg.implicit ? ctx->f[RX_F_JAC] : nullptr)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_sst_source(rx_ctx* ctx) {
  if (!is_sst(ctx)) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_SST_SOURCE);
  const rx_ctx* fl = ctx->flow;
  if (ctx->Nd > 0) {
    RX_ND_SWITCH(ctx->nDim, (k_sst_source<ND_><<<blocks(ctx->Nd), kBlock, 0, ctx->stream>>>(
        (int)ctx->Nd, sst_constants(), ctx->diag, fl->f[RX_F_V], fl->nPV, fl->f[RX_F_GRAD], fl->nG, fl->f[RX_F_EDDY],
        fl->f[RX_F_STRAIN], ctx->f[RX_F_U], ctx->vol, ctx->f[RX_F_WALLDIST], ctx->f[RX_F_F1], ctx->f[RX_F_F2],
        ctx->f[RX_F_CDKW], ctx->f[RX_F_RES], ctx->cfg.implicit ? ctx->f[RX_F_JAC] : nullptr)));
  }
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_sst_postprocessing(rx_ctx* ctx) {
  if (!is_sst(ctx)) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_SST_POST);
  int rc = sst_gradient(ctx);
  if (rc) return rc;
  rx_ctx* fl = ctx->flow;
  RX_ND_SWITCH(ctx->nDim, (k_sst_post<ND_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>(
      (int)ctx->N, sst_constants(), ctx->f[RX_F_U], ctx->f[RX_F_GRAD], fl->f[RX_F_V], fl->nPV, fl->f[RX_F_MU],
      ctx->f[RX_F_WALLDIST], fl->f[RX_F_STRAIN], ctx->f[RX_F_F1], ctx->f[RX_F_F2], ctx->f[RX_F_CDKW],
      ctx->f[RX_F_MUT], fl->f[RX_F_TKE], fl->f[RX_F_OMEGA], fl->f[RX_F_MUT], fl->f[RX_F_EDDY], fl->f[RX_F_SIGMAK],
      fl->f[RX_F_GRADK])));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

}  // extern "C"
