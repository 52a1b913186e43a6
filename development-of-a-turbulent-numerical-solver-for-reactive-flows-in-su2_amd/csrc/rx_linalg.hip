// rx_linalg.hip — block-sparse (BSR) linear algebra of the implicit path on gfx950.
//
// Reference semantics (Common/src/matrix_structure.cpp, linear_solvers_structure.cpp):
//   MatrixVectorProduct :997-1030, Gauss_Elimination :594-643, InverseDiagonalBlock_ILUMatrix
//   :1180-1228, BuildILUPreconditioner :1368-1451 (left-multiply quirk :1432-1436),
//   ComputeILUPreconditioner :1453-1515, ComputeLU_SGSPreconditioner :1673-1709,
//   FGMRES_LinSolver / ModGramSchmidt / Givens / SolveReduced :37-186, 309-463,
//   ImplicitEuler_Iteration SU2_CFD/src/solver_direct_reactive.cpp:2336-2407.
// Triangular sweeps: rx_sweeps.hip; FGMRES: rx_krylov.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "rx_ctx.h"

namespace {

constexpr int kBlock = 256;
inline int blocks(int64_t n, int b = kBlock) { return (int)((n + b - 1) / b); }

// y = A x, one thread per (row, component a): reference order over blocks then columns.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_spmv(int N, const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                 const double* __restrict__ A, const double* __restrict__ x,
                                                 double* __restrict__ y, const int* __restrict__ skip) {
  if (skip && *skip) return;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * NV) return;
  const int i = t / NV, a = t - i * NV;
  double acc = 0.0;
  for (int k = rp[i]; k < rp[i + 1]; ++k) {
    const double* blk = A + (size_t)k * NV * NV + a * NV;
    const double* xv = x + (size_t)col[k] * NV;
#pragma unroll
    for (int c = 0; c < NV; ++c) acc += blk[c] * xv[c];
  }
  y[t] = acc;
}

// ImplicitEuler system build over the owned rows: Aii += V/dt (or identity row when dt <= EPS),
// rhs = -R, x = 0; halo rows get rhs = x = 0 (solver_direct_reactive.cpp:2336-2387).
template <int NV>
__global__ __launch_bounds__(kBlock) void k_build_system(int Nd, int N, const int64_t* __restrict__ diag,
                                                         const double* __restrict__ vol, const double* __restrict__ dt,
                                                         double* __restrict__ A, double* __restrict__ R,
                                                         double* __restrict__ rhs, double* __restrict__ x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if (i >= Nd) {
#pragma unroll
    for (int a = 0; a < NV; ++a) {
      rhs[(size_t)i * NV + a] = 0.0;
      x[(size_t)i * NV + a] = 0.0;
    }
    return;
  }
  double* D = A + diag[i] * NV * NV;
  const bool ok = dt[i] > rx::kEPS;
  if (ok) {
    const double delta = vol[i] / dt[i];
#pragma unroll
    for (int a = 0; a < NV; ++a) D[a * NV + a] += delta;
  } else {
#pragma unroll
    for (int a = 0; a < NV; ++a)
#pragma unroll
      for (int c = 0; c < NV; ++c) D[a * NV + c] = (a == c) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int a = 0; a < NV; ++a) {
    if (!ok) R[(size_t)i * NV + a] = 0.0;
    rhs[(size_t)i * NV + a] = -(R[(size_t)i * NV + a] + 0.0);
    x[(size_t)i * NV + a] = 0.0;
  }
}

// The same system build with one thread per (node, variable): coalesced R / rhs / x rows and NV times the
// threads in flight for the scattered diagonal read-modify-writes. Identical operations per element.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_build_system_elem(int Nd, int N, const int64_t* __restrict__ diag,
                                                              const double* __restrict__ vol,
                                                              const double* __restrict__ dt, double* __restrict__ A,
                                                              double* __restrict__ R, double* __restrict__ rhs,
                                                              double* __restrict__ x,
                                                              const int32_t* __restrict__ skip) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)N * NV) return;
  const int i = (int)(q / NV), a = (int)(q - (int64_t)i * NV);
  x[q] = 0.0;
  if (i >= Nd) {
    rhs[q] = 0.0;
    return;
  }
  // skip != nullptr: the assembly folded the diagonal of the rows with skip[i] == 0 (k_asm_visc, SysFold); their
  // diagonal and zeroed residual are already this kernel's, only rhs and x are left
  const bool folded = skip && !skip[i];
  double* D = A + diag[i] * NV * NV + a * NV;
  if (dt[i] > rx::kEPS) {
    if (!folded) D[a] += vol[i] / dt[i];
    rhs[q] = -(R[q] + 0.0);
  } else {
    if (!folded) {
#pragma unroll
      for (int c = 0; c < NV; ++c) D[c] = (a == c) ? 1.0 : 0.0;
      R[q] = 0.0;
    }
    rhs[q] = -(0.0 + 0.0);
  }
}

// AddClippedSolution: U = clip(U_old + delta) (variable_structure.cpp:207-211) with
//   mode 0 implicit  delta = relax * LinSysSol                          (:2390-2400)
//   mode 1 explicit  delta = -(Res + 0) * dt / Vol                       (:2430-2440)
//   mode 2 RK stage  delta = -(Res + 0) * dt / Vol * alpha_RK, U_old = U0 (ExplicitRK_Iteration :2456-2493)
// wall (optional): isothermal-wall points, whose momentum Solution_Old BC_Isothermal_Wall sets to zero
// (SetVelocity_Old, solver_direct_reactive.cpp:5477, variable_direct_reactive.cpp:950-957); uold mirrors it.
__global__ __launch_bounds__(kBlock) void k_update(int N, int nVar, int nDim, const double* __restrict__ dx,
                                                   double scale, const double* __restrict__ vol,
                                                   const double* __restrict__ dt, int mode,
                                                   const double* __restrict__ U0, double* __restrict__ U,
                                                   const uint8_t* __restrict__ wall, double* __restrict__ uold) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * nVar) return;
  const int i = t / nVar, v = t - i * nVar;
  double delta;
  if (mode == 0) {
    delta = scale * dx[t];
  } else {
    double Delta = 0.0;
    if (vol[i] > rx::kEPS) Delta = dt[i] / vol[i];
    delta = -(dx[t] + 0.0) * Delta;
    if (mode == 2) delta = delta * scale;
  }
  const double lo = (v >= 1 && v <= nDim + 1) ? -1.0 / rx::kEPS : 0.0;
  const double hi = 1.0 / rx::kEPS;
  double base = U0 ? U0[t] : U[t];
  if (wall && wall[i] && v >= 1 && v <= nDim) {
    base = 0.0;
    uold[t] = 0.0;
  }
  const double x = base + delta;
  const double mx = (x < lo) ? lo : x;  // std::min(std::max(x, lo), hi), NaN and signed zeros included
  U[t] = (hi < mx) ? hi : mx;
}

__global__ __launch_bounds__(kBlock) void k_sumsq_cols(int N, int nVar, const double* __restrict__ r,
                                                       double* __restrict__ part) {
  // part[blockIdx.x * nVar + v] = sum over this block's rows of r^2 (fixed order)
  // one pass over the rows with every column's partial in registers (each column's sum in the same row order as a
  // pass per column; nVar <= kMaxCols)
  __shared__ double sh[kBlock];
  constexpr int kMaxCols = 16;
  double acc[kMaxCols];
#pragma unroll
  for (int v = 0; v < kMaxCols; ++v) acc[v] = 0.0;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < N; i += gridDim.x * kBlock) {
#pragma unroll
    for (int v = 0; v < kMaxCols; ++v)
      if (v < nVar) {
        const double x = r[(size_t)i * nVar + v];
        acc[v] += x * x;
      }
  }
#pragma unroll
  for (int v = 0; v < kMaxCols; ++v) {
    if (v < nVar) {  // block-uniform
      sh[threadIdx.x] = acc[v];
      __syncthreads();
      for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
      }
      if (threadIdx.x == 0) part[blockIdx.x * nVar + v] = sh[0];
      __syncthreads();
    }
  }
}

// Per-variable totals of the block partials, summed in block order (one lane per variable).
// The columns' block partials summed in block order. Round 6: the partials (nblk * nVar <= kSumsqStage doubles) are
// staged through LDS by the whole workgroup first — one global round trip instead of nblk dependent loads per column
// (36 us per call at C4, rocprof r06j) — and each column's sum is then the same sequence of adds.
constexpr int kSumsqStage = 256 * 16;
__global__ __launch_bounds__(256) void k_sumsq_total(int nVar, int nblk, const double* __restrict__ part,
                                                     double* __restrict__ out) {
  __shared__ double sp[kSumsqStage];
  const int n = nblk * nVar;
  for (int q = threadIdx.x; q < n; q += blockDim.x) sp[q] = part[q];
  __syncthreads();
  const int v = threadIdx.x;
  if (v >= nVar) return;
  double s = 0.0;
  for (int q = 0; q < nblk; ++q) s += sp[q * nVar + v];
  out[v] = s;
}

#define RX_NV_SWITCH(nv, CALL)                       \
  switch (nv) {                                      \
    case 2: { constexpr int NV_ = 2; CALL; } break;   \
    case 7: { constexpr int NV_ = 7; CALL; } break;   \
    case 8: { constexpr int NV_ = 8; CALL; } break;   \
    case 9: { constexpr int NV_ = 9; CALL; } break;   \
    case 10: { constexpr int NV_ = 10; CALL; } break; \
    case 11: { constexpr int NV_ = 11; CALL; } break; \
    case 12: { constexpr int NV_ = 12; CALL; } break; \
    case 13: { constexpr int NV_ = 13; CALL; } break; \
    case 14: { constexpr int NV_ = 14; CALL; } break; \
    default: return RX_ERR_ARG;                      \
  }


}  // namespace

// MatrixVectorProduct (:997-1029): owned rows, then the halo of the product from the neighbours.
int rx_la_spmv(rx_ctx* ctx, const double* A, const double* x, double* y, const int* skip) {
  RX_NV_SWITCH(ctx->nVar, (k_spmv<NV_><<<blocks(ctx->Nd * NV_), kBlock, 0, ctx->stream>>>((int)ctx->Nd, ctx->rp,
                                                                                           ctx->col, A, x, y, skip)));
  RX_HIP(hipGetLastError());
  return rx_la_exchange(ctx, y, ctx->nVar);
}

int rx_la_build_system(rx_ctx* ctx) {
  static const bool per_node = getenv("RX_BUILD_PER_NODE") != nullptr;  // A/B: the thread-per-node build
  const int32_t* skip = ctx->sys_folded ? ctx->fold_skip : nullptr;
  ctx->sys_folded = 0;
  if (per_node && !skip) {
    RX_NV_SWITCH(ctx->nVar, (k_build_system<NV_><<<blocks(ctx->N), kBlock, 0, ctx->stream>>>(
                                (int)ctx->Nd, (int)ctx->N, ctx->diag, ctx->vol, ctx->f[RX_F_DT], ctx->f[RX_F_JAC],
                                ctx->f[RX_F_RES], ctx->f[RX_F_RHS], ctx->f[RX_F_SOL])));
  } else {
    RX_NV_SWITCH(ctx->nVar, (k_build_system_elem<NV_><<<blocks(ctx->N * NV_), kBlock, 0, ctx->stream>>>(
                                (int)ctx->Nd, (int)ctx->N, ctx->diag, ctx->vol, ctx->f[RX_F_DT], ctx->f[RX_F_JAC],
                                ctx->f[RX_F_RES], ctx->f[RX_F_RHS], ctx->f[RX_F_SOL], skip)));
  }
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// SetResidual_RMS (solver_structure.cpp:184-230): per-variable sums of r^2 over the owned rows
// (fixed order), all-reduced over ranks into rms_sum[16..), read back and finished on the host by
// rx_la_rms_read with the global owned-point count.
constexpr int kRmsBlocks = 256;
constexpr int64_t kRmsOff = 1024;  // ctx->red[0..1023] is the inner-product scratch

int rx_la_rms_enqueue(rx_ctx* ctx, const double* r) {
  k_sumsq_cols<<<kRmsBlocks, kBlock, 0, ctx->stream>>>((int)ctx->Nd, ctx->nVar, r, ctx->red + kRmsOff);
  static_assert(kRmsBlocks * 16 <= kSumsqStage, "the RMS partials fit the LDS stage (nVar <= 16)");
  k_sumsq_total<<<1, 256, 0, ctx->stream>>>(ctx->nVar, kRmsBlocks, ctx->red + kRmsOff, ctx->rms_sum);
  RX_HIP(hipGetLastError());
  return rx_la_allreduce(ctx, ctx->rms_sum, ctx->rms_sum + 16, ctx->nVar);
}

int rx_la_rms_read(rx_ctx* ctx, double* rms) {
  int rc = rx_la_rms_copy(ctx);
  if (!rc) rc = rx_la_host_wait(ctx);
  if (!rc) rx_la_rms_finish(ctx, rms);
  return rc;
}
// the read-back in two halves, so that one host wait covers it and the FGMRES state (implicit_solve)
int rx_la_rms_copy(rx_ctx* ctx) {
  const double* src = ctx->rms_sum + (ctx->distributed() ? 16 : 0);
  RX_HIP(hipMemcpyAsync(ctx->h_red, src, sizeof(double) * ctx->nVar, hipMemcpyDeviceToHost, ctx->stream));
  return RX_OK;
}
void rx_la_rms_finish(const rx_ctx* ctx, double* rms) {
  for (int v = 0; v < ctx->nVar; ++v)
    rms[v] = std::max(rx::kEPS * rx::kEPS, std::sqrt(ctx->h_red[v] / (double)ctx->n_global));
}

// Owned points, then Set_MPI_Solution (solver_direct_reactive.cpp:2403, 2445).
int rx_la_implicit_update(rx_ctx* ctx) {
  const int64_t n = ctx->Nd * ctx->nVar;
  // Solution_Old (Set_OldSolution) for SetPrimVar's non-physical restart
  RX_HIP(hipMemcpyAsync(ctx->uold, ctx->f[RX_F_U], sizeof(double) * ctx->N * ctx->nVar, hipMemcpyDeviceToDevice,
                        ctx->stream));
  k_update<<<blocks(n), kBlock, 0, ctx->stream>>>((int)ctx->Nd, ctx->nVar, ctx->nDim, ctx->f[RX_F_SOL],
                                                  ctx->cfg.relaxation, ctx->vol, ctx->f[RX_F_DT], 0, nullptr,
                                                  ctx->f[RX_F_U], ctx->bc_wall, ctx->uold);
  RX_HIP(hipGetLastError());
  // with RCCL, implicit_solve starts the exchange on comm_stream after the solve (rx_la_u_exchange_begin)
  return rx_u_exchange_deferred(ctx) ? RX_OK : rx_la_exchange(ctx, ctx->f[RX_F_U], ctx->nVar);
}

int rx_la_explicit_update(rx_ctx* ctx) {
  const int64_t n = ctx->Nd * ctx->nVar;
  RX_HIP(hipMemcpyAsync(ctx->uold, ctx->f[RX_F_U], sizeof(double) * ctx->N * ctx->nVar, hipMemcpyDeviceToDevice,
                        ctx->stream));
  k_update<<<blocks(n), kBlock, 0, ctx->stream>>>((int)ctx->Nd, ctx->nVar, ctx->nDim, ctx->f[RX_F_RES], 1.0,
                                                  ctx->vol, ctx->f[RX_F_DT], 1, nullptr, ctx->f[RX_F_U], ctx->bc_wall,
                                                  ctx->uold);
  RX_HIP(hipGetLastError());
  return rx_u_exchange_deferred(ctx) ? rx_la_u_exchange_begin(ctx) : rx_la_exchange(ctx, ctx->f[RX_F_U], ctx->nVar);
}

// ExplicitRK_Iteration stage: Set_OldSolution at stage 0 (integration_time.cpp:162), then
// U = clip(U_old - Res dt/Vol alpha), Set_MPI_Solution (:2488).
int rx_la_rk_update(rx_ctx* ctx, int stage, double alpha) {
  const int64_t n = ctx->Nd * ctx->nVar;
  if (stage == 0)
    RX_HIP(hipMemcpyAsync(ctx->uold, ctx->f[RX_F_U], sizeof(double) * ctx->N * ctx->nVar, hipMemcpyDeviceToDevice,
                          ctx->stream));
  k_update<<<blocks(n), kBlock, 0, ctx->stream>>>((int)ctx->Nd, ctx->nVar, ctx->nDim, ctx->f[RX_F_RES], alpha,
                                                  ctx->vol, ctx->f[RX_F_DT], 2, ctx->uold, ctx->f[RX_F_U], ctx->bc_wall,
                                                  ctx->uold);
  RX_HIP(hipGetLastError());
  return rx_u_exchange_deferred(ctx) ? rx_la_u_exchange_begin(ctx) : rx_la_exchange(ctx, ctx->f[RX_F_U], ctx->nVar);
}
