// rx_krylov.hip — device-resident FGMRES (CSysSolve::FGMRES_LinSolver,
// Common/src/linear_solvers_structure.cpp:309-463, ModGramSchmidt :87-186, ApplyGivens /
// GenerateGivens :37-71, SolveReduced :73-85) and the captured implicit solve.
//
// Every scalar of the Krylov recurrence (norms, Hessenberg entries, Givens rotations, the
// stop/breakdown decisions and the re-orthogonalisation test of MGS) lives in device memory and is
// updated by single-lane kernels in the reference's operation order, so the whole solve is a fixed
// sequence of kernels with no host round trip: the host launches it (or replays it as one hipGraph)
// and reads the iteration count / residual once at the end. Kernels after a stop decision see the
// `done` flag and return immediately. Inner products are fixed-order tree reductions (bitwise
// reproducible); the reference sums sequentially, so results agree to rounding.
#include <hip/hip_runtime.h>

#include <cmath>

#include "rx_ctx.h"

namespace {

constexpr int kBlock = 256;
constexpr int kRedBlocks = 512;
constexpr int kMaxM = 64;
inline int blocks(int64_t n, int b = kBlock) { return (int)((n + b - 1) / b); }

struct KState {
  double tol, norm0, beta, nrm, thr, prod, dot, resid;
  int done, noreo, iters, diverged;
  double H[(kMaxM + 1) * kMaxM];  // H[k][i] at k * kMaxM + i
  double g[kMaxM + 1], cs[kMaxM + 1], sn[kMaxM + 1], y[kMaxM];
};

__device__ inline double& Hk(KState* s, int k, int i) { return s->H[k * kMaxM + i]; }

// ---- vector kernels (skip when *skip != 0)
__global__ __launch_bounds__(kBlock) void k_dot_part(int64_t n, const double* __restrict__ a,
                                                     const double* __restrict__ b, double* __restrict__ part,
                                                     const int* __restrict__ skip) {
  if (skip && *skip) return;
  __shared__ double sh[kBlock];
  double s = 0.0;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < n; q += (int64_t)gridDim.x * kBlock)
    s += a[q] * b[q];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

__global__ __launch_bounds__(kBlock) void k_dot_fin(const double* __restrict__ part, double* __restrict__ out,
                                                    const int* __restrict__ skip) {
  if (skip && *skip) return;
  __shared__ double sh[kBlock];
  sh[threadIdx.x] = part[threadIdx.x] + part[threadIdx.x + kBlock];
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sh[0];
}

// y += sign * (*alpha) * x
__global__ __launch_bounds__(kBlock) void k_axpy_dev(int64_t n, const double* __restrict__ alpha, double sign,
                                                     const double* __restrict__ x, double* __restrict__ y,
                                                     const int* __restrict__ skip) {
  if (skip && *skip) return;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < n) y[q] += (sign * *alpha) * x[q];
}
// y /= *d
__global__ __launch_bounds__(kBlock) void k_div_dev(int64_t n, const double* __restrict__ d, double* __restrict__ y,
                                                    const int* __restrict__ skip) {
  if (skip && *skip) return;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < n) y[q] /= *d;
}
__global__ __launch_bounds__(kBlock) void k_sub_vec(int64_t n, const double* __restrict__ b, double* __restrict__ y) {
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < n) y[q] -= b[q];
}
// x += sum_k y_k z_k, k ascending (the reference's per-k vector updates, element by element)
__global__ __launch_bounds__(kBlock) void k_fg_update_x(int64_t n, const KState* __restrict__ s,
                                                        const double* __restrict__ Z, double* __restrict__ x) {
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int it = s->iters;
  if (q >= n || it == 0 || s->diverged) return;
  double v = x[q];
  for (int k = 0; k < it; ++k) v += s->y[k] * Z[(int64_t)k * n + q];
  x[q] = v;
}

// ---- single-lane recurrence kernels
__global__ void k_fg_reset(KState* s, double tol) {
  s->tol = tol;
  s->done = 0;
  s->noreo = 1;
  s->iters = 0;
  s->diverged = 0;
  s->resid = 0.0;
}
// after dot(b,b) -> norm0 slot and dot(w0,w0) -> dot slot
__global__ void k_fg_start(KState* s) {
  s->norm0 = sqrt(s->norm0);
  s->beta = sqrt(s->dot);
  const double epsm = 2.220446049250313e-16;
  if ((s->beta < s->tol * s->norm0) || (s->beta < epsm)) {
    s->done = 1;
    s->resid = s->beta;
    return;
  }
  s->prod = -s->beta;  // w0 /= -beta
  s->g[0] = s->beta;
  s->norm0 = s->beta;
}
__global__ void k_fg_begin(KState* s) {
  if (s->done) return;
  if (s->beta < s->tol * s->norm0) s->done = 1;
}
// after dot(w_{i+1}, w_{i+1}) -> dot
__global__ void k_fg_mgs_begin(KState* s) {
  if (s->done) return;
  s->nrm = s->dot;
  s->thr = s->nrm * 0.98;
  if ((s->nrm <= 0.0) || (s->nrm != s->nrm)) {
    s->diverged = 1;
    s->done = 1;
  }
}
// after dot(w_{i+1}, w_k) -> dot: H[k][i] = prod, decide re-orthogonalisation
__global__ void k_fg_proj(KState* s, int k, int i) {
  if (s->done) {
    s->noreo = 1;
    return;
  }
  s->prod = s->dot;
  Hk(s, k, i) = s->prod;
  s->noreo = (s->prod * s->prod > s->thr) ? 0 : 1;
}
// after the optional second projection (dot -> dot when it ran)
__global__ void k_fg_reo(KState* s, int k, int i) {
  if (s->done) return;
  if (!s->noreo) {
    s->prod = s->dot;
    Hk(s, k, i) += s->prod;
  }
}
__global__ void k_fg_nrm_update(KState* s, int k, int i) {
  if (s->done) return;
  s->nrm -= Hk(s, k, i) * Hk(s, k, i);
  if (s->nrm < 0.0) s->nrm = 0.0;
  s->thr = s->nrm * 0.98;
}
__device__ inline void apply_givens(double sn, double cs, double& h1, double& h2) {
  const double t = cs * h1 + sn * h2;
  h2 = cs * h2 - sn * h1;
  h1 = t;
}
__device__ inline double sign_of(double a, double b) { return b == 0.0 ? 0.0 : (b < 0 ? -fabs(a) : fabs(a)); }
// after dot(w_{i+1}, w_{i+1}) -> dot: H[i+1][i], Givens, beta
__global__ void k_fg_close(KState* s, int i) {
  if (s->done) return;
  s->nrm = sqrt(s->dot);
  Hk(s, i + 1, i) = s->nrm;
  for (int k = 0; k < i; ++k) apply_givens(s->sn[k], s->cs[k], Hk(s, k, i), Hk(s, k + 1, i));
  double& dx = Hk(s, i, i);
  double& dy = Hk(s, i + 1, i);
  if ((dx == 0.0) && (dy == 0.0)) {
    s->cs[i] = 1.0;
    s->sn[i] = 0.0;
  } else if (fabs(dy) > fabs(dx)) {
    const double tmp = dx / dy;
    dx = sqrt(1.0 + tmp * tmp);
    s->sn[i] = sign_of(1.0 / dx, dy);
    s->cs[i] = tmp * s->sn[i];
  } else if (fabs(dy) <= fabs(dx)) {
    const double tmp = dy / dx;
    dy = sqrt(1.0 + tmp * tmp);
    s->cs[i] = sign_of(1.0 / dy, dx);
    s->sn[i] = tmp * s->cs[i];
  } else {
    dx = dy = 0.0;
    s->cs[i] = 1.0;
    s->sn[i] = 0.0;
  }
  dx = fabs(dx * dy);
  dy = 0.0;
  apply_givens(s->sn[i], s->cs[i], s->g[i], s->g[i + 1]);
  s->beta = fabs(s->g[i + 1]);
  s->iters = i + 1;
}
__global__ void k_fg_solve(KState* s) {
  if (s->diverged) return;
  const int it = s->iters;
  if (it > 0 || !s->done) s->resid = s->beta;
  for (int k = 0; k < it; ++k) s->y[k] = s->g[k];
  for (int k = it - 1; k >= 0; --k) {
    s->y[k] /= Hk(s, k, k);
    for (int j = k - 1; j >= 0; --j) s->y[j] -= Hk(s, j, k) * s->y[k];
  }
}

}  // namespace

int rx_la_krylov_alloc(rx_ctx* ctx, int m) {
  const int64_t n = ctx->N * ctx->nVar;
  if (m < 1 || m > kMaxM) return RX_ERR_ARG;
  if (ctx->krylov_m < m) {
    if (ctx->kw) (void)hipFree(ctx->kw);
    if (ctx->kz) (void)hipFree(ctx->kz);
    ctx->kw = ctx->kz = nullptr;
    RX_HIP(hipMalloc(&ctx->kw, sizeof(double) * n * (m + 1)));
    RX_HIP(hipMalloc(&ctx->kz, sizeof(double) * n * (m + 1)));
    ctx->krylov_m = m;
  }
  if (!ctx->kstate) {
    RX_HIP(hipMalloc(&ctx->kstate, sizeof(KState)));
    RX_HIP(hipMemsetAsync(ctx->kstate, 0, sizeof(KState), ctx->stream));
    RX_HIP(hipHostMalloc(&ctx->h_kstate, sizeof(KState)));
  }
  return RX_OK;
}

// Enqueue FGMRES(m) on JAC * SOL = RHS (SOL = initial guess) without any host synchronisation.
int rx_la_fgmres_enqueue(rx_ctx* ctx, double tol, int m) {
  int rc = rx_la_krylov_alloc(ctx, m);
  if (rc) return rc;
  const int64_t n = ctx->N * ctx->nVar;
  hipStream_t st = ctx->stream;
  KState* s = static_cast<KState*>(ctx->kstate);
  double* A = ctx->f[RX_F_JAC];
  double* b = ctx->f[RX_F_RHS];
  double* x = ctx->f[RX_F_SOL];
  double* part = ctx->red;
  auto W = [&](int k) { return ctx->kw + (int64_t)k * n; };
  auto Z = [&](int k) { return ctx->kz + (int64_t)k * n; };
  const int* done = &s->done;
  const int* noreo = &s->noreo;
  auto dot = [&](const double* a, const double* c, double* out, const int* skip) -> int {
    k_dot_part<<<kRedBlocks, kBlock, 0, st>>>(n, a, c, part, skip);
    k_dot_fin<<<1, kBlock, 0, st>>>(part, out, skip);
    return RX_OK;
  };
  k_fg_reset<<<1, 1, 0, st>>>(s, tol);
  dot(b, b, &s->norm0, nullptr);
  if ((rc = rx_la_spmv(ctx, A, x, W(0), nullptr))) return rc;
  k_sub_vec<<<blocks(n), kBlock, 0, st>>>(n, b, W(0));
  dot(W(0), W(0), &s->dot, nullptr);
  k_fg_start<<<1, 1, 0, st>>>(s);
  k_div_dev<<<blocks(n), kBlock, 0, st>>>(n, &s->prod, W(0), done);
  for (int i = 0; i < m; ++i) {
    k_fg_begin<<<1, 1, 0, st>>>(s);
    if (ctx->cfg.lin_prec == 1) {
      if ((rc = rx_la_ilu_apply(ctx, W(i), Z(i), done))) return rc;
    } else {
      if ((rc = rx_la_lusgs(ctx, A, W(i), Z(i), done))) return rc;
    }
    if ((rc = rx_la_spmv(ctx, A, Z(i), W(i + 1), done))) return rc;
    dot(W(i + 1), W(i + 1), &s->dot, done);
    k_fg_mgs_begin<<<1, 1, 0, st>>>(s);
    for (int k = 0; k <= i; ++k) {
      dot(W(i + 1), W(k), &s->dot, done);
      k_fg_proj<<<1, 1, 0, st>>>(s, k, i);
      k_axpy_dev<<<blocks(n), kBlock, 0, st>>>(n, &s->prod, -1.0, W(k), W(i + 1), done);
      dot(W(i + 1), W(k), &s->dot, noreo);
      k_fg_reo<<<1, 1, 0, st>>>(s, k, i);
      k_axpy_dev<<<blocks(n), kBlock, 0, st>>>(n, &s->prod, -1.0, W(k), W(i + 1), noreo);
      k_fg_nrm_update<<<1, 1, 0, st>>>(s, k, i);
    }
    dot(W(i + 1), W(i + 1), &s->dot, done);
    k_fg_close<<<1, 1, 0, st>>>(s, i);
    k_div_dev<<<blocks(n), kBlock, 0, st>>>(n, &s->nrm, W(i + 1), done);
  }
  k_fg_solve<<<1, 1, 0, st>>>(s);
  k_fg_update_x<<<blocks(n), kBlock, 0, st>>>(n, s, ctx->kz, x);
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// Read back the outcome of the last enqueued FGMRES (synchronises the stream).
int rx_la_fgmres_result(rx_ctx* ctx, int* iters, double* resid) {
  if (!ctx->kstate) return RX_ERR_STATE;
  KState* h = static_cast<KState*>(ctx->h_kstate);
  RX_HIP(hipMemcpyAsync(h, ctx->kstate, offsetof(KState, H), hipMemcpyDeviceToHost, ctx->stream));
  RX_HIP(hipStreamSynchronize(ctx->stream));
  if (iters) *iters = h->iters;
  if (resid) *resid = h->resid;
  return h->diverged ? RX_ERR_DIVERGED : RX_OK;
}

int rx_la_fgmres(rx_ctx* ctx, double tol, int m, int* iters, double* resid) {
  int rc = rx_la_fgmres_enqueue(ctx, tol, m);
  if (rc) return rc;
  return rx_la_fgmres_result(ctx, iters, resid);
}

void rx_la_krylov_free(rx_ctx* ctx) {
  if (ctx->kstate) (void)hipFree(ctx->kstate);
  if (ctx->h_kstate) (void)hipHostFree(ctx->h_kstate);
  ctx->kstate = ctx->h_kstate = nullptr;
}
