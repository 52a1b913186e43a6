// rx_sweeps.hip — triangular work of the implicit path: ILU(0) factorisation and application,
// LU-SGS, diagonal-block factorisations. One workgroup per partition ("rank").
//
// Reference semantics (Common/src/matrix_structure.cpp):
//   BuildILUPreconditioner :1368-1451 (left-multiply quirk :1432-1436), ComputeILUPreconditioner
//   :1453-1515, InverseDiagonalBlock_ILUMatrix :1180-1228, Gauss_Elimination :594-643,
//   ComputeLU_SGSPreconditioner :1673-1709 with Lower/Upper/DiagonalProduct :743-792.
//
// Partitions are contiguous row ranges that stand for the reference's MPI ranks: each rank runs the
// sequential row loops over its own domain rows; ILU(0) ignores halo columns, LU-SGS's backward sweep
// reads halo columns at their forward-sweep (x*) values (see oracle/rx_oracle.cpp, struct Parts).
// A rank never waits on another, so a rank maps to one workgroup: the workgroup walks the rank's
// dependency levels (rows of a level are independent) with a workgroup barrier between levels, and
// inside a row the arithmetic is the reference's, operation for operation (bitwise equal results).
//
// Block factorisations run in one wavefront with lane k holding column k of the block; pivots and
// multipliers are broadcast with v_readlane (compile-time lanes), so the elimination order is the
// scalar reference's.
#include <hip/hip_runtime.h>

#include "rx_ctx.h"

namespace {

template <int NV>
struct Blk {
  static constexpr int N2 = NV * NV;
};

// Lanes of one wavefront exchanging data through LDS: order the LDS traffic at wavefront scope.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double bcast(double v, int lane) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), lane);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// In-wave Gauss elimination of a block (Gauss_Elimination :594-643, matrix part). On entry lane k
// (k < NV) holds column k in col[0..NV-1]; on exit col[r] holds U[r][k] for r <= k and the multiplier
// w[r][k] for r > k (the slot the reference leaves as an unused, eliminated entry).
template <int NV>
__device__ __forceinline__ void wave_factor(double (&col)[NV], int lane) {
#pragma unroll
  for (int ii = 1; ii < NV; ++ii) {
#pragma unroll
    for (int jj = 0; jj < ii; ++jj) {
      const double w = bcast(col[ii], jj) / bcast(col[jj], jj);
      if (lane > jj) col[ii] -= w * col[jj];
      if (lane == jj) col[ii] = w;
    }
  }
}

// Solve with a factorised block held as in wave_factor: rhs (one vector per lane) is overwritten by
// the solution, with the reference's rhs operation order (forward with multipliers, then back
// substitution with U).
template <int NV>
__device__ __forceinline__ void wave_solve(const double (&col)[NV], double (&rhs)[NV]) {
#pragma unroll
  for (int ii = 1; ii < NV; ++ii)
#pragma unroll
    for (int jj = 0; jj < ii; ++jj) rhs[ii] -= bcast(col[ii], jj) * rhs[jj];
  rhs[NV - 1] = rhs[NV - 1] / bcast(col[NV - 1], NV - 1);
#pragma unroll
  for (int ii = NV - 2; ii >= 0; --ii) {
    double aux = 0.0;
#pragma unroll
    for (int jj = ii + 1; jj < NV; ++jj) aux += bcast(col[ii], jj) * rhs[jj];
    rhs[ii] = (rhs[ii] - aux) / bcast(col[ii], ii);
  }
}

// Serial solve with a stored factorisation (row-major LU[r][k] as produced by k_diag_factor).
template <int NV>
__device__ __forceinline__ void lu_solve(const double* __restrict__ LU, double (&rhs)[NV]) {
#pragma unroll
  for (int ii = 1; ii < NV; ++ii)
#pragma unroll
    for (int jj = 0; jj < ii; ++jj) rhs[ii] -= LU[ii * NV + jj] * rhs[jj];
  rhs[NV - 1] = rhs[NV - 1] / LU[NV * NV - 1];
#pragma unroll
  for (int ii = NV - 2; ii >= 0; --ii) {
    double aux = 0.0;
#pragma unroll
    for (int jj = ii + 1; jj < NV; ++jj) aux += LU[ii * NV + jj] * rhs[jj];
    rhs[ii] = (rhs[ii] - aux) / LU[ii * NV + ii];
  }
}

// Factorise every diagonal block once (LU-SGS uses Gauss_Elimination on the same, unchanged diagonal
// block for every row and every call, so one factorisation per matrix is bitwise equivalent).
// One wavefront per row.
template <int NV>
__global__ __launch_bounds__(256) void k_diag_factor(int N, const int64_t* __restrict__ diag,
                                                     const double* __restrict__ A, double* __restrict__ LU) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= N) return;
  const double* D = A + diag[i] * (NV * NV);
  double col[NV];
#pragma unroll
  for (int r = 0; r < NV; ++r) col[r] = lane < NV ? D[r * NV + lane] : 1.0;
  wave_factor<NV>(col, lane);
  if (lane < NV) {
#pragma unroll
    for (int r = 0; r < NV; ++r) LU[(size_t)i * NV * NV + r * NV + lane] = col[r];
  }
}

// ---------------------------------------------------------------------------------------------
// ILU(0) factorisation, one workgroup per partition, one wavefront per row.
// F holds a copy of A on entry. invD receives inv(D_i) of every finished row (the reference recomputes
// exactly this inverse from the same finished block whenever it needs it).
// LDS per wave: row blocks [rowmax][NV2] + W [NV2] + staging [NV2].
template <int NV>
__global__ __launch_bounds__(1024) void k_ilu_build_part(const int32_t* __restrict__ part_lvl,
                                                         const int32_t* __restrict__ lvl_ptr,
                                                         const int32_t* __restrict__ rows,
                                                         const int32_t* __restrict__ col,
                                                         const int32_t* __restrict__ klo,
                                                         const int32_t* __restrict__ khi,
                                                         const int64_t* __restrict__ diag, double* __restrict__ F,
                                                         double* __restrict__ invD, int rowmax) {
  constexpr int NV2 = NV * NV;
  extern __shared__ double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  double* rowbuf = lds + (size_t)wave * (rowmax + 2) * NV2;
  double* Wb = rowbuf + (size_t)rowmax * NV2;
  double* S = Wb + NV2;
  const int p = blockIdx.x;
  for (int l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
    for (int r = lvl_ptr[l] + wave; r < lvl_ptr[l + 1]; r += nwave) {
      const int i = rows[r];
      const int k0 = klo[i], k1 = khi[i], kd = (int)diag[i];
      const int nbk = k1 - k0;
      for (int q = lane; q < nbk * NV2; q += 64) rowbuf[q] = F[(size_t)k0 * NV2 + q];
      wave_sync();
      for (int k = k0; k < kd; ++k) {
        const int j = col[k];
        for (int q = lane; q < NV2; q += 64) S[q] = invD[(size_t)j * NV2 + q];
        wave_sync();
        const double* Bij = rowbuf + (size_t)(k - k0) * NV2;
        // W = A_ij * inv(A_jj)  (MatrixMatrixProduct, sum from 0.0 over q ascending)
        for (int e = lane; e < NV2; e += 64) {
          const int a = e / NV, c = e - a * NV;
          double s = 0.0;
#pragma unroll
          for (int q = 0; q < NV; ++q) s += Bij[a * NV + q] * S[q * NV + c];
          Wb[e] = s;
        }
        wave_sync();
        // A_ik -= A_jk * W for the upper blocks of row j (left-multiply quirk). The diagonal of row j
        // would update A_ij, which is overwritten by W below, so it is skipped.
        const int kdj = (int)diag[j], k1j = khi[j];
        for (int kk = kdj + 1; kk < k1j; ++kk) {
          const int kp = col[kk];
          int pos = -1;
          for (int q = k0; q < k1; ++q)
            if (col[q] == kp) {
              pos = q;
              break;
            }
          if (pos < 0) continue;
          for (int q = lane; q < NV2; q += 64) S[q] = F[(size_t)kk * NV2 + q];
          wave_sync();
          double* Bik = rowbuf + (size_t)(pos - k0) * NV2;
          for (int e = lane; e < NV2; e += 64) {
            const int a = e / NV, c = e - a * NV;
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < NV; ++q) s += S[a * NV + q] * Wb[q * NV + c];
            Bik[e] -= s;
          }
          wave_sync();
        }
        double* dst = rowbuf + (size_t)(k - k0) * NV2;
        for (int e = lane; e < NV2; e += 64) dst[e] = Wb[e];
        wave_sync();
      }
      // inv(D_i): Gauss elimination of each unit column (InverseDiagonalBlock_ILUMatrix)
      {
        const double* D = rowbuf + (size_t)(kd - k0) * NV2;
        double cl[NV], rhs[NV];
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) cl[rr] = lane < NV ? D[rr * NV + lane] : 1.0;
        wave_factor<NV>(cl, lane);
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) rhs[rr] = (rr == lane) ? 1.0 : 0.0;
        wave_solve<NV>(cl, rhs);
        if (lane < NV) {
#pragma unroll
          for (int rr = 0; rr < NV; ++rr) invD[(size_t)i * NV2 + rr * NV + lane] = rhs[rr];
        }
      }
      for (int q = lane; q < nbk * NV2; q += 64) F[(size_t)k0 * NV2 + q] = rowbuf[q];
      wave_sync();
    }
    __syncthreads();
  }
}

// ILU(0) forward substitution x = b - L x per partition; one thread per (row, component).
template <int NV>
__global__ __launch_bounds__(256) void k_ilu_fwd_part(const int32_t* __restrict__ part_lvl,
                                                      const int32_t* __restrict__ lvl_ptr,
                                                      const int32_t* __restrict__ rows,
                                                      const int32_t* __restrict__ col,
                                                      const int32_t* __restrict__ klo,
                                                      const int64_t* __restrict__ diag,
                                                      const double* __restrict__ F, const double* __restrict__ b,
                                                      double* __restrict__ x,
    const int* __restrict__ skip) {
  if (skip && *skip) return;
  constexpr int NV2 = NV * NV, RPB = 256 / NV;
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  for (int l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
    const int r1 = lvl_ptr[l + 1];
    for (int r = lvl_ptr[l] + rl; r < r1 && rl < RPB; r += RPB) {
      const int i = rows[r];
      double xi = b[(size_t)i * NV + a];
      const int kd = (int)diag[i];
      for (int k = klo[i]; k < kd; ++k) {
        const double* blk = F + (size_t)k * NV2 + a * NV;
        const double* xj = x + (size_t)col[k] * NV;
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) s += blk[c] * xj[c];
        xi -= s;
      }
      x[(size_t)i * NV + a] = xi;
    }
    __syncthreads();
  }
}

// ILU(0) backward substitution x_i = inv(D_i) (x_i - sum_{j>i} U_ij x_j) per partition.
template <int NV>
__global__ __launch_bounds__(256) void k_ilu_bwd_part(const int32_t* __restrict__ part_lvl,
                                                      const int32_t* __restrict__ lvl_ptr,
                                                      const int32_t* __restrict__ rows,
                                                      const int32_t* __restrict__ col,
                                                      const int32_t* __restrict__ khi,
                                                      const int64_t* __restrict__ diag,
                                                      const double* __restrict__ F,
                                                      const double* __restrict__ invD, double* __restrict__ x,
    const int* __restrict__ skip) {
  if (skip && *skip) return;
  constexpr int NV2 = NV * NV, RPB = 256 / NV;
  __shared__ double v[RPB * NV];
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  for (int l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    for (int base = r0; base < r1; base += RPB) {
      const int r = base + rl;
      const bool act = rl < RPB && r < r1;
      int i = 0;
      if (act) {
        i = rows[r];
        double sum = 0.0;
        const int k1 = khi[i];
        for (int k = (int)diag[i] + 1; k < k1; ++k) {
          const double* blk = F + (size_t)k * NV2 + a * NV;
          const double* xj = x + (size_t)col[k] * NV;
          double s = 0.0;
#pragma unroll
          for (int c = 0; c < NV; ++c) s += blk[c] * xj[c];
          sum += s;
        }
        v[rl * NV + a] = x[(size_t)i * NV + a] - sum;
      }
      __syncthreads();
      if (act) {
        const double* inv = invD + (size_t)i * NV2 + a * NV;
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) s += inv[c] * v[rl * NV + c];
        x[(size_t)i * NV + a] = s;
      }
      __syncthreads();
    }
  }
}

// LU-SGS forward sweep (D+L) x* = b per partition: products per (row, component), then one thread
// per row solves with the stored factorisation of D.
template <int NV>
__global__ __launch_bounds__(256) void k_lusgs_fwd_part(const int32_t* __restrict__ part_lvl,
                                                        const int32_t* __restrict__ lvl_ptr,
                                                        const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ col,
                                                        const int32_t* __restrict__ klo,
                                                        const int64_t* __restrict__ diag,
                                                        const double* __restrict__ A, const double* __restrict__ DLU,
                                                        const double* __restrict__ b, double* __restrict__ xs,
    const int* __restrict__ skip) {
  if (skip && *skip) return;
  constexpr int NV2 = NV * NV, RPB = 256 / NV;
  __shared__ double v[RPB * NV];
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  for (int l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    for (int base = r0; base < r1; base += RPB) {
      const int r = base + rl;
      if (rl < RPB && r < r1) {
        const int i = rows[r];
        double prv = 0.0;
        const int kd = (int)diag[i];
        for (int k = klo[i]; k < kd; ++k) {
          const double* blk = A + (size_t)k * NV2 + a * NV;
          const double* xj = xs + (size_t)col[k] * NV;
          double pb = 0.0;
#pragma unroll
          for (int c = 0; c < NV; ++c) pb += blk[c] * xj[c];
          prv += pb;
        }
        v[rl * NV + a] = b[(size_t)i * NV + a] - prv;
      }
      __syncthreads();
      if (threadIdx.x < RPB && base + (int)threadIdx.x < r1) {
        const int i = rows[base + threadIdx.x];
        double rhs[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) rhs[c] = v[threadIdx.x * NV + c];
        lu_solve<NV>(DLU + (size_t)i * NV2, rhs);
#pragma unroll
        for (int c = 0; c < NV; ++c) xs[(size_t)i * NV + c] = rhs[c];
      }
      __syncthreads();
    }
  }
}

// LU-SGS backward sweep (D+U) x = D x*: own-partition upper columns at their final values, halo
// columns (other partitions) at their forward-sweep values xs.
template <int NV>
__global__ __launch_bounds__(256) void k_lusgs_bwd_part(const int32_t* __restrict__ part_lvl,
                                                        const int32_t* __restrict__ lvl_ptr,
                                                        const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ rp,
                                                        const int32_t* __restrict__ col,
                                                        const int32_t* __restrict__ klo,
                                                        const int32_t* __restrict__ khi,
                                                        const int64_t* __restrict__ diag,
                                                        const double* __restrict__ A, const double* __restrict__ DLU,
                                                        const double* __restrict__ xs, double* __restrict__ x,
    const int* __restrict__ skip) {
  if (skip && *skip) return;
  constexpr int NV2 = NV * NV, RPB = 256 / NV;
  __shared__ double v[RPB * NV];
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  for (int l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    for (int base = r0; base < r1; base += RPB) {
      const int r = base + rl;
      if (rl < RPB && r < r1) {
        const int i = rows[r];
        const int kd = (int)diag[i];
        double aux;
        {
          const double* blk = A + (size_t)kd * NV2 + a * NV;
          const double* xi = xs + (size_t)i * NV;
          double pb = 0.0;
#pragma unroll
          for (int c = 0; c < NV; ++c) pb += blk[c] * xi[c];
          aux = pb;  // DiagonalProduct: 0 + block * x*
        }
        double prv = 0.0;
        auto prod = [&](int k, const double* xv) {
          const double* blk = A + (size_t)k * NV2 + a * NV;
          const double* xj = xv + (size_t)col[k] * NV;
          double pb = 0.0;
#pragma unroll
          for (int c = 0; c < NV; ++c) pb += blk[c] * xj[c];
          prv += pb;
        };
        const int k1 = khi[i];
        for (int k = kd + 1; k < k1; ++k) prod(k, x);
        const int k0 = klo[i];
        for (int k = rp[i]; k < k0; ++k) prod(k, xs);
        const int ke = rp[i + 1];
        for (int k = k1; k < ke; ++k) prod(k, xs);
        v[rl * NV + a] = aux - prv;
      }
      __syncthreads();
      if (threadIdx.x < RPB && base + (int)threadIdx.x < r1) {
        const int i = rows[base + threadIdx.x];
        double rhs[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) rhs[c] = v[threadIdx.x * NV + c];
        lu_solve<NV>(DLU + (size_t)i * NV2, rhs);
#pragma unroll
        for (int c = 0; c < NV; ++c) x[(size_t)i * NV + c] = rhs[c];
      }
      __syncthreads();
    }
  }
}

#define RX_NV_SWITCH(nv, CALL)                       \
  switch (nv) {                                      \
    case 7: { constexpr int NV_ = 7; CALL; } break;   \
    case 8: { constexpr int NV_ = 8; CALL; } break;   \
    case 11: { constexpr int NV_ = 11; CALL; } break; \
    case 13: { constexpr int NV_ = 13; CALL; } break; \
    default: return RX_ERR_ARG;                      \
  }

}  // namespace

double* rx_invd_buf(rx_ctx* ctx) { return ctx->f[RX_F_ILU] + ctx->nnzb * (int64_t)ctx->nVar * ctx->nVar; }

int rx_la_ilu_build(rx_ctx* ctx) {
  const int nv = ctx->nVar;
  const int64_t nb = ctx->nnzb * (int64_t)nv * nv;
  RX_HIP(hipMemcpyAsync(ctx->f[RX_F_ILU], ctx->f[RX_F_JAC], nb * sizeof(double), hipMemcpyDeviceToDevice,
                        ctx->stream));
  const int waves = ctx->ilu_waves;
  const size_t shm = sizeof(double) * (size_t)waves * (ctx->rowmax + 2) * nv * nv;
  RX_NV_SWITCH(nv, (k_ilu_build_part<NV_><<<ctx->npart, 64 * waves, shm, ctx->stream>>>(
                       ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->fs.rows, ctx->col, ctx->klo, ctx->khi, ctx->diag,
                       ctx->f[RX_F_ILU], rx_invd_buf(ctx), ctx->rowmax)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_la_ilu_apply(rx_ctx* ctx, const double* b, double* x, const int* skip) {
  RX_NV_SWITCH(ctx->nVar, (k_ilu_fwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->fs.rows, ctx->col, ctx->klo, ctx->diag,
                              ctx->f[RX_F_ILU], b, x, skip)));
  RX_NV_SWITCH(ctx->nVar, (k_ilu_bwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->bs.part_lvl, ctx->bs.lvl_ptr, ctx->bs.rows, ctx->col, ctx->khi, ctx->diag,
                              ctx->f[RX_F_ILU], rx_invd_buf(ctx), x, skip)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_la_diag_factor(rx_ctx* ctx, const double* A) {
  RX_NV_SWITCH(ctx->nVar, (k_diag_factor<NV_><<<(int)((ctx->N + 3) / 4), 256, 0, ctx->stream>>>(
                              (int)ctx->N, ctx->diag, A, ctx->dlu)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_la_lusgs(rx_ctx* ctx, const double* A, const double* b, double* x, const int* skip) {
  RX_NV_SWITCH(ctx->nVar, (k_lusgs_fwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->fs.rows, ctx->col, ctx->klo, ctx->diag, A,
                              ctx->dlu, b, ctx->xstar, skip)));
  RX_NV_SWITCH(ctx->nVar, (k_lusgs_bwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->bs.part_lvl, ctx->bs.lvl_ptr, ctx->bs.rows, ctx->rp, ctx->col, ctx->klo, ctx->khi,
                              ctx->diag, A, ctx->dlu, ctx->xstar, x, skip)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}
