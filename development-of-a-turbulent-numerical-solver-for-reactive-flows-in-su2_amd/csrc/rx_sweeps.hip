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

#include <type_traits>

#include <algorithm>
#include <cstdlib>

#include "rx_ctx.h"

namespace {

template <int NV>
struct Blk {
  static constexpr int N2 = NV * NV;
};

// LDS-only synchronisation. Lanes of one wavefront exchanging data through LDS need their LDS
// operations complete (lgkmcnt(0)); outstanding global loads (prefetches into registers) are left in
// flight — a fence would also wait vmcnt(0). The empty asm keeps the compiler from moving LDS
// accesses across. lds_barrier() is the same for all waves of the workgroup (s_barrier); it is only
// used where the data shared between waves lives in LDS.
__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// FGMRES hooks of the sweeps: skip when the solve is done; the first kernel of an iteration also
// turns the previous iteration's convergence flag into `done` (rx_krylov.hip).
__device__ __forceinline__ bool skip_sweep(int* done, const int* conv) {
  if (!done) return false;
  if (*done) return true;
  if (conv && *conv) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *done = 1;
    return true;
  }
  return false;
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

// Right-looking form of the same elimination, lane r holding ROW r: for every pivot jj the rows
// ii > jj compute their multiplier LU[ii][jj] / LU[jj][jj] and update LU[ii][kk] -= w * LU[jj][kk]
// (kk > jj) in parallel. Each (ii, jj) step sees exactly the operands of the reference's row-by-row
// loop (row jj is final when pivot jj is used, row ii has had steps 0..jj-1), so the result is bitwise
// the same while the dependent chain shrinks from NV(NV-1)/2 divisions to NV-1.
// On exit row[kk] holds U[r][kk] (kk >= r) or the multiplier w[r][kk] (kk < r).
template <int NV>
__device__ __forceinline__ void wave_factor_rows(double (&row)[NV], int lane) {
#pragma unroll
  for (int jj = 0; jj < NV - 1; ++jj) {
    const double piv = bcast(row[jj], jj);
    const double w = row[jj] / piv;
    if (lane > jj) {
#pragma unroll
      for (int kk = jj + 1; kk < NV; ++kk) row[kk] -= w * bcast(row[kk], jj);
      row[jj] = w;
    }
  }
}

// Solve with a factorisation held as in wave_factor_rows (lane r holds row r); one rhs per lane.
template <int NV>
__device__ __forceinline__ void wave_solve_rows(const double (&row)[NV], double (&rhs)[NV]) {
#pragma unroll
  for (int ii = 1; ii < NV; ++ii)
#pragma unroll
    for (int jj = 0; jj < ii; ++jj) rhs[ii] -= bcast(row[jj], ii) * rhs[jj];
  rhs[NV - 1] = rhs[NV - 1] / bcast(row[NV - 1], NV - 1);
#pragma unroll
  for (int ii = NV - 2; ii >= 0; --ii) {
    double aux = 0.0;
#pragma unroll
    for (int jj = ii + 1; jj < NV; ++jj) aux += bcast(row[jj], ii) * rhs[jj];
    rhs[ii] = (rhs[ii] - aux) / bcast(row[ii], ii);
  }
}

// The same solve with the factorisation in LDS (row-major LU[r][k], written by the lanes of wave_factor_rows):
// every lane reads the entries at one address (LDS broadcast), and those reads do not depend on the solve, so
// they are issued ahead instead of two readlanes per entry.
template <int NV>
__device__ __forceinline__ void wave_solve_lds(const double* LU, double (&rhs)[NV]) {
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
  double row[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) row[k] = lane < NV ? D[lane * NV + k] : 1.0;
  wave_factor_rows<NV>(row, lane);
  if (lane < NV) {
#pragma unroll
    for (int k = 0; k < NV; ++k) LU[(size_t)i * NV * NV + lane * NV + k] = row[k];
  }
}

// ---------------------------------------------------------------------------------------------
// ILU(0) factorisation, one workgroup per partition, one wavefront per row.
// Reads A, writes the factor F (the reference's copy into ILU_matrix is fused). invD receives inv(D_i)
// of every finished row (the reference recomputes exactly this inverse from the same finished block
// whenever it needs it).
//
// Row plan (host-built, rx_ctx_create; one 32-int record per forward-schedule slot):
//   [0] i [1] k0=klo [2] kd=diag [3] k1=khi [4] rp[i] [5] rp[i+1] [6] nlow (-1: use the general plan)
//   [7] npair [8..10] j of the lower blocks k0.. [11..13] update count per lower block
//   [14..31] (kk, pos) pairs: kk = (j, kp) an upper block of row j with kp in row i at BSR index pos,
//   in the reference's loop order (:1421-1443; kp = j is left out: it only touches A_ij, which is
//   then overwritten by W). The general plan is upd_ptr/upd per lower block.
// Per row: its own A blocks and plan were prefetched during the previous row; one round trip stages
// inv(A_jj) and every A_jk it reads from finished rows; the products run from LDS; inv(D_i) is the
// right-looking Gauss elimination with pivot rows broadcast through LDS.
// LDS per wave: row blocks [rowmax][NV2] + W + staging [kStage][NV2] + plan[32].
#ifndef RX_ILU_STAGE
#define RX_ILU_STAGE 6
#endif
constexpr int kStage = RX_ILU_STAGE;
constexpr int kPlan = 32;
constexpr int kPrefA = 10;  // doubles per lane of the next row's A blocks held in registers

// inv(D) of the block in LDS at D (row-major), written to out (global) — Gauss elimination of every
// unit column (InverseDiagonalBlock_ILUMatrix :1180-1228 via Gauss_Elimination :594-643), right-looking
// as wave_factor_rows, pivot rows and the factors exchanged through the LDS scratch L (NV2 doubles).
template <int NV>
__device__ __forceinline__ void wave_inverse_lds(const double* D, double* L, double* __restrict__ out, int lane) {
  constexpr int NV2 = NV * NV;
  double row[NV];
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) row[kk] = lane < NV ? D[lane * NV + kk] : 1.0;
#pragma unroll
  for (int jj = 0; jj < NV - 1; ++jj) {
    if (lane == jj) {
#pragma unroll
      for (int kk = jj; kk < NV; ++kk) L[jj * NV + kk] = row[kk];
    }
    wave_sync();
    const double w = row[jj] / L[jj * NV + jj];
    if (lane > jj && lane < NV) {
#pragma unroll
      for (int kk = jj + 1; kk < NV; ++kk) row[kk] -= w * L[jj * NV + kk];
      row[jj] = w;
    }
    wave_sync();
  }
  if (lane < NV) {
#pragma unroll
    for (int kk = 0; kk < NV; ++kk) L[lane * NV + kk] = row[kk];
  }
  wave_sync();
  // lane c: column c of the inverse
  double rhs[NV];
#pragma unroll
  for (int rr = 0; rr < NV; ++rr) rhs[rr] = (rr == lane) ? 1.0 : 0.0;
#pragma unroll
  for (int ii = 1; ii < NV; ++ii)
#pragma unroll
    for (int jj = 0; jj < ii; ++jj) rhs[ii] -= L[ii * NV + jj] * rhs[jj];
  rhs[NV - 1] = rhs[NV - 1] / L[NV2 - 1];
#pragma unroll
  for (int ii = NV - 2; ii >= 0; --ii) {
    double aux = 0.0;
#pragma unroll
    for (int jj = ii + 1; jj < NV; ++jj) aux += L[ii * NV + jj] * rhs[jj];
    rhs[ii] = (rhs[ii] - aux) / L[ii * NV + ii];
  }
  if (lane < NV) {
#pragma unroll
    for (int rr = 0; rr < NV; ++rr) out[rr * NV + lane] = rhs[rr];
  }
  wave_sync();
}

#ifndef RX_ILU_LB
#define RX_ILU_LB 768  // 12 wavefronts (rx_ilu_max_waves)
#endif
// Staging loads of one row of the ILU(0) build (plan record in prec, lane q of record slot q): inv(A_jj) of its
// nlow lower blocks, then the A_jk blocks of its npair updates, one NV^2 block per stg slot.
template <int NV>
__device__ __forceinline__ void stage_loads(double (&stg)[kStage][(NV * NV + 63) / 64], int prec, int nlow, int npair,
                                            const double* invD, const double* F, int lane) {
  constexpr int NV2 = NV * NV, PER = (NV2 + 63) / 64;
#pragma unroll
  for (int t = 0; t < kStage; ++t) {
    const double* src = nullptr;
    if (t < nlow) src = invD + (size_t)__builtin_amdgcn_readlane(prec, 8 + (t < 3 ? t : 0)) * NV2;
    else if (t < nlow + npair) src = F + (size_t)__builtin_amdgcn_readlane(prec, 14 + 2 * (t - nlow)) * NV2;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int q = lane + 64 * u;
      if (src && q < NV2) stg[t][u] = src[q];
    }
  }
}

template <int NV>
__global__ __launch_bounds__(RX_ILU_LB) void k_ilu_build_part(const int32_t* __restrict__ part_lvl,
                                                         const int32_t* __restrict__ lvl_ptr,
                                                         const int32_t* __restrict__ plan,
                                                         const int32_t* __restrict__ col,
                                                         const int32_t* __restrict__ upd_ptr,
                                                         const int2* __restrict__ upd, const double* __restrict__ A,
                                                         double* __restrict__ F, double* __restrict__ invD,
                                                         int rowmax, long long* __restrict__ trace) {
  constexpr int NV2 = NV * NV;
  constexpr int PA = NV <= 11 ? kPrefA : 8;
  extern __shared__ double lds[];
  // optional phase trace of block 0 (tools/ilu_trace.py): per row of wave w: 5 stamps
  long long* tr = (trace && blockIdx.x == 0 && (threadIdx.x & 63) == 0) ? trace + 1 + (threadIdx.x >> 6) * 5 * 64
                                                                          : nullptr;
  int trow = 0;
#define RX_STAMP(ph)                                                                        \
  do {                                                                                      \
    if (tr && trow < 64) tr[trow * 5 + (ph)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  double* rowbuf = lds + (size_t)wave * ((rowmax + 1 + kStage) * NV2 + kPlan / 2);
  double* Wb = rowbuf + (size_t)rowmax * NV2;
  double* S = Wb + NV2;
  int* rec = reinterpret_cast<int*>(S + kStage * NV2);
  const int p = blockIdx.x;
  const int l0 = part_lvl[p], l1 = part_lvl[p + 1];
  // next row of this wave after slot r of level l (same level, else a later level), -1 if none
  auto next_slot = [&](int r, int l) -> int {
    if (r + nwave < lvl_ptr[l + 1]) return r + nwave;
    for (int ll = l + 1; ll < l1; ++ll)
      if (lvl_ptr[ll] + wave < lvl_ptr[ll + 1]) return lvl_ptr[ll] + wave;
    return -1;
  };
  int pr = -1;  // first slot of this wave
  for (int ll = l0; ll < l1 && pr < 0; ++ll)
    if (lvl_ptr[ll] + wave < lvl_ptr[ll + 1]) pr = lvl_ptr[ll] + wave;
  int prec = 0;
  double pa[PA];
#pragma unroll
  for (int t = 0; t < PA; ++t) pa[t] = 0.0;
  if (pr >= 0) {
    if (lane < kPlan) prec = plan[(size_t)pr * kPlan + lane];
    const int k0 = __builtin_amdgcn_readlane(prec, 1), k1 = __builtin_amdgcn_readlane(prec, 3);
#pragma unroll
    for (int t = 0; t < PA; ++t) {
      const int q = lane + 64 * t;
      if (q < (k1 - k0) * NV2) pa[t] = A[(size_t)k0 * NV2 + q];
    }
  }
  constexpr int PER = (NV2 + 63) / 64;
  double stg[kStage][PER];  // staged inv(A_jj) / A_jk of the row (loaded ahead for a same-level next row)
  bool stg_ready = false;
  for (int l = l0; l < l1; ++l) {
    for (int r = lvl_ptr[l] + wave; r < lvl_ptr[l + 1]; r += nwave) {
      RX_STAMP(0);
      // this row's plan and A blocks (prefetched)
      if (lane < kPlan) rec[lane] = prec;
      const int i = __builtin_amdgcn_readlane(prec, 0), k0 = __builtin_amdgcn_readlane(prec, 1),
                kd = __builtin_amdgcn_readlane(prec, 2), k1 = __builtin_amdgcn_readlane(prec, 3),
                ra = __builtin_amdgcn_readlane(prec, 4), rb = __builtin_amdgcn_readlane(prec, 5),
                nlow = __builtin_amdgcn_readlane(prec, 6), npair = __builtin_amdgcn_readlane(prec, 7);
      const int nbk = k1 - k0;
#pragma unroll
      for (int t = 0; t < PA; ++t) {
        const int q = lane + 64 * t;
        if (q < nbk * NV2) rowbuf[q] = pa[t];
      }
      for (int q = lane + 64 * PA; q < nbk * NV2; q += 64) rowbuf[q] = A[(size_t)k0 * NV2 + q];
      // blocks of the row outside the partition are copied unchanged (SetBlock_ILUMatrix :1378-1389)
      for (int q = lane; q < (k0 - ra) * NV2; q += 64) F[(size_t)ra * NV2 + q] = A[(size_t)ra * NV2 + q];
      for (int q = lane; q < (rb - k1) * NV2; q += 64) F[(size_t)k1 * NV2 + q] = A[(size_t)k1 * NV2 + q];
      const bool fast = nlow >= 0 && nlow + npair <= kStage;
      if (fast) {  // one round trip: inv(A_jj) of every lower block, then the plan's A_jk blocks
        if (!stg_ready) stage_loads<NV>(stg, prec, nlow, npair, invD, F, lane);
#pragma unroll
        for (int t = 0; t < kStage; ++t)
          if (t < nlow + npair) {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
              const int q = lane + 64 * u;
              if (q < NV2) S[t * NV2 + q] = stg[t][u];
            }
          }
      }
      stg_ready = false;
      // prefetch the next row's plan and A blocks (inputs only)
      const int nr = next_slot(r, l);
      if (nr >= 0) {
        if (lane < kPlan) prec = plan[(size_t)nr * kPlan + lane];
        const int nk0 = __builtin_amdgcn_readlane(prec, 1), nk1 = __builtin_amdgcn_readlane(prec, 3);
#pragma unroll
        for (int t = 0; t < PA; ++t) {
          const int q = lane + 64 * t;
          if (q < (nk1 - nk0) * NV2) pa[t] = A[(size_t)nk0 * NV2 + q];
        }
      }
      wave_sync();
      RX_STAMP(1);
      int pcur = 0;
      for (int k = k0; k < kd; ++k) {
        const int t = k - k0;
        const double* Sinv;
        int u0 = 0, u1 = 0;
        if (fast) {
          Sinv = S + (size_t)t * NV2;
        } else {
          const int j = col[k];
          u0 = upd_ptr[k];
          u1 = upd_ptr[k + 1];
          for (int q = lane; q < NV2; q += 64) S[q] = invD[(size_t)j * NV2 + q];
          wave_sync();
          Sinv = S;
        }
        const double* Bij = rowbuf + (size_t)t * NV2;
        // W = A_ij * inv(A_jj)  (MatrixMatrixProduct, sum from 0.0 over q ascending)
        for (int e = lane; e < NV2; e += 64) {
          const int a = e / NV, c = e - a * NV;
          double s = 0.0;
#pragma unroll
          for (int q = 0; q < NV; ++q) s += Bij[a * NV + q] * Sinv[q * NV + c];
          Wb[e] = s;
        }
        wave_sync();
        // A_ik -= A_jk * W (left-multiply quirk), in increasing kk
        const int nu = fast ? rec[11 + t] : (u1 - u0);
        for (int h = 0; h < nu; ++h) {
          const double* Bjk;
          int pos;
          if (fast) {
            Bjk = S + (size_t)(nlow + pcur) * NV2;
            pos = rec[14 + 2 * pcur + 1];
            ++pcur;
          } else {
            const int2 hh = upd[u0 + h];
            wave_sync();
            for (int q = lane; q < NV2; q += 64) S[NV2 + q] = F[(size_t)hh.x * NV2 + q];
            wave_sync();
            Bjk = S + NV2;
            pos = hh.y;
          }
          double* Bik = rowbuf + (size_t)(pos - k0) * NV2;
          for (int e = lane; e < NV2; e += 64) {
            const int a = e / NV, c = e - a * NV;
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < NV; ++q) s += Bjk[a * NV + q] * Wb[q * NV + c];
            Bik[e] -= s;
          }
        }
        wave_sync();
        double* dst = rowbuf + (size_t)t * NV2;
        for (int e = lane; e < NV2; e += 64) dst[e] = Wb[e];
        wave_sync();
      }
      RX_STAMP(2);
      // a next row of the same level depends only on finished levels: its staging loads are issued now and land
      // while this row's inverse runs
      if (nr >= 0 && nr < lvl_ptr[l + 1]) {
        const int nl = __builtin_amdgcn_readlane(prec, 6), np = __builtin_amdgcn_readlane(prec, 7);
        if (nl >= 0 && nl + np <= kStage) {
          stage_loads<NV>(stg, prec, nl, np, invD, F, lane);
          stg_ready = true;
        }
      }
      {  // inv(D_i): right-looking elimination with register broadcasts, then one unit column per lane
        const double* D = rowbuf + (size_t)(kd - k0) * NV2;
        double row[NV];
#pragma unroll
        for (int kk = 0; kk < NV; ++kk) row[kk] = lane < NV ? D[lane * NV + kk] : 1.0;
        wave_factor_rows<NV>(row, lane);
#ifndef RX_ILU_SOLVE_READLANE
        if (lane < NV) {  // the factorisation to LDS (W is free here) for the broadcast solve
#pragma unroll
          for (int kk = 0; kk < NV; ++kk) Wb[lane * NV + kk] = row[kk];
        }
        wave_sync();
#endif
        double rhs[NV];
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) rhs[rr] = (rr == lane) ? 1.0 : 0.0;
#ifndef RX_ILU_SOLVE_READLANE
        wave_solve_lds<NV>(Wb, rhs);
#else
        wave_solve_rows<NV>(row, rhs);
#endif
        if (lane < NV) {
#pragma unroll
          for (int rr = 0; rr < NV; ++rr) invD[(size_t)i * NV2 + rr * NV + lane] = rhs[rr];
        }
      }
      RX_STAMP(3);
      for (int q = lane; q < nbk * NV2; q += 64) F[(size_t)k0 * NV2 + q] = rowbuf[q];
      wave_sync();
      RX_STAMP(4);
      ++trow;
    }
    __syncthreads();
  }
  if (trace && blockIdx.x == 0 && threadIdx.x == 0) trace[0] = (long long)__builtin_amdgcn_s_memtime();
#undef RX_STAMP
}

// ---------------------------------------------------------------------------------------------
// ILU(0) factorisation with four rows per wavefront (round 3; the flow systems, 5 <= NV <= 16).
// A 16-lane group (one DPP row) owns one row of a dependency level; lane c of the group holds COLUMN c of the
// blocks it works on, so every global access of a block is a run of consecutive doubles across the lanes:
//   W = A_ij inv(A_jj):   lane c: W[a][c] = sum_q A_ij[a][q] inv(A_jj)[q][c] with column c of inv(A_jj) in
//                         registers and A_ij in the group's LDS slot (group-uniform, i.e. broadcast, reads);
//   A_ii -= A_ji W:       lane c: column c of W in registers, A_ji in the LDS slot;
//   inv(D_i):             D_i transposed through the slot, wave_factor_rows within the group (pivot row
//                         broadcast by DPP row_newbcast), the factorisation back through the slot, lane c
//                         solving unit column c.
// Every sum is the reference's (from 0.0, q ascending; the elimination of Gauss_Elimination :594-643), so the
// factor is bitwise k_ilu_build_part's. The kernel takes meshes whose lower blocks (at most six per row) each update
// only the diagonal (ctx->ilu_grp_ok: 5-point quad / 7-point hex stencils, i.e. the jet meshes, where no two
// neighbours of a point are neighbours of each other; its row plans ctx->ilu_gplan: [8 + t] the column of lower
// block t, [14 + t] the position of its A_ji); others keep k_ilu_build_part. There ILU(0) changes no upper block and
// no block outside the partition, so those are not copied: the triangular sweeps read the upper blocks from the
// matrix itself (rx_ilu_upper), and rx_download("ILU") materialises the copies (k_ilu_materialize). One level
// is one round of all groups (48 per workgroup), so the rows of a level run concurrently instead of in rounds
// of one row per wavefront.
template <int L>
__device__ __forceinline__ double grp_bcast(double v) {  // lane L of the lane's 16-lane row
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, 0x150 + L, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0x150 + L, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// wave_factor_rows within a 16-lane group: lane a holds row a. The broadcasts run on every lane (DPP reads a
// source lane that must be active), the update only on the rows below the pivot.
template <int NV, int JJ = 0>
__device__ __forceinline__ void grp_factor_rows(double (&d)[NV], int a) {
  if constexpr (JJ < NV - 1) {
    double pr[NV];
#pragma unroll
    for (int kk = JJ; kk < NV; ++kk) pr[kk] = grp_bcast<JJ>(d[kk]);
    const double w = d[JJ] / pr[JJ];
    if (a > JJ) {
#pragma unroll
      for (int kk = JJ + 1; kk < NV; ++kk) d[kk] -= w * pr[kk];
      d[JJ] = w;
    }
    grp_factor_rows<NV, JJ + 1>(d, a);
  }
}

// Row offset of an LDS operand, tied to a value computed two rows earlier: the reads of row ii cannot be issued
// before `dep` exists, so an unrolled product / solve keeps about two rows of operands in flight instead of
// issuing all NV^2 reads up front (which spills).
__device__ __forceinline__ int lds_row(int off, double dep) {
  asm volatile("" : "+v"(off) : "v"(dep));
  return off;
}
// The same tied to every accumulator of a block product: row q's operand reads wait for row q-1's updates of all
// NV accumulators (tied to one of them, the compiler finishes that one chain first and defers the others).
template <int NV>
__device__ __forceinline__ int lds_row_tied(int off, const double (&v)[NV]) {
#pragma unroll
  for (int c = 0; c < NV; ++c) asm volatile("" : "+v"(off) : "v"(v[c]));
  return off;
}

// acc[e] += S[q + e NV] * v[q] for q ascending (a block product's column, the reference's order: sums from the
// accumulator, q ascending) with row q + 1's LDS reads issued before row q's products: they are tied to the
// accumulators after row q - 1, so one row of operands is in flight (the reads are not all hoisted, which spills) and
// the LDS latency of a row hides behind the previous row's products instead of adding to them.
template <int NV>
__device__ __forceinline__ void lds_colprod(const double* S, const double (&v)[NV], double (&acc)[NV]) {
  double cur[NV];
  {
    const int o = lds_row_tied<NV>(0, acc);
#pragma unroll
    for (int e = 0; e < NV; ++e) cur[e] = S[o + e * NV];
  }
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double nxt[NV];
    if (q + 1 < NV) {
      const int o = lds_row_tied<NV>(q + 1, acc);
#pragma unroll
      for (int e = 0; e < NV; ++e) nxt[e] = S[o + e * NV];
    }
#pragma unroll
    for (int e = 0; e < NV; ++e) acc[e] += cur[e] * v[q];
    if (q + 1 < NV) {
#pragma unroll
      for (int e = 0; e < NV; ++e) cur[e] = nxt[e];
    }
  }
}

// wave_solve_lds with the factorisation stored at row stride NP.
template <int NV, int NP>
__device__ __forceinline__ void grp_solve_lds(const double* LU, double (&rhs)[NV]) {
#pragma unroll
  for (int ii = 1; ii < NV; ++ii) {
    const int o = lds_row(ii * NP, rhs[ii >= 2 ? ii - 2 : 0]);
#pragma unroll
    for (int jj = 0; jj < ii; ++jj) rhs[ii] -= LU[o + jj] * rhs[jj];
  }
  rhs[NV - 1] = rhs[NV - 1] / LU[(NV - 1) * NP + NV - 1];
#pragma unroll
  for (int ii = NV - 2; ii >= 0; --ii) {
    const int o = lds_row(ii * NP, rhs[ii + 2 < NV ? ii + 2 : NV - 1]);
    double aux = 0.0;
#pragma unroll
    for (int jj = ii + 1; jj < NV; ++jj) aux += LU[o + jj] * rhs[jj];
    rhs[ii] = (rhs[ii] - aux) / LU[o + ii];
  }
}

// Wavefronts per workgroup: 12 (3 per SIMD, 168 VGPRs) for blocks up to 9x9; 8 (256 VGPRs) for larger blocks, whose
// prefetched next-row blocks spill at 168 (C3, 11x11: 3.59 ms with 12 waves before the prefetch, 4.34 ms with it
// and 31 spills, 3.21 ms with 8 waves).
#ifndef RX_GRP_WAVES
#define RX_GRP_WAVES 12
#endif
// build knob: 1 = the grouped build stores each row's eliminated diagonal block D_i in the factor (ILU_matrix's
// diagonal); 0 (default, round 5) = it does not — no sweep reads it (they read inv(D_i)) — and a download of the ILU
// field remakes it from the matrix and the stored W blocks with the build's arithmetic (k_ilu_diag_materialize)
#ifndef RX_GRP_DIAG_STORE
#define RX_GRP_DIAG_STORE 0
#endif
#ifndef RX_GRP_WAVES_BIG
#define RX_GRP_WAVES_BIG 8
#endif
// timing probe (build variants only; wrong numerics): bit 0 = every inv(A_jj) load reads row 0's block (an L1/L2 hit
// instead of the block a group of the previous level just stored), bit 1 = the second and later lower blocks' A_ij /
// A_ji loads read block 0
#ifndef RX_GRP_PROBE
#define RX_GRP_PROBE 0
#endif
constexpr int kGrpMaxWaves = RX_GRP_WAVES > RX_GRP_WAVES_BIG ? RX_GRP_WAVES : RX_GRP_WAVES_BIG;
template <int NV>
constexpr int grp_waves() { return NV >= 10 ? RX_GRP_WAVES_BIG : RX_GRP_WAVES; }
constexpr int kGrpTraceRows = 64, kGrpTraceGroups = 64, kGrpTraceLevels = 512;  // >= 4 * kGrpMaxWaves groups
template <int NV>
constexpr int grp_np() { return (NV + 1) & ~1; }
template <int NV>
constexpr int grp_slot_doubles() { return NV * grp_np<NV>() + kPlan; }  // + two plan records (this row, the next)

// Round 6: an LDS ring of inv(D) (ring_w rows per level parity; the host plan's [6] / [20 + t] slots). A row stores its
// inv(D_i) to the ring besides the factor, and a row of the next level reads its lower blocks' inv(A_jj) from there
// instead of from memory. A level none of whose rows reads an inv(A_jj) from memory (gfull[l] = 0) is then entered
// through an LDS barrier: the global stores of the level before (W, inv(D)) no longer have to be acknowledged first
// (__syncthreads waits vmcnt(0)), and no inv(A_jj) load queues behind them (vmcnt retires in issue order). A level
// with such a row (its lower neighbour two or more levels back, or past the ring's width) keeps the full barrier.
// The same values in the same operations: the factor is bitwise the same.
// PAIR (round 6): two groups per row — lane group 2q + role of the workgroup takes row slot q, group `role` makes
// lower block `role` (W = A_ij inv(A_jj), X = A_ji W) and the helper hands its X to the primary through its LDS slot,
// which subtracts X_0 then X_1 from D_i in the reference's order and factors D_i alone. The two blocks' products run
// side by side instead of one after the other (the row's chain is its LDS / FP64 latency, not its loads), for half as
// many rows per round: the host takes it for the meshes whose rows have at most two lower blocks and whose widest level
// a round of the pairs covers in at most a few rounds (ctx->ilu_pair, rx_api.hip). The same operations on the same
// values: the factor is bitwise the same.
template <int NV, bool PAIR>
__global__ __launch_bounds__(64 * grp_waves<NV>()) void k_ilu_build_grp(const int32_t* __restrict__ part_lvl,
                                                                    const int32_t* __restrict__ lvl_ptr,
                                                                    const int32_t* __restrict__ plan,
                                                                    const double* __restrict__ A,
                                                                    double* __restrict__ F, double* __restrict__ invD,
                                                                    long long* __restrict__ trace,
                                                                    const int32_t* __restrict__ gfull, int ring_w) {
  constexpr int NV2 = NV * NV, NP = grp_np<NV>();
  extern __shared__ double lds[];
  const int a = threadIdx.x & 15, grp = threadIdx.x >> 4, ngrp = blockDim.x >> 4;
  const int role = PAIR ? (grp & 1) : 0, gslot = PAIR ? (grp >> 1) : grp, nslot = PAIR ? (ngrp >> 1) : ngrp;
  double* S = lds + (size_t)grp * grp_slot_doubles<NV>();  // inv(A_jj), then W, then the LU of D_i
  int* const recb = reinterpret_cast<int*>(S + NV * NP);   // plan records: this row's and the next row's
  const int p = blockIdx.x, l0 = part_lvl[p], l1 = part_lvl[p + 1];
  // the inv(D) ring behind the group slots, then the partition's level pointers: the loop bounds and the next-row
  // search read them every row
  double* ring = lds + (size_t)ngrp * grp_slot_doubles<NV>();
  int* lp = reinterpret_cast<int*>(ring + (size_t)2 * ring_w * NV2) - l0;
  for (int l = l0 + (int)threadIdx.x; l <= l1; l += blockDim.x) lp[l] = lvl_ptr[l];
  __syncthreads();
  auto next_slot = [&](int r, int l, int& ln) -> int {  // the group's next row after slot r of level l (its level
    if (r + nslot < lp[l + 1]) {                        // in ln), -1 if none
      ln = l;
      return r + nslot;
    }
    for (int ll = l + 1; ll < l1; ++ll)
      if (lp[ll] + gslot < lp[ll + 1]) {
        ln = ll;
        return lp[ll] + gslot;
      }
    return -1;
  };
  constexpr int PB = (NV2 + 15) / 16;  // doubles per lane of a block loaded lane-contiguously
  // The A blocks a row reads first — its diagonal (column per lane), its first lower block A_ij and that block's
  // A_ji — are inputs, so they are loaded for the group's NEXT row while this row factors its diagonal: plain loads
  // stay in flight across the level barrier. Only inv(A_jj) (a row of an earlier level) waits for the barrier.
  auto prefetch = [&](const int* rc, int lane, double (&pd)[NV], double (&pbl)[PB], double (&pjl)[PB]) {
    const int pc = lane < NV ? lane : 0;
    const int pk0 = rc[1] + role, pkd = rc[2];  // (PAIR: the helper's block is the row's second)
#pragma unroll
    for (int q = 0; q < NV; ++q) pd[q] = A[(size_t)pkd * NV2 + q * NV + pc];
    if (pkd > pk0) {
#pragma unroll
      for (int u = 0; u < PB; ++u)
        if (16 * u + lane < NV2) pbl[u] = A[(size_t)pk0 * NV2 + 16 * u + lane];
      if (rc[14 + role] >= 0) {
#pragma unroll
        for (int u = 0; u < PB; ++u)
          if (16 * u + lane < NV2) pjl[u] = A[(size_t)rc[14 + role] * NV2 + 16 * u + lane];
      }
    }
  };
  // the second lower block and its A_ji (issued at the row start with both inv(A_jj))
  auto load_second = [&](const int* rc, int lane, double (&pbl2)[PB], double (&pjl2)[PB]) {
    const int pk0 = rc[1], pkd = rc[2];
    if (pkd > pk0 + 1) {
#pragma unroll
      for (int u = 0; u < PB; ++u)
        if (16 * u + lane < NV2) pbl2[u] = A[(size_t)(pk0 + 1) * NV2 + 16 * u + lane];
      if (rc[15] >= 0) {
        const int kk = rc[15];
#pragma unroll
        for (int u = 0; u < PB; ++u)
          if (16 * u + lane < NV2) pjl2[u] = A[(size_t)kk * NV2 + 16 * u + lane];
      }
    }
  };
  double d[NV], bl[PB], jl[PB];  // the current row's prefetched blocks
  int2 prec = make_int2(0, 0);   // the plan of the group's row after the current one
  int cur = 0;                   // recb slot of the current row's plan
  {
    int pr = -1, pl = 0;
    for (int ll = l0; ll < l1 && pr < 0; ++ll)
      if (lp[ll] + gslot < lp[ll + 1]) {
        pr = lp[ll] + gslot;
        pl = ll;
      }
    if (pr >= 0) {
      reinterpret_cast<int2*>(recb)[a] = reinterpret_cast<const int2*>(plan + (size_t)pr * kPlan)[a];
      wave_sync();
      prefetch(recb, a, d, bl, jl);
      int ln;
      const int nr = next_slot(pr, pl, ln);
      if (nr >= 0) prec = reinterpret_cast<const int2*>(plan + (size_t)nr * kPlan)[a];
    }
  }
  // optional phase trace of block 0 (tools/ilu_trace.py --grp): per group, per row 4 stamps; then one per level
  long long* tr = (trace && blockIdx.x == 0 && a == 0) ? trace + 1 + (size_t)grp * kGrpTraceRows * 8 : nullptr;
  int trow = 0;
#define RX_GSTAMP(ph)                                                                             \
  do {                                                                                            \
    if (tr && trow < kGrpTraceRows) tr[trow * 8 + (ph)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
  for (int l = l0; l < l1; ++l) {
    for (int r = lp[l] + gslot; r < lp[l + 1]; r += nslot) {
      RX_GSTAMP(0);
      // the lane's column, laundered per row so that nothing derived from it is hoisted out of the row loop
      // (the hoisted unit vectors / addresses otherwise spill)
      int al = a;
      asm volatile("" : "+v"(al));
      const bool act = al < NV;
      const int ac = act ? al : 0;  // lanes NV..15 of a group load column 0 and store nothing
      const int* rec = recb + cur * kPlan;
      int nl = l;
      const int nr = next_slot(r, l, nl);  // the group's next row (its plan is in prec)
      const int i = rec[0], k0 = rec[1], kd = rec[2];
      // the first two lower blocks' inv(A_jj) (finished rows) and the second block's A_ij / A_ji; d and the first
      // block's A_ij / A_ji were prefetched
      double s[NV], s2[NV], bl2[PB], jl2[PB];
#ifdef RX_GRP_EARLY2
      load_second(rec, al, bl2, jl2);
#endif
      const int rs_own = rec[6];
      if (kd > k0 + role) {
        const int j0 = (RX_GRP_PROBE & 1) ? 0 : rec[8 + role], rs0 = rec[20 + role];
        if (rs0 >= 0) {
#pragma unroll
          for (int q = 0; q < NV; ++q) s[q] = ring[(size_t)rs0 * NV2 + q * NV + ac];
        } else {
#pragma unroll
          for (int q = 0; q < NV; ++q) s[q] = invD[(size_t)j0 * NV2 + q * NV + ac];
        }
      }
#ifdef RX_GRP_EARLY2
      if (kd > k0 + 1) {
        const int j1 = rec[9];
#pragma unroll
        for (int q = 0; q < NV; ++q) s2[q] = invD[(size_t)j1 * NV2 + q * NV + ac];
      }
#endif
      constexpr int kstep = PAIR ? 2 : 1;  // PAIR: the primary takes blocks 0, 2, .., the helper 1, 3, ..
      for (int k = k0 + role; k < kd; k += kstep) {
        const int t = k - k0, nu = rec[14 + t] >= 0 ? 1 : 0;
        wave_sync();
#pragma unroll
        for (int u = 0; u < PB; ++u)
          if (16 * u + al < NV2) S[16 * u + al] = bl[u];  // A_ij, row-major (stride NV)
        wave_sync();
        if (t < 2) RX_GSTAMP(4 + 2 * t);
        // W = A_ij * inv(A_jj)  (MatrixMatrixProduct, sum from 0.0 over q ascending): column c of W
        double w[NV];
#pragma unroll
        for (int e = 0; e < NV; ++e) w[e] = 0.0;
#ifdef RX_GRP_TIED1  // A/B: each row's reads wait for the previous row's products
#pragma unroll
        for (int q = 0; q < NV; ++q) {
          const int o = lds_row_tied<NV>(q, w);
#pragma unroll
          for (int e = 0; e < NV; ++e) w[e] += S[o + e * NV] * s[q];
        }
#else
        lds_colprod<NV>(S, s, w);
#endif
        if (t < 2) RX_GSTAMP(5 + 2 * t);
        wave_sync();
        if (nu > 0) {
#pragma unroll
          for (int u = 0; u < PB; ++u)
            if (16 * u + al < NV2) S[16 * u + al] = jl[u];  // A_ji
        }
        wave_sync();
#ifndef RX_GRP_EARLY2
        if (false) {
#else
        if (t == 0 && k + 1 < kd) {  // the second block: loaded at the row start
#endif
#pragma unroll
          for (int q = 0; q < NV; ++q) s[q] = s2[q];
#pragma unroll
          for (int u = 0; u < PB; ++u) {
            bl[u] = bl2[u];
            jl[u] = jl2[u];
          }
        } else if (k + kstep < kd) {  // further lower blocks' loads (not on quad / hex meshes), into the registers
                                       // just freed (before W's store, so that waiting for them does not wait for it)
          const int tn = t + kstep;
          const int jn = (RX_GRP_PROBE & 1) ? 0 : rec[8 + tn], rsn = rec[20 + tn];
          if (rsn >= 0) {
#pragma unroll
            for (int q = 0; q < NV; ++q) s[q] = ring[(size_t)rsn * NV2 + q * NV + ac];
          } else {
#pragma unroll
            for (int q = 0; q < NV; ++q) s[q] = invD[(size_t)jn * NV2 + q * NV + ac];
          }
          const size_t kb = (RX_GRP_PROBE & 2) ? 0 : (size_t)(k + kstep);
#pragma unroll
          for (int u = 0; u < PB; ++u)
            if (16 * u + al < NV2) bl[u] = A[kb * NV2 + 16 * u + al];
          if (rec[14 + tn] >= 0) {
            const int kk = (RX_GRP_PROBE & 2) ? 0 : rec[14 + tn];
#pragma unroll
            for (int u = 0; u < PB; ++u)
              if (16 * u + al < NV2) jl[u] = A[(size_t)kk * NV2 + 16 * u + al];
          }
        }
        if (act) {
#pragma unroll
          for (int e = 0; e < NV; ++e) F[(size_t)k * NV2 + e * NV + al] = w[e];
        }
        // D_i -= A_ji * W (left-multiply quirk; the block's one update hits the diagonal)
        double x[NV];
        if (nu > 0) {
#pragma unroll
          for (int e = 0; e < NV; ++e) x[e] = 0.0;
#ifdef RX_GRP_TIED1
#pragma unroll
          for (int q = 0; q < NV; ++q) {
            const int o = lds_row_tied<NV>(q, x);
#pragma unroll
            for (int e = 0; e < NV; ++e) x[e] += S[o + e * NV] * w[q];
          }
#else
          lds_colprod<NV>(S, w, x);
#endif
          if (!PAIR) {
#pragma unroll
            for (int e = 0; e < NV; ++e) d[e] -= x[e];
          }
        }
        if (PAIR) {  // blocks t (primary) and t + 1 (helper): the helper's X to its slot, the primary subtracts its
                     // own X, then the helper's — the reference's block order
          wave_sync();
          if (role == 1 && nu > 0 && act) {
#pragma unroll
            for (int e = 0; e < NV; ++e) S[e * NV + al] = x[e];
          }
          wave_sync();
          if (role == 0) {
            if (nu > 0) {
#pragma unroll
              for (int e = 0; e < NV; ++e) d[e] -= x[e];
            }
            if (k + 1 < kd && rec[15 + t] >= 0) {
              const double* Sh = S + grp_slot_doubles<NV>();  // the partner's (helper's) slot
#pragma unroll
              for (int e = 0; e < NV; ++e) d[e] -= Sh[e * NV + ac];
            }
          }
        }
      }
      if (act && role == 0 && RX_GRP_DIAG_STORE) {  // (the sweeps read inv(D_i) only: rx_la_ilu_materialize remakes D_i)
#pragma unroll
        for (int e = 0; e < NV; ++e) F[(size_t)kd * NV2 + e * NV + al] = d[e];
      }
      RX_GSTAMP(1);
      // inv(D_i): D_i transposed through the slot (lane a then holds row a), the right-looking elimination in the
      // group, the factorisation back to the slot, one unit column per lane
      wave_sync();
      if (act) {
#pragma unroll
        for (int e = 0; e < NV; ++e) S[e * NP + al] = d[e];
      }
      // the next row's plan into the other record, its input blocks into d / bl / jl (dead from here on), and the
      // plan of the row after it
      int* nrec = recb + (cur ^ 1) * kPlan;
      reinterpret_cast<int2*>(nrec)[al] = prec;
      wave_sync();
      if (nr >= 0) {
        prefetch(nrec, al, d, bl, jl);
        int nnl;
        const int nnr = next_slot(nr, nl, nnl);
        if (nnr >= 0) prec = reinterpret_cast<const int2*>(plan + (size_t)nnr * kPlan)[al];
      }
      cur ^= 1;
      double rw[NV];
#pragma unroll
      for (int e = 0; e < NV; ++e) rw[e] = S[ac * NP + e];
      grp_factor_rows<NV>(rw, al);
      RX_GSTAMP(2);
      wave_sync();
      if (act) {
#pragma unroll
        for (int e = 0; e < NV; ++e) S[al * NP + e] = rw[e];
      }
      wave_sync();
      double rhs[NV];
#pragma unroll
      for (int rr = 0; rr < NV; ++rr) rhs[rr] = (rr == al) ? 1.0 : 0.0;
      grp_solve_lds<NV, NP>(S, rhs);
      if (act && role == 0) {
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) invD[(size_t)i * NV2 + rr * NV + al] = rhs[rr];
        if (rs_own >= 0) {
#pragma unroll
          for (int rr = 0; rr < NV; ++rr) ring[(size_t)rs_own * NV2 + rr * NV + al] = rhs[rr];
        }
      }
      RX_GSTAMP(3);
      ++trow;
    }
    if (l + 1 >= l1 || gfull[l + 1]) {
      __syncthreads();
    } else {  // the next level reads inv(A_jj) from the ring only: an LDS barrier
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    if (trace && blockIdx.x == 0 && threadIdx.x == 0 && l - l0 < kGrpTraceLevels)
      trace[1 + kGrpTraceGroups * kGrpTraceRows * 8 + (l - l0)] = (long long)__builtin_amdgcn_s_memtime();
  }
  if (trace && blockIdx.x == 0 && threadIdx.x == 0) trace[0] = (long long)__builtin_amdgcn_s_memtime();
#undef RX_GSTAMP
}

// ILU(0) factorisation for small blocks (NV <= 4, the SST system's 2x2): one thread per row, rows of a
// dependency level spread over the workgroup. Same arithmetic as k_ilu_build_part: W = A_ij inv(A_jj)
// (sums from 0.0, q ascending), A_ik -= A_jk W over the update plan in the reference's order, then
// inv(D_i) by Gauss elimination of every unit column (the factor computed once, left-looking per row:
// each (ii, jj) step sees the operands of Gauss_Elimination :594-643). The thread updates its row in F
// directly; rows of later levels read finished rows after the level barrier.
template <int NV>
__global__ __launch_bounds__(256) void k_ilu_build_small(const int32_t* __restrict__ part_lvl,
                                                         const int32_t* __restrict__ lvl_ptr,
                                                         const int4* __restrict__ slot,
                                                         const int32_t* __restrict__ rp,
                                                         const int32_t* __restrict__ col,
                                                         const int32_t* __restrict__ upd_ptr,
                                                         const int2* __restrict__ upd, const double* __restrict__ A,
                                                         double* __restrict__ F, double* __restrict__ invD) {
  constexpr int NV2 = NV * NV;
  const int p = blockIdx.x;
  for (int l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
    for (int r = lvl_ptr[l] + threadIdx.x; r < lvl_ptr[l + 1]; r += blockDim.x) {
      const int4 sl = slot[r];
      const int i = sl.x, k0 = sl.y, kd = sl.z, k1 = sl.w;
      const int ra = rp[i], rb = rp[i + 1];
      for (int q = ra * NV2; q < rb * NV2; ++q) F[q] = A[q];
      for (int k = k0; k < kd; ++k) {
        const int j = col[k];
        double Sinv[NV2], Bij[NV2], W[NV2];
#pragma unroll
        for (int q = 0; q < NV2; ++q) {
          Sinv[q] = invD[(size_t)j * NV2 + q];
          Bij[q] = F[(size_t)k * NV2 + q];
        }
#pragma unroll
        for (int a = 0; a < NV; ++a)
#pragma unroll
          for (int c = 0; c < NV; ++c) {
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < NV; ++q) s += Bij[a * NV + q] * Sinv[q * NV + c];
            W[a * NV + c] = s;
          }
        for (int u = upd_ptr[k]; u < upd_ptr[k + 1]; ++u) {
          const int2 h = upd[u];
          double Bjk[NV2];
#pragma unroll
          for (int q = 0; q < NV2; ++q) Bjk[q] = F[(size_t)h.x * NV2 + q];
          double* Bik = F + (size_t)h.y * NV2;
#pragma unroll
          for (int a = 0; a < NV; ++a)
#pragma unroll
            for (int c = 0; c < NV; ++c) {
              double s = 0.0;
#pragma unroll
              for (int q = 0; q < NV; ++q) s += Bjk[a * NV + q] * W[q * NV + c];
              Bik[a * NV + c] -= s;
            }
        }
#pragma unroll
        for (int q = 0; q < NV2; ++q) F[(size_t)k * NV2 + q] = W[q];
      }
      double L[NV2];
#pragma unroll
      for (int q = 0; q < NV2; ++q) L[q] = F[(size_t)kd * NV2 + q];
#pragma unroll
      for (int ii = 1; ii < NV; ++ii)
#pragma unroll
        for (int jj = 0; jj < ii; ++jj) {
          const double w = L[ii * NV + jj] / L[jj * NV + jj];
#pragma unroll
          for (int kk = jj + 1; kk < NV; ++kk) L[ii * NV + kk] -= w * L[jj * NV + kk];
          L[ii * NV + jj] = w;
        }
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        double rhs[NV];
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) rhs[rr] = (rr == c) ? 1.0 : 0.0;
        lu_solve<NV>(L, rhs);
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) invD[(size_t)i * NV2 + rr * NV + c] = rhs[rr];
      }
    }
    __syncthreads();
  }
}

// 2x2 fast path of k_ilu_build_small driven by the compact row plan (ilu_plan, nlow <= 3, npair <= 9): every
// load a row needs (its A blocks, inv(D_j) of its lower neighbours, the A_jk of the plan) is issued at once,
// the row lives in registers (runtime block indices resolved by selects), and the row is stored once. Rows
// without a compact plan take the general per-block path. Same arithmetic as k_ilu_build_small.
constexpr int kSmallMaxB = 12;
__global__ __launch_bounds__(256) void k_ilu_build_2(const int32_t* __restrict__ part_lvl,
                                                     const int32_t* __restrict__ lvl_ptr,
                                                     const int32_t* __restrict__ plan, const int4* __restrict__ slot,
                                                     const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                     const int32_t* __restrict__ upd_ptr,
                                                     const int2* __restrict__ upd, const double* __restrict__ A,
                                                     double* __restrict__ F, double* __restrict__ invD,
                                                     bool diag_regs, const int32_t* __restrict__ gplan) {
  constexpr int NV = 2, NV2 = 4;
  const int p = blockIdx.x;
  for (int l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
    for (int r = lvl_ptr[l] + threadIdx.x; r < lvl_ptr[l + 1]; r += blockDim.x) {
      const int4* pr = reinterpret_cast<const int4*>(plan + (size_t)r * 32);
      int rec[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int4 v = pr[q];
        rec[4 * q] = v.x;
        rec[4 * q + 1] = v.y;
        rec[4 * q + 2] = v.z;
        rec[4 * q + 3] = v.w;
      }
      const int i = rec[0], k0 = rec[1], kd = rec[2], k1 = rec[3], ra = rec[4], rb = rec[5];
      const int nlow = rec[6], npair = rec[7], nbk = k1 - k0;
      double L[NV2];
      bool have_d = false;  // the factored D_i still in registers (register path): no reload of what was just stored
      for (int q = ra * NV2; q < k0 * NV2; ++q) F[q] = A[q];
      for (int q = k1 * NV2; q < rb * NV2; ++q) F[q] = A[q];
      if (nlow < 0 && gplan) {
        // more lower blocks than the compact plan holds (3-D: four at C5), on a mesh whose lower blocks each update
        // only the diagonal (k_ilu_build_grp's plan): the general path's arithmetic, block by block
        const int32_t* g = gplan + (size_t)r * 32;
        for (int q = (kd + 1) * NV2; q < k1 * NV2; ++q) F[q] = A[q];
        double D[NV2];
#pragma unroll
        for (int q = 0; q < NV2; ++q) D[q] = A[(size_t)kd * NV2 + q];
        for (int k = k0; k < kd; ++k) {
          const int t = k - k0, kk = g[14 + t];
          double Sinv[NV2], Bij[NV2], W[NV2];
#pragma unroll
          for (int q = 0; q < NV2; ++q) {
            Sinv[q] = invD[(size_t)g[8 + t] * NV2 + q];
            Bij[q] = A[(size_t)k * NV2 + q];
          }
#pragma unroll
          for (int a = 0; a < NV; ++a)
#pragma unroll
            for (int c = 0; c < NV; ++c) {
              double sm = 0.0;
#pragma unroll
              for (int q = 0; q < NV; ++q) sm += Bij[a * NV + q] * Sinv[q * NV + c];
              W[a * NV + c] = sm;
            }
          if (kk >= 0) {
            const double* Bjk = F + (size_t)kk * NV2;
#pragma unroll
            for (int a = 0; a < NV; ++a)
#pragma unroll
              for (int c = 0; c < NV; ++c) {
                double sm = 0.0;
#pragma unroll
                for (int q = 0; q < NV; ++q) sm += Bjk[a * NV + q] * W[q * NV + c];
                D[a * NV + c] -= sm;
              }
          }
#pragma unroll
          for (int q = 0; q < NV2; ++q) F[(size_t)k * NV2 + q] = W[q];
        }
#pragma unroll
        for (int q = 0; q < NV2; ++q) {
          F[(size_t)kd * NV2 + q] = D[q];
          L[q] = D[q];
        }
        have_d = true;
      } else if (nlow < 0 || nbk > kSmallMaxB) {  // general per-block path
        for (int q = k0 * NV2; q < k1 * NV2; ++q) F[q] = A[q];
        for (int k = k0; k < kd; ++k) {
          const int j = col[k];
          double Sinv[NV2], Bij[NV2], W[NV2];
#pragma unroll
          for (int q = 0; q < NV2; ++q) {
            Sinv[q] = invD[(size_t)j * NV2 + q];
            Bij[q] = F[(size_t)k * NV2 + q];
          }
#pragma unroll
          for (int a = 0; a < NV; ++a)
#pragma unroll
            for (int c = 0; c < NV; ++c) {
              double sm = 0.0;
#pragma unroll
              for (int q = 0; q < NV; ++q) sm += Bij[a * NV + q] * Sinv[q * NV + c];
              W[a * NV + c] = sm;
            }
          for (int u = upd_ptr[k]; u < upd_ptr[k + 1]; ++u) {
            const int2 h = upd[u];
            double* Bik = F + (size_t)h.y * NV2;
            const double* Bjk = F + (size_t)h.x * NV2;
#pragma unroll
            for (int a = 0; a < NV; ++a)
#pragma unroll
              for (int c = 0; c < NV; ++c) {
                double sm = 0.0;
#pragma unroll
                for (int q = 0; q < NV; ++q) sm += Bjk[a * NV + q] * W[q * NV + c];
                Bik[a * NV + c] -= sm;
              }
          }
#pragma unroll
          for (int q = 0; q < NV2; ++q) F[(size_t)k * NV2 + q] = W[q];
        }
      } else {
        double B[kSmallMaxB][NV2], S[3][NV2], J[9][NV2];
#pragma unroll
        for (int b = 0; b < kSmallMaxB; ++b)
          if (b < nbk)
#pragma unroll
            for (int q = 0; q < NV2; ++q) B[b][q] = A[(size_t)(k0 + b) * NV2 + q];
#pragma unroll
        for (int t = 0; t < 3; ++t)
          if (t < nlow)
#pragma unroll
            for (int q = 0; q < NV2; ++q) S[t][q] = invD[(size_t)rec[8 + t] * NV2 + q];
#pragma unroll
        for (int u = 0; u < 9; ++u)
          if (u < npair)
#pragma unroll
            for (int q = 0; q < NV2; ++q) J[u][q] = F[(size_t)rec[14 + 2 * u] * NV2 + q];
        int pc = 0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          if (t < nlow) {
            double W[NV2];
#pragma unroll
            for (int a = 0; a < NV; ++a)
#pragma unroll
              for (int c = 0; c < NV; ++c) {
                double sm = 0.0;
#pragma unroll
                for (int q = 0; q < NV; ++q) sm += B[t][a * NV + q] * S[t][q * NV + c];
                W[a * NV + c] = sm;
              }
            const int nu = rec[11 + t];
#pragma unroll
            for (int u = 0; u < 9; ++u) {
              if (u >= pc && u < pc + nu) {
                const int pos = rec[14 + 2 * u + 1] - k0;
                double prod[NV2];
#pragma unroll
                for (int a = 0; a < NV; ++a)
#pragma unroll
                  for (int c = 0; c < NV; ++c) {
                    double sm = 0.0;
#pragma unroll
                    for (int q = 0; q < NV; ++q) sm += J[u][a * NV + q] * W[q * NV + c];
                    prod[a * NV + c] = sm;
                  }
#pragma unroll
                for (int b = 0; b < kSmallMaxB; ++b)
                  if (b == pos)
#pragma unroll
                    for (int q = 0; q < NV2; ++q) B[b][q] -= prod[q];
              }
            }
            pc += nu;
#pragma unroll
            for (int q = 0; q < NV2; ++q) B[t][q] = W[q];
          }
        }
#pragma unroll
        for (int b = 0; b < kSmallMaxB; ++b)
          if (b < nbk) {
#pragma unroll
            for (int q = 0; q < NV2; ++q) F[(size_t)(k0 + b) * NV2 + q] = B[b][q];
            if (diag_regs && b == kd - k0) {
#pragma unroll
              for (int q = 0; q < NV2; ++q) L[q] = B[b][q];
              have_d = true;
            }
          }
      }
      // inv(D_i) (Gauss elimination per unit column, factor once)
      if (!have_d) {
#pragma unroll
        for (int q = 0; q < NV2; ++q) L[q] = F[(size_t)kd * NV2 + q];
      }
      {
        const double w = L[2] / L[0];
        L[3] -= w * L[1];
        L[2] = w;
      }
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        double rhs[NV] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0};
        lu_solve<NV>(L, rhs);
        invD[(size_t)i * NV2 + c] = rhs[0];
        invD[(size_t)i * NV2 + NV + c] = rhs[1];
      }
    }
    __syncthreads();
  }
}

// The SST's 2x2 ILU(0) on triangle-free meshes (ctx->ilu_grp_ok: every lower block A_ij updates only the diagonal,
// D_i = A_ii - sum_t A_ji (A_ij inv(D_j)), k_ilu_build_2's gplan branch), one wavefront per partition (VERDICT r03
// #7). k_ilu_build_2 ran one thread per row on 256-thread workgroups: a level's ~27 rows are one wavefront, whose
// per-row instruction stream (compact plans with runtime block positions resolved by selects) and the global
// round trips of inv(D_j) set the time (0.87 ms at C3 for ~146 levels). Here:
//   * the pass's rows (<= 64 rows of one level, the schedule's pass table) are the wavefront's lanes, so no
//     barrier is needed: a later pass of the same wavefront sees this pass's LDS stores;
//   * inv(D_j) of the partition's rows stays in LDS (partition-local index, 32 B per row), written by the pass that
//     factors row j and read by the passes of its lower neighbours' rows;
//   * every load a pass needs is an input (its plan, A_ii, A_ij, A_ji), so the plan of pass q + 2 and the blocks of
//     pass q + 1 are issued before pass q is computed (all loads unconditional, from clamped valid addresses, so
//     the wait counts stay static);
//   * the upper blocks and the blocks outside the partition are the matrix's own and are neither copied nor
//     rewritten (rx_ilu_upper: the sweeps read them from the Jacobian; rx_la_ilu_materialize for a download).
// Rows with more than kB2 lower blocks (3-D: up to six) take the extra blocks with direct loads. Arithmetic as
// k_ilu_build_2's gplan branch, operation for operation.
constexpr int kB2 = 3;
#ifndef RX_SST_BB2
#define RX_SST_BB2 2  // build knob: passes of blocks in flight ahead of the pass being factored
#endif
struct Plan2 {
  int4 h;        // i, klo, kd, khi
  int j[kB2];    // columns of the first lower blocks
  int kk[kB2];   // A_ji positions (-1: no update)
};
struct Blk2 {
  double d[4], a[kB2][4], u[kB2][4];  // A_ii, A_ij, A_ji
};
__device__ __forceinline__ Plan2 plan2_load(const int32_t* __restrict__ gplan, int r) {
  const int4* g = reinterpret_cast<const int4*>(gplan + (size_t)r * 32);
  Plan2 P;
  P.h = g[0];
  const int4 c = g[2], k3 = g[3], k4 = g[4];  // [8..11] columns, [14..16] A_ji positions
  P.j[0] = c.x;
  P.j[1] = c.y;
  P.j[2] = c.z;
  P.kk[0] = k3.z;
  P.kk[1] = k3.w;
  P.kk[2] = k4.x;
  return P;
}
__device__ __forceinline__ void blk2_load(const double* __restrict__ A, const Plan2& P, Blk2& B) {
  const int kd = P.h.z, nlow = P.h.z - P.h.y;
  const double2* a2 = reinterpret_cast<const double2*>(A);
  double2 x0 = a2[(size_t)kd * 2], x1 = a2[(size_t)kd * 2 + 1];
  B.d[0] = x0.x, B.d[1] = x0.y, B.d[2] = x1.x, B.d[3] = x1.y;
#pragma unroll
  for (int t = 0; t < kB2; ++t) {
    const int k = t < nlow ? P.h.y + t : kd;
    const int u = (t < nlow && P.kk[t] >= 0) ? P.kk[t] : kd;
    double2 y0 = a2[(size_t)k * 2], y1 = a2[(size_t)k * 2 + 1], z0 = a2[(size_t)u * 2], z1 = a2[(size_t)u * 2 + 1];
    B.a[t][0] = y0.x, B.a[t][1] = y0.y, B.a[t][2] = y1.x, B.a[t][3] = y1.y;
    B.u[t][0] = z0.x, B.u[t][1] = z0.y, B.u[t][2] = z1.x, B.u[t][3] = z1.y;
  }
}
// W = Bij inv(D_j), D -= Bji W (each product summed from 0.0, q ascending)
__device__ __forceinline__ void ilu2_lower(const double (&Bij)[4], const double* Sinv, const double (&Bji)[4],
                                          bool upd, double (&D)[4], double (&W)[4]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      double sm = 0.0;
#pragma unroll
      for (int q = 0; q < 2; ++q) sm += Bij[a * 2 + q] * Sinv[q * 2 + c];
      W[a * 2 + c] = sm;
    }
  if (upd) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        double sm = 0.0;
#pragma unroll
        for (int q = 0; q < 2; ++q) sm += Bji[a * 2 + q] * W[q * 2 + c];
        D[a * 2 + c] -= sm;
      }
  }
}
__global__ __launch_bounds__(64) void k_ilu_build_2w(const int32_t* __restrict__ part_ptr,
                                                     const int32_t* __restrict__ part_pass,
                                                     const int32_t* __restrict__ pass_lo,
                                                     const int32_t* __restrict__ gplan, const double* __restrict__ A,
                                                     double* __restrict__ F, double* __restrict__ invD) {
  extern __shared__ double sinv[];  // [partition rows][4]
  const int p = blockIdx.x, lane = threadIdx.x;
  const int p0 = part_ptr[p];
  const int q0 = part_pass[p], q1 = part_pass[p + 1];
  if (q0 >= q1) return;
  const int rlast = pass_lo[q1] - 1;  // clamp target: a valid slot of this partition
  auto slot_of = [&](int q) {
    const int qq = q < q1 ? q : q1 - 1;
    const int r = pass_lo[qq] + lane;
    return r < pass_lo[qq + 1] ? r : rlast;
  };
  // pipeline: the plans of passes q .. q + kPB2 - 1 (a register ring shifted every pass) and the blocks of passes
  // q .. q + kBB2 - 1 are in flight while pass q is computed; a pass's blocks are loaded from a plan that arrived
  // passes earlier, so no load waits on another one
  constexpr int kBB2 = RX_SST_BB2, kPB2 = kBB2 + 4 > 6 ? kBB2 + 4 : 6;
  Plan2 Pr[kPB2];
#pragma unroll
  for (int d = 0; d < kPB2; ++d) Pr[d] = plan2_load(gplan, slot_of(q0 + d));
  Blk2 Br[kBB2];
#pragma unroll
  for (int d = 0; d < kBB2; ++d) blk2_load(A, Pr[d], Br[d]);
  for (int q = q0; q < q1; ++q) {
    const bool act = pass_lo[q] + lane < pass_lo[q + 1];
    const Plan2 P = Pr[0];
    const Blk2 B = Br[0];
#pragma unroll
    for (int d = 0; d + 1 < kPB2; ++d) Pr[d] = Pr[d + 1];
    Pr[kPB2 - 1] = plan2_load(gplan, slot_of(q + kPB2));
#pragma unroll
    for (int d = 0; d + 1 < kBB2; ++d) Br[d] = Br[d + 1];
    blk2_load(A, Pr[kBB2 - 1], Br[kBB2 - 1]);
    if (act) {
      const int i = P.h.x, klo = P.h.y, kd = P.h.z, nlow = kd - klo;
      double D[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) D[e] = B.d[e];
#pragma unroll
      for (int t = 0; t < kB2; ++t) {
        if (t < nlow) {
          double W[4];
          ilu2_lower(B.a[t], sinv + (size_t)(P.j[t] - p0) * 4, B.u[t], P.kk[t] >= 0, D, W);
          double2* f2 = reinterpret_cast<double2*>(F + (size_t)(klo + t) * 4);
          f2[0] = make_double2(W[0], W[1]);
          f2[1] = make_double2(W[2], W[3]);
        }
      }
      for (int t = kB2; t < nlow; ++t) {  // rows past the plan's register blocks (3-D)
        const int32_t* g = gplan + (size_t)(pass_lo[q] + lane) * 32;
        const int kk = g[14 + t];
        double Bij[4], Bji[4], W[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          Bij[e] = A[(size_t)(klo + t) * 4 + e];
          Bji[e] = kk >= 0 ? A[(size_t)kk * 4 + e] : 0.0;
        }
        ilu2_lower(Bij, sinv + (size_t)(g[8 + t] - p0) * 4, Bji, kk >= 0, D, W);
#pragma unroll
        for (int e = 0; e < 4; ++e) F[(size_t)(klo + t) * 4 + e] = W[e];
      }
      double2* fd = reinterpret_cast<double2*>(F + (size_t)kd * 4);
      fd[0] = make_double2(D[0], D[1]);
      fd[1] = make_double2(D[2], D[3]);
      // inv(D_i): Gauss elimination of D_i, then one unit column at a time (k_ilu_build_2)
      {
        const double w = D[2] / D[0];
        D[3] -= w * D[1];
        D[2] = w;
      }
      double inv[4];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        double rhs[2] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0};
        lu_solve<2>(D, rhs);
        inv[c] = rhs[0];
        inv[2 + c] = rhs[1];
      }
      double2* iv = reinterpret_cast<double2*>(invD + (size_t)i * 4);
      iv[0] = make_double2(inv[0], inv[1]);
      iv[1] = make_double2(inv[2], inv[3]);
      double2* sv = reinterpret_cast<double2*>(sinv + (size_t)(i - p0) * 4);
      sv[0] = make_double2(inv[0], inv[1]);
      sv[1] = make_double2(inv[2], inv[3]);
    }
  }
}

// The SST's 2x2 ILU(0) apply, forward and backward sweeps in one launch, one wavefront per partition (VERDICT r03
// #7): the partition's vector lives in LDS from b to x (loaded and stored once, coalesced), the sweeps run pass by
// pass (<= 64 rows of one level, one row per lane, no barrier). A pass's slot record is loaded kS2 passes ahead
// (a register ring shifted every pass) and its blocks, column indices and inv(D_i) kD2 passes ahead, from that
// slot, so no load of the pass being computed waits on another load; every load is unconditional (clamped valid
// addresses) so the wait counts stay static. Rows with more than kB2 blocks on a side take the rest with direct
// loads. Arithmetic as k_ilu_fwd_wide / k_ilu_bwd_wide, operation for operation.
#ifndef RX_SST_D2
#define RX_SST_D2 4  // build knob: passes of blocks in flight ahead of the pass being computed (divides 8: RX_SST_UNROLL)
#endif
#ifndef RX_SST_UNROLL
#define RX_SST_UNROLL 1  // build knob: unroll the 2x2 sweeps' pass loop by the slot ring's length (8), so that the
#endif                   // rings of slots and blocks rotate by renaming instead of register moves (kD2 must divide 8;
                         // SST_SOLVE 0.85 -> 0.68 ms at C3, profiles/r06_ab_ap.txt)
constexpr int kD2 = RX_SST_D2, kS2 = RX_SST_UNROLL ? 8 : (kD2 + 5 > 8 ? kD2 + 5 : 8);
static_assert(!RX_SST_UNROLL || (8 % kD2 == 0 && kD2 < 8), "RX_SST_UNROLL: kD2 must divide the slot ring");
struct Row2 {
  int c[kB2];        // block columns
  double f[kB2][4];  // blocks
  double inv[4];     // inv(D_i) (backward)
};
template <bool BWD>
__device__ __forceinline__ void row2_load(const int4& s, const int32_t* __restrict__ col,
                                          const double* __restrict__ F, const double* __restrict__ invD, Row2& R) {
  const int k0 = BWD ? s.z + 1 : s.y, k1 = BWD ? s.w : s.z;
  const double2* f2 = reinterpret_cast<const double2*>(F);
#pragma unroll
  for (int t = 0; t < kB2; ++t) {
    const int k = k0 + t < k1 ? k0 + t : s.z;  // clamped to the diagonal block (always present)
    R.c[t] = col[k];
    const double2 a = f2[(size_t)k * 2], b = f2[(size_t)k * 2 + 1];
    R.f[t][0] = a.x, R.f[t][1] = a.y, R.f[t][2] = b.x, R.f[t][3] = b.y;
  }
  if (BWD) {
    const double2* i2 = reinterpret_cast<const double2*>(invD);
    const double2 a = i2[(size_t)s.x * 2], b = i2[(size_t)s.x * 2 + 1];
    R.inv[0] = a.x, R.inv[1] = a.y, R.inv[2] = b.x, R.inv[3] = b.y;
  }
}
template <bool BWD>
__device__ __forceinline__ void sweep2(const int4* __restrict__ slot, const int32_t* __restrict__ col,
                                       const double* __restrict__ F, const double* __restrict__ invD,
                                       const int32_t* __restrict__ pass_lo, int q0, int q1, int p0, double* xs) {
  const int lane = threadIdx.x;
  const int rlast = pass_lo[q1] - 1;
  auto slot_of = [&](int q) {
    const int qq = q < q1 ? q : q1 - 1;
    const int r = pass_lo[qq] + lane;
    return slot[r < pass_lo[qq + 1] ? r : rlast];
  };
  int4 S[kS2];  // slots of passes q .. q + kS2 - 1
#pragma unroll
  for (int d = 0; d < kS2; ++d) S[d] = slot_of(q0 + d);
  Row2 R[kD2];  // blocks of passes q .. q + kD2 - 1
#pragma unroll
  for (int d = 0; d < kD2; ++d) row2_load<BWD>(S[d], col, F, invD, R[d]);
#if RX_SST_UNROLL
#pragma unroll 8
#endif
  for (int q = q0; q < q1; ++q) {
    const bool act = pass_lo[q] + lane < pass_lo[q + 1];
    const int4 sc = S[0];
    const Row2 Rc = R[0];
#pragma unroll
    for (int d = 0; d + 1 < kS2; ++d) S[d] = S[d + 1];
    S[kS2 - 1] = slot_of(q + kS2);
#pragma unroll
    for (int d = 0; d + 1 < kD2; ++d) R[d] = R[d + 1];
    row2_load<BWD>(S[kD2 - 1], col, F, invD, R[kD2 - 1]);
    if (!act) continue;
    const int i = sc.x;
    const int k0 = BWD ? sc.z + 1 : sc.y, k1 = BWD ? sc.w : sc.z;
    double* xi = xs + (size_t)(i - p0) * 2;
    double acc[2];
    if (BWD) {
      acc[0] = 0.0;
      acc[1] = 0.0;
    } else {
      acc[0] = xi[0];
      acc[1] = xi[1];
    }
    auto take = [&](const double* blk, int j) {
      const double* xj = xs + (size_t)(j - p0) * 2;
      const double x0 = xj[0], x1 = xj[1];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        double sm = 0.0;
        sm += blk[a * 2] * x0;
        sm += blk[a * 2 + 1] * x1;
        if (BWD) acc[a] += sm;
        else acc[a] -= sm;
      }
    };
#pragma unroll
    for (int t = 0; t < kB2; ++t)
      if (k0 + t < k1) take(Rc.f[t], Rc.c[t]);
    for (int k = k0 + kB2; k < k1; ++k) {  // more blocks than the registers hold
      double blk[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) blk[e] = F[(size_t)k * 4 + e];
      take(blk, col[k]);
    }
    if (BWD) {
      const double v0 = xi[0] - acc[0], v1 = xi[1] - acc[1];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        double sm = 0.0;
        sm += Rc.inv[a * 2] * v0;
        sm += Rc.inv[a * 2 + 1] * v1;
        acc[a] = sm;
      }
    }
    xi[0] = acc[0];
    xi[1] = acc[1];
  }
}
__global__ __launch_bounds__(64) void k_ilu_apply_2w(const int32_t* __restrict__ part_ptr,
                                                     const int32_t* __restrict__ fpart, const int32_t* __restrict__ fpass,
                                                     const int4* __restrict__ fslot, const int32_t* __restrict__ bpart,
                                                     const int32_t* __restrict__ bpass, const int4* __restrict__ bslot,
                                                     const int32_t* __restrict__ col, const double* __restrict__ L,
                                                     const double* __restrict__ U, const double* __restrict__ invD,
                                                     const double* __restrict__ b, double* __restrict__ x,
                                                     int* __restrict__ done, const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
  extern __shared__ double xs[];  // [partition rows][2]
  const int p = blockIdx.x;
  const int p0 = part_ptr[p], n = (part_ptr[p + 1] - p0) * 2;
  for (int q = threadIdx.x; q < n; q += 64) xs[q] = b[(size_t)p0 * 2 + q];
  if (fpart[p] < fpart[p + 1]) sweep2<false>(fslot, col, L, invD, fpass, fpart[p], fpart[p + 1], p0, xs);
  if (bpart[p] < bpart[p + 1]) sweep2<true>(bslot, col, U, invD, bpass, bpart[p], bpart[p + 1], p0, xs);
  for (int q = threadIdx.x; q < n; q += 64) x[(size_t)p0 * 2 + q] = xs[q];
}

// Small-block ILU(0) with the whole partition resident in LDS (the SST system's 2x2 blocks: a 390-row
// partition is ~2 000 blocks = 64 KB). The workgroup loads the partition rows' A blocks once, every
// dependency level then reads finished rows' blocks and inverses from LDS (no global round trip between
// levels), and the factor and inv(D) are stored once at the end. One thread per row of a level; the row
// plan of the thread's next-level row is prefetched during the current level. Arithmetic as
// k_ilu_build_small (general per-block update plan, reference order).
template <int NV>
__global__ __launch_bounds__(256) void k_ilu_build_lds(const int32_t* __restrict__ part_ptr,
                                                       const int32_t* __restrict__ part_lvl,
                                                       const int32_t* __restrict__ lvl_ptr,
                                                       const int4* __restrict__ slot, const int32_t* __restrict__ rp,
                                                       const int32_t* __restrict__ col,
                                                       const int32_t* __restrict__ upd_ptr,
                                                       const int2* __restrict__ upd, const double* __restrict__ A,
                                                       double* __restrict__ F, double* __restrict__ invD) {
  constexpr int NV2 = NV * NV;
  extern __shared__ double lds[];
  const int p = blockIdx.x;
  const int lo = part_ptr[p], hi = part_ptr[p + 1];
  const int kb = rp[lo], ke = rp[hi];
  double* Fl = lds;                                // [ke - kb][NV2]
  double* Il = lds + (size_t)(ke - kb) * NV2;      // [hi - lo][NV2]
  for (int q = threadIdx.x; q < (ke - kb) * NV2; q += blockDim.x) Fl[q] = A[(size_t)kb * NV2 + q];
  __syncthreads();
  const int l0 = part_lvl[p], l1 = part_lvl[p + 1];
  int4 nxt = make_int4(-1, 0, 0, 0);
  if (l0 < l1 && lvl_ptr[l0] + (int)threadIdx.x < lvl_ptr[l0 + 1]) nxt = slot[lvl_ptr[l0] + threadIdx.x];
  for (int l = l0; l < l1; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    int4 cur = nxt;
    nxt = make_int4(-1, 0, 0, 0);
    if (l + 1 < l1 && lvl_ptr[l + 1] + (int)threadIdx.x < lvl_ptr[l + 2]) nxt = slot[lvl_ptr[l + 1] + threadIdx.x];
    for (int r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
      const int4 sl = (r == r0 + (int)threadIdx.x) ? cur : slot[r];
      const int i = sl.x, k0 = sl.y, kd = sl.z;
      for (int k = k0; k < kd; ++k) {
        const int j = col[k];
        const double* Sinv = Il + (size_t)(j - lo) * NV2;
        double* Bij = Fl + (size_t)(k - kb) * NV2;
        double W[NV2];
#pragma unroll
        for (int a = 0; a < NV; ++a)
#pragma unroll
          for (int c = 0; c < NV; ++c) {
            double sm = 0.0;
#pragma unroll
            for (int q = 0; q < NV; ++q) sm += Bij[a * NV + q] * Sinv[q * NV + c];
            W[a * NV + c] = sm;
          }
        for (int u = upd_ptr[k]; u < upd_ptr[k + 1]; ++u) {
          const int2 h = upd[u];
          const double* Bjk = Fl + (size_t)(h.x - kb) * NV2;
          double* Bik = Fl + (size_t)(h.y - kb) * NV2;
#pragma unroll
          for (int a = 0; a < NV; ++a)
#pragma unroll
            for (int c = 0; c < NV; ++c) {
              double sm = 0.0;
#pragma unroll
              for (int q = 0; q < NV; ++q) sm += Bjk[a * NV + q] * W[q * NV + c];
              Bik[a * NV + c] -= sm;
            }
        }
#pragma unroll
        for (int q = 0; q < NV2; ++q) Bij[q] = W[q];
      }
      double L[NV2];
#pragma unroll
      for (int q = 0; q < NV2; ++q) L[q] = Fl[(size_t)(kd - kb) * NV2 + q];
#pragma unroll
      for (int ii = 1; ii < NV; ++ii)
#pragma unroll
        for (int jj = 0; jj < ii; ++jj) {
          const double w = L[ii * NV + jj] / L[jj * NV + jj];
#pragma unroll
          for (int kk = jj + 1; kk < NV; ++kk) L[ii * NV + kk] -= w * L[jj * NV + kk];
          L[ii * NV + jj] = w;
        }
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        double rhs[NV];
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) rhs[rr] = (rr == c) ? 1.0 : 0.0;
        lu_solve<NV>(L, rhs);
#pragma unroll
        for (int rr = 0; rr < NV; ++rr) Il[(size_t)(i - lo) * NV2 + rr * NV + c] = rhs[rr];
      }
    }
    __syncthreads();
  }
  for (int q = threadIdx.x; q < (ke - kb) * NV2; q += blockDim.x) F[(size_t)kb * NV2 + q] = Fl[q];
  for (int q = threadIdx.x; q < (hi - lo) * NV2; q += blockDim.x) invD[(size_t)lo * NV2 + q] = Il[q];
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
    int* __restrict__ done, const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
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
    int* __restrict__ done, const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
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

// Row a of the blocks k0..k1-1 of one row times their x segments: f(s_k) with s_k = sum_c F_k[a][c] x_col(k)[c]
// (from 0.0, c ascending), k ascending. Small blocks (NV <= 4, the SST's 2x2) are taken four at a time with every
// load of the chunk issued before the first product (clamped, always valid addresses; the blocks past the row's
// end are skipped), as in the SpMV.
template <int NV, typename Fn>
__device__ __forceinline__ void row_blocks(const double* __restrict__ F, const int32_t* __restrict__ col,
                                           const double* x, int k0, int k1, int a, Fn f) {
#ifndef RX_ROWCH_BIG
#define RX_ROWCH_BIG 1
#endif
  constexpr int NV2 = NV * NV, CH = NV <= 4 ? 4 : RX_ROWCH_BIG;
  for (int k = k0; k < k1; k += CH) {
    double av[CH][NV], xv[CH][NV];
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int kk = k + t < k1 ? k + t : k;
      const double* blk = F + (size_t)kk * NV2 + a * NV;
      const double* xj = x + (size_t)col[kk] * NV;
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        av[t][c] = blk[c];
        xv[t][c] = xj[c];
      }
    }
#pragma unroll
    for (int t = 0; t < CH; ++t)
      if (k + t < k1) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) s += av[t][c] * xv[t][c];
        f(s);
      }
  }
}

// Wide variants of the two sweeps for partitions whose vector does not fit in LDS: TB threads per
// workgroup (TB / NV rows in flight, so a level of the C3 jet's 62-row-wide partitions is one pass instead
// of three), row metadata from the schedule's slot records {i, klo, diag, khi} (one load instead of
// rows -> klo / diag), and the first pass's slot of level l+1 loaded while level l runs. Same arithmetic,
// operation for operation, as k_ilu_fwd_part / k_ilu_bwd_part.
template <int NV, int TB>
__device__ __forceinline__ void fwd_wide_body(const int32_t* __restrict__ part_lvl, const int32_t* __restrict__ lvl_ptr,
                                              const int4* __restrict__ slot, const int32_t* __restrict__ col,
                                              const double* __restrict__ F, const double* __restrict__ b,
                                              double* __restrict__ x) {
  constexpr int NV2 = NV * NV, RPB = TB / NV;
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  const bool lane = rl < RPB;
  const int l0 = part_lvl[p], l1 = part_lvl[p + 1];
  int4 nxt = make_int4(-1, 0, 0, 0);
  if (lane && l0 < l1 && lvl_ptr[l0] + rl < lvl_ptr[l0 + 1]) nxt = slot[lvl_ptr[l0] + rl];
  for (int l = l0; l < l1; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    const int4 cur = nxt;
    nxt = make_int4(-1, 0, 0, 0);
    if (lane && l + 1 < l1 && r1 + rl < lvl_ptr[l + 2]) nxt = slot[r1 + rl];
    for (int r = r0 + rl; lane && r < r1; r += RPB) {
      const int4 sl = (r == r0 + rl) ? cur : slot[r];
      const int i = sl.x;
      double xi = b[(size_t)i * NV + a];
      row_blocks<NV>(F, col, x, sl.y, sl.z, a, [&](double s) { xi -= s; });
      x[(size_t)i * NV + a] = xi;
    }
    __syncthreads();
  }
}

template <int NV, int TB>
__device__ __forceinline__ void bwd_wide_body(const int32_t* __restrict__ part_lvl, const int32_t* __restrict__ lvl_ptr,
                                              const int4* __restrict__ slot, const int32_t* __restrict__ col,
                                              const double* __restrict__ F, const double* __restrict__ invD,
                                              double* __restrict__ x) {
  // Rows are laid out wavefront by wavefront (64 / NV rows per wavefront, the last 64 mod NV lanes idle), so that a
  // row's lanes never straddle two wavefronts: the exchange of v between the two halves of a level is then
  // wavefront-local (wave_sync) instead of a workgroup barrier. RX_BWD_BLOCK_ROWS restores the dense layout.
#ifdef RX_BWD_BLOCK_ROWS
  constexpr bool kWaveRows = false;
#else
  constexpr bool kWaveRows = true;
#endif
  constexpr int NV2 = NV * NV, RW = 64 / NV, RPB = kWaveRows ? (TB / 64) * RW : TB / NV;
  __shared__ double v[RPB * NV];
  const int p = blockIdx.x;
  const int wl = threadIdx.x & 63;
  const int rl = kWaveRows ? (int)(threadIdx.x >> 6) * RW + wl / NV : (int)threadIdx.x / NV;
  const int a = kWaveRows ? wl - (wl / NV) * NV : (int)threadIdx.x - rl * NV;
  const bool lane = kWaveRows ? wl < RW * NV : rl < RPB;
  const int l0 = part_lvl[p], l1 = part_lvl[p + 1];
  int4 nxt = make_int4(-1, 0, 0, 0);
  if (lane && l0 < l1 && lvl_ptr[l0] + rl < lvl_ptr[l0 + 1]) nxt = slot[lvl_ptr[l0] + rl];
  for (int l = l0; l < l1; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    const int4 cur = nxt;
    nxt = make_int4(-1, 0, 0, 0);
    if (lane && l + 1 < l1 && r1 + rl < lvl_ptr[l + 2]) nxt = slot[r1 + rl];
    for (int base = r0; base < r1; base += RPB) {
      const int r = base + rl;
      const bool act = lane && r < r1;
      int i = 0;
      double inv[NV];  // row a of inv(D_i): an input, loaded with the row's blocks (it stays in flight across the
                       // barrier) instead of after it, one global round trip less per level
      if (act) {
        const int4 sl = (base == r0) ? cur : slot[r];
        i = sl.x;
#ifndef RX_BWD_LATE_INV
#pragma unroll
        for (int c = 0; c < NV; ++c) inv[c] = invD[(size_t)i * NV2 + a * NV + c];
#endif
        double sum = 0.0;
        row_blocks<NV>(F, col, x, sl.z + 1, sl.w, a, [&](double s) { sum += s; });
        v[rl * NV + a] = x[(size_t)i * NV + a] - sum;
      }
      if (kWaveRows) wave_sync();
      else __syncthreads();
      if (act) {
#ifdef RX_BWD_LATE_INV
#pragma unroll
        for (int c = 0; c < NV; ++c) inv[c] = invD[(size_t)i * NV2 + a * NV + c];
#endif
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) s += inv[c] * v[rl * NV + c];
        x[(size_t)i * NV + a] = s;
      }
      __syncthreads();
    }
  }
}

template <int NV, int TB>
__global__ __launch_bounds__(TB) void k_ilu_fwd_wide(const int32_t* __restrict__ part_lvl,
                                                     const int32_t* __restrict__ lvl_ptr,
                                                     const int4* __restrict__ slot, const int32_t* __restrict__ col,
                                                     const double* __restrict__ F, const double* __restrict__ b,
                                                     double* __restrict__ x, int* __restrict__ done,
                                                     const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
  fwd_wide_body<NV, TB>(part_lvl, lvl_ptr, slot, col, F, b, x);
}
template <int NV, int TB>
__global__ __launch_bounds__(TB) void k_ilu_bwd_wide(const int32_t* __restrict__ part_lvl,
                                                     const int32_t* __restrict__ lvl_ptr,
                                                     const int4* __restrict__ slot, const int32_t* __restrict__ col,
                                                     const double* __restrict__ F, const double* __restrict__ invD,
                                                     double* __restrict__ x, int* __restrict__ done,
                                                     const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
  bwd_wide_body<NV, TB>(part_lvl, lvl_ptr, slot, col, F, invD, x);
}
// Both sweeps of a partition in one launch: the block-Jacobi partitions are independent, so the
// backward sweep of partition p needs only p's forward sweep, and a barrier (which makes the forward sweep's x
// stores visible to the workgroup, as between the levels) replaces the grid-wide boundary between two launches;
// the partition's x is then read back from the L2 it was just written to, and the kernel's time is the slowest
// partition's forward + backward instead of the slowest forward + the slowest backward. Same arithmetic.
template <int NV, int TB>
__global__ __launch_bounds__(TB) void k_ilu_apply_wide(const int32_t* __restrict__ fpart_lvl,
                                                       const int32_t* __restrict__ flvl_ptr,
                                                       const int4* __restrict__ fslot,
                                                       const int32_t* __restrict__ bpart_lvl,
                                                       const int32_t* __restrict__ blvl_ptr,
                                                       const int4* __restrict__ bslot, const int32_t* __restrict__ col,
                                                       const double* __restrict__ L, const double* __restrict__ U,
                                                       const double* __restrict__ invD, const double* __restrict__ b,
                                                       double* __restrict__ x, int* __restrict__ done,
                                                       const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
  fwd_wide_body<NV, TB>(fpart_lvl, flvl_ptr, fslot, col, L, b, x);
  __syncthreads();
  bwd_wide_body<NV, TB>(bpart_lvl, blvl_ptr, bslot, col, U, invD, x);
}

// Both sweeps of a partition with the sweep's recent results in an LDS ring (round 5). In the wide sweeps each level
// reads its x segments from global memory after the previous level's stores, so a level's time is the chain
// column index -> x -> product -> store -> barrier (which waits for the stores, and with them for every load issued
// before it). Here every result is also written to LDS: into the ring row (level mod kIluRing, position in the level),
// and, when some row more than kIluRing - 1 levels later reads it, into the partition's far row (the host's plan,
// rx_api.hip: ring_xoff per block, {ring, far} per schedule slot). The sweeps then read x only from LDS, the global
// stores of x are never waited for inside a sweep, and the level barrier is an LDS barrier (lgkmcnt). So the next
// level's factor rows, column offsets and b / inv(D) / forward result are loaded during this level and stay in flight
// across the barrier. One row per lane group and level (the widest level fits the workgroup's rows); MB blocks of a
// row come from registers, further ones are loaded when used. Same arithmetic, operation for operation, as the wide
// sweeps (row_blocks: each block's sum from 0.0, c ascending; blocks ascending).
#ifndef RX_RING_PROBE
#define RX_RING_PROBE 0  // timing probes of k_ilu_apply_ring (build variants only; bit 0: no factor-block loads)
#endif
// round 6: a level's global x store issued after the next level's loads (row, factor and slot loads) instead of
// before them. vmcnt retires loads and stores in issue order, so with the store first, waiting for those loads at
// the wavefront's next level also waited for the store's write acknowledgement; issued last, it is younger than them.
#ifndef RX_RING_LATE_STORE
#define RX_RING_LATE_STORE 1
#endif
template <int NV, int TB>
constexpr int ring_rpb() {
  return (TB / 64) * (64 / NV);  // rows per pass: whole rows per wavefront (the backward's v exchange is wave-local)
}
// G > 1 (round 5): the workgroup's wavefronts form G groups that take turns by level (group l mod G computes level l),
// so a wavefront's loads for its next level are issued G levels ahead: G - 1 other levels run while they are in flight,
// with the same registers per wavefront. A group holds rows per pass / G rows; the host splits wider levels into
// sub-levels (rx_api.hip), which the level tables passed here describe.
template <int NV, int TB, int MB, int G>
__global__ __launch_bounds__(TB) void k_ilu_apply_ring(
    const int32_t* __restrict__ fpart_lvl, const int32_t* __restrict__ flvl_ptr, const int4* __restrict__ fslot,
    const int2* __restrict__ fring, const int32_t* __restrict__ bpart_lvl, const int32_t* __restrict__ blvl_ptr,
    const int4* __restrict__ bslot, const int2* __restrict__ bring, const int32_t* __restrict__ xoff,
    const double* __restrict__ L, const double* __restrict__ U, const double* __restrict__ invD,
    const double* __restrict__ b, double* __restrict__ x, int* __restrict__ done, const int* __restrict__ conv,
    int ring_rows) {
  if (skip_sweep(done, conv)) return;
  constexpr int NV2 = NV * NV, RW = 64 / NV, RPB = ring_rpb<NV, TB>();
  extern __shared__ double lds[];
  double* xs = lds;                                               // [ring_rows][NV]
  double* v = lds + (size_t)ring_rows * NV;                       // [RPB][NV] backward: x_i - sum, per row
  int32_t* lp = reinterpret_cast<int32_t*>(v + (size_t)RPB * NV);  // the sweep's level table for this partition
  constexpr int WPG = (TB / 64) / G;  // wavefronts per group
  static_assert(G >= 1 && (TB / 64) % G == 0, "whole wavefronts per group");
  const int p = blockIdx.x;
  const int wl = threadIdx.x & 63, wave = (int)(threadIdx.x >> 6);
  const int g = wave / WPG;                       // this wavefront's group: it computes the levels l = g mod G
  const int rl = (wave % WPG) * RW + wl / NV;      // row of the level within the group
  const int vr = wave * RW + wl / NV;              // the backward's v row (exchanged inside the wavefront)
  const int a = wl - (wl / NV) * NV;
  const bool lane = wl < RW * NV;
  // ---- forward: x_i = b_i - sum_k L_ik x_col(k)
  {
    const int l0 = fpart_lvl[p], nl = fpart_lvl[p + 1] - l0;
    for (int q = threadIdx.x; q <= nl; q += TB) lp[q] = flvl_ptr[l0 + q];
    __syncthreads();
    // the slot loads — the last memory operations of a level — are issued by every lane on every path (a clamped,
    // valid address when out of range): the loads a level issues before them are then always followed by exactly
    // these two, so the compiler's vmcnt waits count them exactly and the next level's loads stay in flight (a slot
    // load on some paths only made it wait for all of them, vmcnt(0), right after they were issued). The row loads
    // themselves stay predicated (idle rows and missing blocks issue nothing).
    auto slot_at = [&](int l, int4& sl, int2& w) {
      const int lc = l < nl ? l : nl - 1;
      const int r = lp[lc] + rl;
      const bool ok = lane && l < nl && r < lp[lc + 1];
      sl = fslot[ok ? r : 0];
      w = fring[ok ? r : 0];
      return ok;
    };
    int4 sl = make_int4(0, 0, 0, 0), sln = sl;
    int2 w = make_int2(0, -1), wn = w;
    double F[MB][NV], bi = 0.0, xst = 0.0;
    int xo[MB];
    auto issue = [&]() {  // this lane's loads of row sl (its level is the next one computed)
      bi = b[(size_t)sl.x * NV + a];
#pragma unroll
      for (int t = 0; t < MB; ++t)
        if (sl.y + t < sl.z) {
#if RX_RING_PROBE & 1  // timing probe (build variant only): no factor-block loads
          xo[t] = 0;
#pragma unroll
          for (int c = 0; c < NV; ++c) F[t][c] = 0.0;
#else
          xo[t] = xoff[sl.y + t];
          const double* blk = L + (size_t)(sl.y + t) * NV2 + a * NV;
#pragma unroll
          for (int c = 0; c < NV; ++c) F[t][c] = blk[c];
#endif
        }
    };
    bool act = slot_at(g, sl, w);
    if (act) issue();
    bool actn = slot_at(g + G, sln, wn);
    for (int l = 0; l < nl; ++l) {
      if (G > 1 && l % G != g) {  // another group's level (wavefront-uniform)
        lds_barrier();
        continue;
      }
      if (act) {
        double xi = bi;
#pragma unroll
        for (int t = 0; t < MB; ++t)
          if (sl.y + t < sl.z) {
            const double* xj = xs + xo[t] * NV;
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < NV; ++c) s += F[t][c] * xj[c];
            xi -= s;
          }
        for (int k = sl.y + MB; k < sl.z; ++k) {  // rows with more than MB lower blocks
          const double* blk = L + (size_t)k * NV2 + a * NV;
          const double* xj = xs + xoff[k] * NV;
          double s = 0.0;
#pragma unroll
          for (int c = 0; c < NV; ++c) s += blk[c] * xj[c];
          xi -= s;
        }
        xs[w.x * NV + a] = xi;
        if (w.y >= 0) xs[w.y * NV + a] = xi;
        if (!RX_RING_LATE_STORE) x[(size_t)sl.x * NV + a] = xi;
        xst = xi;
      }
      const bool st = act;
      const int xrow = sl.x;
      act = actn;
      sl = sln;
      w = wn;
      if (act) issue();
      actn = slot_at(l + 2 * G, sln, wn);
      if (RX_RING_LATE_STORE && st) x[(size_t)xrow * NV + a] = xst;
      lds_barrier();
    }
  }
  __syncthreads();  // the forward's global x stores (the backward reads x_i) and its level-table reads are done
  // ---- backward: x_i = inv(D_i) (x_i - sum_k U_ik x_col(k))
  {
    const int l0 = bpart_lvl[p], nl = bpart_lvl[p + 1] - l0;
    for (int q = threadIdx.x; q <= nl; q += TB) lp[q] = blvl_ptr[l0 + q];
    __syncthreads();
    auto slot_at = [&](int l, int4& sl, int2& w) {  // unconditional loads, as in the forward sweep
      const int lc = l < nl ? l : nl - 1;
      const int r = lp[lc] + rl;
      const bool ok = lane && l < nl && r < lp[lc + 1];
      sl = bslot[ok ? r : 0];
      w = bring[ok ? r : 0];
      return ok;
    };
    int4 sl = make_int4(0, 0, 0, 0), sln = sl;
    int2 w = make_int2(0, -1), wn = w;
    double F[MB][NV], inv[NV], xf = 0.0, xst = 0.0;
    int xo[MB];
    auto issue = [&]() {
      xf = x[(size_t)sl.x * NV + a];
#pragma unroll
      for (int c = 0; c < NV; ++c) inv[c] = invD[(size_t)sl.x * NV2 + a * NV + c];
#pragma unroll
      for (int t = 0; t < MB; ++t)
        if (sl.z + 1 + t < sl.w) {
#if RX_RING_PROBE & 1
          xo[t] = 0;
#pragma unroll
          for (int c = 0; c < NV; ++c) F[t][c] = 0.0;
#else
          xo[t] = xoff[sl.z + 1 + t];
          const double* blk = U + (size_t)(sl.z + 1 + t) * NV2 + a * NV;
#pragma unroll
          for (int c = 0; c < NV; ++c) F[t][c] = blk[c];
#endif
        }
    };
    bool act = slot_at(g, sl, w);
    if (act) issue();
    bool actn = slot_at(g + G, sln, wn);
    for (int l = 0; l < nl; ++l) {
      if (G > 1 && l % G != g) {
        lds_barrier();
        continue;
      }
      if (act) {
        double sum = 0.0;
#pragma unroll
        for (int t = 0; t < MB; ++t)
          if (sl.z + 1 + t < sl.w) {
            const double* xj = xs + xo[t] * NV;
            double s = 0.0;
#pragma unroll
            for (int c = 0; c < NV; ++c) s += F[t][c] * xj[c];
            sum += s;
          }
        for (int k = sl.z + 1 + MB; k < sl.w; ++k) {
          const double* blk = U + (size_t)k * NV2 + a * NV;
          const double* xj = xs + xoff[k] * NV;
          double s = 0.0;
#pragma unroll
          for (int c = 0; c < NV; ++c) s += blk[c] * xj[c];
          sum += s;
        }
        v[vr * NV + a] = xf - sum;
      }
      wave_sync();
      if (act) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) s += inv[c] * v[vr * NV + c];
        xs[w.x * NV + a] = s;
        if (w.y >= 0) xs[w.y * NV + a] = s;
        if (!RX_RING_LATE_STORE) x[(size_t)sl.x * NV + a] = s;
        xst = s;
      }
      const bool st = act;
      const int xrow = sl.x;
      act = actn;
      sl = sln;
      w = wn;
      if (act) issue();
      actn = slot_at(l + 2 * G, sln, wn);
      if (RX_RING_LATE_STORE && st) x[(size_t)xrow * NV + a] = xst;
      lds_barrier();
    }
  }
}

// ILU(0) application with the partition's vector resident in LDS: b is loaded once, the forward
// and backward substitutions run level by level on the LDS copy, and x is stored once. The row
// metadata of both schedules and the partition's column indices (local) are staged in LDS too, so the
// only global loads inside a level are the factor blocks, and those of level l+1 are issued before
// level l is computed (register double buffer, kPF blocks per row; longer rows load the rest
// directly). Same arithmetic as k_ilu_fwd_part / k_ilu_bwd_part.
// LDS: xs[rows][NV] + v[RPB][NV] + fslot/bslot[rows][4] + colL[partition nnzb].
constexpr int kPF = 3;
template <int NV>
struct RowPF {
  double f[kPF][NV];
};
template <int NV>
__device__ __forceinline__ void pf_load(RowPF<NV>& d, const double* __restrict__ F, int k0, int k1, int a) {
#pragma unroll
  for (int t = 0; t < kPF; ++t)
    if (k0 + t < k1) {
      const double* blk = F + (size_t)(k0 + t) * NV * NV + a * NV;
#pragma unroll
      for (int c = 0; c < NV; ++c) d.f[t][c] = blk[c];
    }
}

template <int NV, bool GMETA>
__global__ __launch_bounds__(256) void k_ilu_apply_lds(const int32_t* __restrict__ part_ptr,
                                                       const int32_t* __restrict__ rp,
                                                       const int32_t* __restrict__ f_part_lvl,
                                                       const int32_t* __restrict__ f_lvl_ptr,
                                                       const int4* __restrict__ f_slot,
                                                       const int32_t* __restrict__ b_part_lvl,
                                                       const int32_t* __restrict__ b_lvl_ptr,
                                                       const int4* __restrict__ b_slot,
                                                       const int32_t* __restrict__ col, const double* __restrict__ F,
                                                       const double* __restrict__ Fu,
                                                       const double* __restrict__ invD, const double* __restrict__ b,
                                                       double* __restrict__ x, int* __restrict__ done,
                                                       const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
  constexpr int NV2 = NV * NV, RPB = 256 / NV;
  extern __shared__ double lds[];
  const int p = blockIdx.x;
  const int lo = part_ptr[p], hi = part_ptr[p + 1], nr = hi - lo;
  const int kb = rp[lo], ke = rp[hi];
  double* xs = lds;
  double* v = xs + (size_t)nr * NV;
  // rows of partition p occupy slots [f_lvl_ptr[f_part_lvl[p]], +nr) in both schedules
  const int fl0 = f_part_lvl[p], fl1 = f_part_lvl[p + 1], bl0 = b_part_lvl[p], bl1 = b_part_lvl[p + 1];
  const int fr0 = f_lvl_ptr[fl0], br0 = b_lvl_ptr[bl0];
  // GMETA: only the vector lives in LDS; the slot records and column indices are read from the global tables
  // (L2-resident, a few tens of KB per partition) — the partitions whose metadata does not fit beside the vector
  int4* fsl_l = reinterpret_cast<int4*>(lds + (((size_t)nr * NV + RPB * NV + 1) & ~(size_t)1));  // 16-B aligned
  int4* bsl_l = fsl_l + nr;
  int* colL_l = reinterpret_cast<int*>(bsl_l + nr);
  const int4* fsl = GMETA ? f_slot + fr0 : fsl_l;
  const int4* bsl = GMETA ? b_slot + br0 : bsl_l;
  auto colx = [&](int k) { return GMETA ? col[k] - lo : colL_l[k - kb]; };
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  const bool lane_ok = rl < RPB;
  RowPF<NV> cur, nxt;
  int4 csl = make_int4(0, 0, 0, 0), nsl = csl;  // the first-pass slot records of this level and the next (GMETA)
  // first forward level's factor rows straight from the global slot table
  if (lane_ok && fr0 + rl < f_lvl_ptr[fl0 + 1]) {
    csl = f_slot[fr0 + rl];
    pf_load<NV>(cur, F, csl.y, csl.z, a);
  }
  for (int q = threadIdx.x; q < nr * NV; q += blockDim.x) xs[q] = b[(size_t)lo * NV + q];
  if (!GMETA) {
    for (int q = threadIdx.x; q < nr; q += blockDim.x) {
      fsl_l[q] = f_slot[fr0 + q];
      bsl_l[q] = b_slot[br0 + q];
    }
    for (int q = threadIdx.x; q < ke - kb; q += blockDim.x) colL_l[q] = col[kb + q] - lo;
  }
  lds_barrier();
  for (int l = fl0; l < fl1; ++l) {
    const int r0 = f_lvl_ptr[l], r1 = f_lvl_ptr[l + 1];
    if (lane_ok && l + 1 < fl1 && r1 + rl < f_lvl_ptr[l + 2]) {
      nsl = fsl[r1 + rl - fr0];
      pf_load<NV>(nxt, F, nsl.y, nsl.z, a);
    }
    for (int r = r0 + rl; r < r1 && lane_ok; r += RPB) {
      const int4 sl = (GMETA && r == r0 + rl) ? csl : fsl[r - fr0];
      const int li = sl.x - lo;
      double xi = xs[li * NV + a];
      for (int k = sl.y; k < sl.z; ++k) {
        const int t = k - sl.y;
        const double* xj = xs + colx(k) * NV;
        double s = 0.0;
        if (r == r0 + rl && t < kPF) {
#pragma unroll
          for (int tt = 0; tt < kPF; ++tt)
            if (tt == t) {
#pragma unroll
              for (int c = 0; c < NV; ++c) s += cur.f[tt][c] * xj[c];
            }
        } else {
          const double* blk = F + (size_t)k * NV2 + a * NV;
#pragma unroll
          for (int c = 0; c < NV; ++c) s += blk[c] * xj[c];
        }
        xi -= s;
      }
      xs[li * NV + a] = xi;
    }
    lds_barrier();
    cur = nxt;
    csl = nsl;
  }
  // backward: upper blocks + the row of inv(D_i)
  RowPF<NV> ucur, unxt;
  double icur[NV], inxt[NV];
  int4 bcsl = make_int4(0, 0, 0, 0), bnsl = bcsl;
  if (lane_ok && br0 + rl < b_lvl_ptr[bl0 + 1]) {
    bcsl = bsl[rl];
    pf_load<NV>(ucur, Fu, bcsl.z + 1, bcsl.w, a);
#pragma unroll
    for (int c = 0; c < NV; ++c) icur[c] = invD[(size_t)bcsl.x * NV2 + a * NV + c];
  }
  for (int l = bl0; l < bl1; ++l) {
    const int r0 = b_lvl_ptr[l], r1 = b_lvl_ptr[l + 1];
    if (lane_ok && l + 1 < bl1 && r1 + rl < b_lvl_ptr[l + 2]) {
      bnsl = bsl[r1 + rl - br0];
      pf_load<NV>(unxt, Fu, bnsl.z + 1, bnsl.w, a);
#pragma unroll
      for (int c = 0; c < NV; ++c) inxt[c] = invD[(size_t)bnsl.x * NV2 + a * NV + c];
    }
    for (int base = r0; base < r1; base += RPB) {
      const int r = base + rl;
      const bool act = lane_ok && r < r1;
      const bool first = base == r0;
      int i = 0, li = 0;
      if (act) {
        const int4 sl = (GMETA && first) ? bcsl : bsl[r - br0];
        i = sl.x;
        li = i - lo;
        double sum = 0.0;
        for (int k = sl.z + 1; k < sl.w; ++k) {
          const int t = k - sl.z - 1;
          const double* xj = xs + colx(k) * NV;
          double s = 0.0;
          if (first && t < kPF) {
#pragma unroll
            for (int tt = 0; tt < kPF; ++tt)
              if (tt == t) {
#pragma unroll
                for (int c = 0; c < NV; ++c) s += ucur.f[tt][c] * xj[c];
              }
          } else {
            const double* blk = Fu + (size_t)k * NV2 + a * NV;
#pragma unroll
            for (int c = 0; c < NV; ++c) s += blk[c] * xj[c];
          }
          sum += s;
        }
        v[rl * NV + a] = xs[li * NV + a] - sum;
      }
      lds_barrier();
      if (act) {
        double s = 0.0;
        if (first) {
#pragma unroll
          for (int c = 0; c < NV; ++c) s += icur[c] * v[rl * NV + c];
        } else {
          const double* inv = invD + (size_t)i * NV2 + a * NV;
#pragma unroll
          for (int c = 0; c < NV; ++c) s += inv[c] * v[rl * NV + c];
        }
        xs[li * NV + a] = s;
      }
      lds_barrier();
    }
    ucur = unxt;
    bcsl = bnsl;
#pragma unroll
    for (int c = 0; c < NV; ++c) icur[c] = inxt[c];
  }
  for (int q = threadIdx.x; q < nr * NV; q += blockDim.x) x[(size_t)lo * NV + q] = xs[q];
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
    int* __restrict__ done, const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
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
    int* __restrict__ done, const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
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

template <int NV>
void launch_ilu_build_grp(rx_ctx* ctx, int gwaves) {
  if constexpr (NV >= 5) {
    const size_t shm = sizeof(double) * (size_t)(4 * gwaves) * grp_slot_doubles<NV>() +
                       sizeof(double) * (size_t)2 * ctx->ilu_ring_w * NV * NV +
                       sizeof(int32_t) * (size_t)(ctx->fs.maxlev + 1);
    auto kern = ctx->ilu_pair ? &k_ilu_build_grp<NV, true> : &k_ilu_build_grp<NV, false>;
    kern<<<ctx->npart, 64 * gwaves, shm, ctx->stream>>>(
        ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->ilu_gplan, ctx->f[RX_F_JAC], ctx->f[RX_F_ILU],
        ctx->f[RX_F_ILU] + ctx->nnzb * (int64_t)NV * NV, ctx->ilu_trace, ctx->ilu_gfull, ctx->ilu_ring_w);
    ctx->ilu_diag_deferred = RX_GRP_DIAG_STORE ? 0 : 1;
  }
}

}  // namespace

double* rx_invd_buf(rx_ctx* ctx) { return ctx->f[RX_F_ILU] + ctx->nnzb * (int64_t)ctx->nVar * ctx->nVar; }

// The factorisation runs k_ilu_build_grp (the factor's upper blocks and the blocks outside the partition are
// then the matrix's own, and are not copied).
static bool ilu_grouped(const rx_ctx* ctx) {
  static const bool rowwave = getenv("RX_ILU_ROWWAVE") != nullptr;  // A/B: one row per wavefront
  return ctx->nVar >= 5 && ctx->ilu_grp_ok && !rowwave;
}
// The one-wavefront 2x2 build (k_ilu_build_2w): triangle-free meshes whose partitions' inv(D) fit LDS.
static bool ilu2_wave(const rx_ctx* ctx) {
  static const bool old = getenv("RX_ILU2_OLD") != nullptr;  // A/B: k_ilu_build_lds / k_ilu_build_2
  return ctx->nVar == 2 && ctx->ilu_grp_ok && !old && (size_t)ctx->maxpart * 4 * sizeof(double) <= (size_t)ctx->lds_max;
}
// Where the triangular sweeps read the factor's upper blocks.
const double* rx_ilu_upper(rx_ctx* ctx) {
  return (ilu_grouped(ctx) || ilu2_wave(ctx)) ? ctx->f[RX_F_JAC] : ctx->f[RX_F_ILU];
}

namespace {
// ILU_matrix as the reference holds it (rx_download of the ILU field after k_ilu_build_grp): the blocks ILU(0)
// leaves unchanged (outside [klo, diag]) copied from the matrix. One wavefront per row.
template <int NV>
__global__ __launch_bounds__(256) void k_ilu_materialize(int N, const int32_t* __restrict__ rp,
                                                         const int32_t* __restrict__ klo,
                                                         const int64_t* __restrict__ diag,
                                                         const double* __restrict__ A, double* __restrict__ F) {
  constexpr int NV2 = NV * NV;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= N) return;
  const int kd = (int)diag[i];
  for (int k = rp[i]; k < rp[i + 1]; ++k)
    if (k < klo[i] || k > kd)
      for (int q = lane; q < NV2; q += 64) F[(size_t)k * NV2 + q] = A[(size_t)k * NV2 + q];
}
}  // namespace

// D_i = A_ii - sum_k A_ji W_k over the row's lower blocks in order, each product summed from 0.0 with q ascending and
// subtracted entry by entry: k_ilu_build_grp's arithmetic on the same operands (the matrix, unchanged since the build,
// and the W blocks it stored), so the block is bitwise the one the build eliminated. One wavefront per plan slot,
// lane c = column c.
template <int NV>
__global__ __launch_bounds__(256) void k_ilu_diag_materialize(int n, const int32_t* __restrict__ plan,
                                                              const double* __restrict__ A, double* __restrict__ F) {
  constexpr int NV2 = NV * NV;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), c = threadIdx.x & 63;
  if (r >= n || c >= NV) return;
  const int32_t* rec = plan + (size_t)r * kPlan;
  const int k0 = rec[1], kd = rec[2];
  double d[NV];
#pragma unroll
  for (int e = 0; e < NV; ++e) d[e] = A[(size_t)kd * NV2 + e * NV + c];
  for (int k = k0; k < kd; ++k) {
    const int kk = rec[14 + (k - k0)];
    if (kk < 0) continue;
    double x[NV];
#pragma unroll
    for (int e = 0; e < NV; ++e) x[e] = 0.0;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const double w = F[(size_t)k * NV2 + q * NV + c];
#pragma unroll
      for (int e = 0; e < NV; ++e) x[e] += A[(size_t)kk * NV2 + e * NV + q] * w;
    }
#pragma unroll
    for (int e = 0; e < NV; ++e) d[e] -= x[e];
  }
#pragma unroll
  for (int e = 0; e < NV; ++e) F[(size_t)kd * NV2 + e * NV + c] = d[e];
}

int rx_la_ilu_materialize(rx_ctx* ctx) {
  if ((!ilu_grouped(ctx) && !ilu2_wave(ctx)) || !ctx->f[RX_F_ILU]) return RX_OK;
  if (ctx->ilu_diag_deferred && ctx->nVar >= 5) {
    RX_NV_SWITCH(ctx->nVar, (k_ilu_diag_materialize<NV_><<<(int)((ctx->Nd + 3) / 4), 256, 0, ctx->stream>>>(
                                (int)ctx->Nd, ctx->ilu_gplan, ctx->f[RX_F_JAC], ctx->f[RX_F_ILU])));
    RX_HIP(hipGetLastError());
    ctx->ilu_diag_deferred = 0;
  }
  RX_NV_SWITCH(ctx->nVar, (k_ilu_materialize<NV_><<<(int)((ctx->Nd + 3) / 4), 256, 0, ctx->stream>>>(
                              (int)ctx->Nd, ctx->rp, ctx->klo, ctx->diag, ctx->f[RX_F_JAC], ctx->f[RX_F_ILU])));
  RX_HIP(hipGetLastError());
  return RX_OK;
}
#ifndef RX_ILU_MAX_WAVES
#define RX_ILU_MAX_WAVES 12
#endif
int rx_ilu_stage() { return kStage; }
int rx_ilu_ring_rpb(int nv, int tb) { return (tb / 64) * (64 / nv); }  // ring_rpb<nv, tb>()
// The ring sweeps' shape: 1 024 threads with two factor blocks of a row in registers (2-D: two lower / upper blocks
// per row on the quad meshes), or 768 threads (3 waves per SIMD, room for the registers) with three (3-D: the hex
// meshes' rows have three), so that a row's blocks are all loaded a level ahead instead of the third inside its level.
// RX_RING_3D=0 gives 3-D the 2-D shape (A/B).
int rx_ilu_ring_tb(const rx_ctx* ctx) {
  static const bool off = getenv("RX_RING_3D") && getenv("RX_RING_3D")[0] == '0';
  return ctx->nDim == 3 && !off ? 768 : 1024;
}
// RX_ILU_RING_G=1: every wavefront at every level (the first ring kernel, A/B); 4 / 8 (round 6, the 1 024-thread shape):
// more groups, each a level's loads further ahead, for the small partitions of a C4 rank (levels of ~10-25 rows)
int rx_ilu_ring_groups() {
  static const int g = [] {
    const int v = getenv("RX_ILU_RING_G") ? atoi(getenv("RX_ILU_RING_G")) : 2;
    return v == 1 || v == 4 || v == 8 ? v : 2;
  }();
  return g;
}
int rx_ilu_max_waves() { return RX_ILU_MAX_WAVES; }

// Raise the dynamic-LDS limit of the LDS-resident kernels to what the device allows (once).
int rx_la_prepare(rx_ctx* ctx) {
  RX_NV_SWITCH(ctx->nVar, {
    RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_lds<NV_, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
    RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_lds<NV_, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
    RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_build_part<NV_>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
    if constexpr (NV_ >= 5) {
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_ring<NV_, 1024, 2, 1>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_ring<NV_, 1024, 2, 2>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_ring<NV_, 768, 3, 1>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_ring<NV_, 768, 3, 2>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_ring<NV_, 1024, 2, 4>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_ring<NV_, 1024, 2, 8>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
    }
    if constexpr (NV_ >= 5) {
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_build_grp<NV_, false>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_build_grp<NV_, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
    }
    if (NV_ <= 4)
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_build_lds<NV_>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
    if (NV_ == 2) {
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_build_2w),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
      RX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ilu_apply_2w),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, ctx->lds_max));
    }
  });
  return RX_OK;
}

// Rows per level parity of the grouped build's inv(D) ring: as many of the widest level's rows as the LDS left by the
// group slots and the level table holds (RX_GRP_RING=0 or fewer than 8: no ring); 0 when not instantiated.
#ifndef RX_GRP_RING
#define RX_GRP_RING 1
#endif
static size_t grp_base_lds(const rx_ctx* ctx, int nv, size_t slot_doubles, int waves_cap) {
  const int gwaves = std::max(1, std::min(waves_cap, (ctx->fs.maxwidth + 3) / 4));
  (void)nv;
  return sizeof(double) * (size_t)(4 * gwaves) * slot_doubles + sizeof(int32_t) * (size_t)(ctx->fs.maxlev + 1);
}
int rx_ilu_grp_ring_w(const rx_ctx* ctx) {
  int w = 0;
  auto f = [&](auto nvc) {
    constexpr int NV = decltype(nvc)::value;
    if constexpr (NV >= 5) {
      const size_t base = grp_base_lds(ctx, NV, grp_slot_doubles<NV>(), grp_waves<NV>());
      const size_t per = sizeof(double) * 2 * (size_t)NV * NV;
      const size_t room = (size_t)ctx->lds_max > base ? (size_t)ctx->lds_max - base : 0;
      w = (int)std::min<size_t>((size_t)ctx->fs.maxwidth, room / per);
      if (!RX_GRP_RING || w < 8) w = 0;
    }
  };
  switch (ctx->nVar) {
    case 7: f(std::integral_constant<int, 7>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 9: f(std::integral_constant<int, 9>{}); break;
    case 10: f(std::integral_constant<int, 10>{}); break;
    case 11: f(std::integral_constant<int, 11>{}); break;
    case 12: f(std::integral_constant<int, 12>{}); break;
    case 13: f(std::integral_constant<int, 13>{}); break;
    case 14: f(std::integral_constant<int, 14>{}); break;
    default: break;
  }
  return w;
}

// Dynamic LDS of the grouped build at its launch configuration (launch_ilu_build_grp); 0 when not instantiated.
size_t rx_ilu_grp_lds(const rx_ctx* ctx) {
  size_t shm = 0;
  auto f = [&](auto nvc) {
    constexpr int NV = decltype(nvc)::value;
    if constexpr (NV >= 5) {
      const int gwaves = std::max(1, std::min(grp_waves<NV>(), (ctx->fs.maxwidth + 3) / 4));
      shm = sizeof(double) * (size_t)(4 * gwaves) * grp_slot_doubles<NV>() + sizeof(int32_t) * (size_t)(ctx->fs.maxlev + 1) +
            sizeof(double) * (size_t)2 * ctx->ilu_ring_w * NV * NV;
    }
  };
  switch (ctx->nVar) {
    case 7: f(std::integral_constant<int, 7>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 9: f(std::integral_constant<int, 9>{}); break;
    case 10: f(std::integral_constant<int, 10>{}); break;
    case 11: f(std::integral_constant<int, 11>{}); break;
    case 12: f(std::integral_constant<int, 12>{}); break;
    case 13: f(std::integral_constant<int, 13>{}); break;
    case 14: f(std::integral_constant<int, 14>{}); break;
    default: break;
  }
  return shm;
}

static int ilu_build_impl(rx_ctx* ctx);
int rx_la_ilu_build(rx_ctx* ctx) {
  const int rc = ilu_build_impl(ctx);
  ctx->ilu_valid = rc == RX_OK;
  return rc;
}

static int ilu_build_impl(rx_ctx* ctx) {
  const int nv = ctx->nVar;
  ctx->ilu_diag_deferred = 0;  // (set again by a grouped build that does not store the diagonal blocks)
  if (ilu2_wave(ctx) && !ctx->ilu_trace) {
    k_ilu_build_2w<<<ctx->npart, 64, (size_t)ctx->maxpart * 4 * sizeof(double), ctx->stream>>>(
        ctx->part_ptr, ctx->fs.part_pass, ctx->fs.pass_lo, ctx->ilu_gplan, ctx->f[RX_F_JAC], ctx->f[RX_F_ILU],
        rx_invd_buf(ctx));
    RX_HIP(hipGetLastError());
    return RX_OK;
  }
  const size_t shm_small = sizeof(double) * (size_t)nv * nv * (ctx->maxpart_nnzb + ctx->maxpart);
  if (nv <= 4 && !ctx->ilu_trace && shm_small <= (size_t)ctx->lds_max) {
    RX_NV_SWITCH(nv, (k_ilu_build_lds<NV_><<<ctx->npart, 256, shm_small, ctx->stream>>>(
                         ctx->part_ptr, ctx->fs.part_lvl, ctx->fs.lvl_ptr, reinterpret_cast<const int4*>(ctx->fs.slot),
                         ctx->rp, ctx->col, ctx->upd_ptr, reinterpret_cast<const int2*>(ctx->upd), ctx->f[RX_F_JAC],
                         ctx->f[RX_F_ILU], rx_invd_buf(ctx))));
    RX_HIP(hipGetLastError());
    return RX_OK;
  }
  if (nv == 2 && !ctx->ilu_trace) {
    k_ilu_build_2<<<ctx->npart, 256, 0, ctx->stream>>>(ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->ilu_plan,
                                                       reinterpret_cast<const int4*>(ctx->fs.slot), ctx->rp, ctx->col,
                                                       ctx->upd_ptr, reinterpret_cast<const int2*>(ctx->upd),
                                                       ctx->f[RX_F_JAC], ctx->f[RX_F_ILU], rx_invd_buf(ctx),
                                                       getenv("RX_ILU2_RELOAD") == nullptr,
                                                       ctx->ilu_grp_ok ? ctx->ilu_gplan : nullptr);
    RX_HIP(hipGetLastError());
    return RX_OK;
  }
  if (nv <= 4 && !ctx->ilu_trace) {
    RX_NV_SWITCH(nv, (k_ilu_build_small<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                         ctx->fs.part_lvl, ctx->fs.lvl_ptr, reinterpret_cast<const int4*>(ctx->fs.slot), ctx->rp,
                         ctx->col, ctx->upd_ptr, reinterpret_cast<const int2*>(ctx->upd), ctx->f[RX_F_JAC],
                         ctx->f[RX_F_ILU], rx_invd_buf(ctx))));
    RX_HIP(hipGetLastError());
    return RX_OK;
  }
  if (ilu_grouped(ctx)) {
    RX_NV_SWITCH(nv, (launch_ilu_build_grp<NV_>(ctx, std::max(1, std::min(grp_waves<NV_>(), (ctx->fs.maxwidth + 3) / 4)))));
    RX_HIP(hipGetLastError());
    return RX_OK;
  }
  const int waves = ctx->ilu_waves;
  const size_t shm = sizeof(double) * (size_t)waves * ((ctx->rowmax + 1 + kStage) * nv * nv + kPlan / 2);
  RX_NV_SWITCH(nv, (k_ilu_build_part<NV_><<<ctx->npart, 64 * waves, shm, ctx->stream>>>(
                       ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->ilu_plan, ctx->col, ctx->upd_ptr,
                       reinterpret_cast<const int2*>(ctx->upd), ctx->f[RX_F_JAC], ctx->f[RX_F_ILU],
                       rx_invd_buf(ctx), ctx->rowmax, ctx->ilu_trace)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// The one-wavefront 2x2 apply (k_ilu_apply_2w): partitions whose vector fits LDS.
static bool ilu2_apply_wave(const rx_ctx* ctx) {
  static const bool old = getenv("RX_ILU2_APPLY_OLD") != nullptr;  // A/B: the LDS-resident / wide sweeps
  return ctx->nVar == 2 && !old && (size_t)ctx->maxpart * 2 * sizeof(double) <= (size_t)ctx->lds_max;
}

// whether the ring sweeps take precedence over the LDS-resident apply where both fit (round 6: yes; RX_RING_FIRST=0
// restores the LDS-resident apply there). At a C4 rank's 490-row partitions (tools/c4_rank_floor.py, gpurun_out r06h,
// one box) SOLVE 2.28 -> 1.80 ms per step: the LDS-resident apply loads a level's factor blocks one level ahead from
// 256 threads, the ring two levels ahead per wavefront group from 1 024
bool rx_ilu_ring_first(const rx_ctx* ctx) {
  (void)ctx;
  static const bool on = !(getenv("RX_RING_FIRST") && getenv("RX_RING_FIRST")[0] == '0');
  return on;
}

int rx_la_ilu_apply(rx_ctx* ctx, const double* b, double* x, int* done, const int* conv) {
  const int nv = ctx->nVar;
  if (ilu2_apply_wave(ctx)) {
    k_ilu_apply_2w<<<ctx->npart, 64, (size_t)ctx->maxpart * 2 * sizeof(double), ctx->stream>>>(
        ctx->part_ptr, ctx->fs.part_pass, ctx->fs.pass_lo, reinterpret_cast<const int4*>(ctx->fs.slot),
        ctx->bs.part_pass, ctx->bs.pass_lo, reinterpret_cast<const int4*>(ctx->bs.slot), ctx->col, ctx->f[RX_F_ILU],
        rx_ilu_upper(ctx), rx_invd_buf(ctx), b, x, done, conv);
    RX_HIP(hipGetLastError());
    return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);
  }
  const size_t shm = sizeof(double) * ((size_t)ctx->maxpart * nv + (size_t)(256 / nv) * nv + 1) +
                     sizeof(int32_t) * (8 * (size_t)ctx->maxpart + (size_t)ctx->maxpart_nnzb);
  static const bool no_lds = getenv("RX_NO_LDS_APPLY") != nullptr;  // diagnosis: force the global sweeps
  if (shm <= (size_t)ctx->lds_max && !no_lds && !rx_ilu_ring_first(ctx)) {
    RX_NV_SWITCH(nv, (k_ilu_apply_lds<NV_, false><<<ctx->npart, 256, shm, ctx->stream>>>(
                         ctx->part_ptr, ctx->rp, ctx->fs.part_lvl, ctx->fs.lvl_ptr,
                         reinterpret_cast<const int4*>(ctx->fs.slot), ctx->bs.part_lvl, ctx->bs.lvl_ptr,
                         reinterpret_cast<const int4*>(ctx->bs.slot), ctx->col, ctx->f[RX_F_ILU], rx_ilu_upper(ctx),
                         rx_invd_buf(ctx), b, x, done, conv)));
    RX_HIP(hipGetLastError());
    return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);  // ComputeILUPreconditioner's closing SendReceive_Solution (:1513)
  }
  // RX_LDS_GMETA=1 (measured, not the default): when the vector alone fits (the SST's 2x2 system at C3 / C5, 62 KB
  // per partition), the LDS-resident apply with slot records and columns read from the global tables. Bitwise the
  // same, but slower than the wide sweeps below: SST_SOLVE 1.78 -> 1.90 ms at C3, 2.79 -> 3.41 ms at C5 (the
  // global metadata loads become the level's dependent chain at one wavefront per SIMD)
  const size_t shm_v = sizeof(double) * ((size_t)ctx->maxpart * nv + (size_t)(256 / nv) * nv + 1);
  static const bool gmeta = getenv("RX_LDS_GMETA") != nullptr;
  if (shm_v <= (size_t)ctx->lds_max && !no_lds && gmeta) {
    RX_NV_SWITCH(nv, (k_ilu_apply_lds<NV_, true><<<ctx->npart, 256, shm_v, ctx->stream>>>(
                         ctx->part_ptr, ctx->rp, ctx->fs.part_lvl, ctx->fs.lvl_ptr,
                         reinterpret_cast<const int4*>(ctx->fs.slot), ctx->bs.part_lvl, ctx->bs.lvl_ptr,
                         reinterpret_cast<const int4*>(ctx->bs.slot), ctx->col, ctx->f[RX_F_ILU], rx_ilu_upper(ctx),
                         rx_invd_buf(ctx), b, x, done, conv)));
    RX_HIP(hipGetLastError());
    return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);
  }
  static const bool narrow = getenv("RX_NARROW_APPLY") != nullptr;  // diagnosis: the 256-thread sweeps
  const int width = std::max(ctx->fs.maxwidth, ctx->bs.maxwidth);
  // the LDS-ring sweeps (round 5) when the widest level fits one pass and the ring fits the LDS; RX_ILU_NO_RING=1
  // restores the wide sweeps below (A/B)
  static const bool no_ring = getenv("RX_ILU_NO_RING") != nullptr;
  // (its sub-level plan splits the levels wider than one group's rows)
  const int tb = rx_ilu_ring_tb(ctx);
  const size_t ring_shm = sizeof(double) * ((size_t)std::max(ctx->fs.ring_rows, ctx->bs.ring_rows) * nv +
                                            (size_t)rx_ilu_ring_rpb(nv, tb) * nv) +
                          sizeof(int32_t) * (size_t)(std::max(ctx->fs.rmaxlev, ctx->bs.rmaxlev) + 1);
  if (!no_ring && !narrow && nv >= 5 && width * nv > 256 && width <= 2 * rx_ilu_ring_rpb(nv, tb) &&
      ring_shm <= (size_t)ctx->lds_max) {
    const int4* fsl = reinterpret_cast<const int4*>(ctx->fs.slot);
    const int4* bsl = reinterpret_cast<const int4*>(ctx->bs.slot);
    const int2* fr = reinterpret_cast<const int2*>(ctx->fs.ring);
    const int2* br = reinterpret_cast<const int2*>(ctx->bs.ring);
    const int rr = std::max(ctx->fs.ring_rows, ctx->bs.ring_rows);
    const int g = rx_ilu_ring_groups();
#define RX_RING_LAUNCH(TB_, MB_, G_)                                                                                \
  RX_NV_SWITCH(nv, (k_ilu_apply_ring<NV_, TB_, MB_, G_><<<ctx->npart, TB_, ring_shm, ctx->stream>>>(                \
                       ctx->fs.rpart_lvl, ctx->fs.rlvl_ptr, fsl, fr, ctx->bs.rpart_lvl, ctx->bs.rlvl_ptr, bsl, br,   \
                       ctx->ring_xoff, ctx->f[RX_F_ILU], rx_ilu_upper(ctx), rx_invd_buf(ctx), b, x, done, conv, rr)))
    if (tb == 768) {
      if (g == 1) {
        RX_RING_LAUNCH(768, 3, 1);
      } else {
        RX_RING_LAUNCH(768, 3, 2);
      }
    } else if (g == 1) {
      RX_RING_LAUNCH(1024, 2, 1);
    } else if (g == 4) {
      RX_RING_LAUNCH(1024, 2, 4);
    } else if (g == 8) {
      RX_RING_LAUNCH(1024, 2, 8);
    } else {
      RX_RING_LAUNCH(1024, 2, 2);
    }
#undef RX_RING_LAUNCH
    RX_HIP(hipGetLastError());
    return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);
  }
  static const bool split = getenv("RX_ILU_SPLIT") != nullptr;  // A/B: the two sweeps as separate launches
  if (!narrow && width * nv > 256 && !split) {
    const int4* fsl = reinterpret_cast<const int4*>(ctx->fs.slot);
    const int4* bsl = reinterpret_cast<const int4*>(ctx->bs.slot);
    RX_NV_SWITCH(nv, (k_ilu_apply_wide<NV_, 1024><<<ctx->npart, 1024, 0, ctx->stream>>>(
                         ctx->fs.part_lvl, ctx->fs.lvl_ptr, fsl, ctx->bs.part_lvl, ctx->bs.lvl_ptr, bsl, ctx->col,
                         ctx->f[RX_F_ILU], rx_ilu_upper(ctx), rx_invd_buf(ctx), b, x, done, conv)));
    RX_HIP(hipGetLastError());
    return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);
  }
  if (!narrow && width * nv > 256) {
    const int4* fsl = reinterpret_cast<const int4*>(ctx->fs.slot);
    const int4* bsl = reinterpret_cast<const int4*>(ctx->bs.slot);
    RX_NV_SWITCH(nv, (k_ilu_fwd_wide<NV_, 1024><<<ctx->npart, 1024, 0, ctx->stream>>>(
                         ctx->fs.part_lvl, ctx->fs.lvl_ptr, fsl, ctx->col, ctx->f[RX_F_ILU], b, x, done, conv)));
    RX_NV_SWITCH(nv, (k_ilu_bwd_wide<NV_, 1024><<<ctx->npart, 1024, 0, ctx->stream>>>(
                         ctx->bs.part_lvl, ctx->bs.lvl_ptr, bsl, ctx->col, rx_ilu_upper(ctx), rx_invd_buf(ctx), x,
                         done, conv)));
    RX_HIP(hipGetLastError());
    return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);
  }
  static const bool narrow_small = getenv("RX_NARROW_SMALL") != nullptr;  // diagnosis: the part sweeps below
  if (!narrow && !narrow_small) {  // levels narrower than 256 / NV rows: the same wide sweeps on 256 threads
    const int4* fsl = reinterpret_cast<const int4*>(ctx->fs.slot);
    const int4* bsl = reinterpret_cast<const int4*>(ctx->bs.slot);
    RX_NV_SWITCH(nv, (k_ilu_fwd_wide<NV_, 256><<<ctx->npart, 256, 0, ctx->stream>>>(
                         ctx->fs.part_lvl, ctx->fs.lvl_ptr, fsl, ctx->col, ctx->f[RX_F_ILU], b, x, done, conv)));
    RX_NV_SWITCH(nv, (k_ilu_bwd_wide<NV_, 256><<<ctx->npart, 256, 0, ctx->stream>>>(
                         ctx->bs.part_lvl, ctx->bs.lvl_ptr, bsl, ctx->col, rx_ilu_upper(ctx), rx_invd_buf(ctx), x,
                         done, conv)));
    RX_HIP(hipGetLastError());
    return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);
  }
  RX_NV_SWITCH(ctx->nVar, (k_ilu_fwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->fs.rows, ctx->col, ctx->klo, ctx->diag,
                              ctx->f[RX_F_ILU], b, x, done, conv)));
  RX_NV_SWITCH(ctx->nVar, (k_ilu_bwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->bs.part_lvl, ctx->bs.lvl_ptr, ctx->bs.rows, ctx->col, ctx->khi, ctx->diag,
                              rx_ilu_upper(ctx), rx_invd_buf(ctx), x, done, conv)));
  RX_HIP(hipGetLastError());
  return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, nv);
}

int rx_la_diag_factor(rx_ctx* ctx, const double* A) {
  if (!ctx->dlu) return RX_ERR_STATE;  // LU-SGS factor storage (allocated with the LU_SGS preconditioner)
  RX_NV_SWITCH(ctx->nVar, (k_diag_factor<NV_><<<(int)((ctx->Nd + 3) / 4), 256, 0, ctx->stream>>>(
                              (int)ctx->Nd, ctx->diag, A, ctx->dlu)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_la_lusgs(rx_ctx* ctx, const double* A, const double* b, double* x, int* done, const int* conv) {
  if (!ctx->dlu) return RX_ERR_STATE;
  RX_NV_SWITCH(ctx->nVar, (k_lusgs_fwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->fs.rows, ctx->col, ctx->klo, ctx->diag, A,
                              ctx->dlu, b, ctx->xstar, done, conv)));
  // halo x* between the sweeps (ComputeLU_SGSPreconditioner :1689)
  int rc = rx_la_exchange(ctx, ctx->xstar, ctx->nVar);
  if (rc) return rc;
  RX_NV_SWITCH(ctx->nVar, (k_lusgs_bwd_part<NV_><<<ctx->npart, 256, 0, ctx->stream>>>(
                              ctx->bs.part_lvl, ctx->bs.lvl_ptr, ctx->bs.rows, ctx->rp, ctx->col, ctx->klo, ctx->khi,
                              ctx->diag, A, ctx->dlu, ctx->xstar, x, done, conv)));
  RX_HIP(hipGetLastError());
  return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, ctx->nVar);  // :1707
}

namespace {
// BuildJacobiPreconditioner (matrix_structure.cpp:1230-1246): invM_i = InverseDiagonalBlock (:1129-1143), column c
// the Gauss_Elimination (:594-643) of the unit vector e_c. One wavefront per row: the block is factorised with
// lane r holding row r (wave_factor_rows, the reference's elimination order), then lane c < NV solves e_c with the
// stored multipliers and U (wave_solve_rows, the reference's rhs order) and writes column c of the inverse.
template <int NV>
__global__ __launch_bounds__(256) void k_jacobi_build(int N, const int64_t* __restrict__ diag,
                                                      const double* __restrict__ A, double* __restrict__ inv) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= N) return;
  const double* D = A + diag[i] * (NV * NV);
  double row[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) row[k] = lane < NV ? D[lane * NV + k] : 1.0;
  wave_factor_rows<NV>(row, lane);
  double rhs[NV];
#pragma unroll
  for (int r = 0; r < NV; ++r) rhs[r] = (r == lane) ? 1.0 : 0.0;
  wave_solve_rows<NV>(row, rhs);
  if (lane < NV) {
#pragma unroll
    for (int r = 0; r < NV; ++r) inv[(size_t)i * NV * NV + r * NV + lane] = rhs[r];
  }
}

// ComputeJacobiPreconditioner (:1249-1266): prod_ia = 0.0 + sum_c invM_i[a][c] vec_ic (c ascending), owned rows.
// One thread per element; the rows of invM are read whole (NV consecutive doubles).
template <int NV>
__global__ __launch_bounds__(256) void k_jacobi_apply(int N, const double* __restrict__ inv,
                                                      const double* __restrict__ b, double* __restrict__ x,
                                                      int* __restrict__ done, const int* __restrict__ conv) {
  if (skip_sweep(done, conv)) return;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (int64_t)N * NV) return;
  const int64_t i = q / NV;
  const double* m = inv + (size_t)q * NV;  // row a of block i: (i * NV + a) * NV
  const double* v = b + i * NV;
  double acc = 0.0;
#pragma unroll
  for (int c = 0; c < NV; ++c) acc += m[c] * v[c];
  x[q] = acc;
}

// Jacobi_Smoother's update (:1331-1337): x_ia += invM_i[a][c] r_ic, accumulated into x itself (c ascending).
template <int NV>
__global__ __launch_bounds__(256) void k_jacobi_smooth(int N, const double* __restrict__ inv,
                                                       const double* __restrict__ r, double* __restrict__ x,
                                                       const int* __restrict__ done) {
  if (*done) return;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (int64_t)N * NV) return;
  const int64_t i = q / NV;
  const double* m = inv + (size_t)q * NV;
  const double* v = r + i * NV;
  double acc = x[q];
#pragma unroll
  for (int c = 0; c < NV; ++c) acc += m[c] * v[c];
  x[q] = acc;
}
}  // namespace

int rx_la_jacobi_build(rx_ctx* ctx, const double* A) {
  if (!ctx->jinv) return RX_ERR_STATE;  // allocated with the JACOBI preconditioner / SMOOTHER_JACOBI
  RX_NV_SWITCH(ctx->nVar, (k_jacobi_build<NV_><<<(int)((ctx->Nd + 3) / 4), 256, 0, ctx->stream>>>(
                              (int)ctx->Nd, ctx->diag, A, ctx->jinv)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

int rx_la_jacobi_apply(rx_ctx* ctx, const double* b, double* x, int* done, const int* conv) {
  if (!ctx->jinv) return RX_ERR_STATE;
  const int64_t n = ctx->Nd * ctx->nVar;
  RX_NV_SWITCH(ctx->nVar, (k_jacobi_apply<NV_><<<(int)((n + 255) / 256), 256, 0, ctx->stream>>>(
                              (int)ctx->Nd, ctx->jinv, b, x, done, conv)));
  RX_HIP(hipGetLastError());
  return ctx->defer_exchange ? RX_OK : rx_la_exchange(ctx, x, ctx->nVar);  // :1264
}

int rx_la_jacobi_smooth(rx_ctx* ctx, const double* r, double* x, const int* done) {
  if (!ctx->jinv) return RX_ERR_STATE;
  const int64_t n = ctx->Nd * ctx->nVar;
  RX_NV_SWITCH(ctx->nVar, (k_jacobi_smooth<NV_><<<(int)((n + 255) / 256), 256, 0, ctx->stream>>>(
                              (int)ctx->Nd, ctx->jinv, r, x, done)));
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// The preconditioner of CSysSolve::Solve (linear_solvers_structure.cpp:633-653) applied to b -> x, with x's halo
// exchanged unless ctx->defer_exchange.
int rx_la_eff_prec(const rx_ctx* ctx) {
  switch (ctx->cfg.lin_solver) {
    case RX_LIN_SMOOTHER_LUSGS: return RX_PREC_LU_SGS;
    case RX_LIN_SMOOTHER_JACOBI: return RX_PREC_JACOBI;
    case RX_LIN_SMOOTHER_ILU: return RX_PREC_ILU;
    default: return ctx->cfg.lin_prec;
  }
}

int rx_la_prec_build(rx_ctx* ctx) {
  switch (rx_la_eff_prec(ctx)) {
    case RX_PREC_ILU: return rx_la_ilu_build(ctx);  // BuildILUPreconditioner (:1368)
    case RX_PREC_LU_SGS: return rx_la_diag_factor(ctx, ctx->f[RX_F_JAC]);  // Gauss_Elimination's factor, once
    case RX_PREC_JACOBI: return rx_la_jacobi_build(ctx, ctx->f[RX_F_JAC]);  // BuildJacobiPreconditioner (:1230)
    default: return RX_ERR_ARG;
  }
}

int rx_la_prec_apply(rx_ctx* ctx, const double* b, double* x, int* done, const int* conv) {
  switch (rx_la_eff_prec(ctx)) {
    case RX_PREC_ILU: {
      RxPhase ph(ctx, RX_K_ILU_APPLY);
      return rx_la_ilu_apply(ctx, b, x, done, conv);
    }
    case RX_PREC_LU_SGS:
      return rx_la_lusgs(ctx, ctx->f[RX_F_JAC], b, x, done, conv);
    case RX_PREC_JACOBI:
      return rx_la_jacobi_apply(ctx, b, x, done, conv);
    default:
      return RX_ERR_ARG;
  }
}

// Debug: trace the phases of the ILU(0) factorisation of partition 0 (see tools/ilu_trace.py).
extern "C" int rx_debug_ilu_trace(rx_ctx* ctx, long long* host, int64_t n) {
  const int64_t need = std::max<int64_t>(1 + 16 * 5 * 64, 1 + kGrpTraceGroups * kGrpTraceRows * 8 + kGrpTraceLevels);
  if (!ctx || n < need) return RX_ERR_ARG;
  if (!ctx->ilu_trace) {
    RX_HIP(hipMalloc(&ctx->ilu_trace, sizeof(long long) * need));
  }
  RX_HIP(hipMemsetAsync(ctx->ilu_trace, 0, sizeof(long long) * need, ctx->stream));
  int rc = rx_la_ilu_build(ctx);
  if (rc) return rc;
  RX_HIP(hipMemcpyAsync(host, ctx->ilu_trace, sizeof(long long) * need, hipMemcpyDeviceToHost, ctx->stream));
  RX_HIP(hipStreamSynchronize(ctx->stream));
  (void)hipFree(ctx->ilu_trace);
  ctx->ilu_trace = nullptr;
  return RX_OK;
}

#ifdef RX_PROBE
// Probe build only (tools/sweep_probe.py, librx_probe.so): timing variants of the wide forward sweep that break
// its semantics on purpose, to locate where a level's time goes. MODE bits: 1 = x read from b (no dependence on
// the level's results), 2 = no workgroup barrier between levels, 4 = factor blocks not loaded (a constant).
namespace {
template <int NV, int TB, int MODE>
__global__ __launch_bounds__(TB) void k_probe_fwd(const int32_t* __restrict__ part_lvl, const int32_t* __restrict__ lvl_ptr,
                                                  const int4* __restrict__ slot, const int32_t* __restrict__ col,
                                                  const double* __restrict__ F, const double* __restrict__ b,
                                                  double* __restrict__ x) {
  constexpr int NV2 = NV * NV, RPB = TB / NV;
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  const bool lane = rl < RPB;
  const int l0 = part_lvl[p], l1 = part_lvl[p + 1];
  const double* xs = (MODE & 1) ? b : x;
  for (int l = l0; l < l1; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    for (int r = r0 + rl; lane && r < r1; r += RPB) {
      const int4 sl = slot[r];
      const int i = sl.x;
      double xi = b[(size_t)i * NV + a];
      for (int k = sl.y; k < sl.z; ++k) {
        const double* blk = F + (size_t)k * NV2 + a * NV;
        const double* xj = xs + (size_t)col[k] * NV;
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) s += ((MODE & 4) ? 1e-3 : blk[c]) * xj[c];
        xi -= s;
      }
      x[(size_t)i * NV + a] = xi;
    }
    if (!(MODE & 2)) __syncthreads();
  }
}
// Compact sweep layouts (modes 10 / 11): the blocks a sweep reads, copied in schedule order, so that a level's
// blocks are one contiguous run. Forward: the lower blocks [klo, diag) of slot r at Lc[off[r]..]; backward: the upper
// blocks (diag, khi) and then inv(D_i) of slot r at Uc[off[r]..].
template <int NV>
__global__ __launch_bounds__(256) void k_probe_gather(int n, const int4* __restrict__ slot, const int64_t* __restrict__ off,
                                                      int bwd, const double* __restrict__ A,
                                                      const double* __restrict__ invD, double* __restrict__ dst) {
  constexpr int NV2 = NV * NV;
  const int r = blockIdx.x;
  if (r >= n) return;
  const int4 sl = slot[r];
  const int k0 = bwd ? sl.z + 1 : sl.y, k1 = bwd ? sl.w : sl.z;
  double* o = dst + (size_t)off[r] * NV2;
  for (int q = threadIdx.x; q < (k1 - k0) * NV2; q += 256) o[q] = A[(size_t)k0 * NV2 + q];
  if (bwd)
    for (int q = threadIdx.x; q < NV2; q += 256) o[(size_t)(k1 - k0) * NV2 + q] = invD[(size_t)sl.x * NV2 + q];
}

template <int NV, int TB>
__global__ __launch_bounds__(TB) void k_probe_fwd_c(const int32_t* __restrict__ part_lvl,
                                                    const int32_t* __restrict__ lvl_ptr, const int4* __restrict__ slot,
                                                    const int32_t* __restrict__ col, const double* __restrict__ Lc,
                                                    const int64_t* __restrict__ off, const double* __restrict__ b,
                                                    double* __restrict__ x) {
  constexpr int NV2 = NV * NV, RPB = TB / NV;
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  const bool lane = rl < RPB;
  const int l0 = part_lvl[p], l1 = part_lvl[p + 1];
  for (int l = l0; l < l1; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    for (int r = r0 + rl; lane && r < r1; r += RPB) {
      const int4 sl = slot[r];
      const int i = sl.x;
      double xi = b[(size_t)i * NV + a];
      row_blocks<NV>(Lc + ((int64_t)off[r] - sl.y) * NV2, col, x, sl.y, sl.z, a, [&](double s) { xi -= s; });
      x[(size_t)i * NV + a] = xi;
    }
    __syncthreads();
  }
}

template <int NV, int TB>
__global__ __launch_bounds__(TB) void k_probe_bwd_c(const int32_t* __restrict__ part_lvl,
                                                    const int32_t* __restrict__ lvl_ptr, const int4* __restrict__ slot,
                                                    const int32_t* __restrict__ col, const double* __restrict__ Uc,
                                                    const int64_t* __restrict__ off, double* __restrict__ x) {
  constexpr int NV2 = NV * NV, RPB = TB / NV;
  __shared__ double v[RPB * NV];
  const int p = blockIdx.x;
  const int rl = threadIdx.x / NV, a = threadIdx.x - rl * NV;
  const bool lane = rl < RPB;
  const int l0 = part_lvl[p], l1 = part_lvl[p + 1];
  for (int l = l0; l < l1; ++l) {
    const int r0 = lvl_ptr[l], r1 = lvl_ptr[l + 1];
    for (int base = r0; base < r1; base += RPB) {
      const int r = base + rl;
      const bool act = lane && r < r1;
      int i = 0;
      const double* inv = nullptr;
      if (act) {
        const int4 sl = slot[r];
        i = sl.x;
        double sum = 0.0;
        row_blocks<NV>(Uc + ((int64_t)off[r] - (sl.z + 1)) * NV2, col, x, sl.z + 1, sl.w, a, [&](double s) { sum += s; });
        v[rl * NV + a] = x[(size_t)i * NV + a] - sum;
        inv = Uc + ((size_t)off[r] + (sl.w - sl.z - 1)) * NV2 + a * NV;
      }
      __syncthreads();
      if (act) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < NV; ++c) s += inv[c] * v[rl * NV + c];
        x[(size_t)i * NV + a] = s;
      }
      __syncthreads();
    }
  }
}
}  // namespace

// builds the compact copies once per context (probe only; leaked)
static int probe_compact(rx_ctx* ctx, int bwd, double** buf, int64_t** off) {
  const int n = (int)ctx->Nd, nv = ctx->nVar;
  const rx_ctx::Sched& S = bwd ? ctx->bs : ctx->fs;
  std::vector<int> h((size_t)4 * n);
  RX_HIP(hipMemcpy(h.data(), S.slot, sizeof(int) * 4 * (size_t)n, hipMemcpyDeviceToHost));
  std::vector<int64_t> o((size_t)n + 1, 0);
  for (int r = 0; r < n; ++r) {
    const int* sl = &h[(size_t)4 * r];
    o[r + 1] = o[r] + (bwd ? (sl[3] - sl[2] - 1 + 1) : (sl[2] - sl[1]));
  }
  RX_HIP(hipMalloc(off, sizeof(int64_t) * (n + 1)));
  RX_HIP(hipMemcpy(*off, o.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
  RX_HIP(hipMalloc(buf, sizeof(double) * (size_t)o[n] * nv * nv + 64));
  RX_NV_SWITCH(nv, (k_probe_gather<NV_><<<n, 256, 0, ctx->stream>>>(
                       n, reinterpret_cast<const int4*>(S.slot), *off, bwd, bwd ? rx_ilu_upper(ctx) : ctx->f[RX_F_ILU],
                       rx_invd_buf(ctx), *buf)));
  RX_HIP(hipStreamSynchronize(ctx->stream));
  return RX_OK;
}

extern "C" int rx_debug_sweep_probe(rx_ctx* ctx, int mode, int reps, double* ms) {
  if (!ctx || !ctx->cfg.implicit || ctx->nVar != 11) return RX_ERR_ARG;
  const int4* fsl = reinterpret_cast<const int4*>(ctx->fs.slot);
  double* b = ctx->f[RX_F_RHS];
  double* x = ctx->f[RX_F_SOL];
  static double *Lc = nullptr, *Uc = nullptr;
  static int64_t *loff = nullptr, *uoff = nullptr;
  if (mode >= 10 && !Lc) {
    int rc = probe_compact(ctx, 0, &Lc, &loff);
    if (!rc) rc = probe_compact(ctx, 1, &Uc, &uoff);
    if (rc) return rc;
  }
  hipEvent_t e0, e1;
  RX_HIP(hipEventCreate(&e0));
  RX_HIP(hipEventCreate(&e1));
  RX_HIP(hipEventRecord(e0, ctx->stream));
  for (int q = 0; q < reps; ++q) {
#define RX_PROBE_CASE(M)                                                                                          \
  case M:                                                                                                         \
    k_probe_fwd<11, 1024, M><<<ctx->npart, 1024, 0, ctx->stream>>>(ctx->fs.part_lvl, ctx->fs.lvl_ptr, fsl, ctx->col, \
                                                                  ctx->f[RX_F_ILU], b, x);                        \
    break;
    switch (mode) {
      RX_PROBE_CASE(0)
      RX_PROBE_CASE(1)
      RX_PROBE_CASE(2)
      RX_PROBE_CASE(3)
      RX_PROBE_CASE(4)
      RX_PROBE_CASE(5)
      RX_PROBE_CASE(6)
      RX_PROBE_CASE(7)
      case 8:  // the production forward sweep
        k_ilu_fwd_wide<11, 1024><<<ctx->npart, 1024, 0, ctx->stream>>>(ctx->fs.part_lvl, ctx->fs.lvl_ptr, fsl,
                                                                        ctx->col, ctx->f[RX_F_ILU], b, x, nullptr,
                                                                        nullptr);
        break;
      case 9:  // the production backward sweep
        k_ilu_bwd_wide<11, 1024><<<ctx->npart, 1024, 0, ctx->stream>>>(
            ctx->bs.part_lvl, ctx->bs.lvl_ptr, reinterpret_cast<const int4*>(ctx->bs.slot), ctx->col,
            rx_ilu_upper(ctx), rx_invd_buf(ctx), x, nullptr, nullptr);
        break;
      case 10:  // forward sweep on the compact lower blocks
        k_probe_fwd_c<11, 1024><<<ctx->npart, 1024, 0, ctx->stream>>>(ctx->fs.part_lvl, ctx->fs.lvl_ptr, fsl, ctx->col,
                                                                       Lc, loff, b, x);
        break;
      case 11:  // backward sweep on the compact upper blocks + inv(D)
        k_probe_bwd_c<11, 1024><<<ctx->npart, 1024, 0, ctx->stream>>>(
            ctx->bs.part_lvl, ctx->bs.lvl_ptr, reinterpret_cast<const int4*>(ctx->bs.slot), ctx->col, Uc, uoff, x);
        break;
      default:
        return RX_ERR_ARG;
    }
#undef RX_PROBE_CASE
  }
  RX_HIP(hipEventRecord(e1, ctx->stream));
  RX_HIP(hipEventSynchronize(e1));
  float t = 0.0f;
  RX_HIP(hipEventElapsedTime(&t, e0, e1));
  *ms = t / reps;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return RX_OK;
}
#endif
