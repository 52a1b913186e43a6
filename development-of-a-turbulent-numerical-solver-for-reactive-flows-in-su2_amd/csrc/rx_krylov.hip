// rx_krylov.hip — device-resident FGMRES (CSysSolve::FGMRES_LinSolver,
// Common/src/linear_solvers_structure.cpp:309-463, ModGramSchmidt :87-186, ApplyGivens /
// GenerateGivens :37-71, SolveReduced :73-85).
//
// Every scalar of the Krylov recurrence (norms, Hessenberg entries, Givens rotations, the
// stop/breakdown decisions and the re-orthogonalisation test of MGS) lives in device memory and is
// updated by the lead lane of the kernel that produces it, in the reference's operation order; the
// other lanes evaluate the same decisions from the same inputs. The solve is therefore a fixed
// sequence of kernels with no host round trip (replayed as one hipGraph by rx_implicit_euler), and
// kernels after a stop decision see the `done` flag and return.
//
// Fusion: every vector kernel also produces the inner product the recurrence needs next
// (SpMV -> |w|^2 and <w, w_0>; projection k -> <w, w_{k+1}> or |w|^2 or, when MGS re-orthogonalises,
// <w, w_k>), reduced inside the launch: each of the 512 blocks reduces its grid-stride partial with a
// fixed tree, publishes it with a write-through (sc1) store, takes an arrival ticket, and the last
// block to arrive sums the partials in a fixed tree (MI355X_MICROARCH.md, inter-workgroup hand-off
// with sc1 stores/loads). The summation order is fixed (independent of arrival order); the oracle's
// orc_dot mode 1 restates it. The reference sums sequentially, so results agree to rounding.
//
// Distributed (one rank per GPU): every reducing kernel publishes its rank-local sums in
// KState::loc[4] (slots not produced are zero), and an out-of-place all-reduce loc -> the landing
// slots {norm0_in, dot, dotn, dot2} follows each reducing launch (dotProd's MPI_Allreduce,
// Common/src/vector_structure.cpp:397-419). A skipped kernel leaves loc unchanged, so the
// all-reduce after it is idempotent and every rank takes the same decisions. Single rank: the
// reducer writes the landing slots itself and no collective is issued. Vectors have N*nVar rows;
// inner products and updates run over the owned prefix Nd*nVar, the preconditioned vector z_i gets
// its halo from the neighbours before the SpMV reads it (MatrixVectorProduct :997-1029 +
// SendReceive_Solution :794).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "rx_ctx.h"

namespace {

constexpr int kBlock = 256;
constexpr int kRedBlocks = 512;  // every reducing kernel runs exactly this grid (grid-stride loops)
constexpr int kMaxM = 64;
inline int blocks(int64_t n, int b = kBlock) { return (int)((n + b - 1) / b); }

struct KState {
  double tol, norm0, beta, nrm, thr2[2], prod, resid;  // thr2: read thr2[k&1], write thr2[(k+1)&1]
  double norm0_in, dot, dotn, dot2;  // inner-product landing slots (all-reduced), contiguous
  double loc[4];                     // rank-local sums in landing-slot order
  int done, noreo, iters, diverged, conv;
  unsigned int ticket;          // arrival counter of the in-launch reductions
  double bnorm;                 // |b| of the solve (RESTARTED_FGMRES's tolerance update reads it)
  double bc_alpha, bc_omega, bc_rho[2];  // BCGSTAB scalars; rho of iteration i in bc_rho[i & 1]
  double H[(kMaxM + 1) * kMaxM];  // H[k][i] at k * kMaxM + i
  double g[kMaxM + 1], cs[kMaxM + 1], sn[kMaxM + 1], y[kMaxM];
};

__device__ inline double& Hk(KState* s, int k, int i) { return s->H[k * kMaxM + i]; }
__device__ inline bool lead() { return blockIdx.x == 0 && threadIdx.x == 0; }

// Block tree (256 lanes, halving) of NR values; results in sh[r * kBlock].
template <int NR>
__device__ inline void block_tree(double* sh) {
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
#pragma unroll
      for (int r = 0; r < NR; ++r) sh[r * kBlock + threadIdx.x] += sh[r * kBlock + threadIdx.x + w];
    }
    __syncthreads();
  }
}

enum Slot { kNorm0In = 0, kDot = 1, kDotN = 2, kDot2 = 3 };
__device__ inline double* land(KState* s) { return &s->norm0_in; }

// In-launch grid reduction of NR partial sums into landing slots slot[r] (see header); the other
// landing slots are zeroed in loc. part: [NR][kRedBlocks].
template <int NR>
__device__ inline void grid_reduce(const double (&v)[NR], double* __restrict__ part, KState* __restrict__ s,
                                   const int (&slot)[NR], bool dist) {
  unsigned int* ticket = &s->ticket;
  __shared__ double sh[NR * kBlock + 1];
  int* last = reinterpret_cast<int*>(sh + NR * kBlock);
#pragma unroll
  for (int r = 0; r < NR; ++r) sh[r * kBlock + threadIdx.x] = v[r];
  block_tree<NR>(sh);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int r = 0; r < NR; ++r)
      __hip_atomic_store(part + r * kRedBlocks + blockIdx.x, sh[r * kBlock], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = (t == kRedBlocks - 1);
  }
  __syncthreads();
  if (!*last) return;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const double a =
        __hip_atomic_load(part + r * kRedBlocks + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double b =
        __hip_atomic_load(part + r * kRedBlocks + kBlock + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh[r * kBlock + threadIdx.x] = a + b;
  }
  block_tree<NR>(sh);
  if (threadIdx.x == 0) {
    double* dst = dist ? s->loc : land(s);
    for (int r = 0; r < 4; ++r) dst[r] = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) dst[slot[r]] = sh[r * kBlock];
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

#define GRID_LOOP(q, n) \
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < (n); q += (int64_t)kRedBlocks * kBlock)

// The same grid-stride walk, kU elements per round: every load of the round is issued before the first element's
// arithmetic, then the elements are processed in the walk's order (q, q + S, ..., S = the reduction grid's thread
// count), so each thread's partial sums and stores are GRID_LOOP's, operation for operation. The 512-block reduction
// grid runs 2 wavefronts per SIMD; with one element per round each thread had a single load chain in flight.
#ifndef RX_FG_U
#define RX_FG_U 4
#endif
constexpr int kU = RX_FG_U;
constexpr int64_t kGridS = (int64_t)kRedBlocks * kBlock;
#define GRID_LOOP_U(q0, n) for (int64_t q0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; q0 < (n); q0 += kU * kGridS)

// Row-block product of y = A x for element q = (row i, component a): the reference's
// MatrixVectorProduct order (blocks of the row in column order, columns c ascending).
// Small blocks (the SST's 2x2) are taken kSpmvChunk at a time: the chunk's column indices, then all of its
// matrix-row and x loads, are issued before the first product (loads from clamped, always valid addresses; the
// sums of the blocks past the row's end are skipped). Measured on one box at C3: the SST solve 2.14 -> 2.05 ms;
// for the 11x11 flow blocks chunks of 3 / 5 made the solve slower (15.40 -> 16.14 / 15.70 ms), so those keep
// one block at a time.
#ifndef RX_SPMV_CHUNK_BIG
#define RX_SPMV_CHUNK_BIG 1  // build knob: blocks per chunk for NV > 4
#endif
template <int NV>
constexpr int rx_spmv_chunk() {
  return NV <= 4 ? 5 : RX_SPMV_CHUNK_BIG;
}
template <int NV>
__device__ inline double spmv_elem(int64_t q, const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
                                   const double* __restrict__ A, const double* __restrict__ x) {
  constexpr int kSpmvChunk = rx_spmv_chunk<NV>();
  const int i = (int)(q / NV), a = (int)(q - (int64_t)i * NV);
  const int k0 = rp[i], k1 = rp[i + 1];
  double acc = 0.0;
  for (int k = k0; k < k1; k += kSpmvChunk) {
    int cc[kSpmvChunk];
#pragma unroll
    for (int t = 0; t < kSpmvChunk; ++t) cc[t] = col[k + t < k1 ? k + t : k];
    double av[kSpmvChunk][NV], xv[kSpmvChunk][NV];
#pragma unroll
    for (int t = 0; t < kSpmvChunk; ++t) {
      const double* blk = A + (size_t)(k + t < k1 ? k + t : k) * NV * NV + a * NV;
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        av[t][c] = blk[c];
        xv[t][c] = x[(size_t)cc[t] * NV + c];
      }
    }
#pragma unroll
    for (int t = 0; t < kSpmvChunk; ++t)
      if (k + t < k1) {
#pragma unroll
        for (int c = 0; c < NV; ++c) acc += av[t][c] * xv[t][c];
      }
  }
  return acc;
}

// |b|^2 -> norm0_in, w0 = A x - b and |w0|^2 -> dot (owned rows Nd)
template <int NV>
__global__ __launch_bounds__(kBlock) void k_fg_residual(int Nd, const int32_t* __restrict__ rp,
                                                        const int32_t* __restrict__ col, const double* __restrict__ A,
                                                        const double* __restrict__ x, const double* __restrict__ b,
                                                        double* __restrict__ w, double* __restrict__ part,
                                                        KState* __restrict__ s, bool dist) {
  const int64_t n = (int64_t)Nd * NV;
  double v[2] = {0.0, 0.0};
  GRID_LOOP(q, n) {
    const double bq = b[q];
    v[0] += bq * bq;
    double y = spmv_elem<NV>(q, rp, col, A, x);
    y -= bq;
    w[q] = y;
    v[1] += y * y;
  }
  const int sl[2] = {kNorm0In, kDot};
  grid_reduce<2>(v, part, s, sl, dist);
}

// k_fg_residual for x = 0 (ImplicitEuler_Iteration zeroes LinSysSol before the solve, solver_direct_reactive.cpp:2373 / :2384): A x is then
// +0.0 in every element for a FINITE A (spmv_elem sums from +0.0, so +0 + (+-0) = +0), and w0 = +0.0 - b is the
// same double as the product path gives, with the same grid loop and reduction, without streaming the matrix.
// For a non-finite A (Inf / NaN entries) the reference's A * 0 makes w0 NaN at the first residual; here w0 stays
// -b and the NaN enters at the first SpMV, one Krylov step later. Either way the update is non-finite and the
// following SetPrimitive_Variables / rx_sync report it; RX_FG_X_PRODUCT=1 restores the product path.
__global__ __launch_bounds__(kBlock) void k_fg_residual0(int64_t n, const double* __restrict__ b,
                                                         double* __restrict__ w, double* __restrict__ part,
                                                         KState* __restrict__ s, bool dist) {
  double v[2] = {0.0, 0.0};
  GRID_LOOP_U(q0, n) {
    double bb[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) bb[u] = b[q0 + u * kGridS];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) {
        const double bq = bb[u];
        v[0] += bq * bq;
        const double y = 0.0 - bq;
        w[q0 + u * kGridS] = y;
        v[1] += y * y;
      }
  }
  const int sl[2] = {kNorm0In, kDot};
  grid_reduce<2>(v, part, s, sl, dist);
}

// w_{i+1} = A z_i on a full grid (one thread per element, every CU filled like k_spmv); the inner products follow
// in k_fg_spmv_dots.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_fg_spmv_full(int Nd, const int32_t* __restrict__ rp,
                                                         const int32_t* __restrict__ col, const double* __restrict__ A,
                                                         const double* __restrict__ z, double* __restrict__ w,
                                                         const KState* __restrict__ s) {
  if (s->done) return;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < (int64_t)Nd * NV) w[q] = spmv_elem<NV>(q, rp, col, A, z);
}

// k_fg_spmv_full for the flow blocks (NV > 4) with the blocks staged through LDS (round 5). Element (row i, component
// a) on one lane reads row a of each block: 88 contiguous bytes per lane, so each of a wavefront's six block loads
// touched ~44 cache lines for 1 KiB (the kernel's waves were 72 % waiting on instruction issue, r05_c3_stall.json).
// Here a wavefront owns NN = 64 / NV whole rows of the system and walks their blocks by position s (s-th block of each
// row at once): the NN blocks are copied to the wavefront's LDS slot by consecutive lanes (each load 512 contiguous
// bytes but for a row boundary), the NN x columns gathered one double per lane, then lane (row, a) makes its sum from
// LDS. Every sum is spmv_elem's: the blocks of the row in column order, columns ascending, from +0.0, so w is bitwise
// k_fg_spmv_full's.
// Same box at C3 (profiles/r05_ab_s.txt, two runs each): 949 / 963 us per SpMV with k_fg_spmv_full, 918 / 915 staged,
// 897 / 886 staged with the column indices read once and the next step's blocks loaded during this one (the default);
// C5 1 448 -> 1 430 -> 1 413 us.
#ifndef RX_SPMV_STAGE
#define RX_SPMV_STAGE 2  // build knob: 0 = k_fg_spmv_full for every block size; 1 = staged, one step's loads at a time
#endif
#ifndef RX_SPMV_XCD
#define RX_SPMV_XCD 0  // build knob: 1 = consecutive workgroups' rows on one XCD (its L2 then holds their x columns)
#endif
__device__ inline int spmv_block(int b, int nb) {  // workgroup b's position: XCD x = b mod 8 takes the x-th eighth
  if (!RX_SPMV_XCD) return b;
  constexpr int kXcd = 8;
  const int x = b % kXcd, idx = b / kXcd, q = nb / kXcd, r = nb % kXcd;
  return x < r ? x * (q + 1) + idx : r * (q + 1) + (x - r) * q + idx;
}
template <int NV>
__global__ __launch_bounds__(kBlock) void k_fg_spmv_stage(int n_rows, const int32_t* __restrict__ rows,
                                                          const int32_t* __restrict__ rp,
                                                          const int32_t* __restrict__ col,
                                                          const double* __restrict__ A, const double* __restrict__ z,
                                                          double* __restrict__ w, const KState* __restrict__ s) {
  // rows == nullptr: the system's rows 0 .. n_rows - 1; else the row list rows[0 .. n_rows) (a distributed solve's
  // interior / rank-boundary rows, k_fg_spmv_rows's)
  constexpr int NN = 64 / NV, B2 = NV * NV, CH = NN * B2, NL = (CH + 63) / 64, WPB = kBlock / 64;
  __shared__ double sa[WPB][CH];
  __shared__ double sx[WPB][NN * NV];
  if (s->done) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l0 = (spmv_block(blockIdx.x, gridDim.x) * WPB + wv) * NN;  // the wavefront's first row (of the list)
  if (l0 >= n_rows) return;                      // (uniform over the wavefront)
  // lane j < NN: the wavefront's j-th row, its first block and its block count (none past the end)
  const bool lv = lane < NN && l0 + lane < n_rows;
  const int rowl = lv ? (rows ? rows[l0 + lane] : l0 + lane) : 0;
  const int kb = lv ? rp[rowl] : 0, kd = lv ? rp[rowl + 1] - kb : 0;
  int rb[NN], rd[NN];
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    rb[j] = __builtin_amdgcn_readfirstlane(__shfl(kb, j));
    rd[j] = __builtin_amdgcn_readfirstlane(__shfl(kd, j));
  }
  int maxdeg = 0;
#pragma unroll
  for (int j = 0; j < NN; ++j) maxdeg = max(maxdeg, rd[j]);
  // this lane's share of a step's chunk: element e = u * 64 + lane is entry off of row j's block
  int64_t base[NL];
  int deg[NL];
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    const int e = u * 64 + lane, j = e < CH ? e / B2 : 0, off = e < CH ? e - j * B2 : 0;
    int rj = rb[0], dj = rd[0];
#pragma unroll
    for (int q = 1; q < NN; ++q)
      if (j == q) {
        rj = rb[q];
        dj = rd[q];
      }
    base[u] = (int64_t)rj * B2 + off;
    deg[u] = e < CH ? dj : 0;
  }
  // the x gather: lane l < NN NV fetches component l % NV of row l / NV's s-th column
  const int xj = lane < NN * NV ? lane / NV : 0, xc = lane - xj * NV;
  int xr = rb[0], xd = rd[0];
#pragma unroll
  for (int q = 1; q < NN; ++q)
    if (xj == q) {
      xr = rb[q];
      xd = rd[q];
    }
  if (lane >= NN * NV) xd = 0;
  // this lane's element
  const int n = lane / NV, a = lane - n * NV;
  const bool act = n < NN && l0 + n < n_rows;
  const int i = __shfl(rowl, n < NN ? n : 0);
  int nd = 0;
#pragma unroll
  for (int q = 0; q < NN; ++q)
    if (n == q) nd = rd[q];
  double acc = 0.0;
  double* sw = sa[wv];
  double* sxw = sx[wv];
  // RX_SPMV_STAGE=2: the rows' column indices read once up front (when the wavefront's rows are one contiguous range
  // of at most 64 blocks, else from global memory at each step) and each step's blocks loaded during the previous step
  const int r0 = rb[0], rng = rows ? 65 : rp[min(l0 + NN, n_rows)] - r0;
  const int cl = RX_SPMV_STAGE == 2 && lane < rng && lane < 64 && !rows ? col[r0 + lane] : 0;
  const bool cpre = RX_SPMV_STAGE == 2 && rng <= 64;
  double v[NL];
  auto load = [&](int st) {
#pragma unroll
    for (int u = 0; u < NL; ++u) v[u] = st < deg[u] ? A[base[u] + (int64_t)st * B2] : 0.0;
  };
  if (RX_SPMV_STAGE == 2) load(0);
  for (int st = 0; st < maxdeg; ++st) {
    if (RX_SPMV_STAGE != 2) load(st);
    // (the permute runs on every lane, from a lane index kept in range; the global reads only where the row has an
    // st-th block)
    const int xcp = RX_SPMV_STAGE == 2 ? __shfl(cl, min(max(xr + st - r0, 0), 63)) : 0;
    const double xv = st < xd ? z[(int64_t)(cpre ? xcp : col[xr + st]) * NV + xc] : 0.0;
#pragma unroll
    for (int u = 0; u < NL; ++u)
      if (u * 64 + lane < CH) sw[u * 64 + lane] = v[u];
    if (RX_SPMV_STAGE == 2 && st + 1 < maxdeg) load(st + 1);
    if (lane < NN * NV) sxw[lane] = xv;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (act && st < nd) {
      const double* ar = sw + n * B2 + a * NV;
      const double* xr_ = sxw + n * NV;
#pragma unroll
      for (int c = 0; c < NV; ++c) acc += ar[c] * xr_[c];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  if (act) w[(int64_t)i * NV + a] = acc;
}

// k_fg_spmv_full over a row list (rows[0..n)): the same element arithmetic at the same positions. A distributed
// solve computes the rows without halo columns while the preconditioned vector's halo is in flight, then the rest.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_fg_spmv_rows(int n, const int32_t* __restrict__ rows,
                                                         const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                         const double* __restrict__ A, const double* __restrict__ z,
                                                         double* __restrict__ w, const KState* __restrict__ s) {
  if (s->done) return;
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (int64_t)n * NV) return;
  const int r = (int)(t / NV), a = (int)(t - (int64_t)r * NV);
  const int64_t q = (int64_t)rows[r] * NV + a;
  w[q] = spmv_elem<NV>(q, rp, col, A, z);
}

// |w_{i+1}|^2 -> dotn and <w_{i+1}, w_0> -> dot over the stored product, in k_fg_spmv's grid-stride order (each
// thread sums the same elements in the same order, then the same fixed trees): bitwise k_fg_spmv's sums.
__global__ __launch_bounds__(kBlock) void k_fg_spmv_dots(int64_t n, const double* __restrict__ w0,
                                                         const double* __restrict__ w, double* __restrict__ part,
                                                         KState* __restrict__ s, bool dist) {
  if (s->done) return;
  double v[2] = {0.0, 0.0};
  GRID_LOOP_U(q0, n) {
    double y[kU], z[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t q = q0 + u * kGridS;
      if (q < n) {
        y[u] = w[q];
        z[u] = w0[q];
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) {
        v[0] += y[u] * y[u];
        v[1] += y[u] * z[u];
      }
  }
  const int sl[2] = {kDotN, kDot};
  grid_reduce<2>(v, part, s, sl, dist);
}

// w_{i+1} = A z_i with |w_{i+1}|^2 -> dotn and <w_{i+1}, w_0> -> dot (one launch on the 512-block reduction grid;
// RX_FG_FUSED_SPMV=1 selects it instead of k_fg_spmv_full + k_fg_spmv_dots)
template <int NV>
__global__ __launch_bounds__(kBlock) void k_fg_spmv(int Nd, const int32_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col, const double* __restrict__ A,
                                                    const double* __restrict__ z, const double* __restrict__ w0,
                                                    double* __restrict__ w, double* __restrict__ part,
                                                    KState* __restrict__ s, bool dist) {
  if (s->done) return;
  const int64_t n = (int64_t)Nd * NV;
  double v[2] = {0.0, 0.0};
  GRID_LOOP(q, n) {
    const double y = spmv_elem<NV>(q, rp, col, A, z);
    w[q] = y;
    v[0] += y * y;
    v[1] += y * w0[q];
  }
  const int sl[2] = {kDotN, kDot};
  grid_reduce<2>(v, part, s, sl, dist);
}

// w0 = w0 / (-beta) after the start decision (:318-330), evaluated identically by every lane.
__global__ __launch_bounds__(kBlock) void k_fg_start_div(int64_t n, KState* __restrict__ s, double* __restrict__ w0) {
  const double norm0 = sqrt(s->norm0_in);
  const double beta = sqrt(s->dot);
  const double epsm = 2.220446049250313e-16;
  const bool early = (beta < s->tol * norm0) || (beta < epsm);
  if (early) {
    if (lead()) {
      s->done = 1;
      s->resid = beta;
      s->beta = beta;
      s->norm0 = norm0;
      s->bnorm = norm0;
    }
    return;
  }
  if (lead()) {
    s->bnorm = norm0;
    s->g[0] = beta;
    s->norm0 = beta;
    s->beta = beta;
  }
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < n) w0[q] /= -beta;
}

// w -= prod * wk over this thread's walk, with the partial sum of y * wn (wn null: y * y) in walk order.
__device__ __forceinline__ void proj_walk(int64_t n, double prod, const double* wk, double* w, const double* wn,
                                          double& acc) {
  GRID_LOOP_U(q0, n) {
    double a[kU], b[kU], c[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t q = q0 + u * kGridS;
      if (q < n) {
        a[u] = w[q];
        b[u] = wk[q];
        if (wn) c[u] = wn[q];
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t q = q0 + u * kGridS;
      if (q < n) {
        const double y = a[u] + (-1.0 * prod) * b[u];
        w[q] = y;
        acc += y * (wn ? c[u] : y);
      }
    }
  }
}

// ModGramSchmidt (:87-186) projection k of iteration i: H[k][i] = prod = <w, w_k> (in s->dot),
// w -= prod w_k, the re-orthogonalisation test prod^2 > thr, and the inner product the recurrence
// needs next: <w, w_k> (re-orthogonalise), else <w, w_{k+1}> (k < i) or |w|^2 (k == i).
// For k = 0 also ModGramSchmidt's entry: nrm = |w|^2 (s->dotn), thr = 0.98 nrm, breakdown test.
__global__ __launch_bounds__(kBlock) void k_fg_proj(int64_t n, int64_t ld, KState* __restrict__ s, int k, int i,
                                                    double* __restrict__ W, double* __restrict__ part, bool dist) {
  if (s->done) return;
  double nrm0 = 0.0;
  if (k == 0) {
    nrm0 = s->dotn;
    if ((nrm0 <= 0.0) || (nrm0 != nrm0)) {
      if (lead()) {
        s->diverged = 1;
        s->done = 1;
      }
      return;
    }
  }
  const double prod = s->dot;
  const double thr = (k == 0) ? nrm0 * 0.98 : s->thr2[k & 1];
  const bool reo = prod * prod > thr;
  const double* wk = W + (int64_t)k * ld;
  double* w = W + (int64_t)(i + 1) * ld;
  const double* wn = reo ? wk : (k < i ? W + (int64_t)(k + 1) * ld : nullptr);
  double v[1] = {0.0};
  proj_walk(n, prod, wk, w, wn, v[0]);
  if (lead()) {
    if (k == 0) s->nrm = nrm0;
    Hk(s, k, i) = prod;
    s->prod = prod;
    s->noreo = reo ? 0 : 1;
    if (!reo) {
      s->nrm -= Hk(s, k, i) * Hk(s, k, i);
      if (s->nrm < 0.0) s->nrm = 0.0;
      s->thr2[(k + 1) & 1] = s->nrm * 0.98;
    }
  }
  const int sl[1] = {reo ? kDot2 : (k < i ? kDot : kDotN)};
  grid_reduce<1>(v, part, s, sl, dist);
}

// Second projection when the test fired: H[k][i] += prod2, w -= prod2 w_k, norm update, and the
// next inner product (<w, w_{k+1}> or |w|^2).
__global__ __launch_bounds__(kBlock) void k_fg_reo(int64_t n, int64_t ld, KState* __restrict__ s, int k, int i,
                                                   double* __restrict__ W, double* __restrict__ part, bool dist) {
  if (s->done || s->noreo) return;
  const double prod = s->dot2;
  const double* wk = W + (int64_t)k * ld;
  double* w = W + (int64_t)(i + 1) * ld;
  const double* wn = k < i ? W + (int64_t)(k + 1) * ld : nullptr;
  double v[1] = {0.0};
  proj_walk(n, prod, wk, w, wn, v[0]);
  if (lead()) {
    Hk(s, k, i) += prod;
    s->nrm -= Hk(s, k, i) * Hk(s, k, i);
    if (s->nrm < 0.0) s->nrm = 0.0;
    s->thr2[(k + 1) & 1] = s->nrm * 0.98;
  }
  const int sl[1] = {k < i ? kDot : kDotN};
  grid_reduce<1>(v, part, s, sl, dist);
}

__device__ inline void apply_givens(double sn, double cs, double& h1, double& h2) {
  const double t = cs * h1 + sn * h2;
  h2 = cs * h2 - sn * h1;
  h1 = t;
}
__device__ inline double sign_of(double a, double b) { return b == 0.0 ? 0.0 : (b < 0 ? -fabs(a) : fabs(a)); }

// H[i+1][i] = |w|, Givens rotations (:37-71), beta = |g[i+1]|, and the stop test of the next
// iteration's top (:339), published in `conv` (the next iteration's first kernel turns it into done).
__device__ void fg_close(KState* s, int i) {
  s->nrm = sqrt(s->dotn);
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
  if (s->beta < s->tol * s->norm0) s->conv = 1;
}

// w_{i+1} /= |w_{i+1}| (all lanes) and fg_close (lead lane).
__global__ __launch_bounds__(kBlock) void k_fg_close_div(int64_t n, KState* __restrict__ s, int i,
                                                         double* __restrict__ w) {
  if (s->done) return;
  const double nrm = sqrt(s->dotn);
  GRID_LOOP_U(q0, n) {
    double a[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) a[u] = w[q0 + u * kGridS];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) w[q0 + u * kGridS] = a[u] / nrm;
  }
  if (lead()) fg_close(s, i);
}

// Per-solve initialisation; g = 0 as the reference's std::vector<su2double> g(m+1, 0.0) (:349):
// the Givens update of column i reads g[i+1] before writing it.
__global__ void k_fg_reset(KState* s, double tol) {
  for (int k = threadIdx.x; k <= kMaxM; k += blockDim.x) s->g[k] = 0.0;
  if (threadIdx.x != 0) return;
  s->tol = tol;
  s->done = 0;
  s->conv = 0;
  s->noreo = 1;
  s->iters = 0;
  s->diverged = 0;
  s->resid = 0.0;
  s->bc_alpha = s->bc_omega = 1.0;  // BCGSTAB_LinSolver :509
  s->bc_rho[0] = s->bc_rho[1] = 1.0;
}

// SolveReduced (:73-85) and x += sum_k y_k z_k (k ascending, element by element as the reference's
// per-k vector updates). Every block solves the small triangular system itself.
__global__ __launch_bounds__(kBlock) void k_fg_finish(int64_t n, int64_t ld, KState* __restrict__ s,
                                                      const double* __restrict__ Z, double* __restrict__ x) {
  if (s->diverged) return;
  __shared__ double y[kMaxM];
  const int it = s->iters;
  if (threadIdx.x == 0) {
    for (int k = 0; k < it; ++k) y[k] = s->g[k];
    for (int k = it - 1; k >= 0; --k) {
      y[k] /= Hk(s, k, k);
      for (int j = k - 1; j >= 0; --j) y[j] -= Hk(s, j, k) * y[k];
    }
  }
  __syncthreads();
  if (lead()) {
    if (it > 0 || !s->done) s->resid = s->beta;
    for (int k = 0; k < it; ++k) s->y[k] = y[k];
  }
  if (it == 0) return;
  GRID_LOOP_U(q0, n) {
    double v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) v[u] = x[q0 + u * kGridS];
    for (int k = 0; k < it; ++k) {
      double zz[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (q0 + u * kGridS < n) zz[u] = Z[(int64_t)k * ld + q0 + u * kGridS];
#pragma unroll
      for (int u = 0; u < kU; ++u) v[u] += y[k] * zz[u];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) x[q0 + u * kGridS] = v[u];
  }
}

// ---- BCGSTAB_LinSolver (linear_solvers_structure.cpp:465-599) and the smoothers of Solve's non-Krylov branch
// (:683-708; LU_SGS_Smoother / Jacobi_Smoother / ILU0_Smoother, matrix_structure.cpp:1711 / :1268 / :1517).
// The same device-resident scheme as FGMRES: scalars in KState, updated by lead lanes in the reference's operation
// order, every lane evaluating the decisions from the same inputs, inner products reduced inside the launch.

// r = b - A x (x_zero: b - 0.0, the +0.0 product of A * 0 for a finite A; see k_fg_residual0) with |b|^2 ->
// norm0_in and |r|^2 -> dot; BCGSTAB also copies r_0 = r and starts p = v = b (its CSysVector p(b), v(b), :486-499).
template <int NV, bool XZ>
__global__ __launch_bounds__(kBlock) void k_lin_resid(int Nd, const int32_t* __restrict__ rp,
                                                      const int32_t* __restrict__ col, const double* __restrict__ A,
                                                      const double* __restrict__ x, const double* __restrict__ b,
                                                      double* __restrict__ r, double* __restrict__ r0,
                                                      double* __restrict__ p, double* __restrict__ v,
                                                      double* __restrict__ part, KState* __restrict__ s, bool dist) {
  if (s->done) return;
  const int64_t n = (int64_t)Nd * NV;
  double acc[2] = {0.0, 0.0};
  GRID_LOOP(q, n) {
    const double bq = b[q];
    acc[0] += bq * bq;
    double ax = 0.0;
    if constexpr (!XZ) ax = spmv_elem<NV>(q, rp, col, A, x);
    const double y = bq - ax;
    r[q] = y;
    if (r0) r0[q] = y;
    if (p) p[q] = bq;
    if (v) v[q] = bq;
    acc[1] += y * y;
  }
  const int sl[2] = {kNorm0In, kDot};
  grid_reduce<2>(acc, part, s, sl, dist);
}

// the start test (:500-505 / :1302-1307): norm_r = |r|, norm0 = |b|; solved by the initial guess -> done, 0
// iterations; else norm0 = norm_r (:513)
__global__ void k_lin_start(KState* s) {
  const double norm_r = sqrt(s->dot), norm0 = sqrt(s->norm0_in);
  const double epsm = 2.220446049250313e-16;  // numeric_limits<su2double>::epsilon() (matrix_structure.hpp:49)
  s->bnorm = norm0;
  s->resid = norm_r;
  s->iters = 0;
  if ((norm_r < s->tol * norm0) || (norm_r < epsm)) {
    s->done = 1;
    return;
  }
  s->norm0 = norm_r;
}

// the convergence test closing iteration i (:575-576 / :1352-1353): break with i iterations, else i + 1
__global__ void k_lin_check(KState* s, int i, int slot) {
  if (s->done) return;
  const double norm_r = sqrt(land(s)[slot]);
  s->resid = norm_r;
  if (norm_r < s->tol * s->norm0) {
    s->done = 1;
    s->iters = i;
  } else {
    s->iters = i + 1;
  }
}

// rho_i = <r, r_0> -> dot (:533)
__global__ __launch_bounds__(kBlock) void k_bc_rho(int64_t n, const double* __restrict__ r,
                                                   const double* __restrict__ r0, double* __restrict__ part,
                                                   KState* __restrict__ s, bool dist) {
  if (s->done) return;
  double acc[1] = {0.0};
  GRID_LOOP_U(q0, n) {
    double a[kU], c[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) {
        a[u] = r[q0 + u * kGridS];
        c[u] = r0[q0 + u * kGridS];
      }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (q0 + u * kGridS < n) acc[0] += a[u] * c[u];
  }
  const int sl[1] = {kDot};
  grid_reduce<1>(acc, part, s, sl, dist);
}

// beta = (rho_i / rho_{i-1}) (alpha / omega), p = beta p + (-beta omega) v, p += 1.0 r (:529-543)
__global__ __launch_bounds__(kBlock) void k_bc_p(int64_t n, KState* __restrict__ s, int i,
                                                 const double* __restrict__ r, const double* __restrict__ v,
                                                 double* __restrict__ p) {
  if (s->done) return;
  const double rho = s->dot, rho_prime = s->bc_rho[(i + 1) & 1];
  const double beta = (rho / rho_prime) * (s->bc_alpha / s->bc_omega);
  const double beta_omega = -beta * s->bc_omega;
  if (lead()) s->bc_rho[i & 1] = rho;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < n) {
    const double t = beta * p[q] + beta_omega * v[q];
    p[q] = t + 1.0 * r[q];
  }
}

// alpha = rho_i / <r_0, v> (:552-553), s = 1.0 r + (-alpha) v (:557)
__global__ __launch_bounds__(kBlock) void k_bc_s(int64_t n, KState* __restrict__ s, int i,
                                                 const double* __restrict__ r, const double* __restrict__ v,
                                                 double* __restrict__ sv) {
  if (s->done) return;
  const double alpha = s->bc_rho[i & 1] / s->dot;
  if (lead()) s->bc_alpha = alpha;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < n) sv[q] = 1.0 * r[q] + (-alpha) * v[q];
}

// omega = <t, s> / <t, t> (:566), x += alpha phat, x += omega shat (:570), r = 1.0 s + (-omega) t (:571) and
// |r|^2 -> dot2 (:575)
__global__ __launch_bounds__(kBlock) void k_bc_x(int64_t n, KState* __restrict__ s, double* __restrict__ x,
                                                 const double* __restrict__ ph, const double* __restrict__ sh,
                                                 const double* __restrict__ sv, const double* __restrict__ t,
                                                 double* __restrict__ r, double* __restrict__ part, bool dist) {
  if (s->done) return;
  const double omega = s->dot / s->dotn, alpha = s->bc_alpha;
  double acc[1] = {0.0};
  GRID_LOOP(q, n) {
    double xq = x[q];
    xq += alpha * ph[q];
    xq += omega * sh[q];
    x[q] = xq;
    const double y = 1.0 * sv[q] + (-omega) * t[q];
    r[q] = y;
    acc[0] += y * y;
  }
  if (lead()) s->bc_omega = omega;
  const int sl[1] = {kDot2};
  grid_reduce<1>(acc, part, s, sl, dist);
}

// the LU_SGS / ILU0 smoothers' update x.Plus_AX(omega = 1.0, M^-1 r) (matrix_structure.cpp:1805 / :1642)
__global__ __launch_bounds__(kBlock) void k_sm_add(int64_t n, const KState* __restrict__ s,
                                                   const double* __restrict__ z, double* __restrict__ x) {
  if (s->done) return;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < n) x[q] += 1.0 * z[q];
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

// device address of the landing slots (host-side pointer arithmetic on the device KState)
double* land_host(KState* s) { return &s->norm0_in; }

// distributed: the preconditioner's closing halo exchange (SendReceive_Solution, matrix_structure.cpp:1513 / :1707 /
// :1264) is deferred and overlaps the SpMV rows that read no halo column (on comm_stream with RCCL)
bool spmv_split(const rx_ctx* ctx) {
  static const bool off = getenv("RX_NO_SPMV_SPLIT") != nullptr;
  return ctx->distributed() && ctx->spmv_rows && !off;
}

// CSysSolve's `precond(in, z)` + `mat_vec(z, w)` pair: z = M^-1 in (halo exchanged), w = A z over the owned rows
// (MatrixVectorProduct :997-1029). RxPhase records only outside a graph capture: an eager solve (RX_NO_GRAPH=1,
// bench.py's kernel-timing pass) times the in-solve preconditioner applies and SpMVs themselves.
int prec_spmv(rx_ctx* ctx, const double* in, double* z, double* w, KState* s) {
  hipStream_t st = ctx->stream;
  const double* A = ctx->f[RX_F_JAC];
  const bool split = spmv_split(ctx);
  ctx->defer_exchange = split;
  int rc = rx_la_prec_apply(ctx, in, z, &s->done, &s->conv);
  ctx->defer_exchange = false;
  if (rc) return rc;
  if (!split) {
    RxPhase ph(ctx, RX_K_SPMV);
    if (RX_SPMV_STAGE && ctx->nVar > 4) {
      RX_NV_SWITCH(ctx->nVar, (k_fg_spmv_stage<NV_><<<blocks(ctx->Nd, (kBlock / 64) * (64 / NV_)), kBlock, 0, st>>>(
                                  (int)ctx->Nd, nullptr, ctx->rp, ctx->col, A, z, w, s)));
    } else {
      RX_NV_SWITCH(ctx->nVar, (k_fg_spmv_full<NV_><<<blocks(ctx->Nd * NV_), kBlock, 0, st>>>((int)ctx->Nd, ctx->rp,
                                                                                            ctx->col, A, z, w, s)));
    }
    return RX_OK;
  }
  const bool overlap = ctx->comm_stream != nullptr && !ctx->has_hcomm;
  if (overlap) {
    RX_HIP(hipEventRecord(ctx->comm_fork, st));
    RX_HIP(hipStreamWaitEvent(ctx->comm_stream, ctx->comm_fork, 0));
    if ((rc = rx_la_exchange_on(ctx, z, ctx->nVar, ctx->comm_stream))) return rc;
    RX_HIP(hipEventRecord(ctx->comm_join, ctx->comm_stream));
  } else if ((rc = rx_la_exchange(ctx, z, ctx->nVar))) {
    return rc;
  }
  const int ni = (int)ctx->n_spmv_int, nb_rows = (int)(ctx->Nd - ctx->n_spmv_int);
  RxPhase ph(ctx, RX_K_SPMV);
  auto rows_spmv = [&](int n, const int32_t* rows) -> int {
    if (RX_SPMV_STAGE && ctx->nVar > 4) {
      RX_NV_SWITCH(ctx->nVar, (k_fg_spmv_stage<NV_><<<blocks(n, (kBlock / 64) * (64 / NV_)), kBlock, 0, st>>>(
                                  n, rows, ctx->rp, ctx->col, A, z, w, s)));
    } else {
      RX_NV_SWITCH(ctx->nVar, (k_fg_spmv_rows<NV_><<<blocks((int64_t)n * NV_), kBlock, 0, st>>>(
                                  n, rows, ctx->rp, ctx->col, A, z, w, s)));
    }
    return RX_OK;
  };
  if (ni > 0 && (rc = rows_spmv(ni, ctx->spmv_rows))) return rc;
  if (overlap) RX_HIP(hipStreamWaitEvent(st, ctx->comm_join, 0));
  if (nb_rows > 0 && (rc = rows_spmv(nb_rows, ctx->spmv_rows + ni))) return rc;
  return RX_OK;
}

}  // namespace

int rx_la_krylov_alloc(rx_ctx* ctx, int m) {
  const int64_t n = ctx->N * ctx->nVar;
  if (m < 1 || m > kMaxM) return RX_ERR_ARG;
  if (ctx->krylov_m < m) {
    rx_graph_reset(ctx);  // a captured solve reads kw / kz
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
int rx_la_fgmres_enqueue(rx_ctx* ctx, double tol, int m, bool x_zero) {
  return rx_la_fgmres_enqueue_part(ctx, tol, m, x_zero, 0, m, true);
}

// Iterations [i0, i1) of that FGMRES(m): i0 == 0 adds the reset and the start (r = b - A x, beta), finish the
// solution update. Enqueued in two parts with the host reading the state between them (implicit_solve), it is the
// same kernel sequence with the same arguments as the whole, so the same doubles.
int rx_la_fgmres_enqueue_part(rx_ctx* ctx, double tol, int m, bool x_zero, int i0, int i1, bool finish) {
  if (i0 < 0 || i1 > m || i0 > i1) return RX_ERR_ARG;
  int rc = rx_la_krylov_alloc(ctx, m);
  if (rc) return rc;
  const int64_t ld = ctx->N * ctx->nVar;  // vector length (owned + halo)
  const int64_t n = ctx->Nd * ctx->nVar;  // owned prefix
  const int nb = blocks(n);
  const bool dist = ctx->distributed();
  hipStream_t st = ctx->stream;
  KState* s = static_cast<KState*>(ctx->kstate);
  double* A = ctx->f[RX_F_JAC];
  double* b = ctx->f[RX_F_RHS];
  double* x = ctx->f[RX_F_SOL];
  double* part = ctx->red;  // [2][kRedBlocks]
  auto W = [&](int k) { return ctx->kw + (int64_t)k * ld; };
  auto Z = [&](int k) { return ctx->kz + (int64_t)k * ld; };
  auto reduce = [&]() { return dist ? rx_la_allreduce(ctx, s->loc, land_host(s), 4) : RX_OK; };
  if (i0 == 0) {
    k_fg_reset<<<1, 64, 0, st>>>(s, tol);
    if (x_zero) {
      k_fg_residual0<<<kRedBlocks, kBlock, 0, st>>>(n, b, W(0), part, s, dist);
    } else {
      RX_NV_SWITCH(ctx->nVar, (k_fg_residual<NV_><<<kRedBlocks, kBlock, 0, st>>>((int)ctx->Nd, ctx->rp, ctx->col, A,
                                                                                 x, b, W(0), part, s, dist)));
    }
    if ((rc = reduce())) return rc;
    k_fg_start_div<<<nb, kBlock, 0, st>>>(n, s, W(0));
  }
  // the product on a full grid (the 512-block reduction grid left 2 waves per SIMD, 91 % parked),
  // then the two inner products in the reduction's own order; RX_FG_FUSED_SPMV=1: one launch on the reduction grid
  static const bool fused_spmv = getenv("RX_FG_FUSED_SPMV") != nullptr;
  for (int i = i0; i < i1; ++i) {
    if (fused_spmv && !spmv_split(ctx)) {
      if ((rc = rx_la_prec_apply(ctx, W(i), Z(i), &s->done, &s->conv))) return rc;
      RX_NV_SWITCH(ctx->nVar, (k_fg_spmv<NV_><<<kRedBlocks, kBlock, 0, st>>>((int)ctx->Nd, ctx->rp, ctx->col, A, Z(i),
                                                                             W(0), W(i + 1), part, s, dist)));
    } else {
      if ((rc = prec_spmv(ctx, W(i), Z(i), W(i + 1), s))) return rc;
      k_fg_spmv_dots<<<kRedBlocks, kBlock, 0, st>>>(n, W(0), W(i + 1), part, s, dist);
    }
    if ((rc = reduce())) return rc;
    for (int k = 0; k <= i; ++k) {
      k_fg_proj<<<kRedBlocks, kBlock, 0, st>>>(n, ld, s, k, i, ctx->kw, part, dist);
      if ((rc = reduce())) return rc;
#ifndef RX_FG_NOREO_PROBE  // timing probe (build variant only): the second projection's launches left out
      k_fg_reo<<<kRedBlocks, kBlock, 0, st>>>(n, ld, s, k, i, ctx->kw, part, dist);
      if ((rc = reduce())) return rc;
#endif
    }
    k_fg_close_div<<<kRedBlocks, kBlock, 0, st>>>(n, s, i, W(i + 1));
  }
  if (finish) k_fg_finish<<<kRedBlocks, kBlock, 0, st>>>(n, ld, s, ctx->kz, x);
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// The state after a partial enqueue (synchronises the stream): 1 when the FGMRES has stopped (converged, broken
// down or diverged), so the iterations left would all return at their first instruction.
int rx_la_fgmres_stopped(rx_ctx* ctx, bool* stopped) {
  if (!ctx->kstate) return RX_ERR_STATE;
  KState* h = static_cast<KState*>(ctx->h_kstate);
  RX_HIP(hipMemcpyAsync(h, ctx->kstate, offsetof(KState, H), hipMemcpyDeviceToHost, ctx->stream));
  if (int rc = rx_la_host_wait(ctx)) return rc;
  *stopped = h->done || h->conv || h->diverged;
  return RX_OK;
}

// The host waits for the stream's work so far (polling an event instead measured the same: profiles/r06_ab_aj.txt)
int rx_la_host_wait(rx_ctx* ctx) {
  RX_HIP(hipStreamSynchronize(ctx->stream));
  return RX_OK;
}

// Read back the outcome of the last enqueued FGMRES (synchronises the stream).
int rx_la_fgmres_result(rx_ctx* ctx, int* iters, double* resid) {
  if (!ctx->kstate) return RX_ERR_STATE;
  KState* h = static_cast<KState*>(ctx->h_kstate);
  RX_HIP(hipMemcpyAsync(h, ctx->kstate, offsetof(KState, H), hipMemcpyDeviceToHost, ctx->stream));
  if (int rc = rx_la_host_wait(ctx)) return rc;
  if (iters) *iters = h->iters;
  if (resid) *resid = h->resid;
  return h->diverged ? RX_ERR_DIVERGED : RX_OK;
}

int rx_la_fgmres(rx_ctx* ctx, double tol, int m, int* iters, double* resid) {
  int rc = rx_la_fgmres_enqueue(ctx, tol, m, false);
  if (rc) return rc;
  return rx_la_fgmres_result(ctx, iters, resid);
}

namespace {
// r = b - A x (+ the BCGSTAB copies) and the start test; x's halo is the caller's (x_zero: not read)
int lin_start(rx_ctx* ctx, double tol, bool x_zero, double* r, double* r0, double* p, double* v) {
  KState* s = static_cast<KState*>(ctx->kstate);
  hipStream_t st = ctx->stream;
  const bool dist = ctx->distributed();
  const double* A = ctx->f[RX_F_JAC];
  k_fg_reset<<<1, 64, 0, st>>>(s, tol);
  if (x_zero) {
    RX_NV_SWITCH(ctx->nVar, (k_lin_resid<NV_, true><<<kRedBlocks, kBlock, 0, st>>>(
                                (int)ctx->Nd, ctx->rp, ctx->col, A, ctx->f[RX_F_SOL], ctx->f[RX_F_RHS], r, r0, p, v,
                                ctx->red, s, dist)));
  } else {
    RX_NV_SWITCH(ctx->nVar, (k_lin_resid<NV_, false><<<kRedBlocks, kBlock, 0, st>>>(
                                (int)ctx->Nd, ctx->rp, ctx->col, A, ctx->f[RX_F_SOL], ctx->f[RX_F_RHS], r, r0, p, v,
                                ctx->red, s, dist)));
  }
  int rc = dist ? rx_la_allreduce(ctx, s->loc, land_host(s), 4) : RX_OK;
  if (rc) return rc;
  k_lin_start<<<1, 1, 0, st>>>(s);
  return RX_OK;
}
}  // namespace

// BCGSTAB_LinSolver (linear_solvers_structure.cpp:465-599) on JAC * SOL = RHS with the configured preconditioner,
// m iterations at most, no host synchronisation. Vectors: r, r_0, v, t in kw[0..3], p, s, phat, shat in kz[0..3].
int rx_la_bcgstab_enqueue(rx_ctx* ctx, double tol, int m, bool x_zero) {
  if (m < 1) return RX_ERR_ARG;  // :475-484
  int rc = rx_la_krylov_alloc(ctx, std::max(3, std::min(ctx->krylov_m, kMaxM)));
  if (rc) return rc;
  const int64_t ld = ctx->N * ctx->nVar, n = ctx->Nd * ctx->nVar;
  const int nb = blocks(n);
  const bool dist = ctx->distributed();
  hipStream_t st = ctx->stream;
  KState* s = static_cast<KState*>(ctx->kstate);
  double* part = ctx->red;
  double *r = ctx->kw, *r0 = ctx->kw + ld, *v = ctx->kw + 2 * ld, *t = ctx->kw + 3 * ld;
  double *p = ctx->kz, *sv = ctx->kz + ld, *ph = ctx->kz + 2 * ld, *sh = ctx->kz + 3 * ld;
  double* x = ctx->f[RX_F_SOL];
  auto reduce = [&]() { return dist ? rx_la_allreduce(ctx, s->loc, land_host(s), 4) : RX_OK; };
  if ((rc = lin_start(ctx, tol, x_zero, r, r0, p, v))) return rc;
  for (int i = 0; i < m; ++i) {
    k_bc_rho<<<kRedBlocks, kBlock, 0, st>>>(n, r, r0, part, s, dist);
    if ((rc = reduce())) return rc;
    k_bc_p<<<nb, kBlock, 0, st>>>(n, s, i, r, v, p);
    if ((rc = prec_spmv(ctx, p, ph, v, s))) return rc;  // precond(p, phat); mat_vec(phat, v) (:547-548)
    k_fg_spmv_dots<<<kRedBlocks, kBlock, 0, st>>>(n, r0, v, part, s, dist);  // <r_0, v> -> dot
    if ((rc = reduce())) return rc;
    k_bc_s<<<nb, kBlock, 0, st>>>(n, s, i, r, v, sv);
    if ((rc = prec_spmv(ctx, sv, sh, t, s))) return rc;  // precond(s, shat); mat_vec(shat, t) (:561-562)
    k_fg_spmv_dots<<<kRedBlocks, kBlock, 0, st>>>(n, sv, t, part, s, dist);  // <t, t> -> dotn, <t, s> -> dot
    if ((rc = reduce())) return rc;
    k_bc_x<<<kRedBlocks, kBlock, 0, st>>>(n, s, x, ph, sh, sv, t, r, part, dist);
    if ((rc = reduce())) return rc;
    k_lin_check<<<1, 1, 0, st>>>(s, i, kDot2);
  }
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// The smoothers of Solve's non-Krylov branch (:683-701), m smoothing iterations at most: x += M^-1 r (LU_SGS /
// ILU0: the preconditioner sweeps of ComputeLU_SGSPreconditioner / ComputeILUPreconditioner, whose arithmetic the
// smoothers repeat; JACOBI: accumulated into x itself, k_jacobi_smooth), x's halo exchanged (:1809 / :1646 / :1341),
// r = b - A x, |r| against tol * |r_0|. r in kw[0], M^-1 r in kz[0].
int rx_la_smoother_enqueue(rx_ctx* ctx, double tol, int m, bool x_zero) {
  if (m < 1) return RX_ERR_ARG;  // :1279 / :1531 / :1723
  int rc = rx_la_krylov_alloc(ctx, std::max(1, std::min(ctx->krylov_m, kMaxM)));
  if (rc) return rc;
  const int64_t n = ctx->Nd * ctx->nVar;
  const int nb = blocks(n);
  const bool dist = ctx->distributed();
  hipStream_t st = ctx->stream;
  KState* s = static_cast<KState*>(ctx->kstate);
  double *r = ctx->kw, *z = ctx->kz;
  double* x = ctx->f[RX_F_SOL];
  const double* A = ctx->f[RX_F_JAC];
  const bool jacobi = rx_la_eff_prec(ctx) == RX_PREC_JACOBI;
  if ((rc = lin_start(ctx, tol, x_zero, r, nullptr, nullptr, nullptr))) return rc;
  for (int i = 0; i < m; ++i) {
    if (jacobi) {
      if ((rc = rx_la_jacobi_smooth(ctx, r, x, &s->done))) return rc;
    } else {
      ctx->defer_exchange = true;  // M^-1 r's halo is never read: x's is exchanged below
      rc = rx_la_prec_apply(ctx, r, z, &s->done, nullptr);
      ctx->defer_exchange = false;
      if (rc) return rc;
      k_sm_add<<<nb, kBlock, 0, st>>>(n, s, z, x);
    }
    if ((rc = rx_la_exchange(ctx, x, ctx->nVar))) return rc;
    RX_NV_SWITCH(ctx->nVar, (k_lin_resid<NV_, false><<<kRedBlocks, kBlock, 0, st>>>(
                                (int)ctx->Nd, ctx->rp, ctx->col, A, x, ctx->f[RX_F_RHS], r, nullptr, nullptr, nullptr,
                                ctx->red, s, dist)));
    if (dist && (rc = rx_la_allreduce(ctx, s->loc, land_host(s), 4))) return rc;
    k_lin_check<<<1, 1, 0, st>>>(s, i, kDot);
  }
  RX_HIP(hipGetLastError());
  return RX_OK;
}

// RESTARTED_FGMRES (Solve :662-671): FGMRES cycles of `iter` iterations (the remainder once fewer than `restart`
// are left) from the previous cycle's x, the tolerance scaled by 1 / |b| after each cycle, until `iter` iterations
// are spent or |b| < tol. Each cycle's iteration count decides the next, so the cycles synchronise with the host.
// A cycle that returns 0 iterations has met FGMRES's start test (|r| < eps or |r| < tol |b|, :367-370) and left x as
// it was, so every later cycle would see the same x: the reference's loop then either spins until the growing
// tolerance passes |b| (|b| < 1) or never ends (|b| >= 1). This one stops there with RX_OK: the same x and the same
// iteration count (it used to spin 4096 host-synchronous cycles and report RX_ERR_DIVERGED). kMaxCycles
// stays as a bound on cycles that keep iterating.
int rx_la_restarted_fgmres(rx_ctx* ctx, double tol, int iter, int restart, bool x_zero, int* iters, double* resid) {
  constexpr int kMaxCycles = 4096;
  if (iter < 1 || iter > kMaxM) return RX_ERR_ARG;
  int total = 0, max_iter = iter, rc;
  double stol = tol, res = 0.0;
  for (int cycle = 0; total < iter; ++cycle) {
    if (cycle == kMaxCycles) return RX_ERR_DIVERGED;
    if ((int64_t)total + restart > iter) max_iter = iter - total;
    if ((rc = rx_la_fgmres_enqueue(ctx, stol, max_iter, x_zero && cycle == 0))) return rc;
    int it = 0;
    if ((rc = rx_la_fgmres_result(ctx, &it, &res))) return rc;
    total += it;
    // FGMRES updates x over every element, its halo from the exchanged z (:455-457): the next cycle's A x reads it
    if (ctx->distributed() && (rc = rx_la_exchange(ctx, ctx->f[RX_F_SOL], ctx->nVar))) return rc;
    if (it == 0) break;  // the start test: x is final (above)
    const double bn = static_cast<KState*>(ctx->h_kstate)->bnorm;
    if (bn < stol) break;
    stol = stol * (1.0 / bn);
  }
  if (iters) *iters = total;
  if (resid) *resid = res;
  return RX_OK;
}

bool rx_la_solve_capturable(const rx_ctx* ctx) { return ctx->cfg.lin_solver != RX_LIN_RESTARTED_FGMRES; }

// CSysSolve::Solve's branch for cfg.lin_solver (the preconditioner is built before, rx_la_prec_build)
int rx_la_solve_enqueue(rx_ctx* ctx, bool x_zero) {
  const rx_cfg& c = ctx->cfg;
  ctx->solve_iters = -1;
  switch (c.lin_solver) {
    case RX_LIN_FGMRES:
      return rx_la_fgmres_enqueue(ctx, c.lin_tol, c.lin_iter, x_zero);
    case RX_LIN_BCGSTAB:
      return rx_la_bcgstab_enqueue(ctx, c.lin_tol, c.lin_iter, x_zero);
    case RX_LIN_RESTARTED_FGMRES: {
      int it = 0;
      double res = 0.0;
      const int rc = rx_la_restarted_fgmres(ctx, c.lin_tol, c.lin_iter, c.lin_restart, x_zero, &it, &res);
      ctx->solve_iters = it;
      return rc;
    }
    case RX_LIN_SMOOTHER_LUSGS:
    case RX_LIN_SMOOTHER_JACOBI:
    case RX_LIN_SMOOTHER_ILU:
      return rx_la_smoother_enqueue(ctx, c.lin_tol, c.lin_iter, x_zero);
    default:
      return RX_ERR_ARG;
  }
}

void rx_la_krylov_free(rx_ctx* ctx) {
  if (ctx->kstate) (void)hipFree(ctx->kstate);
  if (ctx->h_kstate) (void)hipHostFree(ctx->h_kstate);
  ctx->kstate = ctx->h_kstate = nullptr;
}
