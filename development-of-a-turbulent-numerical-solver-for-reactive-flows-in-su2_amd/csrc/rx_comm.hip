// rx_comm.hip — multi-GPU plumbing: halo exchange and all-reduce on the context stream, over RCCL
// (graph-capturable: the FGMRES graph contains them) or over a caller-provided host transport. The
// primitive-gradient exchange overlaps the interior gradients on a side stream (rx_grad_lsq).
//
// Halo exchange = the reference's SendReceive_Solution / Set_MPI_Solution / Set_MPI_Primitive_*
// (Common/src/matrix_structure.cpp:794-880; SU2_CFD/src/solver_direct_reactive.cpp:1530-1640,
// 1756-1990): owned values are packed per neighbour and received straight into the halo block
// (halo points are contiguous per owning rank). Inner products and the RMS: dotProd's
// MPI_Allreduce (Common/src/vector_structure.cpp:397-419), SetResidual_RMS (solver_structure.cpp:184-230).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "rx_ctx.h"

namespace {

constexpr int kGatherStride = 64;  // the widest all-reduce (the RMS columns): ctx->gather holds [nranks][<= 64]

__global__ void k_pack(int64_t n, int stride, const int32_t* __restrict__ idx, const double* __restrict__ f,
                       double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * stride) return;
  const int64_t k = t / stride;
  const int c = (int)(t - k * stride);
  out[t] = f[(int64_t)idx[k] * stride + c];
}

// out[c] = sum over ranks r = 0, 1, ... of g[r][c], added in rank order from rank 0's value: the all-reduce's
// result is then a fixed function of the rank sums (the oracle's rank-split inner products restate it,
// oracle/rx_oracle.cpp orc_dot), identical on every rank, independent of the collective's algorithm.
__global__ void k_sum_ranks(int nranks, int count, const double* __restrict__ g, double* __restrict__ out) {
  const int c = threadIdx.x;
  if (c >= count) return;
  double s = g[c];
  for (int r = 1; r < nranks; ++r) s += g[(size_t)r * count + c];  // ncclAllGather: rank r's block at r * count
  out[c] = s;
}

int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? RX_OK : RX_ERR_COMM; }

int gather_alloc(rx_ctx* ctx) {
  if (ctx->gather) return RX_OK;
  RX_HIP(hipMalloc(&ctx->gather, sizeof(double) * (size_t)ctx->nranks * kGatherStride));
  return RX_OK;
}

int stage_alloc(rx_ctx* ctx) {
  if (ctx->h_stage) return RX_OK;
  const size_t n = (size_t)(ctx->n_send + (ctx->N - ctx->Nd)) * ctx->halo_stride + 64;
  RX_HIP(hipHostMalloc(&ctx->h_stage, n * sizeof(double)));
  return RX_OK;
}

}  // namespace

int rx_la_exchange(rx_ctx* ctx, double* f, int stride) { return rx_la_exchange_on(ctx, f, stride, ctx->stream); }

// The flow's post-update Set_MPI_Solution (solver_direct_reactive.cpp:2403) with RCCL: k_update's owned rows are
// final when the solve graph ends, and SetPrimitive_Variables' owned points do not read the halo, so the exchange
// runs on comm_stream while they are computed (rx_set_primitive), and the halo points wait for it.
bool rx_u_exchange_deferred(const rx_ctx* ctx) {
  return ctx->kind == RX_KIND_FLOW && ctx->comm_stream && ctx->u_join && !ctx->has_hcomm && ctx->n_neigh > 0 &&
         getenv("RX_NO_U_OVERLAP") == nullptr;
}

int rx_la_u_exchange_begin(rx_ctx* ctx) {
  RX_HIP(hipEventRecord(ctx->comm_fork, ctx->stream));
  RX_HIP(hipStreamWaitEvent(ctx->comm_stream, ctx->comm_fork, 0));
  const int rc = rx_la_exchange_on(ctx, ctx->f[RX_F_U], ctx->nVar, ctx->comm_stream);
  if (rc) return rc;
  RX_HIP(hipEventRecord(ctx->u_join, ctx->comm_stream));
  ctx->u_pending = true;
  return RX_OK;
}

int rx_settle_u(rx_ctx* ctx) {
  rx_ctx* f = ctx->kind == RX_KIND_SST && ctx->flow ? ctx->flow : ctx;
  if (!f->u_pending) return RX_OK;
  RX_HIP(hipStreamWaitEvent(ctx->stream, f->u_join, 0));  // an SST context shares its flow's stream
  f->u_pending = false;
  return RX_OK;
}

// The exchange on stream st (the context stream, or comm_stream for the overlapped gradient exchange; the host
// transport always runs on the context stream).
int rx_la_exchange_on(rx_ctx* ctx, double* f, int stride, hipStream_t st) {
  if (!ctx->distributed() || ctx->n_neigh == 0) return RX_OK;
  if (stride > ctx->halo_stride) return RX_ERR_ARG;
  if (ctx->has_hcomm) st = ctx->stream;
  if (st == ctx->stream) {  // the send buffer and the communicator are free once a pending U exchange is waited for
    const int rc0 = rx_settle_u(ctx);
    if (rc0) return rc0;
  }
  if (ctx->n_send > 0) {
    const int64_t n = ctx->n_send * stride;
    k_pack<<<(int)((n + 255) / 256), 256, 0, st>>>(ctx->n_send, stride, ctx->send_idx, f, ctx->sendbuf);
    RX_HIP(hipGetLastError());
  }
  double* halo = f + ctx->Nd * stride;
  const int64_t n_recv = ctx->N - ctx->Nd;
  if (ctx->has_hcomm) {
    double* hs = ctx->h_stage;
    double* hr = ctx->h_stage + ctx->n_send * stride;
    RX_HIP(hipMemcpyAsync(hs, ctx->sendbuf, sizeof(double) * ctx->n_send * stride, hipMemcpyDeviceToHost,
                          ctx->stream));
    RX_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->hcomm.sendrecv(ctx->hcomm.user, ctx->n_neigh, ctx->h_neigh.data(), ctx->h_send_ptr.data(), hs,
                            ctx->h_recv_ptr.data(), hr, stride) != 0)
      return RX_ERR_COMM;
    RX_HIP(hipMemcpyAsync(halo, hr, sizeof(double) * n_recv * stride, hipMemcpyHostToDevice, ctx->stream));
    return RX_OK;
  }
  ncclComm_t comm = static_cast<ncclComm_t>(ctx->comm);
  int rc = nccl_rc(ncclGroupStart());
  for (int k = 0; k < ctx->n_neigh && !rc; ++k) {
    const int64_t s0 = ctx->h_send_ptr[k], s1 = ctx->h_send_ptr[k + 1];
    const int64_t r0 = ctx->h_recv_ptr[k], r1 = ctx->h_recv_ptr[k + 1];
    if (s1 > s0)
      rc = nccl_rc(ncclSend(ctx->sendbuf + s0 * stride, (size_t)((s1 - s0) * stride), ncclDouble, ctx->h_neigh[k],
                            comm, st));
    if (!rc && r1 > r0)
      rc = nccl_rc(ncclRecv(halo + r0 * stride, (size_t)((r1 - r0) * stride), ncclDouble, ctx->h_neigh[k], comm, st));
  }
  const int rc2 = nccl_rc(ncclGroupEnd());
  return rc ? rc : rc2;
}

// dotProd's / SetResidual_RMS's MPI_Allreduce (vector_structure.cpp:397-419), as a rank-ordered sum: RCCL all-gather
// of every rank's `count` sums, then k_sum_ranks; the host transport's allreduce callback has the same contract
// (rx_host_comm, include/rx.h).
int rx_la_allreduce(rx_ctx* ctx, const double* in, double* out, int count) {
  if (!ctx->distributed()) return RX_OK;
  if (count > kGatherStride) return RX_ERR_ARG;
  if (int rc0 = rx_settle_u(ctx)) return rc0;  // one RCCL operation of the communicator at a time
  if (ctx->has_hcomm) {
    double* h = ctx->h_stage + (ctx->n_send + (ctx->N - ctx->Nd)) * ctx->halo_stride;
    RX_HIP(hipMemcpyAsync(h, in, sizeof(double) * count, hipMemcpyDeviceToHost, ctx->stream));
    RX_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->hcomm.allreduce(ctx->hcomm.user, h, h, count) != 0) return RX_ERR_COMM;
    RX_HIP(hipMemcpyAsync(out, h, sizeof(double) * count, hipMemcpyHostToDevice, ctx->stream));
    return RX_OK;
  }
  int rc = gather_alloc(ctx);
  if (rc) return rc;
  rc = nccl_rc(ncclAllGather(in, ctx->gather, (size_t)count, ncclDouble, static_cast<ncclComm_t>(ctx->comm),
                             ctx->stream));
  if (rc) return rc;
  k_sum_ranks<<<1, 64, 0, ctx->stream>>>(ctx->nranks, count, ctx->gather, out);
  RX_HIP(hipGetLastError());
  return RX_OK;
}

namespace {

// global owned-point count (RMS normalisation) and a fresh solve graph once a transport is attached
int comm_attached(rx_ctx* ctx) {
  double* d = nullptr;
  RX_HIP(hipMalloc(&d, sizeof(double)));
  double h = (double)ctx->Nd;
  int rc = RX_OK;
  if (hipMemcpyAsync(d, &h, sizeof(double), hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    rc = RX_ERR_HIP;
  if (!rc) rc = rx_la_allreduce(ctx, d, d, 1);
  if (!rc && (hipMemcpyAsync(&h, d, sizeof(double), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
              hipStreamSynchronize(ctx->stream) != hipSuccess))
    rc = RX_ERR_HIP;
  if (!rc) ctx->n_global = (int64_t)h;
  (void)hipFree(d);
  rx_graph_reset(ctx);
  return rc;
}

}  // namespace

extern "C" {

int rx_comm_unique_id(void* id128) {
  if (!id128) return RX_ERR_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return RX_ERR_COMM;
  std::memcpy(id128, &id, sizeof(id));
  return RX_OK;
}

int rx_comm_init(rx_ctx* ctx, int nranks, int rank, const void* id128) {
  if (!ctx || !id128 || nranks < 1 || rank < 0 || rank >= nranks || ctx->distributed()) return RX_ERR_ARG;
  RX_HIP(hipSetDevice(ctx->device));
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  ncclComm_t comm = nullptr;
  if (ncclCommInitRank(&comm, nranks, id, rank) != ncclSuccess) return RX_ERR_COMM;
  ctx->comm = comm;
  ctx->nranks = nranks;
  ctx->rank = rank;
  if (int rc = gather_alloc(ctx)) return rc;  // before any graph capture
  // side stream of the overlapped gradient exchange (rx_grad_lsq)
  RX_HIP(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
  RX_HIP(hipEventCreateWithFlags(&ctx->comm_fork, hipEventDisableTiming));
  RX_HIP(hipEventCreateWithFlags(&ctx->comm_join, hipEventDisableTiming));
  RX_HIP(hipEventCreateWithFlags(&ctx->u_join, hipEventDisableTiming));
  return comm_attached(ctx);
}

int rx_comm_init_host(rx_ctx* ctx, int nranks, int rank, const rx_host_comm* ops) {
  if (!ctx || !ops || !ops->sendrecv || !ops->allreduce || nranks < 1 || rank < 0 || rank >= nranks ||
      ctx->distributed())
    return RX_ERR_ARG;
  int rc = stage_alloc(ctx);
  if (rc) return rc;
  ctx->hcomm = *ops;
  ctx->has_hcomm = true;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return comm_attached(ctx);
}

int rx_halo_exchange(rx_ctx* ctx, rx_field f) {
  if (!ctx || f < 0 || f >= RX_F_COUNT || ctx->fcount[f] % ctx->N != 0) return RX_ERR_ARG;
  if (f == RX_F_JAC || f == RX_F_ILU) return RX_ERR_ARG;
  int rc = rx_settle_u(ctx);
  if (!rc) rc = rx_la_exchange(ctx, ctx->f[f], (int)(ctx->fcount[f] / ctx->N));
  if (rc) return rc;
  RX_HIP(hipStreamSynchronize(ctx->stream));
  return RX_OK;
}

}  // extern "C"

// An SST context shares its flow context's transport (same ranks, same halo plan).
int rx_comm_borrow(rx_ctx* ctx, const rx_ctx* from) {
  ctx->comm = from->comm;
  ctx->comm_owned = false;
  ctx->nranks = from->nranks;
  ctx->rank = from->rank;
  if (from->has_hcomm) {
    const int rc = stage_alloc(ctx);
    if (rc) return rc;
    ctx->hcomm = from->hcomm;
    ctx->has_hcomm = true;
  }
  ctx->n_global = from->n_global;
  if (!ctx->has_hcomm && ctx->comm) return gather_alloc(ctx);  // the SST solve graph all-reduces through it
  return RX_OK;
}

void rx_comm_free(rx_ctx* ctx) {
  if (ctx->comm_stream) {
    (void)hipStreamSynchronize(ctx->comm_stream);
    (void)hipStreamDestroy(ctx->comm_stream);
    (void)hipEventDestroy(ctx->comm_fork);
    (void)hipEventDestroy(ctx->comm_join);
    if (ctx->u_join) (void)hipEventDestroy(ctx->u_join);
    ctx->u_join = nullptr;
    ctx->u_pending = false;
    ctx->comm_stream = nullptr;
  }
  if (ctx->gather) (void)hipFree(ctx->gather);
  ctx->gather = nullptr;
  if (ctx->comm && ctx->comm_owned) (void)ncclCommDestroy(static_cast<ncclComm_t>(ctx->comm));
  ctx->comm = nullptr;
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  ctx->h_stage = nullptr;
  ctx->has_hcomm = false;
}
