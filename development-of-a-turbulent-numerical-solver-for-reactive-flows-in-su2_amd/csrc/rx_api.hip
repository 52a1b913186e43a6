// rx_api.hip — C ABI (include/rx.h): context setup (dual-grid adjacency, BSR pattern, level
// schedule, mechanism upload) and the phase entry points in the reference's call order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "rx_ctx.h"
#include "rx_species.h"

namespace {

// y[i] = rx_recip(x[i]).y: divisors' reciprocals made by the device's own instructions (rx_fdiv.h)
__global__ void k_recip_table(const double* __restrict__ x, double* __restrict__ y, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) y[i] = rx::rx_recip(x[i]).y;
}

template <typename T>
int dalloc(rx_ctx* ctx, T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  RX_HIP(hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)));
  RX_HIP(hipMemsetAsync(*p, 0, n * sizeof(T), ctx->stream));
  return RX_OK;
}

// Allocate + copy on the context stream (ordered after dalloc's memset on the same stream; the
// context stream does not synchronise with the null stream) and wait, so the host buffer may go.
template <typename T>
int dupload(rx_ctx* ctx, T** p, const T* h, size_t n) {
  int rc = dalloc(ctx, p, n);
  if (rc) return rc;
  if (n) {
    RX_HIP(hipMemcpyAsync(*p, h, n * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
    RX_HIP(hipStreamSynchronize(ctx->stream));
  }
  return RX_OK;
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

__global__ void k_fold_mark(int n, const int32_t* __restrict__ rows, int32_t* __restrict__ skip) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) skip[rows[t]] = 1;
}

// fold_skip for the current boundary markers: the owned boundary points k_bc_apply updates after the assembly
int fold_prepare(rx_ctx* ctx) {
  if (ctx->fold_skip && ctx->fold_epoch == ctx->bc_epoch) return RX_OK;
  if (!ctx->fold_skip) RX_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->fold_skip), sizeof(int32_t) * (ctx->N + 1)));
  RX_HIP(hipMemsetAsync(ctx->fold_skip, 0, sizeof(int32_t) * (ctx->N + 1), ctx->stream));
  if (ctx->bc_on && ctx->bc_nbn > 0)
    k_fold_mark<<<(int)((ctx->bc_nbn + 255) / 256), 256, 0, ctx->stream>>>((int)ctx->bc_nbn, ctx->bc_bn,
                                                                          ctx->fold_skip);
  RX_HIP(hipGetLastError());
  ctx->fold_epoch = ctx->bc_epoch;
  return RX_OK;
}

int ensure_assembled(rx_ctx* ctx) {
  if (!ctx->cfg.implicit || ctx->assembled) return RX_OK;
  if (!ctx->phase_conv) return RX_ERR_STATE;
  if (ctx->fold_req && ctx->kind == RX_KIND_FLOW)
    if (int rc0 = fold_prepare(ctx)) return rc0;
  RxPhase ph(ctx, RX_K_ASSEMBLE);
  int rc = rx_launch_assemble(ctx, ctx->phase_visc, ctx->phase_src);
  if (rc) return rc;
  ctx->assembled = 1;
  return RX_OK;
}

}  // namespace

int rx_ensure_assembled(rx_ctx* ctx) { return ensure_assembled(ctx); }

extern "C" {

const char* rx_status_string(int s) {
  switch (s) {
    case RX_OK: return "ok";
    case RX_ERR_ARG: return "invalid argument";
    case RX_ERR_HIP: return "HIP runtime error";
    case RX_ERR_NAN: return "NaN found in the residual";
    case RX_ERR_RANGE: return "temperature out of the property-table range";
    case RX_ERR_NONPHYS: return "non-physical state";
    case RX_ERR_DIVERGED: return "linear solver diverged";
    case RX_ERR_STATE: return "call sequence error";
    case RX_ERR_COMM: return "RCCL communication error";
    case RX_ERR_UNSUPPORTED: return "input not supported on this path";
    default: return "unknown";
  }
}

}  // extern "C"

namespace {

// Context construction shared by the flow context (mech != null) and the SST context (flow != null,
// nVar = 2, borrows the flow context's stream and communicator).
int create_impl(const rx_mesh_desc* mesh, const rx_mech_desc* mech, const rx_cfg* cfg, int device, rx_ctx* flow,
                rx_ctx** out) {
  if (!mesh || !cfg || !out || (!mech && !flow)) return RX_ERR_ARG;
  if (cfg->spatial_order < 0 || cfg->spatial_order > 2) return RX_ERR_ARG;
  if (cfg->implicit && (cfg->lin_solver < RX_LIN_FGMRES || cfg->lin_solver > RX_LIN_SMOOTHER_ILU ||
                        cfg->lin_prec < RX_PREC_LU_SGS || cfg->lin_prec > RX_PREC_JACOBI || cfg->lin_restart < 0 ||
                        cfg->lin_iter < 1))
    return RX_ERR_ARG;
  *out = nullptr;
  if (mesh->n_dim != 2 && mesh->n_dim != 3) return RX_ERR_ARG;
  const bool sst = flow != nullptr;
  const int ns = sst ? 0 : mech->n_species;
  if (!sst && (ns < kMinSpecies || ns > kMaxSpecies)) return RX_ERR_ARG;  // the instantiated counts (rx_species.h)
  if (!sst && mech->n_reactions > rx::kMaxNR) return RX_ERR_ARG;
  if (mesh->n_point >= (1LL << 31) || 2 * mesh->n_edge >= (1LL << 31)) return RX_ERR_ARG;
  if (sst && (mesh->n_point != flow->N || mesh->n_edge != flow->E)) return RX_ERR_ARG;
  rx_ctx* ctx = new rx_ctx();
  ctx->device = sst ? flow->device : device;
  if (hipSetDevice(ctx->device) != hipSuccess) {
    delete ctx;
    return RX_ERR_HIP;
  }
  if (sst) {
    ctx->kind = RX_KIND_SST;
    ctx->flow = flow;
    ++flow->n_children;
    ctx->stream = flow->stream;
    ctx->own_stream = false;
  } else if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return RX_ERR_HIP;
  }
  ctx->cfg = *cfg;
  ctx->nDim = mesh->n_dim;
  ctx->ns = ns;
  if (sst) {  // (k, omega); the gradient has the same two rows
    ctx->cfg.rans = 1;
    ctx->nr = 0;
    ctx->nVar = 2;
    ctx->nPV = 0;
    ctx->nG = 2;
    ctx->nL = 0;
  } else {
    ctx->nr = mech->n_reactions;
    ctx->nVar = ns + ctx->nDim + 2;
    ctx->nPV = ns + ctx->nDim + 5;
    ctx->nG = ns + ctx->nDim + 2;
    ctx->nL = ctx->nDim + 2;
  }
  const int64_t N = mesh->n_point, E = mesh->n_edge, NB = mesh->n_bvert;
  ctx->N = N;
  ctx->E = E;
  ctx->NB = NB;
  ctx->Nd = (mesh->n_domain > 0) ? mesh->n_domain : N;
  if (ctx->Nd > N) {
    rx_ctx_destroy(ctx);
    return RX_ERR_ARG;
  }
  ctx->n_global = ctx->Nd;
  const int nd = ctx->nDim, nv = ctx->nVar;
  int rc = RX_OK;
#define CK(x)        \
  do {               \
    rc = (x);        \
    if (rc) {        \
      rx_ctx_destroy(ctx); \
      return rc;     \
    }                \
  } while (0)

  // ---- edges, incident-edge adjacency (sorted by edge id), BSR pattern
  std::vector<int32_t> e32(2 * E);
  for (int64_t q = 0; q < 2 * E; ++q) {
    if (mesh->edges[q] < 0 || mesh->edges[q] >= N) {
      rx_ctx_destroy(ctx);
      return RX_ERR_ARG;
    }
    e32[q] = (int32_t)mesh->edges[q];
  }
  std::vector<int32_t> adj_ptr(N + 1, 0), adj(2 * E);
  for (int64_t e = 0; e < E; ++e) {
    adj_ptr[e32[2 * e] + 1]++;
    adj_ptr[e32[2 * e + 1] + 1]++;
  }
  for (int64_t i = 0; i < N; ++i) adj_ptr[i + 1] += adj_ptr[i];
  {
    std::vector<int32_t> fill(adj_ptr.begin(), adj_ptr.end() - 1);
    for (int64_t e = 0; e < E; ++e) {  // increasing e => sorted
      adj[fill[e32[2 * e]]++] = (int32_t)(e << 1);
      adj[fill[e32[2 * e + 1]]++] = (int32_t)((e << 1) | 1);
    }
  }
  // BSR: neighbours + diagonal, sorted (matrix_structure.cpp:113-201) by local number, or by global number when the
  // mesh carries it (a shard of a distributed mesh: the rows then sum in the undivided mesh's order). Either way a
  // partition's columns form one run, in increasing local number (owned points keep the global order).
  ctx->h_rp.assign(N + 1, 0);
  std::vector<std::vector<int32_t>> rows(N);
  const int64_t* gid = mesh->global_id;
  auto key = [&](int32_t c) { return gid ? gid[c] : (int64_t)c; };
  for (int64_t i = 0; i < N; ++i) {
    rows[i].push_back((int32_t)i);
    for (int32_t k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
      const int e = adj[k] >> 1, side = adj[k] & 1;
      rows[i].push_back(e32[2 * e + (side ^ 1)]);
    }
    std::sort(rows[i].begin(), rows[i].end(), [&](int32_t a, int32_t b) { return key(a) < key(b); });
    rows[i].erase(std::unique(rows[i].begin(), rows[i].end()), rows[i].end());
    ctx->h_rp[i + 1] = ctx->h_rp[i] + (int64_t)rows[i].size();
  }
  if (gid) {  // owned points must be in increasing global order (partition runs stay contiguous and ascending)
    for (int64_t i = 1; i < ctx->Nd; ++i)
      if (gid[i] <= gid[i - 1]) CK(RX_ERR_ARG);
  }
  auto pos_in = [](const std::vector<int32_t>& r, int32_t c) -> int64_t {
    for (size_t q = 0; q < r.size(); ++q)
      if (r[q] == c) return (int64_t)q;
    return -1;
  };
  ctx->nnzb = ctx->h_rp[N];
  ctx->h_col.resize(ctx->nnzb);
  std::vector<int32_t> rp32(N + 1), col32(ctx->nnzb);
  std::vector<int64_t> diag(N), adj_blk(2 * E), edge_blk(2 * E);
  for (int64_t i = 0; i < N; ++i) {
    rp32[i] = (int32_t)ctx->h_rp[i];
    for (size_t q = 0; q < rows[i].size(); ++q) {
      ctx->h_col[ctx->h_rp[i] + q] = rows[i][q];
      col32[ctx->h_rp[i] + q] = rows[i][q];
      if (rows[i][q] == i) diag[i] = ctx->h_rp[i] + (int64_t)q;
    }
    for (int32_t k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) {
      const int e = adj[k] >> 1, side = adj[k] & 1;
      const int32_t o = e32[2 * e + (side ^ 1)];
      adj_blk[k] = ctx->h_rp[i] + pos_in(rows[i], o);
      edge_blk[2 * e + side] = adj_blk[k];
    }
  }
  rp32[N] = (int32_t)ctx->nnzb;
  // partitions (ranks), per-row intra-partition column ranges and per-partition level schedules
  {
    const int64_t np = (mesh->part_ptr && mesh->n_part > 0) ? mesh->n_part : 1;
    ctx->h_part_ptr.assign(np + 1, 0);
    if (mesh->part_ptr && mesh->n_part > 0) {
      for (int64_t p = 0; p <= np; ++p) ctx->h_part_ptr[p] = mesh->part_ptr[p];
      bool ok = ctx->h_part_ptr[0] == 0 && ctx->h_part_ptr[np] == ctx->Nd;
      for (int64_t p = 0; p < np && ok; ++p) ok = ctx->h_part_ptr[p + 1] > ctx->h_part_ptr[p];
      if (!ok) CK(RX_ERR_ARG);
    } else {
      ctx->h_part_ptr[1] = ctx->Nd;
    }
    ctx->npart = (int)np;
    std::vector<int32_t> klo(N), khi(N);
    for (int64_t i = ctx->Nd; i < N; ++i) klo[i] = khi[i] = (int32_t)diag[i];  // halo rows: no solve
    int rowmax = 1;
    for (int64_t p = 0; p < np; ++p) {
      const int64_t lo = ctx->h_part_ptr[p], hi = ctx->h_part_ptr[p + 1];
      for (int64_t i = lo; i < hi; ++i) {
        // the row's columns inside the partition: one run (see the BSR ordering above)
        const auto& r = rows[i];
        size_t a = 0, b = r.size();
        while (a < r.size() && !(r[a] >= lo && r[a] < hi)) ++a;
        while (b > a && !(r[b - 1] >= lo && r[b - 1] < hi)) --b;
        klo[i] = (int32_t)(ctx->h_rp[i] + (int64_t)a);
        khi[i] = (int32_t)(ctx->h_rp[i] + (int64_t)b);
        rowmax = std::max(rowmax, khi[i] - klo[i]);
      }
    }
    ctx->rowmax = rowmax;
    std::vector<int32_t> ring_xoff(ctx->nnzb, 0);
    auto schedule = [&](bool fwd, rx_ctx::Sched& S) -> int {
      std::vector<int32_t> lv(N, 0), pos(N, 0), part_lvl(np + 1, 0), lvl_ptr(1, 0), order;
      order.reserve(N);
      for (int64_t p = 0; p < np; ++p) {
        const int64_t lo = ctx->h_part_ptr[p], hi = ctx->h_part_ptr[p + 1];
        int32_t maxl = 0;
        if (fwd) {
          for (int64_t i = lo; i < hi; ++i) {
            int32_t l = 0;
            for (int32_t k = klo[i]; k < (int32_t)diag[i]; ++k) l = std::max(l, lv[col32[k]] + 1);
            lv[i] = l;
            maxl = std::max(maxl, l);
          }
        } else {
          for (int64_t i = hi - 1; i >= lo; --i) {
            int32_t l = 0;
            for (int32_t k = (int32_t)diag[i] + 1; k < khi[i]; ++k) l = std::max(l, lv[col32[k]] + 1);
            lv[i] = l;
            maxl = std::max(maxl, l);
          }
        }
        std::vector<int32_t> cnt(maxl + 2, 0);
        for (int64_t i = lo; i < hi; ++i) cnt[lv[i] + 1]++;
        for (int32_t l = 0; l <= maxl; ++l) cnt[l + 1] += cnt[l];
        std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1), loc(hi - lo);
        for (int64_t i = lo; i < hi; ++i) {
          pos[i] = fill[lv[i]] - cnt[lv[i]];  // position within its level
          loc[fill[lv[i]]++] = (int32_t)i;
        }
        const int32_t base = (int32_t)order.size();
        for (int32_t l = 0; l <= maxl; ++l) {
          lvl_ptr.push_back(base + cnt[l + 1]);
          S.maxwidth = std::max(S.maxwidth, cnt[l + 1] - cnt[l]);
        }
        order.insert(order.end(), loc.begin(), loc.end());
        part_lvl[p + 1] = part_lvl[p] + maxl + 1;
        S.maxlev = std::max(S.maxlev, maxl + 1);
      }
      S.nlevels = part_lvl[np];
      std::vector<int32_t> slot(4 * order.size());
      for (size_t r = 0; r < order.size(); ++r) {
        const int32_t i = order[r];
        slot[4 * r] = i;
        slot[4 * r + 1] = klo[i];
        slot[4 * r + 2] = (int32_t)diag[i];
        slot[4 * r + 3] = khi[i];
      }
      // passes of <= 64 rows within one level (the one-wavefront 2x2 kernels, rx_sweeps.hip)
      std::vector<int32_t> pass_lo, part_pass(np + 1, 0);
      for (int64_t p = 0; p < np; ++p) {
        for (int32_t l = part_lvl[p]; l < part_lvl[p + 1]; ++l)
          for (int32_t b = lvl_ptr[l]; b < lvl_ptr[l + 1]; b += 64) pass_lo.push_back(b);
        part_pass[p + 1] = (int32_t)pass_lo.size();
      }
      pass_lo.push_back((int32_t)order.size());
      // k_ilu_apply_ring's plan. Its wavefronts take turns by level in G groups (rx_ilu_ring_groups), so a level has
      // at most cap = rows per pass / G rows: a wider level is split into ceil(width / cap) consecutive sub-levels of
      // nearly equal width (the rows of a level are independent, so any split keeps every row's arithmetic; the rows
      // keep their schedule order). Row j's result goes to ring row (sub-level(j) mod R) W + position(j) (W = the
      // widest sub-level); a block (i, j) of a dependency less than R sub-levels back reads it there, a farther one
      // from j's far row R W + (its index among the partition's far sources), written by j as well
      {
        const int cap = std::max(1, rx_ilu_ring_rpb(ctx->nVar, rx_ilu_ring_tb(ctx)) / rx_ilu_ring_groups());
        std::vector<int32_t> slv(N, 0), spos(N, 0), rpart_lvl(np + 1, 0), rlvl_ptr(1, 0);
        int W = 1;
        S.rmaxlev = 0;
        for (int64_t p = 0; p < np; ++p) {
          int32_t nsub_p = 0;
          for (int32_t l = part_lvl[p]; l < part_lvl[p + 1]; ++l) {
            const int32_t c = lvl_ptr[l + 1] - lvl_ptr[l];
            const int32_t nsub = (c + cap - 1) / cap, chunk = (c + nsub - 1) / nsub;
            for (int32_t q = 0; q < c; ++q) {
              const int32_t i = order[lvl_ptr[l] + q];
              slv[i] = nsub_p + q / chunk;
              spos[i] = q % chunk;
            }
            for (int32_t s = 0; s < nsub; ++s) {
              const int32_t e = std::min(c, (s + 1) * chunk);
              rlvl_ptr.push_back(lvl_ptr[l] + e);
              W = std::max(W, e - s * chunk);
            }
            nsub_p += nsub;
          }
          rpart_lvl[p + 1] = rpart_lvl[p] + nsub_p;
          S.rmaxlev = std::max(S.rmaxlev, nsub_p);
        }
        S.rmaxwidth = W;
        const int R = kIluRing;
        std::vector<int32_t> farid(N, -1);
        int32_t nfar_max = 0;
        for (int64_t p = 0; p < np; ++p) {
          int32_t nfar = 0;
          for (int64_t i = ctx->h_part_ptr[p]; i < ctx->h_part_ptr[p + 1]; ++i) {
            const int32_t k0 = fwd ? klo[i] : (int32_t)diag[i] + 1, k1 = fwd ? (int32_t)diag[i] : khi[i];
            for (int32_t k = k0; k < k1; ++k) {
              const int32_t j = col32[k];
              if (slv[i] - slv[j] < R) {
                ring_xoff[k] = (slv[j] % R) * W + spos[j];
              } else {
                if (farid[j] < 0) farid[j] = nfar++;
                ring_xoff[k] = R * W + farid[j];
              }
            }
          }
          nfar_max = std::max(nfar_max, nfar);
        }
        std::vector<int32_t> ring(2 * order.size());
        for (size_t r = 0; r < order.size(); ++r) {
          const int32_t i = order[r];
          ring[2 * r] = (slv[i] % R) * W + spos[i];
          ring[2 * r + 1] = farid[i] >= 0 ? R * W + farid[i] : -1;
        }
        S.ring_rows = R * W + nfar_max;
        int rc3 = dupload(ctx, &S.ring, ring.data(), ring.size());
        if (!rc3) rc3 = dupload(ctx, &S.rpart_lvl, rpart_lvl.data(), rpart_lvl.size());
        if (!rc3) rc3 = dupload(ctx, &S.rlvl_ptr, rlvl_ptr.data(), rlvl_ptr.size());
        if (rc3) return rc3;
      }
      int rc2 = dupload(ctx, &S.pass_lo, pass_lo.data(), pass_lo.size());
      if (!rc2) rc2 = dupload(ctx, &S.part_pass, part_pass.data(), part_pass.size());
      if (!rc2) rc2 = dupload(ctx, &S.part_lvl, part_lvl.data(), part_lvl.size());
      if (!rc2) rc2 = dupload(ctx, &S.lvl_ptr, lvl_ptr.data(), lvl_ptr.size());
      if (!rc2) rc2 = dupload(ctx, &S.rows, order.data(), order.size());
      if (!rc2) rc2 = dupload(ctx, &S.slot, slot.data(), slot.size());
      return rc2;
    };
    {
      std::vector<int32_t> pp32(np + 1);
      int maxpart = 1;
      for (int64_t p = 0; p <= np; ++p) pp32[p] = (int32_t)ctx->h_part_ptr[p];
      int maxnz = 1;
      for (int64_t p = 0; p < np; ++p) {
        maxpart = std::max(maxpart, pp32[p + 1] - pp32[p]);
        maxnz = std::max(maxnz, (int)(ctx->h_rp[pp32[p + 1]] - ctx->h_rp[pp32[p]]));
      }
      ctx->maxpart = maxpart;
      ctx->maxpart_nnzb = maxnz;
      CK(dupload(ctx, &ctx->part_ptr, pp32.data(), pp32.size()));
      int v = 0;
      if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && v > 0)
        ctx->lds_max = v;
      CK(rx_la_prepare(ctx));
    }
    CK(schedule(true, ctx->fs));
    CK(schedule(false, ctx->bs));
    CK(dupload(ctx, &ctx->ring_xoff, ring_xoff.data(), ring_xoff.size()));
    CK(dupload(ctx, &ctx->klo, klo.data(), N));
    CK(dupload(ctx, &ctx->khi, khi.data(), N));
    // ILU(0) update plan: for each intra lower block k = (i, j): upper blocks kk = (j, kp), kp > j
    // inside row i's partition and present in row i, with their BSR index pos in row i
    {
      std::vector<int32_t> uptr(ctx->nnzb + 1, 0), upd;
      for (int64_t i = 0; i < N; ++i) {
        for (int32_t k = (int32_t)ctx->h_rp[i]; k < (int32_t)ctx->h_rp[i + 1]; ++k) {
          if (k >= klo[i] && k < (int32_t)diag[i]) {
            const int32_t j = col32[k];
            for (int32_t kk = (int32_t)diag[j] + 1; kk < khi[j]; ++kk) {
              const int32_t kp = col32[kk];
              const int64_t q = pos_in(rows[i], kp);
              if (q >= 0) {
                const int32_t pos = (int32_t)(ctx->h_rp[i] + q);
                if (pos >= klo[i] && pos < khi[i]) {
                  upd.push_back(kk);
                  upd.push_back(pos);
                }
              }
            }
          }
          uptr[k + 1] = (int32_t)(upd.size() / 2);
        }
      }
      CK(dupload(ctx, &ctx->upd_ptr, uptr.data(), uptr.size()));
      CK(dupload(ctx, &ctx->upd, upd.data(), upd.size()));
      // compact row plans in forward-schedule order (layout: rx_sweeps.hip, k_ilu_build_part); the
      // order is recomputed exactly as schedule() builds it
      const int64_t Nd = ctx->Nd;
      std::vector<int32_t> fo(Nd);
      // a row's dependency level in its partition, its place in the level, and the partition's first (global) level
      std::vector<int32_t> lv(N, 0), lpos(N, 0), lbase(np + 1, 0);
      {
        for (int64_t p = 0; p < np; ++p) {
          const int64_t lo = ctx->h_part_ptr[p], hi = ctx->h_part_ptr[p + 1];
          int32_t maxl = 0;
          for (int64_t i = lo; i < hi; ++i) {
            int32_t l = 0;
            for (int32_t k = klo[i]; k < (int32_t)diag[i]; ++k) l = std::max(l, lv[col32[k]] + 1);
            lv[i] = l;
            maxl = std::max(maxl, l);
          }
          std::vector<int32_t> cnt(maxl + 2, 0);
          for (int64_t i = lo; i < hi; ++i) cnt[lv[i] + 1]++;
          for (int32_t l = 0; l <= maxl; ++l) cnt[l + 1] += cnt[l];
          const std::vector<int32_t> start(cnt);
          for (int64_t i = lo; i < hi; ++i) {
            lpos[i] = cnt[lv[i]] - start[lv[i]];
            fo[lo + cnt[lv[i]]++] = (int32_t)i;
          }
          lbase[p + 1] = lbase[p] + maxl + 1;  // (schedule()'s part_lvl: a level even for an empty partition)
        }
      }
      std::vector<int32_t> plan((size_t)Nd * 32, 0);
      // k_ilu_build_grp's plans (rx_sweeps.hip): rows with at most six lower blocks, each of whose single update
      // (if any) is the diagonal (triangle-free stencils: quads, hexahedra) — [0..5] as plan, [8 + t] the column j
      // of lower block t, [14 + t] the position of A_ji in row j (-1: the block updates nothing)
      // round 6, the LDS ring of inv(D) (rx_ilu_grp_ring_w rows per level parity): [6] the row's own ring slot, [20 + t]
      // the slot of lower block t's inv(A_jj) when row j is in the previous level and in the ring (-1: read from the
      // factor in memory; its level is then flagged in ilu_gfull, so that the barrier before it waits for the stores)
      std::vector<int32_t> gplan((size_t)Nd * 32, 0);
      const int32_t rw = rx_ilu_grp_ring_w(ctx);
      auto ring_slot = [&](int32_t q) { return lpos[q] < rw ? (lv[q] & 1) * rw + lpos[q] : -1; };
      std::vector<int32_t> gfull((size_t)std::max<int32_t>(lbase[np], 0) + 1, 0);
      std::vector<int32_t> part_of(N, 0);
      for (int64_t p = 0; p < np; ++p)
        for (int64_t i = ctx->h_part_ptr[p]; i < ctx->h_part_ptr[p + 1]; ++i) part_of[i] = (int32_t)p;
      bool grp_ok = true;
      for (int64_t r = 0; r < Nd && grp_ok; ++r) {
        const int32_t i = fo[r];
        int32_t* g = gplan.data() + r * 32;
        g[0] = i;
        g[1] = klo[i];
        g[2] = (int32_t)diag[i];
        g[3] = khi[i];
        g[4] = (int32_t)ctx->h_rp[i];
        g[5] = (int32_t)ctx->h_rp[i + 1];
        const int32_t nlow = (int32_t)diag[i] - klo[i];
        grp_ok = nlow <= 6;
        g[6] = ring_slot(i);
        for (int32_t t = 0; t < 6; ++t) g[20 + t] = -1;
        for (int32_t t = 0; t < nlow && grp_ok; ++t) {
          const int32_t k = klo[i] + t;
          const int32_t nu = uptr[k + 1] - uptr[k];
          grp_ok = nu == 0 || (nu == 1 && upd[2 * uptr[k] + 1] == (int32_t)diag[i]);
          g[8 + t] = col32[k];
          g[14 + t] = nu == 1 ? upd[2 * uptr[k]] : -1;  // -1: no update
          if (lv[col32[k]] == lv[i] - 1) g[20 + t] = ring_slot(col32[k]);
          if (g[20 + t] < 0) gfull[lbase[part_of[i]] + lv[i]] = 1;
        }
      }
      for (int64_t r = 0; r < Nd; ++r) {
        const int32_t i = fo[r];
        int32_t* rec = plan.data() + r * 32;
        rec[0] = i;
        rec[1] = klo[i];
        rec[2] = (int32_t)diag[i];
        rec[3] = khi[i];
        rec[4] = (int32_t)ctx->h_rp[i];
        rec[5] = (int32_t)ctx->h_rp[i + 1];
        const int32_t nlow = (int32_t)diag[i] - klo[i];
        int32_t npair = 0;
        bool ok = nlow <= 3;
        for (int32_t t = 0; t < nlow && ok; ++t) {
          const int32_t k = klo[i] + t;
          const int32_t nu = uptr[k + 1] - uptr[k];
          if (nu > 3 || npair + nu > 9) {
            ok = false;
            break;
          }
          rec[8 + t] = col32[k];
          rec[11 + t] = nu;
          for (int32_t u = uptr[k]; u < uptr[k + 1]; ++u, ++npair) {
            rec[14 + 2 * npair] = upd[2 * u];
            rec[14 + 2 * npair + 1] = upd[2 * u + 1];
          }
        }
        rec[6] = ok ? nlow : -1;
        rec[7] = ok ? npair : 0;
      }
      ctx->ilu_grp_ok = grp_ok;
      // the grouped build's LDS (its row slots + the partition's level table) must fit this device's
      // limit; else k_ilu_build_part, and rx_ilu_upper (same predicate) keeps the sweeps on the ILU buffer
      if (grp_ok && rx_ilu_grp_lds(ctx) > (size_t)ctx->lds_max) ctx->ilu_grp_ok = false;
      CK(dupload(ctx, &ctx->ilu_plan, plan.data(), plan.size()));
      if (grp_ok) CK(dupload(ctx, &ctx->ilu_gplan, gplan.data(), gplan.size()));
      if (grp_ok) CK(dupload(ctx, &ctx->ilu_gfull, gfull.data(), gfull.size()));
      ctx->ilu_ring_w = rw;
      // PAIR build (rx_sweeps.hip): meshes whose widest level is at most RX_GRP_PAIR_W rows (the pairs' half as many
      // rows per round then cost at most two rounds where one did; the C4 rank shape, 490-row partitions with 22-row
      // levels, takes it, the C3 shape, 62-row levels, does not); RX_GRP_PAIR=0 / 1 forces it off / on
      {
        const char* ev = getenv("RX_GRP_PAIR");
        const int maxw = getenv("RX_GRP_PAIR_W") ? atoi(getenv("RX_GRP_PAIR_W")) : 32;
        ctx->ilu_pair = grp_ok && (ev ? atoi(ev) != 0 : ctx->fs.maxwidth <= maxw);
      }
    }

    const size_t per_wave = sizeof(double) * ((size_t)(rowmax + 1 + rx_ilu_stage()) * nv * nv + 16);
    if (per_wave > (size_t)ctx->lds_max) CK(RX_ERR_ARG);  // a row with more blocks than one wave's LDS slice
    ctx->ilu_waves = (int)std::max<size_t>(1, std::min<size_t>({(size_t)rx_ilu_max_waves(),
                                                                (size_t)std::max(1, ctx->fs.maxwidth),
                                                                (size_t)ctx->lds_max / per_wave}));
  }
  // halo exchange plan (distributed mesh)
  if (mesh->n_neigh > 0) {
    if (!mesh->neigh || !mesh->send_ptr || !mesh->send_idx || !mesh->recv_ptr) CK(RX_ERR_ARG);
    ctx->n_neigh = mesh->n_neigh;
    ctx->h_neigh.assign(mesh->neigh, mesh->neigh + mesh->n_neigh);
    ctx->h_send_ptr.assign(mesh->send_ptr, mesh->send_ptr + mesh->n_neigh + 1);
    ctx->h_recv_ptr.assign(mesh->recv_ptr, mesh->recv_ptr + mesh->n_neigh + 1);
    if (ctx->h_recv_ptr.back() != N - ctx->Nd) CK(RX_ERR_ARG);
    ctx->n_send = ctx->h_send_ptr.back();
    std::vector<int32_t> si(ctx->n_send);
    for (int64_t q = 0; q < ctx->n_send; ++q) {
      if (mesh->send_idx[q] < 0 || mesh->send_idx[q] >= ctx->Nd) CK(RX_ERR_ARG);
      si[q] = (int32_t)mesh->send_idx[q];
    }
    CK(dupload(ctx, &ctx->send_idx, si.data(), si.size()));
    {  // gradient order of the overlapped exchange: points some neighbour receives, then the others
      std::vector<char> sent(ctx->Nd, 0);
      for (int32_t q : si) sent[q] = 1;
      std::vector<int32_t> gl;
      gl.reserve(ctx->Nd);
      for (int64_t i = 0; i < ctx->Nd; ++i)
        if (sent[i]) gl.push_back((int32_t)i);
      ctx->n_grad_bnd = (int64_t)gl.size();
      for (int64_t i = 0; i < ctx->Nd; ++i)
        if (!sent[i]) gl.push_back((int32_t)i);
      CK(dupload(ctx, &ctx->grad_list, gl.data(), gl.size()));
    }
    {  // SpMV rows: interior (no halo column) first, then the rows on the rank boundary
      std::vector<int32_t> rl;
      rl.reserve(ctx->Nd);
      std::vector<char> bnd(ctx->Nd, 0);
      for (int64_t i = 0; i < ctx->Nd; ++i)
        for (int64_t k = ctx->h_rp[i]; k < ctx->h_rp[i + 1]; ++k)
          if (ctx->h_col[k] >= ctx->Nd) bnd[i] = 1;
      for (int64_t i = 0; i < ctx->Nd; ++i)
        if (!bnd[i]) rl.push_back((int32_t)i);
      ctx->n_spmv_int = (int64_t)rl.size();
      for (int64_t i = 0; i < ctx->Nd; ++i)
        if (bnd[i]) rl.push_back((int32_t)i);
      CK(dupload(ctx, &ctx->spmv_rows, rl.data(), rl.size()));
    }
    // the widest exchangeable node record: D_ij (Ns^2), the primitive gradient (nG x nDim) or V (nPV)
    ctx->halo_stride = std::max({kHaloMaxStride, ctx->ns * ctx->ns, ctx->nG * ctx->nDim, ctx->nPV});
    CK(dalloc(ctx, &ctx->sendbuf, (size_t)std::max<int64_t>(1, ctx->n_send) * ctx->halo_stride));
  }
  CK(dalloc(ctx, &ctx->rms_sum, 32));
  // LSQ neighbour lists (reference order) and boundary vertices per node
  std::vector<int32_t> nptr(N + 1), nbr(mesh->nbr_ptr[N]);
  for (int64_t i = 0; i <= N; ++i) nptr[i] = (int32_t)mesh->nbr_ptr[i];
  for (int64_t q = 0; q < mesh->nbr_ptr[N]; ++q) nbr[q] = (int32_t)mesh->nbr[q];
  ctx->h_bvert.assign(mesh->bvert, mesh->bvert + 2 * NB);
  ctx->h_bnormal.assign(mesh->bvert_normal, mesh->bvert_normal + NB * nd);
  std::vector<int32_t> bvp(N + 1, 0);
  std::vector<double> bvn((size_t)std::max<int64_t>(NB, 1) * nd);
  {
    for (int64_t b = 0; b < NB; ++b) bvp[mesh->bvert[2 * b + 1] + 1]++;
    for (int64_t i = 0; i < N; ++i) bvp[i + 1] += bvp[i];
    std::vector<int32_t> f(bvp.begin(), bvp.end() - 1);
    for (int64_t b = 0; b < NB; ++b) {  // input is in (marker, vertex) order: stable per node
      const int64_t p = mesh->bvert[2 * b + 1];
      const int32_t slot = f[p]++;
      for (int d = 0; d < nd; ++d) bvn[(size_t)slot * nd + d] = mesh->bvert_normal[b * nd + d];
    }
  }
  CK(dupload(ctx, &ctx->edges, e32.data(), 2 * E));
  CK(dupload(ctx, &ctx->normal, mesh->edge_normal, E * nd));
  CK(dupload(ctx, &ctx->coord, mesh->coord, N * nd));
  CK(dupload(ctx, &ctx->vol, mesh->volume, N));
  CK(dupload(ctx, &ctx->adj_ptr, adj_ptr.data(), N + 1));
  CK(dupload(ctx, &ctx->adj, adj.data(), 2 * E));
  CK(dupload(ctx, &ctx->adj_blk, adj_blk.data(), 2 * E));
  CK(dupload(ctx, &ctx->edge_blk, edge_blk.data(), 2 * E));
  for (int64_t i = 0; i < N; ++i) ctx->max_degree = std::max(ctx->max_degree, (int)(adj_ptr[i + 1] - adj_ptr[i]));
  if (ctx->kind == RX_KIND_FLOW) {  // k_asm_es's node runs: consecutive nodes while their edge sides fit the teams
    const int T = rx_asmes_teams(ctx->nVar);
    std::vector<int32_t> wg{0, 0};
    bool ok = ctx->h_rp.back() < (1LL << 31);  // block indices as int32
    for (int64_t n = 0; n < N && ok;) {
      const int64_t lo = n;
      while (n < N && n - lo < T && adj_ptr[n + 1] - adj_ptr[lo] <= T) ++n;
      ok = n > lo;  // a node with more edges than teams
      wg.push_back((int32_t)n);
      wg.push_back((int32_t)adj_ptr[n]);
    }
    if (ok && N > 0) {
      std::vector<int32_t> sr(8 * (size_t)E);
      for (int64_t k = 0; k < 2 * E; ++k) {
        const int64_t e = adj[k] >> 1, side = adj[k] & 1;
        sr[4 * k] = (int32_t)((uint32_t)e | ((uint32_t)side << 31));
        sr[4 * k + 1] = e32[2 * e];
        sr[4 * k + 2] = e32[2 * e + 1];
        sr[4 * k + 3] = (int32_t)edge_blk[2 * e + (side ? 0 : 1)];
      }
      CK(dupload(ctx, &ctx->asmes_wg, wg.data(), wg.size()));
      CK(dupload(ctx, &ctx->asmes_side, sr.data(), sr.size()));
      ctx->asmes_nwg = (int)wg.size() / 2 - 1;
    }
  }
  CK(dupload(ctx, &ctx->nbr_ptr, nptr.data(), N + 1));
  CK(dupload(ctx, &ctx->nbr, nbr.data(), nbr.size()));
  CK(dupload(ctx, &ctx->bv_ptr, bvp.data(), N + 1));
  CK(dupload(ctx, &ctx->bv_normal, bvn.data(), bvn.size()));
  CK(dupload(ctx, &ctx->rp, rp32.data(), N + 1));
  CK(dupload(ctx, &ctx->col, col32.data(), ctx->nnzb));
  CK(dupload(ctx, &ctx->diag, diag.data(), N));

  // ---- mechanism
  if (!sst) {
    rx::DevMech& m = ctx->mech;
    const int nr = mech->n_reactions, nt = mech->n_tab;
    m.ns = ns;
    m.nr = nr;
    m.ntab = nt;
    auto up = [&](const double* h, size_t n) -> const double* {
      double* d = nullptr;
      if (dupload(ctx, &d, h, n)) return nullptr;
      ctx->mech_bufs.push_back(d);
      return d;
    };
    auto upi = [&](const int32_t* h, size_t n) -> const int* {
      int32_t* d = nullptr;
      if (dupload(ctx, &d, h, n)) return nullptr;
      ctx->mech_bufs.push_back(d);
      return d;
    };
    m.mm = up(mech->mmass, ns);
    m.sr = up(mech->stoich_reac, (size_t)ns * nr);
    m.sp = up(mech->stoich_prod, (size_t)ns * nr);
    m.er = up(mech->exp_reac, (size_t)ns * nr);
    m.ep = up(mech->exp_prod, (size_t)ns * nr);
    m.A = up(mech->A, nr);
    m.beta = up(mech->beta, nr);
    m.Ta = up(mech->Ta, nr);
    m.Ab = up(mech->A_back, nr);
    m.betab = up(mech->beta_back, nr);
    m.Tab = up(mech->Ta_back, nr);
    m.rev = upi(mech->reversible, nr);
    m.hasb = upi(mech->has_backward, nr);
    m.tx = up(mech->tab_x, (size_t)5 * ns * nt);
    m.ty = up(mech->tab_y, (size_t)5 * ns * nt);
    m.ty2 = up(mech->tab_y2, (size_t)5 * ns * nt);
    {  // one temperature grid for every (prop, s) row, bitwise: spline_k() shares the interval search (rx_device.h)
      const double* X = mech->tab_x;
      bool same = true;
      for (int r = 1; r < 5 * ns && same; ++r) same = std::memcmp(X, X + (size_t)r * nt, sizeof(double) * nt) == 0;
      const char* e = getenv("RX_SPLINE_SHARED");  // 0: the per-row search everywhere (the parity tests compare both)
      m.xshared = (same && !(e && atoi(e) == 0)) ? 1 : 0;
    }
    {  // the molar masses' reciprocals as the device's division makes them (rx_fdiv.h)
      double* d = nullptr;
      RX_HIP(hipMalloc(&d, sizeof(double) * ns));
      ctx->mech_bufs.push_back(d);
      k_recip_table<<<1, 64, 0, ctx->stream>>>(m.mm, d, ns);
      RX_HIP(hipGetLastError());
      m.rmm = d;
    }
    m.mtot = 0.0;
    for (int s = 0; s < ns; ++s) m.mtot += mech->mmass[s];
    {
      std::vector<double> phic(ns * ns), pw(ns * ns), mij(ns * ns), dvs(ns * ns);
      const double* M = mech->mmass;
      for (int a = 0; a < ns; ++a)
        for (int b = 0; b < ns; ++b) {
          phic[a * ns + b] = std::sqrt(8.0 * (1.0 + M[a] / M[b]));
          pw[a * ns + b] = std::pow(M[b] / M[a], 0.25);
          mij[a * ns + b] = std::sqrt((M[a] * M[b]) / (M[a] + M[b]));
          dvs[a * ns + b] = std::cbrt(mech->diff_vol[a]) + std::cbrt(mech->diff_vol[b]);
        }
      m.phic = up(phic.data(), phic.size());
      double* d = nullptr;  // its reciprocals (rx_fdiv.h)
      RX_HIP(hipMalloc(&d, sizeof(double) * phic.size()));
      ctx->mech_bufs.push_back(d);
      if (m.phic) k_recip_table<<<1, 64, 0, ctx->stream>>>(m.phic, d, (int)phic.size());
      RX_HIP(hipGetLastError());
      m.rphic = d;
      m.pw25 = up(pw.data(), pw.size());
      m.mij = up(mij.data(), mij.size());
      m.dvs = up(dvs.data(), dvs.size());
    }
    for (int r = 0; r < rx::kMaxNR; ++r) m.neg_reac[r] = m.neg_prod[r] = 0;
    for (int r = 0; r < nr; ++r)
      for (int s = 0; s < ns; ++s) {
        if (mech->exp_reac[r * ns + s] < 0.0) m.neg_reac[r] |= (1u << s);
        if (mech->exp_prod[r * ns + s] < 0.0) m.neg_prod[r] |= (1u << s);
      }
    if (!m.mm || !m.tx || !m.ty2) CK(RX_ERR_HIP);
  }

  // ---- fields
  const int64_t nb2 = ctx->nnzb * (int64_t)nv * nv;
  const int64_t imp = ctx->cfg.implicit ? 1 : 0;
  int64_t sizes[RX_F_COUNT] = {};
  if (!sst) {
    const int64_t fl[RX_F_COUNT] = {
        N * nv,                 // U
        N * ctx->nPV,           // V
        N * nv, N * nv,         // dPdU, dTdU
        N, N,                   // mu, kappa
        N * ns * ns,            // Dij
        N * ctx->nG * nd,       // grad
        N * ctx->nL,            // limiter
        N, N, N, N,             // tke, omega, mut, sigmak
        N * nd,                 // gradk
        N,                      // eddy
        N * nv,                 // res
        N, N, N,                // dt, lambda_inv, lambda_visc
        imp * nb2,                       // jac
        imp * (nb2 + N * (int64_t)nv * nv), // ilu (+ inverse diagonals)
        N * nv, N * nv,         // sol, rhs
        N,                      // strain
        0, 0, 0, 0              // SST-only
    };
    std::copy(fl, fl + RX_F_COUNT, sizes);
  } else {
    sizes[RX_F_U] = N * 2;
    sizes[RX_F_GRAD] = N * 2 * nd;
    sizes[RX_F_LIMITER] = N * 2;  // SetSolution_Limiter of (k, omega) (SPATIAL_ORDER_TURB = 2ND_ORDER_LIMITER)
    sizes[RX_F_MUT] = N;
    sizes[RX_F_RES] = N * 2;
    sizes[RX_F_JAC] = imp * nb2;
    sizes[RX_F_ILU] = imp * (nb2 + N * 4);
    sizes[RX_F_SOL] = N * 2;
    sizes[RX_F_RHS] = N * 2;
    sizes[RX_F_F1] = sizes[RX_F_F2] = sizes[RX_F_CDKW] = sizes[RX_F_WALLDIST] = N;
  }
  for (int q = 0; q < RX_F_COUNT; ++q) {
    ctx->fcount[q] = sizes[q];
    CK(dalloc(ctx, &ctx->f[q], sizes[q]));
  }
  ctx->fcount[RX_F_ILU] = imp * nb2;
  if (ctx->cfg.implicit && !sst) {
    // fconv / jconv (the per-edge convective fluxes and blocks, 2 E nVar^2 doubles: 3.9 GB at C3) are allocated by
    // the first k_ausm_edge launch (rx_launch_ausm_edge); the 2-D fused assembly never needs them
    // The per-edge viscous Jacobians and the viscous summary live only between the viscous sweep and the assembly
    // (k_visc_edge -> k_visc_jac -> k_assemble); the ILU(0) factor is written only later, by the ILU build of the
    // implicit step. So both share the ILU buffer when it is large enough (on the jet meshes it is: (2N + 2E) nVar^2
    // doubles against 2E nVar^2 + E (14 + 5 nDim + 9 Ns)): at C5 (8M points, nVar 12) this saves 71.6 GB, which is
    // what lets the whole 1000x400x20 mesh fit one 288 GB MI355X. Otherwise they get their own buffers.
    const int64_t jv_n = E * 2 * (int64_t)nv * nv;
    const int64_t vs_n = (E + rx::kSummTile - 1) / rx::kSummTile * rx::kSummTile *
                         (int64_t)(14 + 5 * ctx->nDim + 9 * ns);  // visc_summary_size<NS, NDIM> per edge, tiled
    const int64_t vs_off = (jv_n + 255) / 256 * 256;             // 2 KiB-aligned summary tiles
    if (vs_off + vs_n <= sizes[RX_F_ILU]) {
      ctx->jvisc = ctx->f[RX_F_ILU];
      ctx->vsumm = ctx->f[RX_F_ILU] + vs_off;
      ctx->scratch_in_ilu = 1;
    } else {
      CK(dalloc(ctx, &ctx->jvisc, jv_n));
      CK(dalloc(ctx, &ctx->vsumm, vs_n));
    }
    CK(dalloc(ctx, &ctx->jsrc, (N + kSrcTile - 1) / kSrcTile * kSrcTile * (int64_t)ctx->ns * nv));
    CK(dalloc(ctx, &ctx->rsrc, N * nv));
  }
  if (ctx->cfg.implicit) {
    // LU-SGS's factorised diagonal blocks: only with the LU_SGS preconditioner (rx_lusgs_apply allocates them on
    // first use otherwise)
    if (rx_la_eff_prec(ctx) == RX_PREC_LU_SGS) CK(dalloc(ctx, &ctx->dlu, N * (int64_t)nv * nv));
    if (rx_la_eff_prec(ctx) == RX_PREC_JACOBI) CK(dalloc(ctx, &ctx->jinv, ctx->Nd * (int64_t)nv * nv));
    CK(dalloc(ctx, &ctx->xstar, N * nv));
  }
  if (!sst && ctx->cfg.spatial_order) CK(dalloc(ctx, &ctx->recon, E * 2 * (int64_t)(ctx->nPV + nv)));
  if (!sst) {
    CK(dalloc(ctx, &ctx->uold, N * nv));
    CK(dalloc(ctx, &ctx->fvisc, E * nv));
    CK(dalloc(ctx, &ctx->lim_mn, N * ctx->nL));
    CK(dalloc(ctx, &ctx->lim_mx, N * ctx->nL));
  }
  CK(dalloc(ctx, &ctx->red, 256 * 32 + 1024));
  CK(dalloc(ctx, &ctx->err, 4));
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_red), sizeof(double) * (256 * 32 + 1024)) != hipSuccess)
    CK(RX_ERR_HIP);
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) CK(RX_ERR_HIP);
  if (sst && flow->distributed()) CK(rx_comm_borrow(ctx, flow));
#undef CK
  *out = ctx;
  return RX_OK;
}

}  // namespace

extern "C" {

int rx_ctx_create(const rx_mesh_desc* mesh, const rx_mech_desc* mech, const rx_cfg* cfg, int device, rx_ctx** out) {
  if (!mech) return RX_ERR_ARG;
  return create_impl(mesh, mech, cfg, device, nullptr, out);
}

int rx_sst_create(const rx_mesh_desc* mesh, rx_ctx* flow, const rx_cfg* cfg, rx_ctx** out) {
  if (!flow || flow->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  return create_impl(mesh, nullptr, cfg, 0, flow, out);
}

int rx_ctx_destroy(rx_ctx* ctx) {
  if (!ctx) return RX_OK;
  if (ctx->n_children > 0) return RX_ERR_STATE;  // an SST context still runs on this stream / communicator
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)rx_settle_u(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  // the captured solve first: a graph holding RCCL work keeps the communicator's persistent resources, and
  // ncclCommDestroy waits for them (the self-halo RCCL test hung here with the graph destroyed after the comm)
  rx_graph_reset(ctx);
  if (ctx->kind == RX_KIND_SST && ctx->flow) --ctx->flow->n_children;
  void* ptrs[] = {ctx->edges, ctx->normal, ctx->coord, ctx->vol, ctx->adj_ptr, ctx->adj, ctx->adj_blk, ctx->edge_blk, ctx->asmes_wg, ctx->asmes_side, ctx->nbr_ptr,
                  ctx->nbr, ctx->bv_ptr, ctx->bv_normal, ctx->rp, ctx->col, ctx->diag, ctx->klo, ctx->khi, ctx->part_ptr, ctx->upd_ptr, ctx->upd, ctx->ilu_plan, ctx->ilu_gplan, ctx->ilu_gfull,
                  ctx->fs.part_lvl, ctx->fs.lvl_ptr, ctx->fs.rows, ctx->bs.part_lvl, ctx->bs.lvl_ptr, ctx->bs.rows,
                  ctx->fs.pass_lo, ctx->fs.part_pass, ctx->bs.pass_lo, ctx->bs.part_pass,
                  ctx->fs.slot, ctx->bs.slot, ctx->fs.ring, ctx->bs.ring, ctx->fs.rpart_lvl, ctx->fs.rlvl_ptr,
                  ctx->bs.rpart_lvl, ctx->bs.rlvl_ptr, ctx->ring_xoff, ctx->send_idx, ctx->grad_list, ctx->spmv_rows, ctx->sendbuf, ctx->rms_sum,
                  ctx->recon, ctx->uold, ctx->fconv, ctx->fvisc, ctx->jconv, ctx->scratch_in_ilu ? nullptr : ctx->jvisc,
                  ctx->scratch_in_ilu ? nullptr : ctx->vsumm, ctx->jsrc, ctx->rsrc, ctx->dlu, ctx->xstar, ctx->jinv,
                  ctx->lim_mn, ctx->lim_mx, ctx->red, ctx->err, ctx->kw, ctx->kz, ctx->fold_skip};
  rx_comm_free(ctx);
  if (ctx->kind == RX_KIND_FLOW) rx_bc_free(ctx);
  rx_la_krylov_free(ctx);
  for (void* p : ptrs) dfree(p);
  for (void* p : ctx->mech_bufs) dfree(p);
  for (int q = 0; q < RX_F_COUNT; ++q) dfree(ctx->f[q]);
  if (ctx->h_red) (void)hipHostFree(ctx->h_red);
  ctx->prof_drain();
  for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
  if (ctx->stream && ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return RX_OK;
}

int rx_set_system_fold(rx_ctx* ctx, int on) {
  if (!ctx) return RX_ERR_ARG;
  static const bool off = getenv("RX_NO_FOLD") && getenv("RX_NO_FOLD")[0] == '1';  // A/B
  ctx->fold_req = on && !off && ctx->kind == RX_KIND_FLOW ? 1 : 0;
  return RX_OK;
}

int rx_field_size(const rx_ctx* ctx, rx_field f, int64_t* count) {
  if (!ctx || f < 0 || f >= RX_F_COUNT || !count) return RX_ERR_ARG;
  *count = ctx->fcount[f];
  return RX_OK;
}

int rx_upload(rx_ctx* ctx, rx_field f, const double* host, int64_t count) {
  if (!ctx || f < 0 || f >= RX_F_COUNT || count != ctx->fcount[f] || !host) return RX_ERR_ARG;
  if (int rc = rx_settle_u(ctx)) return rc;
  RX_HIP(hipMemcpyAsync(ctx->f[f], host, count * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  if (f == RX_F_ILU) {  // a caller-provided factor (its diagonal blocks included)
    ctx->ilu_valid = 1;
    ctx->ilu_diag_deferred = 0;
  }
  // a loaded solution is also the Solution_Old (CVariable construction / LoadRestart)
  if (f == RX_F_U && ctx->kind == RX_KIND_FLOW && ctx->uold)
    RX_HIP(hipMemcpyAsync(ctx->uold, ctx->f[f], count * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
  RX_HIP(hipStreamSynchronize(ctx->stream));
  return RX_OK;
}

int rx_download(rx_ctx* ctx, rx_field f, double* host, int64_t count) {
  if (!ctx || f < 0 || f >= RX_F_COUNT || count != ctx->fcount[f] || !host) return RX_ERR_ARG;
  if (int rc = rx_settle_u(ctx)) return rc;
  if (f == RX_F_RES || f == RX_F_JAC) {
    int rc = ensure_assembled(ctx);
    if (rc && rc != RX_ERR_STATE) return rc;
  }
  // with the viscous scratch aliased onto it, the ILU field holds a factor only after an ILU build
  if (f == RX_F_ILU && !ctx->ilu_valid) return RX_ERR_STATE;
  if (f == RX_F_ILU && ctx->assembled) {  // the factor with the blocks ILU(0) leaves unchanged (rx_sweeps.hip);
    int rc = rx_la_ilu_materialize(ctx);  // while a residual is being assembled the field holds its scratch
    if (rc) return rc;
  }
  RX_HIP(hipMemcpyAsync(host, ctx->f[f], count * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  RX_HIP(hipStreamSynchronize(ctx->stream));
  return RX_OK;
}

int rx_bsr_pattern(const rx_ctx* ctx, int64_t* row_ptr, int64_t* col) {
  if (!ctx) return RX_ERR_ARG;
  if (row_ptr) std::memcpy(row_ptr, ctx->h_rp.data(), sizeof(int64_t) * (ctx->N + 1));
  if (col) std::memcpy(col, ctx->h_col.data(), sizeof(int64_t) * ctx->nnzb);
  return RX_OK;
}

int rx_sync(rx_ctx* ctx) {
  if (!ctx) return RX_ERR_ARG;
  if (int rc = rx_settle_u(ctx)) return rc;
  RX_HIP(hipStreamSynchronize(ctx->stream));
  return rx_check_error(ctx);
}

int64_t rx_last_error_index(const rx_ctx* ctx) { return ctx ? ctx->last_err_index : -1; }

int rx_last_error_phase(const rx_ctx* ctx) { return ctx ? ctx->last_err_phase : RX_ERR_PHASE_CALL; }

int rx_residual_zero(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RX_HIP(hipMemsetAsync(ctx->f[RX_F_RES], 0, sizeof(double) * ctx->fcount[RX_F_RES], ctx->stream));
  ctx->phase_conv = ctx->phase_visc = ctx->phase_src = ctx->offdiag_done = ctx->conv_deferred = 0;
  ctx->assembled = ctx->cfg.implicit ? 0 : 1;
  if (ctx->bc_on && ctx->bc_stream && !ctx->capturing) {
    // the boundary fluxes of the current node records, overlapped with the interior sweeps (rx_bc.hip)
    RX_HIP(hipEventRecord(ctx->bc_fork, ctx->stream));
    RX_HIP(hipStreamWaitEvent(ctx->bc_stream, ctx->bc_fork, 0));
    const int rc = rx_bc_launch_weak(ctx, ctx->bc_stream);
    if (rc) return rc;
    RX_HIP(hipEventRecord(ctx->bc_join, ctx->bc_stream));
    ctx->bc_pending = true;
  }
  return RX_OK;
}

int rx_edge_flux_conv(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_CONV);
  int rc = RX_OK;
  if (ctx->cfg.spatial_order && (rc = rx_launch_muscl(ctx))) return rc;
  ctx->conv_deferred = ctx->cfg.implicit && rx_fuse_conv(ctx->nDim) ? 1 : 0;
  if (!ctx->conv_deferred) rc = ctx->cfg.implicit ? rx_launch_ausm_edge(ctx) : rx_launch_ausm_node(ctx);
  if (rc) return rc;
  ctx->phase_conv = 1;
  ctx->offdiag_done = 0;  // new convective blocks: off-diagonals are (re)assembled from them
  ctx->assembled = ctx->cfg.implicit ? 0 : 1;
  return RX_OK;
}

int rx_edge_flux_visc(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  if (ctx->scratch_in_ilu) ctx->ilu_valid = 0;  // the per-edge viscous Jacobians / summary overwrite the factor
  int rc = rx_launch_visc_edge(ctx);
  if (rc) return rc;
  if (!ctx->cfg.implicit) {
    rc = rx_launch_gather_edge_flux(ctx, ctx->fvisc, -1.0);  // R[i] -= Fv, R[j] += Fv
    if (rc) return rc;
  }
  ctx->phase_visc = 1;
  ctx->assembled = ctx->cfg.implicit ? 0 : 1;
  return RX_OK;
}

int rx_cell_source_pasr(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_SOURCE);
  int rc = rx_launch_source(ctx);
  if (rc) return rc;
  ctx->phase_src = 1;
  ctx->assembled = ctx->cfg.implicit ? 0 : 1;
  return RX_OK;
}

int rx_grad_lsq(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_GRAD);
  const int stride = (int)(ctx->fcount[RX_F_GRAD] / ctx->N);
  if (!ctx->distributed() || !ctx->grad_list) {
    const int rc = rx_launch_grad(ctx, nullptr, ctx->N);
    if (rc) return rc;
    // Set_MPI_Primitive_Gradient (solver_direct_reactive.cpp:5049)
    return rx_la_exchange(ctx, ctx->f[RX_F_GRAD], stride);
  }
  // Distributed: the owned points the neighbours receive first, then their exchange (on comm_stream with
  // RCCL) runs while the remaining owned points are computed; halo rows come only from their owners, as
  // Set_MPI_Primitive_Gradient leaves them. Every point's arithmetic is unchanged (bitwise the same).
  int rc = rx_launch_grad(ctx, ctx->grad_list, ctx->n_grad_bnd);
  if (rc) return rc;
  const bool overlap = ctx->comm_stream != nullptr && !ctx->capturing;
  if (overlap) {
    RX_HIP(hipEventRecord(ctx->comm_fork, ctx->stream));
    RX_HIP(hipStreamWaitEvent(ctx->comm_stream, ctx->comm_fork, 0));
    if ((rc = rx_la_exchange_on(ctx, ctx->f[RX_F_GRAD], stride, ctx->comm_stream))) return rc;
    RX_HIP(hipEventRecord(ctx->comm_join, ctx->comm_stream));
  } else if ((rc = rx_la_exchange(ctx, ctx->f[RX_F_GRAD], stride))) {
    return rc;
  }
  if ((rc = rx_launch_grad(ctx, ctx->grad_list + ctx->n_grad_bnd, ctx->Nd - ctx->n_grad_bnd))) return rc;
  if (overlap) RX_HIP(hipStreamWaitEvent(ctx->stream, ctx->comm_join, 0));
  return RX_OK;
}

int rx_grad_gg(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_GRAD);
  const int rc = rx_launch_grad_gg(ctx);
  if (rc) return rc;
  // Set_MPI_Primitive_Gradient (solver_direct_reactive.cpp:4878)
  return rx_la_exchange(ctx, ctx->f[RX_F_GRAD], (int)(ctx->fcount[RX_F_GRAD] / ctx->N));
}

int rx_limiter_venkat(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_LIMITER);
  const int rc = rx_launch_limiter(ctx);
  if (rc) return rc;
  // Set_MPI_Primitive_Limiter (:1522)
  return rx_la_exchange(ctx, ctx->f[RX_F_LIMITER], (int)(ctx->fcount[RX_F_LIMITER] / ctx->N));
}

int rx_time_step(rx_ctx* ctx) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  RxPhase ph(ctx, RX_K_DT);
  return rx_launch_time_step(ctx);
}

int rx_bsr_spmv(rx_ctx* ctx, rx_field x, rx_field y) {
  if (!ctx || !ctx->cfg.implicit) return RX_ERR_ARG;
  int rc = ensure_assembled(ctx);
  if (rc) return rc;
  RxPhase ph(ctx, RX_K_SPMV);
  return rx_la_spmv(ctx, ctx->f[RX_F_JAC], ctx->f[x], ctx->f[y], nullptr);
}

int rx_ilu0_build(rx_ctx* ctx) {
  if (!ctx || !ctx->cfg.implicit) return RX_ERR_ARG;
  int rc = ensure_assembled(ctx);
  if (rc) return rc;
  RxPhase ph(ctx, RX_K_ILU_BUILD);
  return rx_la_ilu_build(ctx);
}

int rx_ilu0_apply(rx_ctx* ctx, rx_field b, rx_field x) {
  if (!ctx || !ctx->cfg.implicit) return RX_ERR_ARG;
  if (!ctx->ilu_valid) return RX_ERR_STATE;  // no factor since the last viscous sweep (scratch) / never built
  RxPhase ph(ctx, RX_K_ILU_APPLY);
  return rx_la_ilu_apply(ctx, ctx->f[b], ctx->f[x], nullptr, nullptr);
}

int rx_lusgs_apply(rx_ctx* ctx, rx_field b, rx_field x) {
  if (!ctx || !ctx->cfg.implicit) return RX_ERR_ARG;
  int rc = ensure_assembled(ctx);
  if (rc) return rc;
  if (!ctx->dlu) RX_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->dlu), sizeof(double) * ctx->N * ctx->nVar * ctx->nVar));
  RxPhase ph(ctx, RX_K_LUSGS);
  if ((rc = rx_la_diag_factor(ctx, ctx->f[RX_F_JAC]))) return rc;
  return rx_la_lusgs(ctx, ctx->f[RX_F_JAC], ctx->f[b], ctx->f[x], nullptr, nullptr);
}

int rx_fgmres(rx_ctx* ctx, double tol, int m, int* iters, double* resid) {
  if (!ctx || !ctx->cfg.implicit || !iters || !resid) return RX_ERR_ARG;
  int rc = ensure_assembled(ctx);
  if (rc) return rc;
  RxPhase ph(ctx, RX_K_KRYLOV);
  if (rx_la_eff_prec(ctx) != RX_PREC_ILU && (rc = rx_la_prec_build(ctx))) return rc;  // ILU: rx_ilu0_build's factor
  return rx_la_fgmres(ctx, tol, m, iters, resid);
}

// CSysSolve::Solve (linear_solvers_structure.cpp:601-708) on the assembled system: the preconditioner build of the
// configured branch, then cfg.lin_solver with cfg.lin_tol / lin_iter on JAC * SOL = RHS from SOL's current values
// (their halo is the caller's). Synchronous: returns the iteration count and the final residual norm.
int rx_linear_solve(rx_ctx* ctx, int* iters, double* resid) {
  if (!ctx || !ctx->cfg.implicit || !iters || !resid) return RX_ERR_ARG;
  int rc = ensure_assembled(ctx);
  if (rc) return rc;
  const int ls = ctx->cfg.lin_solver;
  if ((rc = rx_la_krylov_alloc(ctx, (ls == RX_LIN_FGMRES || ls == RX_LIN_RESTARTED_FGMRES) ? ctx->cfg.lin_iter : 3)))
    return rc;
  RxPhase ph(ctx, RX_K_KRYLOV);
  if ((rc = rx_la_prec_build(ctx))) return rc;
  if ((rc = rx_la_solve_enqueue(ctx, false))) return rc;
  int it = 0;
  double r = 0.0;
  if ((rc = rx_la_fgmres_result(ctx, &it, &r))) return rc;
  *iters = ctx->solve_iters >= 0 ? ctx->solve_iters : it;
  *resid = r;
  return RX_OK;
}

int rx_explicit_euler(rx_ctx* ctx, double* res_rms) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  int rc = rx_settle_u(ctx);
  if (rc) return rc;
  {
    RxPhase ph(ctx, RX_K_UPDATE);
    if (res_rms && (rc = rx_la_rms_enqueue(ctx, ctx->f[RX_F_RES]))) return rc;
    if ((rc = rx_la_explicit_update(ctx))) return rc;
  }
  return res_rms ? rx_la_rms_read(ctx, res_rms) : RX_OK;
}

// SetPrimitive_Variables (solver_direct_reactive.cpp:985-1040); the residual reset it also does is
// rx_residual_zero.
int rx_set_primitive(rx_ctx* ctx, int ext_iter, int64_t* n_nonphys) {
  if (!ctx || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  {
    RxPhase ph(ctx, RX_K_PRIMITIVE);
    RX_HIP(hipMemsetAsync(ctx->err + 2, 0, sizeof(int), ctx->stream));
    // with the post-update exchange still running on comm_stream (rx_la_u_exchange_begin), the owned points first
    // (they read no halo value), then the halo points once it has arrived; each point's arithmetic is unchanged
    int rc = rx_launch_set_primitive(ctx, ext_iter, 0, ctx->u_pending ? ctx->Nd : ctx->N);
    if (!rc && ctx->u_pending && !(rc = rx_settle_u(ctx))) rc = rx_launch_set_primitive(ctx, ext_iter, ctx->Nd, ctx->N);
    if (rc) return rc;
  }
  if (!n_nonphys) return RX_OK;
  int h = 0;
  RX_HIP(hipMemcpyAsync(&h, ctx->err + 2, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  const int rc = rx_sync(ctx);
  *n_nonphys = h;
  return rc;
}

// ExplicitRK_Iteration (solver_direct_reactive.cpp:2456-2493): stage iRKStep with RK_ALPHA_COEFF[iRKStep].
int rx_explicit_rk(rx_ctx* ctx, int rk_step, double alpha, double* res_rms) {
  if (!ctx || ctx->kind != RX_KIND_FLOW || rk_step < 0) return RX_ERR_ARG;
  int rc = rx_settle_u(ctx);
  if (rc) return rc;
  {
    RxPhase ph(ctx, RX_K_UPDATE);
    if (res_rms && (rc = rx_la_rms_enqueue(ctx, ctx->f[RX_F_RES]))) return rc;
    if ((rc = rx_la_rk_update(ctx, rk_step, alpha))) return rc;
  }
  return res_rms ? rx_la_rms_read(ctx, res_rms) : RX_OK;
}

namespace {
// The linear solve (FGMRES by default), RMS partials and the clipped update: a fixed kernel sequence with no host
// decision (rx_krylov.hip), recorded once as a hipGraph (RESTARTED_FGMRES runs eagerly: its cycles are host decisions). System and preconditioner builds are launched
// before it as single kernels (timed per phase).
int enqueue_solve(rx_ctx* ctx) {
  int rc;
  static const bool x_product = getenv("RX_FG_X_PRODUCT") != nullptr;  // diagnosis: the A x product at x = 0
  if ((rc = rx_la_solve_enqueue(ctx, !x_product))) return rc;
  if ((rc = rx_la_rms_enqueue(ctx, ctx->f[RX_F_RHS]))) return rc;
  return ctx->kind == RX_KIND_SST ? rx_sst_update(ctx) : rx_la_implicit_update(ctx);
}

// The same sequence as enqueue_solve for FGMRES, in two parts: iterations [0, c), then (split_tail) iterations
// [i0, m) + finish + RMS + update. An FGMRES that has stopped after c iterations leaves iterations c .. m - 1 as
// launches that return at their first instruction (≈ 4.4 µs each at the C4 rank shape, one per dependent kernel);
// the SST solve stops after 2 of its 5, so its 3 x (10-14) empty launches are skipped when the host finds it stopped.
int enqueue_solve_head(rx_ctx* ctx, int c) {
  static const bool x_product = getenv("RX_FG_X_PRODUCT") != nullptr;
  ctx->solve_iters = -1;
  return rx_la_fgmres_enqueue_part(ctx, ctx->cfg.lin_tol, ctx->cfg.lin_iter, !x_product, 0, c, false);
}
int enqueue_solve_tail(rx_ctx* ctx, int i0) {
  int rc;
  if ((rc = rx_la_fgmres_enqueue_part(ctx, ctx->cfg.lin_tol, ctx->cfg.lin_iter, false, i0, ctx->cfg.lin_iter, true)))
    return rc;
  if ((rc = rx_la_rms_enqueue(ctx, ctx->f[RX_F_RHS]))) return rc;
  return ctx->kind == RX_KIND_SST ? rx_sst_update(ctx) : rx_la_implicit_update(ctx);
}

// The split point of this solve: 0 (whole) unless FGMRES stopped early in the previous solve (or RX_FG_SPLIT=c).
int solve_split(const rx_ctx* ctx) {
  if (ctx->cfg.lin_solver != RX_LIN_FGMRES) return 0;
  const char* e = getenv("RX_FG_SPLIT");
  const int fixed = (e && e[0]) ? atoi(e) : -1;
  const int c = fixed >= 0 ? fixed : ctx->fg_split;
  return (c > 0 && c < ctx->cfg.lin_iter && c < rx_ctx::kSplitMax) ? c : 0;
}

int enqueue_solve_whole(rx_ctx* ctx, int) { return enqueue_solve(ctx); }

// Run fn(ctx, arg) captured once into (*gr, *ex) and replayed, or eagerly when graphs are off.
int run_graph(rx_ctx* ctx, bool graphs, hipGraph_t* gr, hipGraphExec_t* ex, int (*fn)(rx_ctx*, int), int arg) {
  if (!graphs) return fn(ctx, arg);
  if (!*ex) {
    RX_HIP(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    ctx->capturing = true;
    const int rc = fn(ctx, arg);
    ctx->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    if (e != hipSuccess) return rx_fail_hip(ctx, e);
    *gr = g;
    RX_HIP(hipGraphInstantiate(ex, g, nullptr, nullptr, 0));
  }
  RX_HIP(hipGraphLaunch(*ex, ctx->stream));
  return RX_OK;
}

// The solve is replayed as a graph unless RX_NO_GRAPH=1 or a host-staged transport is attached
// (its exchanges synchronise with the host).
bool graphs_enabled(const rx_ctx* ctx) {
  const char* e = getenv("RX_NO_GRAPH");
  return !(e && e[0] == '1') && !ctx->has_hcomm;
}

}  // namespace

}  // extern "C"

void rx_graph_reset(rx_ctx* ctx) {
  if (ctx->solve_exec) (void)hipGraphExecDestroy(ctx->solve_exec);
  if (ctx->solve_graph) (void)hipGraphDestroy(ctx->solve_graph);
  ctx->solve_exec = nullptr;
  ctx->solve_graph = nullptr;
  for (int p = 0; p < 2; ++p)
    for (int c = 0; c < rx_ctx::kSplitMax; ++c) {
      if (ctx->split_exec[p][c]) (void)hipGraphExecDestroy(ctx->split_exec[p][c]);
      if (ctx->split_graph[p][c]) (void)hipGraphDestroy(ctx->split_graph[p][c]);
      ctx->split_exec[p][c] = nullptr;
      ctx->split_graph[p][c] = nullptr;
    }
}

extern "C" {

namespace {
// Shared by the flow and the SST context: system build, preconditioner build (CSysSolve::Solve
// :601-653), then FGMRES + RMS + update replayed as one hipGraph.
int implicit_solve(rx_ctx* ctx, double* res_rms, int* lin_iters) {
  const bool sst = ctx->kind == RX_KIND_SST;
  int rc = rx_settle_u(ctx);  // (nothing waits on an event recorded outside the capture below)
  if (!rc) rc = ensure_assembled(ctx);
  if (rc) return rc;
  const int ls = ctx->cfg.lin_solver;
  if ((rc = rx_la_krylov_alloc(ctx, (ls == RX_LIN_FGMRES || ls == RX_LIN_RESTARTED_FGMRES) ? ctx->cfg.lin_iter : 3)))
    return rc;
  {
    RxPhase ph(ctx, sst ? RX_K_SST_SYSTEM : RX_K_UPDATE);
    if ((rc = sst ? rx_sst_build_system(ctx) : rx_la_build_system(ctx))) return rc;
  }
  {
    RxPhase ph(ctx, sst ? RX_K_SST_SYSTEM : (rx_la_eff_prec(ctx) == RX_PREC_ILU ? RX_K_ILU_BUILD : RX_K_LUSGS));
    if ((rc = rx_la_prec_build(ctx))) return rc;
  }
  {
    RxPhase ph(ctx, sst ? RX_K_SST_SOLVE : RX_K_SOLVE);
    const bool graphs = graphs_enabled(ctx) && rx_la_solve_capturable(ctx);
    if (graphs) {
      const uint64_t epoch = (sst && ctx->flow ? ctx->flow : ctx)->bc_epoch;
      if (ctx->graph_epoch != epoch) {
        rx_graph_reset(ctx);
        ctx->graph_epoch = epoch;
      }
    }
    const int c = solve_split(ctx);
    if (c == 0) {
      rc = run_graph(ctx, graphs, &ctx->solve_graph, &ctx->solve_exec, enqueue_solve_whole, 0);
    } else {
      bool stopped = false;
      rc = run_graph(ctx, graphs, &ctx->split_graph[0][c], &ctx->split_exec[0][c], enqueue_solve_head, c);
      if (!rc) rc = rx_la_fgmres_stopped(ctx, &stopped);
      const int i0 = stopped ? 0 : c;  // [1][0]: finish + RMS + update alone
      if (!rc)
        rc = run_graph(ctx, graphs, &ctx->split_graph[1][i0], &ctx->split_exec[1][i0],
                       enqueue_solve_tail, stopped ? ctx->cfg.lin_iter : c);
    }
    if (rc) return rc;
    // the flow's Set_MPI_Solution after the update, on comm_stream (rx_u_exchange_deferred), overlapping the owned
    // points of the next SetPrimitive_Variables
    if (rx_u_exchange_deferred(ctx) && (rc = rx_la_u_exchange_begin(ctx))) return rc;
  }
  if (res_rms && (rc = rx_la_rms_copy(ctx))) return rc;
  int it = 0;
  double resid = 0.0;
  rc = rx_la_fgmres_result(ctx, &it, &resid);  // one host wait for both copies
  if (res_rms && (rc == RX_OK || rc == RX_ERR_DIVERGED)) rx_la_rms_finish(ctx, res_rms);
  if (rc) return rc;
  if (lin_iters) *lin_iters = ctx->solve_iters >= 0 ? ctx->solve_iters : it;
  ctx->fg_split = it;  // the next solve's split point (solve_split)
  return RX_OK;
}
}  // namespace

// ImplicitEuler_Iteration (solver_direct_reactive.cpp:2336-2407): system build, ILU0 build if
// selected (CSysSolve::Solve :601-653), FGMRES, clipped relaxed update.
int rx_implicit_euler(rx_ctx* ctx, double* res_rms, int* lin_iters) {
  if (!ctx || !ctx->cfg.implicit || ctx->kind != RX_KIND_FLOW) return RX_ERR_ARG;
  return implicit_solve(ctx, res_rms, lin_iters);
}

// CTurbSolver::ImplicitEuler_Iteration (solver_direct_turbulent.cpp:615-728): A_ii += Vol/(CFLRed*dt),
// rhs = -R, the same preconditioned FGMRES, AddConservativeSolution, Set_MPI_Solution, RMS.
int rx_sst_implicit_euler(rx_ctx* ctx, double* res_rms, int* lin_iters) {
  if (!ctx || !ctx->cfg.implicit || ctx->kind != RX_KIND_SST) return RX_ERR_ARG;
  return implicit_solve(ctx, res_rms, lin_iters);
}

hipEvent_t rx_ctx::prof_event() {
  if (ev_pool.empty()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  hipEvent_t e = ev_pool.back();
  ev_pool.pop_back();
  return e;
}

void rx_ctx::prof_drain() {
  if (prof_pending.empty()) return;
  (void)hipEventSynchronize(prof_pending.back().b);
  for (const ProfRec& r : prof_pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      prof_ms[r.k] += ms;
      prof_n[r.k] += 1;
    }
    ev_pool.push_back(r.a);
    ev_pool.push_back(r.b);
  }
  prof_pending.clear();
}

int rx_profile_enable(rx_ctx* ctx, int on) {
  if (!ctx) return RX_ERR_ARG;
  ctx->prof_drain();
  ctx->prof = on != 0;
  for (int k = 0; k < RX_K_COUNT; ++k) {
    ctx->prof_ms[k] = 0.0;
    ctx->prof_n[k] = 0;
  }
  return RX_OK;
}

int rx_profile_read(rx_ctx* ctx, rx_kernel k, double* total_ms, int64_t* launches) {
  if (!ctx || k < 0 || k >= RX_K_COUNT) return RX_ERR_ARG;
  ctx->prof_drain();
  if (total_ms) *total_ms = ctx->prof_ms[k];
  if (launches) *launches = ctx->prof_n[k];
  return RX_OK;
}

}  // extern "C"
