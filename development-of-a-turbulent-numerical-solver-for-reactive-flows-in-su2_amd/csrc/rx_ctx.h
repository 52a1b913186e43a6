// rx_ctx.h — the device-resident state behind the C ABI (include/rx.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/rx.h"
#include "rx_device.h"

#define RX_HIP(call)                                     \
  do {                                                   \
    hipError_t _e = (call);                              \
    if (_e != hipSuccess) return rx_fail_hip(ctx, _e);   \
  } while (0)

enum rx_kind { RX_KIND_FLOW = 0, RX_KIND_SST = 1 };

constexpr int kSrcTile = 64;  // cells per tile of the source-Jacobian scratch (one wavefront, cell index fastest)

struct rx_ctx {
  int device = 0;
  int kind = RX_KIND_FLOW;
  rx_ctx* flow = nullptr;       // SST context: the flow context it reads (V, MU, EDDY, GRAD, STRAIN, DT)
  hipStream_t stream = nullptr;
  bool own_stream = true;       // SST contexts run on their flow context's stream
  int nDim = 2, ns = 0, nr = 0, nVar = 0, nPV = 0, nG = 0, nL = 0;
  int64_t N = 0, E = 0, NB = 0, nnzb = 0;
  int64_t Nd = 0;               // owned (domain) points; N - Nd halo points follow them
  // ---- distributed: halo plan and RCCL communicator (rx_comm.hip)
  int n_neigh = 0;
  std::vector<int> h_neigh;
  std::vector<int64_t> h_send_ptr, h_recv_ptr;
  int32_t* send_idx = nullptr;  // [n_send] owned points to send, grouped per neighbour
  int64_t n_send = 0;
  double* sendbuf = nullptr;    // [n_send * halo_stride]
  int halo_stride = 64;         // doubles per point of the widest exchangeable node field (>= kHaloMaxStride)
  void* comm = nullptr;         // ncclComm_t
  bool comm_owned = true;       // SST contexts borrow the flow context's communicator
  int n_children = 0;           // live SST contexts on this flow context's stream / communicator
  bool has_hcomm = false;       // host-staged transport (rx_comm_init_host)
  rx_host_comm hcomm{};
  double* h_stage = nullptr;    // pinned [(n_send + N - Nd) * halo_stride + 64]
  int nranks = 1, rank = 0;
  double* gather = nullptr;     // RCCL all-reduce: [nranks][64] all-gathered rank sums, added in rank order
  bool distributed() const { return comm != nullptr || has_hcomm; }
  // compute / communication overlap of the primitive-gradient exchange (rx_grad_lsq): the owned points
  // the neighbours need first (n_grad_bnd of them), then the rest while the exchange runs on comm_stream
  int32_t* grad_list = nullptr; // [Nd]
  int64_t n_grad_bnd = 0;
  // SpMV rows of a distributed context: owned rows with only owned columns first (n_spmv_int of them), then the rows
  // that read halo columns; FGMRES computes the first set while the preconditioned vector's halo is exchanged
  int32_t* spmv_rows = nullptr; // [Nd]
  int64_t n_spmv_int = 0;
  bool defer_exchange = false;  // the preconditioner apply leaves its closing halo exchange to the caller
  hipStream_t comm_stream = nullptr;  // RCCL transport only
  hipEvent_t comm_fork = nullptr, comm_join = nullptr;
  // the flow's post-update Set_MPI_Solution runs on comm_stream after the solve (rx_la_u_exchange_begin) while
  // SetPrimitive_Variables computes the owned points; u_pending until the context stream has waited for u_join
  // (rx_settle_u: at rx_set_primitive's halo points, and before anything else that reads / writes U, exchanges or
  // all-reduces)
  hipEvent_t u_join = nullptr;
  bool u_pending = false;
  int64_t n_global = 0;         // owned points over all ranks
  double* rms_sum = nullptr;    // [32] per-variable sums of squares (device)
  rx_cfg cfg{};

  // ---- dual grid (device)
  int32_t* edges = nullptr;     // [E][2]
  double* normal = nullptr;     // [E][nDim]
  double* coord = nullptr;      // [N][nDim]
  double* vol = nullptr;        // [N]
  int32_t* adj_ptr = nullptr;   // [N+1] incident edges per node, increasing edge id
  int32_t* adj = nullptr;       // [2E] (edge << 1) | (node is the edge's second node)
  int64_t* adj_blk = nullptr;   // [2E] BSR block index of (node, other)
  int64_t* edge_blk = nullptr;  // [E][2] BSR block index of (n0, n1) and (n1, n0)
  int max_degree = 0;           // incident edges of the busiest node
  // k_asm_es (round 6): workgroup g assembles nodes [asmes_wg[2g], asmes_wg[2g+2]), whose adjacency entries (from
  // asmes_wg[2g+1] = adj_ptr of its first node) fit its rx_asmes_teams(nVar) edge-side teams; asmes_side [2E][4] per
  // adjacency entry {edge | side << 31, n0, n1, BSR block of the neighbour row's entry}; null when a node has more
  // edges than teams (k_asm_visc then)
  int32_t* asmes_wg = nullptr;
  int32_t* asmes_side = nullptr;
  int asmes_nwg = 0;
  int32_t* nbr_ptr = nullptr;   // [N+1] LSQ neighbours in the reference order
  int32_t* nbr = nullptr;
  int32_t* bv_ptr = nullptr;    // [N+1] boundary vertices per node in (marker, vertex) order
  double* bv_normal = nullptr;  // [NB][nDim]
  // ---- BSR pattern (device + host copy)
  int32_t* rp = nullptr;        // [N+1]
  int32_t* col = nullptr;       // [nnzb]
  int64_t* diag = nullptr;      // [N] block index of the diagonal
  std::vector<int64_t> h_rp, h_col;
  // partitions (the reference's MPI ranks): contiguous row ranges; per row the BSR index range of
  // the columns inside its own partition [klo, khi) (columns are sorted, partitions contiguous)
  int npart = 1;
  std::vector<int64_t> h_part_ptr;
  int32_t* part_ptr = nullptr;  // [npart+1] device copy
  int maxpart = 1;              // rows of the largest partition
  int maxpart_nnzb = 1;         // BSR blocks of the largest partition's rows
  int lds_max = 65536;          // dynamic LDS bytes a workgroup may use on this device
  int32_t* klo = nullptr;       // [N]
  int32_t* khi = nullptr;       // [N]
  int rowmax = 1;               // max khi - klo
  int32_t* upd_ptr = nullptr;   // [nnzb+1] ILU update plan per lower block (rx_sweeps.hip)
  int32_t* upd = nullptr;       // [2 * n_upd] (kk, pos) pairs
  int32_t* ilu_plan = nullptr;  // [N][32] per forward-schedule slot row plan (rx_sweeps.hip)
  int ilu_waves = 1;            // wavefronts per workgroup of the ILU factorisation
  bool ilu_grp_ok = false;      // every row's plan is compact and updates only its diagonal (k_ilu_build_grp)
  int32_t* ilu_gplan = nullptr; // [N][32] k_ilu_build_grp's row plans (up to 6 lower blocks, one update each)
  int32_t* ilu_gfull = nullptr; // [forward levels + 1] k_ilu_build_grp: 1 = the level reads an inv(A_jj) from memory
  int ilu_ring_w = 0;           // k_ilu_build_grp's LDS ring of inv(D): rows per level parity (0: no ring)
  bool ilu_pair = false;        // k_ilu_build_grp with two lane groups per row (PAIR; rows of <= 2 lower blocks)
  int ilu_diag_deferred = 0;    // the ILU field's diagonal blocks are not stored (k_ilu_build_grp, RX_GRP_DIAG_STORE 0)
  // dependency-level schedules of the per-partition lower (fs) / upper (bs) triangular graphs:
  // partition p owns levels [part_lvl[p], part_lvl[p+1]); level l owns rows[lvl_ptr[l] .. lvl_ptr[l+1])
  struct Sched {
    int32_t* part_lvl = nullptr;
    int32_t* lvl_ptr = nullptr;
    int32_t* rows = nullptr;
    int32_t* slot = nullptr;      // [rows][4] {row, klo, diag, khi} in schedule order
    int32_t* pass_lo = nullptr;   // [npass + 1] schedule positions of the passes: <= 64 rows of one level each
    int32_t* part_pass = nullptr; // [npart + 1] each partition's passes
    int nlevels = 0, maxwidth = 0, maxlev = 0;  // maxlev: most levels of one partition
    // k_ilu_apply_ring (rx_sweeps.hip): per schedule slot {ring row, far row or -1}, the LDS rows the slot's result
    // is written to; its sub-level tables (levels wider than rows per pass / groups split, rx_api.hip) like part_lvl /
    // lvl_ptr; ring_rows = kIluRing * rmaxwidth + the most far rows of one partition
    int32_t* ring = nullptr;
    int32_t* rpart_lvl = nullptr;
    int32_t* rlvl_ptr = nullptr;
    int ring_rows = 0, rmaxlev = 0, rmaxwidth = 0;
  } fs, bs;
  int32_t* ring_xoff = nullptr;  // [nnzb] LDS row of x_col(k) for the blocks the sweeps read (L: fs ring, U: bs ring)
  double* dlu = nullptr;        // [N][nVar^2] factorised diagonal blocks (LU-SGS)
  double* xstar = nullptr;      // [N][nVar] LU-SGS forward-sweep result (halo values)
  double* jinv = nullptr;       // [Nd][nVar^2] invM of the JACOBI preconditioner / SMOOTHER_JACOBI
  long long* ilu_trace = nullptr;  // debug phase trace of the ILU factorisation (rx_debug_ilu_trace)

  // ---- mechanism
  rx::DevMech mech{};
  std::vector<void*> mech_bufs;

  // ---- fields (device), see rx_field
  double* f[RX_F_COUNT] = {};
  int64_t fcount[RX_F_COUNT] = {};

  // ---- scratch
  double* fconv = nullptr;   // [E][nVar]   convective edge fluxes (implicit path)
  double* fvisc = nullptr;   // [E][nVar]   viscous edge fluxes
  double* jconv = nullptr;   // [E][2][nVar*nVar]
  double* jvisc = nullptr;   // [E][2][nVar*nVar]
  double* vsumm = nullptr;   // [E/kSummTile][visc_summary_size][kSummTile] per-edge viscous summary (implicit)
  int scratch_in_ilu = 0;    // jvisc / vsumm alias the ILU buffer (dead before the ILU build writes it)
  int ilu_valid = 0;         // the ILU field holds a factor (set by the ILU build / an upload of the field; cleared when
                             // the viscous sweep writes its scratch there): rx_ilu0_apply / rx_download(ILU) need it
  double* jsrc = nullptr;    // [ceil(N/kSrcTile)][ns*nVar][kSrcTile] species rows of the source Jacobians
  double* rsrc = nullptr;    // [N][nVar] source residual (implicit path)
  double* uold = nullptr;    // [N][nVar] Solution_Old of the RK stages
  double* recon = nullptr;   // [E][2][nPV] reconstructed edge states + [E][2][nVar] their dP/dU (2nd order)
  int phase_conv = 0, phase_visc = 0, phase_src = 0, assembled = 1;
  int offdiag_done = 0;      // k_visc_jac wrote the off-diagonal blocks of this residual (fused assembly)
  int last_err_phase = 0;    // rx_err_phase of the last RX_ERR_NAN (rx_check_error)
  int conv_deferred = 0;     // implicit AUSM left to the assembly (rx_fuse_conv): k_asm_visc or, without it, k_ausm_edge
  int asm_visc = 0;          // this residual's viscous Jacobians are made by the assembly (k_asm_visc), not k_visc_jac
  // the implicit system's V / dt folded into the assembly (rx_set_system_fold, round 5): while fold_req is set the
  // node-centric assembly adds AddVal2Diag's V / dt (or the identity row) to the diagonal of every owned row that no
  // boundary condition changes afterwards (fold_skip[i] = 0), and the system build then leaves those diagonals alone
  int fold_req = 0;
  int sys_folded = 0;                // the last assembly folded (consumed by the next system build)
  int32_t* fold_skip = nullptr;      // [N] 1: a row the boundary conditions change after the assembly
  uint64_t fold_epoch = ~0ull;       // the bc_epoch fold_skip was made for
  double* lim_mn = nullptr;  // [N][nL]
  double* lim_mx = nullptr;
  double* red = nullptr;     // reduction scratch
  double* h_red = nullptr;   // pinned host mirror
  int* err = nullptr;        // [2] code, index (device)
  int64_t last_err_index = -1;
  // Krylov workspace (device-resident FGMRES, rx_krylov.hip)
  int krylov_m = 0;
  double* kw = nullptr;      // [(m+1)][N*nVar]
  double* kz = nullptr;      // [(m+1)][N*nVar]
  void* kstate = nullptr;    // device KState
  void* h_kstate = nullptr;  // pinned host mirror
  int solve_iters = -1;      // iterations of the last host-driven solve (RESTARTED_FGMRES: the cycles' sum), else -1
  // captured implicit solve (system build + preconditioner build + FGMRES + update)
  hipGraphExec_t solve_exec = nullptr;
  // buffers a captured solve graph bakes in: bumped by rx_bc_set (bc arrays reallocated); a graph captured under
  // another epoch of its own (flow) or its flow context's (SST) markers is re-captured
  uint64_t bc_epoch = 0;
  uint64_t graph_epoch = 0;
  hipGraph_t solve_graph = nullptr;
  // the FGMRES solve in two captured parts with a host check between them (implicit_solve): [0][c] iterations
  // [0, c), [1][c] iterations [c, m) + finish + RMS + update, [1][0] finish + RMS + update alone. fg_split: the
  // split point, the previous solve's iteration count (RX_FG_SPLIT: 0 off, n > 0 fixed)
  static constexpr int kSplitMax = 65;
  hipGraphExec_t split_exec[2][kSplitMax] = {};
  hipGraph_t split_graph[2][kSplitMax] = {};
  int fg_split = 0;
  bool capturing = false;

  // ---- boundary conditions (rx_bc.hip, rx_bc_set); the SST context reads its flow context's
  std::vector<int64_t> h_bvert;  // [NB][2] (marker, point) of the mesh, vertex order
  std::vector<double> h_bnormal; // [NB][nDim]
  bool bc_on = false;
  int bc_nmark = 0, bc_W = 0, bc_inlet_kind = 0, bc_nweak = 0, bc_nbn = 0;
  double bc_tke_inf = 0.0, bc_kine_inf = 0.0, bc_omega_inf = 0.0;
  int32_t* bc_mkind = nullptr;   // [n_marker] rx_bc_kind
  double* bc_mdata = nullptr;    // [n_marker][W]
  int32_t* bc_node = nullptr;    // [NB] per vertex: point, normal neighbour, marker
  int32_t* bc_pn = nullptr;
  int32_t* bc_mark = nullptr;
  double* bc_nrm = nullptr;      // [NB][nDim] vertex normals (vertex order)
  int32_t* bc_weak = nullptr;    // [nweak] vertices of the weak (inlet / outlet) markers
  int32_t* bc_bn = nullptr;      // [nbn] owned boundary points
  int32_t* bc_bn_ptr = nullptr;  // [nbn+1] their vertices (bc_bn_vtx) in (marker, vertex) order
  int32_t* bc_bn_vtx = nullptr;
  uint8_t* bc_wall = nullptr;    // [N] isothermal-wall points (SetVelocity_Old in the update)
  double* bc_charac = nullptr;   // [NB][nPV] ghost states (CharacPrimVar)
  double* bc_resc = nullptr;     // [NB][nVar] convective / viscous boundary fluxes
  double* bc_resv = nullptr;
  double* bc_jacc = nullptr;     // [NB][nVar^2] convective Jacobian_i
  double* bc_jacv = nullptr;     // [NB][2][nVar^2] viscous Jacobians (i, j)
  double* bc_summ = nullptr;     // [NB][visc summary]
  double* bc_sv = nullptr;       // [NB][nVar] ghost dT/dU
  // the boundary fluxes (weak markers) only read the node records, so rx_residual_zero launches them on a
  // side stream where they overlap the interior edge sweeps; rx_bc_flow joins before applying them
  hipStream_t bc_stream = nullptr;
  hipEvent_t bc_fork = nullptr, bc_join = nullptr;
  bool bc_pending = false;

  // ---- profiling
  // Phases record an event pair on the context stream without blocking; pairs are resolved
  // (elapsed time accumulated per rx_kernel) when rx_profile_read / rx_sync drain the queue.
  bool prof = false;
  struct ProfRec { hipEvent_t a, b; int k; };
  std::vector<hipEvent_t> ev_pool;   // free events
  std::vector<ProfRec> prof_pending;
  double prof_ms[RX_K_COUNT] = {};
  int64_t prof_n[RX_K_COUNT] = {};
  hipEvent_t prof_event();
  void prof_drain();
};

int rx_fail_hip(rx_ctx* ctx, hipError_t e);
constexpr int kHaloMaxStride = 64;  // minimum doubles per point of the exchange buffers (ctx->halo_stride)
// halo exchange of a device array with `stride` doubles per point (no-op without communicator)
int rx_la_exchange(rx_ctx* ctx, double* f, int stride);
int rx_la_exchange_on(rx_ctx* ctx, double* f, int stride, hipStream_t st);
bool rx_u_exchange_deferred(const rx_ctx* ctx);  // the flow's post-update exchange overlaps SetPrimitive_Variables
int rx_la_u_exchange_begin(rx_ctx* ctx);          // that exchange, on comm_stream
int rx_settle_u(rx_ctx* ctx);                     // the context stream waits for it (an SST context: its flow's)
// out[i] = sum over ranks of in[i] (in == out allowed), ordered on the context stream; no-op
// without communicator
int rx_la_allreduce(rx_ctx* ctx, const double* in, double* out, int count);
void rx_comm_free(rx_ctx* ctx);
int rx_comm_borrow(rx_ctx* ctx, const rx_ctx* from);

// Phase timer: records HIP events around a phase on the context stream when profiling is on.
struct RxPhase {
  rx_ctx* c;
  rx_kernel k;
  hipEvent_t a = nullptr;
  RxPhase(rx_ctx* ctx, rx_kernel kk) : c(ctx), k(kk) {
    if (c->prof && !c->capturing) {
      a = c->prof_event();
      (void)hipEventRecord(a, c->stream);
    }
  }
  ~RxPhase() {
    if (a) {
      hipEvent_t b = c->prof_event();
      (void)hipEventRecord(b, c->stream);
      c->prof_pending.push_back({a, b, (int)k});
      if (c->prof_pending.size() > 4096) c->prof_drain();
    }
  }
};

// kernel launchers (rx_kernels.hip)
int rx_launch_ausm_node(rx_ctx* ctx);
int rx_launch_muscl(rx_ctx* ctx);
int rx_launch_set_primitive(rx_ctx* ctx, int ext_iter, int64_t lo, int64_t hi);  // points [lo, hi)
int rx_launch_ausm_edge(rx_ctx* ctx);
bool rx_fuse_conv(int nDim);
int rx_asmes_teams(int nVar);  // edge-side teams per k_asm_es workgroup
// levels of the ILU(0) sweeps' LDS ring (k_ilu_apply_ring): a row's result is read from the ring slot of its level
// by the rows up to kIluRing - 1 levels later, from a per-partition "far" slot by later ones
constexpr int kIluRing = 4;
int rx_ilu_ring_rpb(int nv, int tb);  // rows per pass of k_ilu_apply_ring (tb threads)
int rx_ilu_ring_tb(const rx_ctx* ctx);  // its workgroup size for this context (1 024, or 768 in 3-D)
int rx_ilu_ring_groups();     // wavefront groups of k_ilu_apply_ring taking turns by level (RX_ILU_RING_G, default 2)
int rx_launch_visc_edge(rx_ctx* ctx);
int rx_launch_gather_edge_flux(rx_ctx* ctx, const double* flux, double sign_first);
int rx_launch_source(rx_ctx* ctx);
int rx_launch_assemble(rx_ctx* ctx, int with_visc, int with_src);
int rx_launch_grad(rx_ctx* ctx, const int32_t* list, int64_t n);
int rx_launch_grad_gg(rx_ctx* ctx);  // list null: points 0..n-1
int rx_launch_limiter(rx_ctx* ctx);
int rx_launch_time_step(rx_ctx* ctx);
int rx_check_error(rx_ctx* ctx);
// linear algebra (rx_linalg.hip)
int rx_la_spmv(rx_ctx* ctx, const double* A, const double* x, double* y, const int* skip);
int rx_la_lusgs(rx_ctx* ctx, const double* A, const double* b, double* x, int* done, const int* conv);
int rx_la_diag_factor(rx_ctx* ctx, const double* A);
int rx_la_ilu_build(rx_ctx* ctx);
int rx_la_prepare(rx_ctx* ctx);
int rx_la_ilu_apply(rx_ctx* ctx, const double* b, double* x, int* done, const int* conv);
double* rx_invd_buf(rx_ctx* ctx);
const double* rx_ilu_upper(rx_ctx* ctx);  // the factor's upper blocks as the sweeps read them
int rx_la_ilu_materialize(rx_ctx* ctx);   // complete ILU field for rx_download
int rx_ilu_stage();      // staged blocks per wave of the ILU(0) build (rx_sweeps.hip kStage)
int rx_ilu_max_waves();  // wavefronts per workgroup cap of the ILU(0) build
int rx_la_krylov_alloc(rx_ctx* ctx, int m);
// Drop the captured solve graph (its kernel arguments point at buffers about to be replaced).
void rx_graph_reset(rx_ctx* ctx);
int rx_la_fgmres_enqueue(rx_ctx* ctx, double tol, int m, bool x_zero);  // x_zero: SOL is all +0.0
int rx_la_fgmres_enqueue_part(rx_ctx* ctx, double tol, int m, bool x_zero, int i0, int i1, bool finish);
int rx_la_fgmres_stopped(rx_ctx* ctx, bool* stopped);  // synchronises: the partial solve has stopped
int rx_la_rms_copy(rx_ctx* ctx);                           // rx_la_rms_read's copy to the host (no wait)
void rx_la_rms_finish(const rx_ctx* ctx, double* rms);  // ... and its RMS from the copied sums
int rx_la_host_wait(rx_ctx* ctx);  // waits for ctx->stream's work so far
int rx_la_fgmres_result(rx_ctx* ctx, int* iters, double* resid);
int rx_la_fgmres(rx_ctx* ctx, double tol, int m, int* iters, double* resid);
// the other Krylov / smoother branches of CSysSolve::Solve (rx_krylov.hip); results via rx_la_fgmres_result
int rx_la_bcgstab_enqueue(rx_ctx* ctx, double tol, int m, bool x_zero);
int rx_la_smoother_enqueue(rx_ctx* ctx, double tol, int m, bool x_zero);
int rx_la_restarted_fgmres(rx_ctx* ctx, double tol, int iter, int restart, bool x_zero, int* iters, double* resid);
int rx_la_solve_enqueue(rx_ctx* ctx, bool x_zero);  // cfg.lin_solver's branch (host-synchronous for RESTARTED)
bool rx_la_solve_capturable(const rx_ctx* ctx);     // the branch is a fixed kernel sequence (graph-capturable)
// JACOBI preconditioner (rx_sweeps.hip): invM build, apply (+ halo exchange unless defer_exchange), smoother update
int rx_la_jacobi_build(rx_ctx* ctx, const double* A);
int rx_la_jacobi_apply(rx_ctx* ctx, const double* b, double* x, int* done, const int* conv);
int rx_la_jacobi_smooth(rx_ctx* ctx, const double* r, double* x, const int* done);
int rx_la_prec_apply(rx_ctx* ctx, const double* b, double* x, int* done, const int* conv);  // by rx_la_eff_prec
// the preconditioner the solve applies: cfg.lin_prec for the Krylov solvers, the smoother's own for SMOOTHER_*
int rx_la_eff_prec(const rx_ctx* ctx);
int rx_la_prec_build(rx_ctx* ctx);  // the preconditioner build CSysSolve::Solve does before the solve
void rx_la_krylov_free(rx_ctx* ctx);
int rx_la_rms_enqueue(rx_ctx* ctx, const double* r);
int rx_la_rms_read(rx_ctx* ctx, double* rms);
int rx_la_implicit_update(rx_ctx* ctx);
int rx_la_explicit_update(rx_ctx* ctx);
int rx_la_rk_update(rx_ctx* ctx, int stage, double alpha);
int rx_la_build_system(rx_ctx* ctx);
// boundary conditions (rx_bc.hip)
void rx_bc_free(rx_ctx* ctx);
int rx_bc_launch_weak(rx_ctx* ctx, hipStream_t st);  // ghost states + boundary fluxes (+ Jacobians)
size_t rx_ilu_grp_lds(const rx_ctx* ctx);  // grouped ILU build's dynamic LDS (rx_sweeps.hip)
int rx_ilu_grp_ring_w(const rx_ctx* ctx);  // rows per level parity of the grouped build's inv(D) ring (rx_sweeps.hip)
int rx_ensure_assembled(rx_ctx* ctx);  // implicit: assemble the residual / BSR Jacobian now (rx_api.hip)
// SST (rx_sst.hip)
int rx_sst_build_system(rx_ctx* ctx);
int rx_sst_update(rx_ctx* ctx);
