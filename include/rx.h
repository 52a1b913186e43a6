/* rx.h — C ABI of the MI355X reactive-RANS hot path (librx.so).
 *
 * Drop-in boundary for the loops the reference runs inside its CSolver overrides. Each entry point
 * replaces one reference loop / operator (paths relative to the reference root):
 *
 *   rx_edge_flux_conv    CReactiveEulerSolver::Upwind_Residual (1st order, or the MUSCL 2nd-order branch
 *                        :2554-2729 when rx_cfg.spatial_order > 0)
 *                        SU2_CFD/src/solver_direct_reactive.cpp:2535-2785 with
 *                        CUpwReactiveAUSM::ComputeResidual SU2_CFD/src/numerics_direct_reactive.cpp:53-378
 *   rx_edge_flux_visc    CReactiveNSSolver::Viscous_Residual solver_direct_reactive.cpp:5305-5386 with
 *                        CAvgGradReactive_Flow::ComputeResidual numerics_direct_reactive.cpp:1425-1678
 *   rx_cell_source_pasr  CReactiveEulerSolver::Source_Residual solver_direct_reactive.cpp:2792-2874 with
 *                        CSourceReactive::ComputeChemistry numerics_direct_reactive.cpp:1728-1879
 *   rx_grad_lsq          CReactiveNSSolver::SetPrimitive_Gradient_LS solver_direct_reactive.cpp:4887-5050
 *   rx_grad_gg           CReactiveNSSolver::SetPrimitive_Gradient_GG solver_direct_reactive.cpp:4784-4880
 *   rx_limiter_venkat    CReactiveEulerSolver::SetPrimitive_Limiter solver_direct_reactive.cpp:1328-1523
 *                        (Venkatakrishnan or Barth-Jespersen by rx_cfg.slope_limiter)
 *   rx_time_step         CReactiveNSSolver::SetTime_Step solver_direct_reactive.cpp:5057-5298
 *   rx_bsr_spmv          CSysMatrix::MatrixVectorProduct Common/src/matrix_structure.cpp:997-1030
 *   rx_ilu0_build        CSysMatrix::BuildILUPreconditioner matrix_structure.cpp:1368-1451
 *   rx_ilu0_apply        CSysMatrix::ComputeILUPreconditioner matrix_structure.cpp:1453-1515
 *   rx_lusgs_apply       CSysMatrix::ComputeLU_SGSPreconditioner matrix_structure.cpp:1673-1709
 *   rx_fgmres            CSysSolve::FGMRES_LinSolver Common/src/linear_solvers_structure.cpp:309-463
 *   rx_linear_solve      CSysSolve::Solve linear_solvers_structure.cpp:601-708 (FGMRES, BCGSTAB :465-599,
 *                        RESTARTED_FGMRES; JACOBI / ILU0 / LU_SGS preconditioners; the LU_SGS / Jacobi / ILU0
 *                        smoothers matrix_structure.cpp:1268-1835)
 *   rx_implicit_euler    CReactiveEulerSolver::ImplicitEuler_Iteration solver_direct_reactive.cpp:2336-2407
 *   rx_explicit_euler    CReactiveEulerSolver::ExplicitEuler_Iteration solver_direct_reactive.cpp:2414-2449
 *   rx_explicit_rk       CReactiveEulerSolver::ExplicitRK_Iteration solver_direct_reactive.cpp:2456-2493
 *
 * Ownership: all device buffers belong to the rx_ctx. Host arrays passed in are copied at the
 * call; no pointer is retained. Every function returns an rx_status; on RX_ERR_NAN /
 * RX_ERR_RANGE the index of the first offending edge/cell is available from rx_last_error_index
 * (reference behaviour: std::runtime_error "NaN found in the ... residual").
 * Layouts are the reference's (row-major per node):
 *   V   [N][nPrimVar]  T, u, v, P, rho, h, a, Y_1..Y_Ns   (nPrimVar = Ns + nDim + 5)
 *   U   [N][nVar]      rho, rho u, rho v, rho E, rho Y_s   (nVar = Ns + nDim + 2)
 *   grad[N][nPrimVarGrad][nDim]  T, u, v, P, X_1..X_Ns    (nPrimVarGrad = Ns + nDim + 2)
 *   Dij [N][Ns][Ns], BSR blocks [nnzb][nVar][nVar] row-major, columns sorted per row (local number, or global
 *   number with rx_mesh_desc.global_id), diagonal included.
 */
#ifndef RX_H
#define RX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  RX_OK = 0,
  RX_ERR_ARG = 1,
  RX_ERR_HIP = 2,
  RX_ERR_NAN = 3,
  RX_ERR_RANGE = 4,
  RX_ERR_NONPHYS = 5,
  RX_ERR_DIVERGED = 6,
  RX_ERR_STATE = 7,
  RX_ERR_COMM = 8,    /* RCCL error */
  RX_ERR_UNSUPPORTED = 9  /* input the path does not implement (rx_case_read: physics / numerics keys of other solvers) */
} rx_status;

typedef struct rx_ctx rx_ctx;

/* Mechanism + property tables (reacting_model_library.cpp Setup/readers output). Tables are
 * [5][Ns][nTab] in property order cp, h, s, mu, kappa with the spline second derivatives. */
typedef struct {
  int32_t n_species, n_reactions, n_tab;
  const double *mmass, *diff_vol;
  const double *stoich_reac, *stoich_prod; /* [Ns][nR] */
  const double *exp_reac, *exp_prod;       /* [nR][Ns] */
  const double *A, *beta, *Ta, *A_back, *beta_back, *Ta_back;
  const int32_t *reversible, *has_backward;
  const double *tab_x, *tab_y, *tab_y2;
} rx_mech_desc;

/* Dual grid (CGeometry edges / dual volumes / boundary vertices). Edge order is the reference's
 * (i < j), normals oriented i -> j. nbr = point neighbour lists in the reference's order.
 * n_dim 2 or 3 (flow contexts: 3 to 9 species in either, csrc/rx_species.h; 3-D node records carry w / rho w after
 * v / rho v). */
typedef struct {
  int32_t n_dim;
  int64_t n_point, n_edge, n_bvert;
  const int64_t *edges;      /* [E][2] */
  const double *edge_normal; /* [E][nDim] */
  const double *coord;       /* [N][nDim] */
  const double *volume;      /* [N] */
  const int64_t *nbr_ptr;    /* [N+1] */
  const int64_t *nbr;        /* [nbr_ptr[N]] */
  const int64_t *bvert;      /* [nB][2] (marker, point) in marker / vertex order */
  const double *bvert_normal;/* [nB][nDim] */
  /* Partitions standing for the reference's MPI ranks (CGeometry partitioning,
   * geometry_structure.cpp:11465-11530): points are numbered partition by partition and
   * part_ptr[p]..part_ptr[p+1] is partition p. The ILU(0)/LU-SGS preconditioners act per partition
   * exactly as each rank's CSysMatrix does (matrix_structure.cpp:1397/1416/1472 skip halo columns;
   * LU-SGS's backward sweep reads halo x*). n_part = 0 or part_ptr = NULL: one partition. */
  int64_t n_part;
  const int64_t *part_ptr;   /* [n_part+1] */
  /* Distributed mesh (one rank per GPU, geometry_structure.cpp:11465-11530 partitioning): the first
   * n_domain points are owned, the rest are halo points grouped by owning rank. n_neigh neighbour
   * ranks; to neighbour k this rank sends its points send_idx[send_ptr[k]..send_ptr[k+1]) and
   * receives halo points n_domain + recv_ptr[k] .. n_domain + recv_ptr[k+1]. n_domain = 0: all
   * points are owned (single rank). Partitions must then cover exactly [0, n_domain). */
  int64_t n_domain;
  int32_t n_neigh;
  const int32_t *neigh;      /* [n_neigh] ranks */
  const int64_t *send_ptr;   /* [n_neigh+1] */
  const int64_t *send_idx;   /* [send_ptr[n_neigh]] local owned point ids */
  const int64_t *recv_ptr;   /* [n_neigh+1] offsets into the halo block */
  /* Distributed mesh, optional: the global number of every local point [n_point] (owned points in increasing
   * global order). When given, each BSR row holds its blocks in increasing global column (rx_bsr_pattern then
   * returns that order) and the caller's local edges keep the global edge order and orientation, so an owned
   * row's residual, Jacobian and SpMV sums run in the undivided mesh's order (meshgen.shard). NULL: columns in
   * increasing local number, as a reference rank's own CSysMatrix (matrix_structure.cpp:113-201). */
  const int64_t *global_id;
} rx_mesh_desc;

typedef struct {
  double mach_inf;                               /* CUpwReactiveAUSM mInfty */
  double T_ref, E_ref, R_ref, rho_ref, t_ref;    /* non-dimensionalisation (all 1 when DIMENSIONAL) */
  double prandtl_lam, prandtl_turb, lewis_turb;  /* CNumerics / config */
  double c_mu, pasr_lb;                          /* PaSR closure */
  double cfl, max_delta_time;                    /* SetTime_Step */
  double ref_elem_length, limiter_coeff;         /* Venkatakrishnan */
  double lin_tol, relaxation;                    /* LINEAR_SOLVER_ERROR, RELAXATION_FACTOR_FLOW */
  int32_t implicit, rans, lin_iter, lin_prec;    /* lin_prec: rx_lin_prec (0 = LU_SGS, 1 = ILU0, 2 = JACOBI) */
  int32_t spatial_order;  /* SPATIAL_ORDER_FLOW: 0 = 1ST_ORDER, 1 = 2ND_ORDER (MUSCL), 2 = 2ND_ORDER_LIMITER
                             (MUSCL with RX_F_LIMITER), Upwind_Residual :2554-2729 */
  int32_t clip_temp;      /* CLIPPING_TEMPRATURE (Cons2PrimVar :711-712) */
  double t_min, t_max;    /* TEMPERATURE_MIN / TEMPERATURE_MAX (Cons2PrimVar secant / bisection bounds) */
  double p_ref, visc_ref, cond_ref, vel_ref, len_ref;  /* Pressure/Viscosity/Conductivity/Velocity/Length_Ref */
  int32_t slope_limiter;  /* SLOPE_LIMITER_FLOW: rx_slope_limiter (SetPrimitive_Limiter :1383 / :1443) */
  /* IGNITION / IGNITION_ITER / IGNITION_TEMPERATURE / FUEL_INDEX / OXIDIZER_INDEX (config_structure.cpp:591-603;
   * defaults 0, 999999, 1700, 0, 2): SetPrimitive_Variables (solver_direct_reactive.cpp:1013-1024) sets the record's
   * temperature to ignition_temp at points with Y_fuel > 0.4, Y_oxidizer > 0.2 and T < ignition_temp while the
   * outer iteration (rx_set_primitive's ext_iter) is below ignition_iter; the rest of the record keeps the
   * secant's temperature. */
  int32_t ignition, fuel_index, oxidizer_index;
  int64_t ignition_iter;
  double ignition_temp;
  /* NUM_METHOD_GRAD (config_structure.cpp:1147): rx_grad_method. The flow's Preprocessing calls rx_grad_lsq or
   * rx_grad_gg by it (solver_direct_reactive.cpp:4717); the SST context's Preprocessing / Postprocessing gradient of
   * (k, omega) follows its own rx_cfg (solver_direct_turbulent.cpp:2944, 2963). */
  int32_t grad_method;
  /* LINEAR_SOLVER (config_structure.cpp:1047, default FGMRES): rx_lin_solver, the Krylov branch of CSysSolve::Solve
   * (linear_solvers_structure.cpp:655-672). LINEAR_SOLVER_RESTART_FREQUENCY (:1056, default 10): RESTARTED_FGMRES's
   * lin_restart. The subspace size / iteration cap is lin_iter (LINEAR_SOLVER_ITER) for every solver. rx_cfg_default:
   * FGMRES, 10. */
  int32_t lin_solver, lin_restart;
} rx_cfg;

typedef enum { RX_GRAD_WEIGHTED_LEAST_SQUARES = 0, RX_GRAD_GREEN_GAUSS = 1 } rx_grad_method;

typedef enum { RX_PREC_LU_SGS = 0, RX_PREC_ILU = 1, RX_PREC_JACOBI = 2 } rx_lin_prec;

/* the SMOOTHER_* kinds are Solve's non-Krylov branch (:683-708): LU_SGS_Smoother / Jacobi_Smoother / ILU0_Smoother
 * (matrix_structure.cpp:1711 / :1268 / :1517) with lin_iter smoothing iterations; lin_prec is not read for them */
typedef enum {
  RX_LIN_FGMRES = 0, RX_LIN_BCGSTAB = 1, RX_LIN_RESTARTED_FGMRES = 2,
  RX_LIN_SMOOTHER_LUSGS = 3, RX_LIN_SMOOTHER_JACOBI = 4, RX_LIN_SMOOTHER_ILU = 5
} rx_lin_solver;

typedef enum { RX_LIMITER_VENKATAKRISHNAN = 0, RX_LIMITER_BARTH_JESPERSEN = 1 } rx_slope_limiter;

typedef enum {
  RX_F_U = 0, RX_F_V, RX_F_DPDU, RX_F_DTDU, RX_F_MU, RX_F_KAPPA, RX_F_DIJ, RX_F_GRAD, RX_F_LIMITER,
  RX_F_TKE, RX_F_OMEGA, RX_F_MUT, RX_F_SIGMAK, RX_F_GRADK, RX_F_EDDY,
  RX_F_RES,        /* LinSysRes [N][nVar] */
  RX_F_DT,         /* local time step [N] */
  RX_F_LAMBDA_INV, RX_F_LAMBDA_VISC,
  RX_F_JAC,        /* BSR blocks [nnzb][nVar][nVar] */
  RX_F_ILU,        /* ILU(0) factor, same layout */
  RX_F_SOL,        /* LinSysSol [N][nVar] */
  RX_F_RHS,        /* linear-system right-hand side [N][nVar] */
  RX_F_STRAIN,     /* flow: StrainMag [N] (CReactiveNSVariable::SetStrainMag) */
  RX_F_F1,         /* SST: Menter blending F1 [N] */
  RX_F_F2,         /* SST: Menter blending F2 [N] */
  RX_F_CDKW,       /* SST: cross diffusion CDkw [N] */
  RX_F_WALLDIST,   /* SST: wall distance [N] (CGeometry::ComputeWall_Distance output) */
  RX_F_COUNT
} rx_field;

int rx_ctx_create(const rx_mesh_desc *mesh, const rx_mech_desc *mech, const rx_cfg *cfg, int device, rx_ctx **out);
int rx_ctx_destroy(rx_ctx *ctx); /* RX_ERR_STATE for a flow context whose SST context (rx_sst_create) is alive:
                                    destroy the SST context first (it runs on the flow's stream / communicator) */
int rx_field_size(const rx_ctx *ctx, rx_field f, int64_t *count);
/* Optimisation hint for a caller that runs the whole ImplicitEuler sequence of an iteration (the loops, BC_*, then
   rx_implicit_euler) with no rx_download / rx_upload of RES or JAC in between (rx.Iterate does): on = 1 lets the
   node-centric assembly add ImplicitEuler_Iteration's AddVal2Diag V/dt (solver_direct_reactive.cpp:2336-2387) to the
   rows no boundary condition changes afterwards, so the system build no longer revisits their diagonal blocks.
   The system is bitwise the same; only the intermediate JAC / RES between the assembly and the implicit step differ
   from the reference's, which is why it is off by default. Flow contexts only (ignored for SST); RX_NO_FOLD=1
   disables it. */
int rx_set_system_fold(rx_ctx *ctx, int on);
int rx_upload(rx_ctx *ctx, rx_field f, const double *host, int64_t count);
int rx_download(rx_ctx *ctx, rx_field f, double *host, int64_t count);
int rx_bsr_pattern(const rx_ctx *ctx, int64_t *row_ptr, int64_t *col); /* host copies, [N+1], [nnzb] */
int rx_sync(rx_ctx *ctx);
int64_t rx_last_error_index(const rx_ctx *ctx);
/* Which reference loop produced the last RX_ERR_NAN that rx_sync / a phase call returned: RX_ERR_PHASE_CALL = the loop
 * of the call itself; RX_ERR_PHASE_UPWIND = Upwind_Residual (solver_direct_reactive.cpp:2746-2757 "NaN found in the
 * upwind residual"): in 2-D and in 3-D (round 5) the implicit AUSM flux and Jacobians are evaluated by the
 * node-centric assembly (k_asm_es / k_asm_visc), which runs at the first call that needs the system (rx_bc_flow,
 * rx_fgmres, a RES / JAC download), not by rx_edge_flux_conv; with RX_ASM_CONV=0 or RX_ASM_VISC=0 in the environment
 * the edge kernel k_ausm_edge evaluates them inside rx_edge_flux_conv again. */
typedef enum { RX_ERR_PHASE_CALL = 0, RX_ERR_PHASE_UPWIND = 1 } rx_err_phase;
int rx_last_error_phase(const rx_ctx *ctx);
const char *rx_status_string(int status);

/* Residual / Jacobian phases (Space_Integration order). */
int rx_residual_zero(rx_ctx *ctx);      /* LinSysRes = 0, Jacobian = 0 (Preprocessing) */
int rx_edge_flux_conv(rx_ctx *ctx);     /* R[i] += F, R[j] -= F (+ Jacobian blocks) */
int rx_edge_flux_visc(rx_ctx *ctx);     /* R[i] -= Fv, R[j] += Fv (+ Jacobian blocks) */
int rx_cell_source_pasr(rx_ctx *ctx);   /* R[i] += S (+ diagonal block) */
int rx_grad_lsq(rx_ctx *ctx);           /* grad from V (weighted least squares) */
/* CReactiveNSSolver::SetPrimitive_Gradient_GG (solver_direct_reactive.cpp:4784-4880): Green-Gauss grad from V, with
 * the reference's node-0 species on both sides of an edge (:4812-4813) */
int rx_grad_gg(rx_ctx *ctx);
int rx_limiter_venkat(rx_ctx *ctx);     /* limiter from V, grad */
int rx_time_step(rx_ctx *ctx);          /* dt, lambda_inv, lambda_visc */

/* Linear algebra on the context's BSR Jacobian (all on device vectors of the context). */
int rx_bsr_spmv(rx_ctx *ctx, rx_field x, rx_field y);
int rx_ilu0_build(rx_ctx *ctx);
int rx_ilu0_apply(rx_ctx *ctx, rx_field b, rx_field x);
int rx_lusgs_apply(rx_ctx *ctx, rx_field b, rx_field x);
int rx_fgmres(rx_ctx *ctx, double tol, int m, int *iters, double *resid); /* solves JAC * SOL = RHS */
/* CSysSolve::Solve (linear_solvers_structure.cpp:601-708): the configured preconditioner build and linear solver
 * (rx_cfg lin_solver / lin_prec / lin_tol / lin_iter / lin_restart) on JAC * SOL = RHS from SOL's current values */
int rx_linear_solve(rx_ctx *ctx, int *iters, double *resid);

/* Multi-GPU (RCCL over xGMI). rx_comm_unique_id on one rank, broadcast the 128 bytes, then
 * rx_comm_init on every rank. With a communicator the context exchanges halo values where the
 * reference calls SendReceive / Set_MPI_* (after the gradient and the limiter, before every SpMV,
 * the LU-SGS halo x*) and all-reduces every FGMRES inner product and the RMS. */
int rx_comm_unique_id(void *id128);
int rx_comm_init(rx_ctx *ctx, int nranks, int rank, const void *id128);

/* Host-staged transport: the reference's own MPI pattern (CSysMatrix::SendReceive_Solution,
 * Common/src/matrix_structure.cpp:794-880, point-to-point host buffers; dotProd's MPI_Allreduce,
 * Common/src/vector_structure.cpp:397-419). Halo values and inner products are staged through pinned
 * host memory and handed to the caller's transport (MPI, gloo, ...). Synchronous: a context with a
 * host transport runs its solve eagerly (no graph).
 *   sendrecv: for every neighbour k, send points [send_ptr[k], send_ptr[k+1]) of `send` (stride
 *             doubles each) to rank neigh[k] and receive points [recv_ptr[k], recv_ptr[k+1]) of
 *             `recv` from it.
 *   allreduce: out[i] = sum over ranks of in[i], i < count (in == out allowed), added in rank order starting from
 *             rank 0's value (((in_0 + in_1) + in_2) + ...), as the RCCL path does (all-gather, then the ordered
 *             sum): every rank gets the same doubles, and the result is a fixed function of the rank sums.
 * Both return 0 on success. */
typedef struct {
  void *user;
  int (*sendrecv)(void *user, int32_t n_neigh, const int32_t *neigh, const int64_t *send_ptr, const double *send,
                  const int64_t *recv_ptr, double *recv, int32_t stride);
  int (*allreduce)(void *user, const double *in, double *out, int32_t count);
} rx_host_comm;
int rx_comm_init_host(rx_ctx *ctx, int nranks, int rank, const rx_host_comm *ops);

/* owned -> halo copies of a node field (every per-point field: U, V, D_ij, GRAD, ...; the exchange buffers are
 * sized for the widest, max(Ns^2, nPrimVarGrad*nDim, nPrimVar, 64) doubles per point). JAC / ILU (per block, not
 * per point) return RX_ERR_ARG. */
int rx_halo_exchange(rx_ctx *ctx, rx_field f);

/* CReactiveEulerSolver::SetPrimitive_Variables (solver_direct_reactive.cpp:985-1040) on every point:
 * CReactiveNSVariable::SetPrimVar(eddy = MUT, k = TKE) (variable_direct_reactive.cpp:1188-1228) — Cons2PrimVar
 * (:550-778) from RX_F_U with the secant started at the current RX_F_V temperature, Cp, dT/dU, dP/dU
 * (:786-853), mu, kappa, Dij (reacting_model_library.cpp:634-766), eddy viscosity. Writes RX_F_V, DPDU,
 * DTDU, MU, KAPPA, DIJ, EDDY (and clamps RX_F_U as the reference does). ext_iter > 0 enables the reference's
 * restart from Solution_Old (kept by the last update) and CLIPPING_TEMPRATURE. n_nonphys (optional, syncs):
 * the reference's ErrorCounter. A failed bisection returns RX_ERR_NONPHYS (the reference throws). */
int rx_set_primitive(rx_ctx *ctx, int ext_iter, int64_t *n_nonphys);

/* Time integration (updates RX_F_U). */
int rx_explicit_euler(rx_ctx *ctx, double *res_rms /* [nVar] or NULL */);
int rx_implicit_euler(rx_ctx *ctx, double *res_rms /* [nVar] or NULL */, int *lin_iters);
/* CReactiveEulerSolver::ExplicitRK_Iteration (solver_direct_reactive.cpp:2456-2493): stage rk_step with
 * alpha = RK_ALPHA_COEFF[rk_step]; stage 0 also stores Solution_Old (Set_OldSolution,
 * integration_time.cpp:162). U = clip(U_old - Res dt/Vol alpha). */
int rx_explicit_rk(rx_ctx *ctx, int rk_step, double alpha, double *res_rms /* [nVar] or NULL */);

/* Menter SST turbulence solver (SURVEY.md §8 a14 + next-2): CTurbSSTSolver / CTurbSolver
 * (SU2_CFD/src/solver_direct_turbulent.cpp) on the flow context's state. A second context with
 * nVar = 2, U = (k, omega) [N][2], GRAD [N][2][nDim], its own BSR Jacobian (2x2 blocks), ILU / LU-SGS
 * and FGMRES, sharing the flow context's stream (and communicator, which must be attached to the flow
 * context before rx_sst_create). rx_cfg fields read: implicit, lin_tol, lin_iter, lin_prec,
 * relaxation (= RELAXATION_FACTOR_TURB), cfl (= CFL_REDUCTION_TURB). Upload RX_F_U, RX_F_WALLDIST and,
 * before the first Upwind, RX_F_F1/F2/CDKW (or run rx_sst_postprocessing). Reads the flow's V, MU,
 * EDDY, GRAD, STRAIN, DT.
 *   rx_strain_mag        (flow ctx) CReactiveNSVariable::SetStrainMag variable_direct_reactive.cpp:1060-1095,
 *                        called from CReactiveNSSolver::Preprocessing solver_direct_reactive.cpp:4720-4735
 *   rx_sst_preprocessing CTurbSSTSolver::Preprocessing solver_direct_turbulent.cpp:2923-2951 (zero +
 *                        CSolver::SetSolution_Gradient_LS solver_structure.cpp:580-720)
 *   rx_sst_upwind        CTurbSolver::Upwind_Residual :429-543 + CUpwSca_TurbSST::ComputeResidual
 *                        numerics_direct_turbulent.cpp:865-922
 *   rx_sst_viscous       CTurbSolver::Viscous_Residual :545-600 + CAvgGradCorrected_TurbSST :1080-1163
 *   rx_sst_source        CTurbSSTSolver::Source_Residual :3018-3080 + CSourcePieceWise_TurbSST :1183-1256
 *   rx_sst_implicit_euler CTurbSolver::ImplicitEuler_Iteration :615-728 (CSysSolve::Solve)
 *   rx_sst_postprocessing CTurbSSTSolver::Postprocessing :2953-3016 (gradient, SetBlendingFunc
 *                        variable_direct_turbulent.cpp:178-203, mu_t); then writes the flow context's
 *                        TKE, OMEGA, MUT, GRADK, SIGMAK and EDDY (the MANGOTURB coupling getters). */
int rx_sst_create(const rx_mesh_desc *mesh, rx_ctx *flow, const rx_cfg *cfg, rx_ctx **out);
int rx_strain_mag(rx_ctx *flow);
int rx_sst_preprocessing(rx_ctx *turb);
int rx_sst_upwind(rx_ctx *turb);
int rx_sst_viscous(rx_ctx *turb);
int rx_sst_source(rx_ctx *turb);
int rx_sst_implicit_euler(rx_ctx *turb, double *res_rms /* [2] or NULL */, int *lin_iters);
int rx_sst_postprocessing(rx_ctx *turb);

/* Boundary conditions of Space_Integration (SURVEY.md §8 next-3 + a8; integration_structure.cpp:95-193: the weak
 * BCs in marker order, then the strong ones), restricted to the markers of the reference's reactive jet:
 *   RX_BC_INLET       CReactiveEulerSolver::BC_Inlet solver_direct_reactive.cpp:3226-3674 (INLET_TYPE TOTAL_CONDITIONS,
 *                     MASS_FLOW, TEMPERATURE_IMPOSE) / CTurbSSTSolver::BC_Inlet solver_direct_turbulent.cpp:3264-3358
 *   RX_BC_OUTLET      CReactiveEulerSolver::BC_Outlet :3808-4123 / CTurbSSTSolver::BC_Outlet :3360-3450
 *   RX_BC_ISOTHERMAL  CReactiveNSSolver::BC_Isothermal_Wall :5393-5711 (strong no-slip, DeleteValsRowi) /
 *                     CTurbSSTSolver::BC_Isothermal_Wall :3142-3196
 * with the boundary numerics CUpwReactiveAUSM + CAvgGradReactive_Boundary::ComputeResidual
 * (numerics_direct_reactive.cpp:478-648, a8) and CUpwSca_TurbSST + CAvgGrad_TurbSST. Marker m of a mesh bvert is
 * rx_mesh_desc.bvert[2b]. data rows [n_marker][6 + Ns]: inlet (Ttotal | density | T, Ptotal | velocity, flow
 * direction[3], mass fractions[Ns]) as MARKER_INLET / INLET_MASS_FRAC, outlet (back pressure), isothermal (wall
 * temperature). RX_BC_NONE: a marker with no action — MARKER_SYM, which the reactive and turbulent solvers leave to
 * the empty CSolver::BC_Sym_Plane (solver_structure.inl:731-732) / CTurbSolver::BC_Sym_Plane
 * (solver_direct_turbulent.cpp:602-606); its vertices still enter SetTime_Step through rx_mesh_desc. */
/* and, for the reference's turbulent flat plate (Test_Cases/TURBOLENT/TURBOLENT_FLAT_PLATE: MARKER_HEATFLUX,
 * MARKER_EULER):
 *   RX_BC_HEATFLUX    CReactiveNSSolver::BC_HeatFlux_Wall :5717-5911 (strong no-slip, rho E residual -= q A, data
 *                     row a = the wall heat flux) / CTurbSSTSolver::BC_HeatFlux_Wall solver_direct_turbulent.cpp:
 *                     3087-3140 (the isothermal wall's k = 0, omega = 60 mu / (rho beta_1 d^2))
 *   RX_BC_EULER       CReactiveEulerSolver::BC_Euler_Wall :2881-2966 (weak: momentum += (p + 2/3 rho k) n A, the
 *                     Jacobian's momentum rows += dP/dU n A) / CTurbSolver::BC_Euler_Wall (no action, :608-613)  *   RX_BC_SUP_INLET   CReactiveEulerSolver::BC_Supersonic_Inlet :2998-3206 (round 6): the whole ghost state imposed,
 *                     data [kind, T, P, velocity[3], Y[Ns]] (MARKER_SUPERSONIC_INLET + INLET_MASS_FRAC); laminar
 *                     contexts only (rans = 0: the reference hands its viscous numerics no turbulence quantities)
 *   RX_BC_SUP_OUTLET  CReactiveEulerSolver::BC_Supersonic_Outlet :3681-3800 (round 6): ghost = the domain state;
 *                     laminar contexts only
 */
typedef enum {
  RX_BC_NONE = 0, RX_BC_INLET = 1, RX_BC_OUTLET = 2, RX_BC_ISOTHERMAL = 3, RX_BC_HEATFLUX = 4, RX_BC_EULER = 5,
  RX_BC_SUP_INLET = 6, RX_BC_SUP_OUTLET = 7
} rx_bc_kind;
typedef enum { RX_INLET_TOTAL_CONDITIONS = 0, RX_INLET_MASS_FLOW = 1, RX_INLET_TEMPERATURE_IMPOSE = 2 } rx_inlet_kind;
typedef struct {
  int32_t n_marker;
  const int32_t *kind;             /* [n_marker] rx_bc_kind */
  const double *data;              /* [n_marker][6 + Ns] */
  const int64_t *normal_neighbor;  /* [n_bvert] CVertex::GetNormal_Neighbor */
  int32_t inlet_kind;              /* rx_inlet_kind (INLET_TYPE) */
  double tke_inf;                  /* CReactiveEulerSolver Tke_Inf (Tke_FreeStreamND; 0 without SST) */
  double kine_inf, omega_inf;      /* CTurbSSTSolver free-stream k, omega (solver_direct_turbulent.cpp:2740-2752) */
} rx_bc_desc;
int rx_bc_set(rx_ctx *flow, const rx_bc_desc *bc);
int rx_bc_flow(rx_ctx *flow); /* after the interior residual loops; implicit: on the assembled Jacobian */
int rx_bc_sst(rx_ctx *turb);  /* after the SST loops, reads the ghost states of the flow's last rx_bc_flow */

/* Per-phase device timing with HIP events on the context stream (for bench roofline). */
typedef enum {
  RX_K_CONV = 0, RX_K_VISC, RX_K_SOURCE, RX_K_GRAD, RX_K_LIMITER, RX_K_DT, RX_K_SPMV, RX_K_ILU_BUILD,
  RX_K_ILU_APPLY, RX_K_LUSGS, RX_K_KRYLOV, RX_K_UPDATE,
  RX_K_SOLVE,    /* rx_implicit_euler's captured solve: FGMRES + RMS + clipped update (one hipGraph) */
  RX_K_VISC_JAC, /* viscous Jacobian kernel (implicit) */
  RX_K_ASSEMBLE, /* residual + BSR Jacobian assembly */
  RX_K_STRAIN,   /* flow StrainMag */
  RX_K_PRIMITIVE, /* SetPrimitive_Variables */
  RX_K_SST_GRAD, /* SST: least-squares gradient of (k, omega) */
  RX_K_SST_UPW, RX_K_SST_VISC, RX_K_SST_SOURCE, /* SST residual + Jacobian loops */
  RX_K_SST_SYSTEM, /* SST: system build + preconditioner build */
  RX_K_SST_SOLVE,  /* SST: FGMRES + RMS + conservative clipped update */
  RX_K_SST_POST,   /* SST: Postprocessing (gradient, blending, mu_t, flow coupling fields) */
  RX_K_BC,         /* flow boundary conditions (rx_bc_flow) */
  RX_K_SST_BC,     /* SST boundary conditions (rx_bc_sst) */
  RX_K_COUNT
} rx_kernel;
int rx_profile_enable(rx_ctx *ctx, int on);
int rx_profile_read(rx_ctx *ctx, rx_kernel k, double *total_ms, int64_t *launches);

#ifdef __cplusplus
}
#endif
#endif /* RX_H */
