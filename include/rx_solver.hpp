/* rx_solver.hpp — C++ host mirror of the reference's CReactiveNSSolver phase surface over the C ABI
 * of rx.h (header-only; link with librx.so).
 *
 * The methods keep the reference's names, call order and error behaviour
 * (SU2_CFD/include/solver_reactive.hpp:141-363, 476-554):
 *   Preprocessing residual reset  -> rx_residual_zero            (LinSysRes.SetValZero, Jacobian.SetValZero)
 *   SetPrimitive_Gradient_LS      -> rx_grad_lsq                 (solver_direct_reactive.cpp:4887-5050)
 *   SetPrimitive_Gradient_GG      -> rx_grad_gg                  (solver_direct_reactive.cpp:4784-4880)
 *   SetPrimitive_Limiter          -> rx_limiter_venkat           (:1328-1523; Venkatakrishnan or Barth-Jespersen by rx_cfg.slope_limiter)
 *   SetTime_Step                  -> rx_time_step                (:5057-5298)
 *   Upwind_Residual               -> rx_edge_flux_conv           (:2535-2785)  throws "NaN found in the upwind residual"
 *   Viscous_Residual              -> rx_edge_flux_visc           (:5305-5386)  throws "NaN found in the viscous residual"
 *   Source_Residual               -> rx_cell_source_pasr         (:2792-2874)  throws "NaN found in the source residual"
 *   ExplicitEuler_Iteration       -> rx_explicit_euler           (:2414-2449)
 *   ExplicitRK_Iteration          -> rx_explicit_rk              (:2456-2493)
 *   ImplicitEuler_Iteration       -> rx_implicit_euler           (:2336-2407)
 *   SetStrainMag                  -> rx_strain_mag               (variable_direct_reactive.cpp:1060-1095)
 *   SetPrimitive_Variables        -> rx_set_primitive            (:985-1040)
 *   BC_Inlet / BC_Outlet / BC_Isothermal_Wall (Space_Integration's marker loops,
 *                                 integration_structure.cpp:95-193) -> rx_bc_flow (:3226-4123, 5393-5711)
 * TurbSSTSolver mirrors CTurbSSTSolver / CTurbSolver (SU2_CFD/include/solver_structure.hpp, turbulent
 * classes; SU2_CFD/src/solver_direct_turbulent.cpp):
 *   Preprocessing                 -> rx_sst_preprocessing        (:2923-2951)
 *   Upwind_Residual               -> rx_sst_upwind               (:429-543)
 *   Viscous_Residual              -> rx_sst_viscous              (:545-600)
 *   Source_Residual               -> rx_sst_source               (:3018-3080)
 *   ImplicitEuler_Iteration       -> rx_sst_implicit_euler       (:615-728)
 *   Postprocessing                -> rx_sst_postprocessing       (:2953-3016)
 *   BC_Inlet / BC_Outlet / BC_Isothermal_Wall -> rx_bc_sst       (:3142-3450)
 * Iterate(flow, turb, ext_iter) is CMeanFlowIteration::Iterate for REACTIVE_RANS (iteration_structure.cpp:486-560);
 * IterateFlow(flow, ext_iter) the laminar REACTIVE_NAVIER_STOKES one (no turbulence model, round 6).
 * A spline lookup outside the property tables throws std::out_of_range (MathTools::GetSpline,
 * Common/src/spline.cpp:62-77); any other failure throws std::runtime_error with rx_status_string.
 * Ownership: the solver owns one rx_ctx (device state); host arrays are copied at construction /
 * upload and never retained.
 */
#ifndef RX_SOLVER_HPP
#define RX_SOLVER_HPP

#include <stdexcept>
#include <string>
#include <vector>

#include "rx.h"

namespace rx {

class ReactiveNSSolver {
 public:
  ReactiveNSSolver(const rx_mesh_desc& mesh, const rx_mech_desc& mech, const rx_cfg& cfg, int device = 0)
      : cfg_(cfg) {
    check(rx_ctx_create(&mesh, &mech, &cfg, device, &ctx_), "rx_ctx_create");
    nvar_ = mech.n_species + mesh.n_dim + 2;
  }
  ~ReactiveNSSolver() { rx_ctx_destroy(ctx_); }
  ReactiveNSSolver(const ReactiveNSSolver&) = delete;
  ReactiveNSSolver& operator=(const ReactiveNSSolver&) = delete;

  rx_ctx* context() const { return ctx_; }
  int nVar() const { return nvar_; }
  const rx_cfg& config() const { return cfg_; }

  // ---- node state (Preprocessing output of the reference: primitives, transport, SST fields)
  void Upload(rx_field f, const std::vector<double>& host) {
    check(rx_upload(ctx_, f, host.data(), (int64_t)host.size()), "rx_upload");
  }
  std::vector<double> Download(rx_field f) const {
    int64_t n = 0;
    check(rx_field_size(ctx_, f, &n), "rx_field_size");
    std::vector<double> h((size_t)n);
    check(rx_download(ctx_, f, h.data(), n), "rx_download");
    return h;
  }

  // ---- phases, reference names
  void Preprocessing() { check(rx_residual_zero(ctx_), "Preprocessing"); }
  void SetPrimitive_Gradient_LS() { check(rx_grad_lsq(ctx_), "SetPrimitive_Gradient_LS"); }
  void SetPrimitive_Gradient_GG() { check(rx_grad_gg(ctx_), "SetPrimitive_Gradient_GG"); }
  // CReactiveNSSolver::Preprocessing's choice by NUM_METHOD_GRAD (solver_direct_reactive.cpp:4714-4718)
  void SetPrimitive_Gradient() {
    if (cfg_.grad_method == RX_GRAD_GREEN_GAUSS) SetPrimitive_Gradient_GG();
    else SetPrimitive_Gradient_LS();
  }
  void SetPrimitive_Limiter() { check(rx_limiter_venkat(ctx_), "SetPrimitive_Limiter"); }
  void SetTime_Step() { check(rx_time_step(ctx_), "SetTime_Step"); }
  void SetStrainMag() { check(rx_strain_mag(ctx_), "SetStrainMag"); }
  void Upwind_Residual() { phase(rx_edge_flux_conv(ctx_), "NaN found in the upwind residual"); }
  void Viscous_Residual() { phase(rx_edge_flux_visc(ctx_), "NaN found in the viscous residual"); }
  void Source_Residual() { phase(rx_cell_source_pasr(ctx_), "NaN found in the source residual"); }
  std::vector<double> ExplicitEuler_Iteration() {
    std::vector<double> rms((size_t)nvar_);
    check(rx_explicit_euler(ctx_, rms.data()), "ExplicitEuler_Iteration");
    return rms;
  }
  std::vector<double> ExplicitRK_Iteration(int rk_step, double alpha) {
    std::vector<double> rms((size_t)nvar_);
    check(rx_explicit_rk(ctx_, rk_step, alpha, rms.data()), "ExplicitRK_Iteration");
    return rms;
  }
  std::vector<double> ImplicitEuler_Iteration(int* lin_iters = nullptr) {
    std::vector<double> rms((size_t)nvar_);
    int it = 0;
    check(rx_implicit_euler(ctx_, rms.data(), &it), "ImplicitEuler_Iteration");
    if (lin_iters) *lin_iters = it;
    return rms;
  }
  void Synchronize() { check(rx_sync(ctx_), "rx_sync"); }
  // CReactiveEulerSolver::SetPrimitive_Variables; returns the non-physical point count (syncs)
  long long SetPrimitive_Variables(int ext_iter) {
    int64_t n = 0;
    const int rc = rx_set_primitive(ctx_, ext_iter, &n);
    if (rc == RX_ERR_NONPHYS) throw std::runtime_error("Convergence not achieved for bisection method");
    check(rc, "SetPrimitive_Variables");
    return (long long)n;
  }
  // boundary markers, then Space_Integration's weak + strong BC loops
  void SetBoundaryConditions(const rx_bc_desc& bc) { check(rx_bc_set(ctx_, &bc), "rx_bc_set"); }
  void BC_Apply() { phase(rx_bc_flow(ctx_), "NaN found in the residual of a boundary condition"); }

  // ---- distributed (one rank per GPU): RCCL communicator or host-staged transport (rx.h)
  void CommInit(int nranks, int rank, const void* unique_id128) {
    check(rx_comm_init(ctx_, nranks, rank, unique_id128), "rx_comm_init");
  }
  void CommInitHost(int nranks, int rank, const rx_host_comm& ops) {
    check(rx_comm_init_host(ctx_, nranks, rank, &ops), "rx_comm_init_host");
  }
  void HaloExchange(rx_field f) { check(rx_halo_exchange(ctx_, f), "rx_halo_exchange"); }

 private:
  void phase(int rc, const char* nan_msg) {
    if (rc == RX_OK) rc = rx_sync(ctx_);
    if (rc == RX_ERR_NAN)  // a NaN of the fused AUSM pass is the upwind loop's, whichever call assembled it
      throw std::runtime_error(rx_last_error_phase(ctx_) == RX_ERR_PHASE_UPWIND ? "NaN found in the upwind residual"
                                                                                 : nan_msg);
    check(rc, nan_msg);
  }
  void check(int rc, const char* what) const {
    if (rc == RX_OK) return;
    if (rc == RX_ERR_RANGE) throw std::out_of_range(std::string(what) + ": " + rx_status_string(rc));
    throw std::runtime_error(std::string(what) + ": " + rx_status_string(rc) + " (index " +
                             std::to_string((long long)rx_last_error_index(ctx_)) + ")");
  }
  rx_ctx* ctx_ = nullptr;
  rx_cfg cfg_;
  int nvar_ = 0;
};

// Menter SST solver bound to a flow solver: its own device context (k, omega), on the flow context's
// stream and communicator (attach the flow's communicator first).
class TurbSSTSolver {
 public:
  TurbSSTSolver(const rx_mesh_desc& mesh, ReactiveNSSolver& flow, const rx_cfg& cfg) {
    check(rx_sst_create(&mesh, flow.context(), &cfg, &ctx_), "rx_sst_create");
  }
  ~TurbSSTSolver() { rx_ctx_destroy(ctx_); }
  TurbSSTSolver(const TurbSSTSolver&) = delete;
  TurbSSTSolver& operator=(const TurbSSTSolver&) = delete;

  rx_ctx* context() const { return ctx_; }
  void Upload(rx_field f, const std::vector<double>& host) {
    check(rx_upload(ctx_, f, host.data(), (int64_t)host.size()), "rx_upload");
  }
  std::vector<double> Download(rx_field f) const {
    int64_t n = 0;
    check(rx_field_size(ctx_, f, &n), "rx_field_size");
    std::vector<double> h((size_t)n);
    check(rx_download(ctx_, f, h.data(), n), "rx_download");
    return h;
  }
  void Preprocessing() { check(rx_sst_preprocessing(ctx_), "Preprocessing"); }
  void Upwind_Residual() { check(rx_sst_upwind(ctx_), "Upwind_Residual"); }
  void Viscous_Residual() { check(rx_sst_viscous(ctx_), "Viscous_Residual"); }
  void Source_Residual() { check(rx_sst_source(ctx_), "Source_Residual"); }
  std::vector<double> ImplicitEuler_Iteration(int* lin_iters = nullptr) {
    std::vector<double> rms(2);
    int it = 0;
    check(rx_sst_implicit_euler(ctx_, rms.data(), &it), "ImplicitEuler_Iteration");
    if (lin_iters) *lin_iters = it;
    return rms;
  }
  void Postprocessing() { check(rx_sst_postprocessing(ctx_), "Postprocessing"); }
  void BC_Apply() { check(rx_bc_sst(ctx_), "BC_Apply"); }

 private:
  void check(int rc, const char* what) const {
    if (rc == RX_OK) return;
    throw std::runtime_error(std::string(what) + ": " + rx_status_string(rc));
  }
  rx_ctx* ctx_ = nullptr;
};

// One outer iteration in the reference's order (CMultiGridIntegration::MultiGrid_Iteration with MGLEVEL = 0,
// integration_time.cpp:40-140: MultiGrid_Cycle's pre-smoothing sweep of iRKLimit stages :144-183, each with its own
// Preprocessing and Space_Integration, Set_OldSolution + SetTime_Step at stage 0, then Time_Integration
// (integration_structure.cpp:325-335), and the Preprocessing(Output = true) of the updated solution; then
// CSingleGridIntegration::SingleGrid_Iteration :770-810 for the SST solver). TIME_DISCRE_FLOW follows the flow
// context's cfg: implicit -> ImplicitEuler_Iteration; explicit with rk_alpha empty -> ExplicitEuler_Iteration
// (EULER_EXPLICIT); explicit with rk_alpha = RK_ALPHA_COEFF -> one ExplicitRK_Iteration per stage
// (RUNGE-KUTTA_EXPLICIT). SPATIAL_ORDER_FLOW = 2ND_ORDER_LIMITER (cfg.spatial_order == 2) adds
// SetPrimitive_Limiter to the non-Output Preprocessing (solver_direct_reactive.cpp:4739-4742).
// Returns the flow RMS (of the last stage); turb_rms gets the SST one.
// The flow's MultiGrid_Iteration alone: laminar REACTIVE_NAVIER_STOKES (KIND_TURB_MODEL= NONE, a flow context with
// cfg.rans = 0): CMeanFlowIteration::Iterate runs no turbulence iteration (iteration_structure.cpp:531-534).
inline std::vector<double> IterateFlow(ReactiveNSSolver& flow, int ext_iter,
                                       const std::vector<double>& rk_alpha = std::vector<double>());

inline std::vector<double> Iterate(ReactiveNSSolver& flow, TurbSSTSolver& turb, int ext_iter,
                                   std::vector<double>* turb_rms = nullptr,
                                   const std::vector<double>& rk_alpha = std::vector<double>()) {
  std::vector<double> rms = IterateFlow(flow, ext_iter, rk_alpha);
  turb.Preprocessing();
  turb.Upwind_Residual();
  turb.Viscous_Residual();
  turb.Source_Residual();
  turb.BC_Apply();
  std::vector<double> trms = turb.ImplicitEuler_Iteration();
  turb.Postprocessing();
  if (turb_rms) *turb_rms = trms;
  return rms;
}

inline std::vector<double> IterateFlow(ReactiveNSSolver& flow, int ext_iter, const std::vector<double>& rk_alpha) {
  const rx_cfg& cfg = flow.config();
  auto preprocess = [&](bool output) {
    flow.SetPrimitive_Variables(ext_iter);
    flow.SetPrimitive_Gradient();
    flow.SetStrainMag();
    if (cfg.spatial_order == 2 && !output) flow.SetPrimitive_Limiter();
  };
  const size_t stages = (!cfg.implicit && !rk_alpha.empty()) ? rk_alpha.size() : 1;
  // nothing reads RES / JAC between the loops and the implicit step here: the assembly may fold the system's V / dt
  // (rx_set_system_fold; the system is bitwise the same), cleared again on every exit
  struct Fold {
    rx_ctx* c;
    ~Fold() { if (c) rx_set_system_fold(c, 0); }
  } fold{cfg.implicit ? flow.context() : nullptr};
  if (fold.c && rx_set_system_fold(fold.c, 1) != RX_OK) throw std::runtime_error("rx_set_system_fold");
  std::vector<double> rms;
  for (size_t k = 0; k < stages; ++k) {
    preprocess(false);
    if (k == 0) flow.SetTime_Step();
    flow.Preprocessing();
    flow.Upwind_Residual();
    flow.Viscous_Residual();
    flow.Source_Residual();
    flow.BC_Apply();
    if (cfg.implicit) rms = flow.ImplicitEuler_Iteration();
    else if (rk_alpha.empty()) rms = flow.ExplicitEuler_Iteration();
    else rms = flow.ExplicitRK_Iteration((int)k, rk_alpha[k]);
  }
  preprocess(true);  // MultiGrid_Iteration's Preprocessing(Output = true) on the updated solution (:124-126)
  return rms;
}

}  // namespace rx

#endif
