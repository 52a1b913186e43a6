// rx_case.cpp — a reference case from its cfg file (host C++, no GPU): the cfg grammar of
// CConfig::SetConfig_Parsing (Common/src/config_structure.cpp: "KEY= value" lines, '%' comments, lists in
// parentheses separated by ',' / ';') for the keys of this path, the mesh (rx_mesh_read_su2, MESH_FILENAME), the
// library (rx_mech_read, CONFIG_LIB_FILE), the flow and SST rx_cfg, the boundary markers in the mesh's marker
// order, and the free-stream turbulence values CReactiveEulerSolver::SetNondimensionalization derives
// (SU2_CFD/src/solver_direct_reactive.cpp:4534-4590) for DIMENSIONAL cases.
//
// Defaults are CConfig's (config_structure.cpp): TIME_DISCRE_FLOW EULER_IMPLICIT (:1026), LINEAR_SOLVER_PREC LU_SGS
// (:1050), LINEAR_SOLVER_ERROR 1e-5 (:1052), LINEAR_SOLVER_ITER 10 (:1054), CFL_NUMBER 1.25 (:981), PASR_LB 1.0
// (:609), SPATIAL_ORDER_FLOW 2ND_ORDER (:1163), INLET_TYPE TOTAL_CONDITIONS (:884), RK_ALPHA_COEFF one stage of
// 1.0 (:3038-3041), IGNITION NO / 999999 / 1700 K / fuel 0 / oxidizer 2 (:591-603). Keys the path does not
// implement are rejected with RX_ERR_UNSUPPORTED (CFL_ADAPT YES, MGLEVEL > 0, other preconditioners / time schemes
// / marker kinds, non-DIMENSIONAL cases), never silently ignored.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <string>
#include <vector>

#include "../../include/rx_io.h"

struct rx_case {
  rx_mesh* mesh = nullptr;
  rx_mech* mech = nullptr;
  rx_cfg flow{}, sst{};
  std::vector<int32_t> kind;
  std::vector<double> data;
  std::vector<int64_t> pn;
  int32_t inlet_kind = RX_INLET_TOTAL_CONDITIONS;
  double tke_inf = 0.0, omega_inf = 0.0;
  std::vector<double> rk;  // RK_ALPHA_COEFF (RUNGE-KUTTA_EXPLICIT), else empty
  double rho_inf = 0.0, mu_inf = 0.0, T_inf = 0.0, P_inf = 0.0;
};

namespace {

thread_local std::string g_err;

constexpr double kRUngas = 6.02214129e23 * 1.3806488e-23 * 1.0e3;  // J/(kmol K) (physical_chemical_library.hpp:571-579)

std::string trim(const std::string& s) {
  const size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

std::string upper(std::string s) {
  for (char& ch : s) ch = (char)std::toupper((unsigned char)ch);
  return s;
}

// list tokens: strip, strip '(' / ')' at both ends, ';' as ','
std::vector<std::string> list(const std::string& v) {
  std::string t = trim(v);
  const size_t a = t.find_first_not_of("()"), b = t.find_last_not_of("()");
  t = a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
  std::replace(t.begin(), t.end(), ';', ',');
  std::vector<std::string> out;
  size_t p = 0;
  while (p <= t.size()) {
    const size_t q = t.find(',', p);
    const std::string tok = trim(t.substr(p, q == std::string::npos ? std::string::npos : q - p));
    if (!tok.empty()) out.push_back(tok);
    if (q == std::string::npos) break;
    p = q + 1;
  }
  return out;
}

struct Cfg {
  std::map<std::string, std::string> kv;
  bool has(const char* k) const { return kv.count(k) != 0; }
  std::string str(const char* k, const char* d) const {
    auto it = kv.find(k);
    return it == kv.end() ? std::string(d) : it->second;
  }
  double num(const char* k, double d) const {
    auto it = kv.find(k);
    return it == kv.end() ? d : std::strtod(it->second.c_str(), nullptr);
  }
};

bool read_cfg(const char* path, Cfg* c) {
  std::ifstream f(path);
  if (!f) return false;
  std::string line;
  while (std::getline(f, line)) {
    const size_t pc = line.find('%');
    if (pc != std::string::npos) line = line.substr(0, pc);
    line = trim(line);
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    c->kv[upper(trim(line.substr(0, eq)))] = trim(line.substr(eq + 1));
  }
  return true;
}

// MathTools::GetSpline (spline.cpp:62-77) on the library tables, with its range check (:63-64)
bool spline(const rx_mech_desc& d, int prop, int s, double T, double* out) {
  const int nt = d.n_tab;
  const size_t o = ((size_t)prop * d.n_species + s) * nt;
  const double *x = d.tab_x + o, *y = d.tab_y + o, *y2 = d.tab_y2 + o;
  if (T < x[0] || T > x[nt - 1]) return false;
  const double h = x[1] - x[0];
  // the reference's klo is nt at T == x[nt - 1] and reads one past the table (spline.cpp:66-70, undefined
  // behaviour); clamped to the last interval, whose b = 1 gives y[nt - 1], the spline's value there
  const unsigned long klo = std::min((unsigned long)((T - x[0]) / h + 1), (unsigned long)(nt - 1));
  const double a = (x[klo] - T) / h, b = (T - x[klo - 1]) / h;
  *out = a * y[klo - 1] + b * y[klo] + ((a * a * a - a) * y2[klo - 1] + (b * b * b - b) * y2[klo]) * (h * h) / 6.0;
  return true;
}

std::string dir_of(const std::string& p) {
  const size_t k = p.find_last_of('/');
  return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

int fail(rx_case* c, int rc, const std::string& msg) {
  g_err = msg;
  rx_case_destroy(c);
  return rc;
}

}  // namespace

extern "C" {

void rx_cfg_default(rx_cfg* c) {
  if (!c) return;
  *c = rx_cfg{};
  c->mach_inf = 0.01819;
  c->T_ref = c->E_ref = c->R_ref = c->rho_ref = c->t_ref = 1.0;
  c->prandtl_lam = 0.72;
  c->prandtl_turb = 0.9;
  c->lewis_turb = 1.2;
  c->c_mu = 0.09;
  c->pasr_lb = 0.2;
  c->cfl = 1.0;  // the bench CFL pinned against the reference (rx.BENCH_CFL, profiles/r05_calibration_c2.json)
  c->max_delta_time = 1e6;
  c->ref_elem_length = 0.1;
  c->limiter_coeff = 0.5;
  c->lin_tol = 1e-6;
  c->relaxation = 1.0;
  c->implicit = 1;
  c->rans = 1;
  c->lin_iter = 5;
  c->lin_prec = 1;
  c->spatial_order = 0;
  c->clip_temp = 0;
  c->t_min = 200.0;
  c->t_max = 6000.0;
  c->p_ref = c->visc_ref = c->cond_ref = c->vel_ref = c->len_ref = 1.0;
  c->slope_limiter = RX_LIMITER_VENKATAKRISHNAN;
  c->ignition = 0;
  c->fuel_index = 0;
  c->oxidizer_index = 2;
  c->ignition_iter = 999999;
  c->ignition_temp = 1700.0;
  c->lin_solver = RX_LIN_FGMRES;
  c->lin_restart = 10;
}

const char* rx_case_error(void) { return g_err.c_str(); }

int rx_case_read(const char* cfg_path, rx_case** out) {
  if (!cfg_path || !out) return RX_ERR_ARG;
  *out = nullptr;
  Cfg c;
  rx_case* k = new rx_case();
  if (!read_cfg(cfg_path, &c)) return fail(k, RX_ERR_STATE, std::string("cannot read ") + cfg_path);
  const std::string base = dir_of(cfg_path);
  if (upper(c.str("REF_DIMENSIONALIZATION", "DIMENSIONAL")) != "DIMENSIONAL")
    return fail(k, RX_ERR_UNSUPPORTED, "only REF_DIMENSIONALIZATION= DIMENSIONAL");
  if (upper(c.str("CFL_ADAPT", "NO")) != "NO") return fail(k, RX_ERR_UNSUPPORTED, "CFL_ADAPT= YES");
  if (std::atoi(c.str("MGLEVEL", "0").c_str()) != 0) return fail(k, RX_ERR_UNSUPPORTED, "MGLEVEL > 0");
  {
    // the solver and numerics this path builds (VERDICT r03 missing #3): anything else is refused by name
    struct Need {
      const char* key;
      const char* dflt;  // CConfig's default ("" = NO_SOLVER / NO_CONVECTIVE: the reference refuses to run)
      const char* want;
      const char* why;
    };
    static const Need need[] = {
        // Kind_Solver (config_structure.cpp:622, default NO_SOLVER); REACTIVE_NAVIER_STOKES + a turbulence model
        // becomes REACTIVE_RANS (:2872-2874), the solver pair driver_structure.cpp:795-822 builds
        {"PHYSICAL_PROBLEM", "", "REACTIVE_NAVIER_STOKES",
         "the outer iteration on this path is REACTIVE_RANS (or laminar REACTIVE_NAVIER_STOKES)"},
        // :626 (default NONE): SA would build CTurbSASolver (driver_structure.cpp:806-814); NONE (round 6) is the
        // laminar CReactiveNSSolver without TURB_SOL (flow_cfg.rans = 0: rx::Iterate / rx.Iterate without an SST
        // context run the flow's MultiGrid_Iteration alone, iteration_structure.cpp:531-534)
        {"KIND_TURB_MODEL", "NONE", "", "SST (REACTIVE_RANS) or NONE (laminar REACTIVE_NAVIER_STOKES)"},
        // :1147 (default WEIGHTED_LEAST_SQUARES): both methods of Gradient_Map (option_structure.hpp:723-725) are
        // built: rx_grad_lsq / rx_grad_gg (SetPrimitive_Gradient_LS / _GG, solver_direct_reactive.cpp:4717) and the
        // SST's SetSolution_Gradient_LS / _GG (solver_direct_turbulent.cpp:2944, 2963)
        {"NUM_METHOD_GRAD", "WEIGHTED_LEAST_SQUARES", "", "WEIGHTED_LEAST_SQUARES or GREEN_GAUSS"},
        // :1160 (default NO_CONVECTIVE): the reactive driver exits for any upwind scheme but AUSM
        // (driver_structure.cpp:1517-1529)
        {"CONV_NUM_METHOD_FLOW", "", "AUSM", "the reactive solvers implement AUSM only"},
        // :1195: the SST convective term is CUpwSca_TurbSST
        {"CONV_NUM_METHOD_TURB", "SCALAR_UPWIND", "SCALAR_UPWIND", "the SST convection is the scalar upwind"},
        // :1030: the SST SingleGrid_Iteration calls ImplicitEuler_Iteration
        {"TIME_DISCRE_TURB", "EULER_IMPLICIT", "EULER_IMPLICIT", "the SST update is the implicit Euler step"},
        // :979 (default STEADY): dual time stepping is not built
        {"UNSTEADY_SIMULATION", "NO", "NO", "steady (local time stepping) only"},
        {"MATH_PROBLEM", "DIRECT", "DIRECT", "the direct problem only"},
    };
    for (const Need& n : need) {
      std::string v = upper(c.str(n.key, n.dflt));
      if (std::string(n.key) == "NUM_METHOD_GRAD") {
        if (v == "WEIGHTED_LEAST_SQUARES" || v == "GREEN_GAUSS") continue;
        return fail(k, RX_ERR_UNSUPPORTED, "NUM_METHOD_GRAD= " + v + ": " + n.why);
      }
      if (std::string(n.key) == "KIND_TURB_MODEL") {
        if (v == "SST" || v == "NONE") continue;
        return fail(k, RX_ERR_UNSUPPORTED, "KIND_TURB_MODEL= " + v + ": " + n.why);
      }
      if (std::string(n.key) == "UNSTEADY_SIMULATION" && v == "STEADY") v = "NO";
      if (std::string(n.key) == "PHYSICAL_PROBLEM" && v == "REACTIVE_RANS") v = "REACTIVE_NAVIER_STOKES";
      if (v != n.want)
        return fail(k, RX_ERR_UNSUPPORTED,
                    std::string(n.key) + "= " + (v.empty() ? std::string("(unset)") : v) + ": " + n.why);
    }
  }
  if (!c.has("MESH_FILENAME") || !c.has("CONFIG_LIB_FILE"))
    return fail(k, RX_ERR_STATE, "MESH_FILENAME / CONFIG_LIB_FILE missing");
  // mesh + library
  int rc = rx_mesh_read_su2((base + "/" + c.str("MESH_FILENAME", "")).c_str(), &k->mesh);
  if (rc) return fail(k, rc, "mesh " + c.str("MESH_FILENAME", ""));
  rc = rx_mech_read(base.c_str(), c.str("CONFIG_LIB_FILE", "").c_str(), &k->mech);
  if (rc) return fail(k, rc, "library " + c.str("CONFIG_LIB_FILE", ""));
  rx_mech_desc md{};
  rx_mech_describe(k->mech, &md);
  const int ns = md.n_species;
  int32_t nd = 0, nmark = 0;
  int64_t npt = 0, ned = 0, nbv = 0;
  rx_mesh_info(k->mesh, &nd, &npt, &ned, &nbv, &nmark);
  {
    const auto order = list(c.str("SPECIES_ORDER", ""));
    if (!order.empty()) {
      if ((int)order.size() != ns) return fail(k, RX_ERR_STATE, "SPECIES_ORDER does not match the library");
      for (int s = 0; s < ns; ++s)
        if (order[s] != rx_mech_species(k->mech, s))
          return fail(k, RX_ERR_STATE, "SPECIES_ORDER does not match the library");
    }
  }
  // solver knobs
  const std::string tf = upper(c.str("TIME_DISCRE_FLOW", "EULER_IMPLICIT"));
  if (tf != "EULER_IMPLICIT" && tf != "EULER_EXPLICIT" && tf != "RUNGE-KUTTA_EXPLICIT")
    return fail(k, RX_ERR_UNSUPPORTED, "TIME_DISCRE_FLOW= " + tf);
  // :1050 (default LU_SGS), Linear_Solver_Prec_Map (option_structure.hpp:1312-1316). LINELET / SMOOTHER_LINELET: the
  // reactive flow solver never builds the linelets (BuildLineletPreconditioner, matrix_structure.cpp:1837, is called
  // by the SST / SA / compressible solvers' constructors, e.g. solver_direct_turbulent.cpp:2691-2694, not by
  // CReactiveEulerSolver / CReactiveNSSolver), so its Solve reads a null LineletBool (ComputeLineletPreconditioner
  // :2049): the reference cannot run the flow solve with them, and they are refused here
  const std::string pk = upper(c.str("LINEAR_SOLVER_PREC", "LU_SGS"));
  if (pk != "ILU" && pk != "ILU0" && pk != "LU_SGS" && pk != "JACOBI")
    return fail(k, RX_ERR_UNSUPPORTED, "LINEAR_SOLVER_PREC= " + pk);
  const int prec = pk == "LU_SGS" ? RX_PREC_LU_SGS : (pk == "JACOBI" ? RX_PREC_JACOBI : RX_PREC_ILU);
  // :1047 (default FGMRES), Linear_Solver_Map (option_structure.hpp:1249-1260): the branches of CSysSolve::Solve
  // (linear_solvers_structure.cpp:626-708); SMOOTHER_LINELET is refused (see above), CONJUGATE_GRADIENT and
  // the point-inversion methods are not solver kinds of Solve (it does nothing for them)
  const std::string lk = upper(c.str("LINEAR_SOLVER", "FGMRES"));
  static const std::pair<const char*, int> lin_map[] = {
      {"FGMRES", RX_LIN_FGMRES}, {"BCGSTAB", RX_LIN_BCGSTAB}, {"RESTARTED_FGMRES", RX_LIN_RESTARTED_FGMRES},
      {"SMOOTHER_LUSGS", RX_LIN_SMOOTHER_LUSGS}, {"SMOOTHER_JACOBI", RX_LIN_SMOOTHER_JACOBI},
      {"SMOOTHER_ILU0", RX_LIN_SMOOTHER_ILU}};
  int lin_solver = -1;
  for (const auto& e : lin_map)
    if (lk == e.first) lin_solver = e.second;
  if (lin_solver < 0) return fail(k, RX_ERR_UNSUPPORTED, "LINEAR_SOLVER= " + lk);
  const int32_t lin_restart = (int32_t)c.num("LINEAR_SOLVER_RESTART_FREQUENCY", 10);
  const std::string so = upper(c.str("SPATIAL_ORDER_FLOW", "2ND_ORDER"));
  const std::string sl = upper(c.str("SLOPE_LIMITER_FLOW", "VENKATAKRISHNAN"));
  if ((so != "1ST_ORDER" && so != "2ND_ORDER" && so != "2ND_ORDER_LIMITER") ||
      (sl != "VENKATAKRISHNAN" && sl != "BARTH_JESPERSEN"))
    return fail(k, RX_ERR_UNSUPPORTED, "SPATIAL_ORDER_FLOW / SLOPE_LIMITER_FLOW");
  rx_cfg& F = k->flow;
  rx_cfg_default(&F);
  F.cfl = c.num("CFL_NUMBER", 1.25);
  F.max_delta_time = c.num("MAX_DELTA_TIME", 1e6);
  F.prandtl_lam = c.num("PRANDTL_LAM", 0.72);
  F.prandtl_turb = c.num("PRANDTL_TURB", 0.9);
  F.lewis_turb = c.num("LEWIS_TURB", 1.2);
  F.c_mu = c.num("C_MU", 0.09);
  F.pasr_lb = c.num("PASR_LB", 1.0);
  F.lin_tol = c.num("LINEAR_SOLVER_ERROR", 1e-5);
  F.lin_iter = (int32_t)c.num("LINEAR_SOLVER_ITER", 10);
  F.lin_prec = prec;
  F.lin_solver = lin_solver;
  F.lin_restart = lin_restart;
  F.relaxation = c.num("RELAXATION_FACTOR_FLOW", 1.0);
  F.implicit = tf == "EULER_IMPLICIT";
  F.rans = upper(c.str("KIND_TURB_MODEL", "NONE")) == "SST";
  F.spatial_order = so == "1ST_ORDER" ? 0 : (so == "2ND_ORDER" ? 1 : 2);
  F.ref_elem_length = c.num("REF_ELEM_LENGTH", 0.1);
  F.limiter_coeff = c.num("LIMITER_COEFF", 0.5);
  F.slope_limiter = sl == "BARTH_JESPERSEN" ? RX_LIMITER_BARTH_JESPERSEN : RX_LIMITER_VENKATAKRISHNAN;
  F.t_min = c.num("TEMPERATURE_MIN", 200.0);
  F.t_max = c.num("TEMPERATURE_MAX", 6000.0);
  F.clip_temp = upper(c.str("CLIPPING_TEMPRATURE", "NO")) == "YES";
  F.ignition = upper(c.str("IGNITION", "NO")) == "YES";
  F.fuel_index = (int32_t)c.num("FUEL_INDEX", 0);
  F.oxidizer_index = (int32_t)c.num("OXIDIZER_INDEX", 2);
  F.ignition_iter = (int64_t)c.num("IGNITION_ITER", 999999);
  F.ignition_temp = c.num("IGNITION_TEMPERATURE", 1700.0);
  F.grad_method = upper(c.str("NUM_METHOD_GRAD", "WEIGHTED_LEAST_SQUARES")) == "GREEN_GAUSS" ? RX_GRAD_GREEN_GAUSS
                                                                                         : RX_GRAD_WEIGHTED_LEAST_SQUARES;
  if (F.ignition && (F.fuel_index < 0 || F.fuel_index >= ns || F.oxidizer_index < 0 || F.oxidizer_index >= ns))
    return fail(k, RX_ERR_STATE, "FUEL_INDEX / OXIDIZER_INDEX out of the mixture");
  // :1189 (default FIRST_ORDER), :1192 (default VENKATAKRISHNAN): the SST upwind's MUSCL branch
  // (solver_direct_turbulent.cpp:464-510) and CSolver::SetSolution_Limiter's branches (solver_structure.cpp:951-1204:
  // VENKATAKRISHNAN; BARTH_JESPERSEN has no branch there, the limiter stays 2.0; SHARP_EDGES and SOLID_WALL_DISTANCE
  // need geometry the path does not build)
  const std::string sot = upper(c.str("SPATIAL_ORDER_TURB", "1ST_ORDER"));
  const std::string slt = upper(c.str("SLOPE_LIMITER_TURB", "VENKATAKRISHNAN"));
  if ((sot != "1ST_ORDER" && sot != "2ND_ORDER" && sot != "2ND_ORDER_LIMITER") ||
      (slt != "VENKATAKRISHNAN" && slt != "BARTH_JESPERSEN"))
    return fail(k, RX_ERR_UNSUPPORTED, "SPATIAL_ORDER_TURB / SLOPE_LIMITER_TURB");
  rx_cfg& S = k->sst;  // SST context: RELAXATION_FACTOR_TURB -> relaxation, CFL_REDUCTION_TURB -> cfl
  rx_cfg_default(&S);
  S.spatial_order = sot == "1ST_ORDER" ? 0 : (sot == "2ND_ORDER" ? 1 : 2);
  S.slope_limiter = slt == "BARTH_JESPERSEN" ? RX_LIMITER_BARTH_JESPERSEN : RX_LIMITER_VENKATAKRISHNAN;
  S.ref_elem_length = F.ref_elem_length;
  S.limiter_coeff = F.limiter_coeff;
  S.implicit = upper(c.str("TIME_DISCRE_TURB", "EULER_IMPLICIT")) == "EULER_IMPLICIT";
  S.lin_tol = F.lin_tol;
  S.lin_iter = F.lin_iter;
  S.lin_prec = prec;
  S.lin_solver = lin_solver;  // the SST's ImplicitEuler_Iteration calls the same System.Solve with the same config
  S.lin_restart = lin_restart;
  S.relaxation = c.num("RELAXATION_FACTOR_TURB", 1.0);
  S.cfl = c.num("CFL_REDUCTION_TURB", 1.0);
  S.grad_method = F.grad_method;
  if (tf == "RUNGE-KUTTA_EXPLICIT") {
    if (c.has("RK_ALPHA_COEFF"))
      for (const auto& t : list(c.str("RK_ALPHA_COEFF", ""))) k->rk.push_back(std::strtod(t.c_str(), nullptr));
    if (k->rk.empty()) k->rk.push_back(1.0);
  }
  // boundary markers (mesh marker order)
  std::map<std::string, std::vector<double>> inlet, inlet_y, sup_in;
  std::map<std::string, double> outlet, iso, hf;
  std::map<std::string, int> euler, sym, sup_out;
  {
    // MARKER_INLET= (tag, a, b, dir[3]); MARKER_SUPERSONIC_INLET= (tag, T, P, velocity[3]) (config_structure.cpp's
    // Marker_Supersonic_Inlet / Inlet_Temperature / Inlet_Pressure / Inlet_Velocity)
    auto six = [&](const char* key, std::map<std::string, std::vector<double>>& m) {
      const auto t = list(c.str(key, ""));
      for (size_t q = 0; q + 5 < t.size(); q += 6) {
        std::vector<double> v;
        for (size_t r = 1; r < 6; ++r) v.push_back(std::strtod(t[q + r].c_str(), nullptr));
        m[t[q]] = v;
      }
    };
    six("MARKER_INLET", inlet);
    six("MARKER_SUPERSONIC_INLET", sup_in);
    std::string fr = trim(c.str("INLET_MASS_FRAC", ""));
    const size_t a = fr.find_first_not_of("()"), b = fr.find_last_not_of("()");
    fr = a == std::string::npos ? std::string() : fr.substr(a, b - a + 1);
    size_t p = 0;
    while (p < fr.size()) {
      const size_t q = fr.find(';', p);
      const auto seg = list(fr.substr(p, q == std::string::npos ? std::string::npos : q - p));
      if (!seg.empty()) {
        std::vector<double> y;
        for (size_t r = 1; r < seg.size() && (int)y.size() < ns; ++r) y.push_back(std::strtod(seg[r].c_str(), nullptr));
        inlet_y[seg[0]] = y;
      }
      if (q == std::string::npos) break;
      p = q + 1;
    }
    auto pairs = [&](const char* key, std::map<std::string, double>& m) {
      const auto u = list(c.str(key, ""));
      for (size_t q = 0; q + 1 < u.size(); q += 2) m[u[q]] = std::strtod(u[q + 1].c_str(), nullptr);
    };
    pairs("MARKER_OUTLET", outlet);
    pairs("MARKER_ISOTHERMAL", iso);
    pairs("MARKER_HEATFLUX", hf);
    for (const auto& u : list(c.str("MARKER_EULER", ""))) euler[u] = 1;
    for (const auto& u : list(c.str("MARKER_SYM", ""))) sym[u] = 1;
    for (const auto& u : list(c.str("MARKER_SUPERSONIC_OUTLET", ""))) sup_out[u] = 1;
  }
  // the reference's supersonic BCs give the viscous numerics no turbulence quantities: laminar cases only (rx_bc_set)
  if ((!sup_in.empty() || !sup_out.empty()) && F.rans)
    return fail(k, RX_ERR_UNSUPPORTED, "MARKER_SUPERSONIC_INLET / _OUTLET with KIND_TURB_MODEL= SST");
  const int W = 6 + ns;
  std::vector<int32_t> is_wall(nmark, 0);
  k->data.assign((size_t)nmark * W, 0.0);
  for (int m = 0; m < nmark; ++m) {
    const std::string tag = rx_mesh_marker_tag(k->mesh, m);
    double* r = k->data.data() + (size_t)m * W;
    if (inlet.count(tag)) {
      k->kind.push_back(RX_BC_INLET);
      const auto& v = inlet[tag];
      for (int q = 0; q < 5; ++q) r[1 + q] = v[q];
      if (inlet_y.count(tag))
        for (size_t s = 0; s < inlet_y[tag].size(); ++s) r[6 + s] = inlet_y[tag][s];
    } else if (sup_in.count(tag)) {
      k->kind.push_back(RX_BC_SUP_INLET);
      const auto& v = sup_in[tag];
      for (int q = 0; q < 5; ++q) r[1 + q] = v[q];
      if (inlet_y.count(tag))
        for (size_t s = 0; s < inlet_y[tag].size(); ++s) r[6 + s] = inlet_y[tag][s];
    } else if (sup_out.count(tag)) {
      k->kind.push_back(RX_BC_SUP_OUTLET);
    } else if (outlet.count(tag)) {
      k->kind.push_back(RX_BC_OUTLET);
      r[1] = outlet[tag];
    } else if (iso.count(tag)) {
      k->kind.push_back(RX_BC_ISOTHERMAL);
      r[1] = iso[tag];
      is_wall[m] = 1;
    } else if (hf.count(tag)) {
      k->kind.push_back(RX_BC_HEATFLUX);
      r[1] = hf[tag];
      is_wall[m] = 1;
    } else if (euler.count(tag)) {
      k->kind.push_back(RX_BC_EULER);
    } else if (sym.count(tag)) {
      k->kind.push_back(RX_BC_NONE);
    } else {
      return fail(k, RX_ERR_UNSUPPORTED, "marker " + tag + ": boundary kind not supported on this path");
    }
  }
  const std::string it = upper(c.str("INLET_TYPE", "TOTAL_CONDITIONS"));
  if (it == "TOTAL_CONDITIONS") k->inlet_kind = RX_INLET_TOTAL_CONDITIONS;
  else if (it == "MASS_FLOW") k->inlet_kind = RX_INLET_MASS_FLOW;
  else if (it == "TEMPERATURE_IMPOSE") k->inlet_kind = RX_INLET_TEMPERATURE_IMPOSE;
  else return fail(k, RX_ERR_UNSUPPORTED, "INLET_TYPE= " + it);
  rx_mesh_wall_distance(k->mesh, is_wall.data());  // ComputeWall_Distance over the HEAT_FLUX / ISOTHERMAL markers
  const int64_t* nn = rx_mesh_normal_neighbor(k->mesh);
  k->pn.assign(nn, nn + nbv);
  // free stream (SetNondimensionalization, DIMENSIONAL)
  const double T_inf = c.num("FREESTREAM_TEMPERATURE", 288.15), P_inf = c.num("FREESTREAM_PRESSURE", 101325.0);
  std::vector<double> Y;
  for (const auto& t : list(c.str("FREESTREAM_MASS_FRAC", ""))) Y.push_back(std::strtod(t.c_str(), nullptr));
  if ((int)Y.size() != ns) return fail(k, RX_ERR_STATE, "FREESTREAM_MASS_FRAC needs one value per species");
  double rgas = 0.0;
  for (int q = 0; q < ns; ++q) rgas += Y[q] * (kRUngas / md.mmass[q]);  // ComputeRgas
  const double rho_inf = P_inf / (rgas * T_inf);
  double cp = 0.0;
  for (int q = 0; q < ns; ++q) {  // ComputeCP
    double v;
    if (!spline(md, 0, q, T_inf, &v)) return fail(k, RX_ERR_RANGE, "FREESTREAM_TEMPERATURE out of the tables");
    cp += Y[q] * (v / md.mmass[q]);
  }
  const double gamma = cp / (cp - rgas);  // ComputeFrozenGamma
  std::vector<double> vel;
  for (const auto& t : list(c.str("FREESTREAM_VELOCITY", "(1.0, 0.0, 0.0)"))) vel.push_back(std::strtod(t.c_str(), nullptr));
  double mv2 = 0.0;
  for (int d = 0; d < nd && d < (int)vel.size(); ++d) mv2 += vel[d] * vel[d];
  const double mod_v = std::sqrt(mv2);
  // mInfty of the AUSM numerics is config->GetMach() (numerics_direct_reactive.cpp:19). The reactive solver
  // overwrites MACH_NUMBER with the frozen-sound-speed Mach (CConfig::SetMach, solver_direct_reactive.cpp:973) only
  // inside its CONSOLE_OUTPUT_VERBOSITY == VERB_HIGH (the default, config_structure.cpp:1384) && rank == MASTER_NODE
  // block; otherwise MACH_NUMBER (default 0.0, :725) stands. In an MPI run of the reference the other ranks keep
  // MACH_NUMBER even with VERB_HIGH; this path gives every rank the master's value.
  if (upper(c.str("CONSOLE_OUTPUT_VERBOSITY", "HIGH")) == "HIGH")
    F.mach_inf = mod_v / std::sqrt(gamma * rgas * T_inf);
  else
    F.mach_inf = c.num("MACH_NUMBER", 0.0);
  std::vector<double> visc(ns), yom(ns);
  for (int s = 0; s < ns; ++s) {
    if (!spline(md, 3, s, T_inf, &visc[s])) return fail(k, RX_ERR_RANGE, "FREESTREAM_TEMPERATURE out of the tables");
    yom[s] = (Y[s] < 0.0 ? 1.0e-30 : Y[s]) / md.mmass[s];
  }
  double eta = 0.0;
  for (int a = 0; a < ns; ++a) {  // ComputeEta (Wilke), SetPrimVar's expression
    double phi = 0.0;
    for (int b = 0; b < ns; ++b) {
      const double t = 1.0 + std::sqrt(visc[a] / visc[b]) * std::pow(md.mmass[b] / md.mmass[a], 0.25);
      phi += yom[b] / std::sqrt(8.0 * (1.0 + md.mmass[a] / md.mmass[b])) * t * t;
    }
    eta += visc[a] * yom[a] / phi;
  }
  const double inten = c.num("FREESTREAM_TURBULENCEINTENSITY", 0.05);
  k->tke_inf = 3.0 / 2.0 * (mod_v * mod_v * inten * inten);
  k->omega_inf = rho_inf * k->tke_inf / (eta * c.num("FREESTREAM_TURB2LAMVISCRATIO", 10.0));
  k->rho_inf = rho_inf;
  k->mu_inf = eta;
  k->T_inf = T_inf;
  k->P_inf = P_inf;
  *out = k;
  return RX_OK;
}

void rx_case_destroy(rx_case* c) {
  if (!c) return;
  if (c->mesh) rx_mesh_destroy(c->mesh);
  if (c->mech) rx_mech_destroy(c->mech);
  delete c;
}

rx_mesh* rx_case_mesh(rx_case* c) { return c ? c->mesh : nullptr; }
rx_mech* rx_case_mech(rx_case* c) { return c ? c->mech : nullptr; }

int rx_case_cfg(const rx_case* c, rx_cfg* flow, rx_cfg* sst) {
  if (!c) return RX_ERR_ARG;
  if (flow) *flow = c->flow;
  if (sst) *sst = c->sst;
  return RX_OK;
}

int rx_case_bc(const rx_case* c, rx_bc_desc* bc) {
  if (!c || !bc) return RX_ERR_ARG;
  bc->n_marker = (int32_t)c->kind.size();
  bc->kind = c->kind.data();
  bc->data = c->data.data();
  bc->normal_neighbor = c->pn.data();
  bc->inlet_kind = c->inlet_kind;
  bc->tke_inf = c->tke_inf;
  bc->kine_inf = c->tke_inf;
  bc->omega_inf = c->omega_inf;
  return RX_OK;
}

int rx_case_rk(const rx_case* c, int32_t* n_stage, const double** alpha) {
  if (!c || !n_stage) return RX_ERR_ARG;
  *n_stage = (int32_t)c->rk.size();
  if (alpha) *alpha = c->rk.empty() ? nullptr : c->rk.data();
  return RX_OK;
}

int rx_case_free_stream(const rx_case* c, double* rho, double* mu, double* T, double* P) {
  if (!c) return RX_ERR_ARG;
  if (rho) *rho = c->rho_inf;
  if (mu) *mu = c->mu_inf;
  if (T) *T = c->T_inf;
  if (P) *P = c->P_inf;
  return RX_OK;
}

}  // extern "C"
