// rx_driver.cpp — C++ host driver in the reference's CIntegration call order over include/rx_solver.hpp.
// Test harness (tests/test_cpp_driver.py): reads a case directory of raw little-endian arrays
// (<name>.f64 / <name>.i64 / <name>.i32), runs one explicit residual evaluation and one implicit
// iteration (mode 0 / 1), or one whole reference outer iteration with the boundary conditions (mode 2,
// rx::Iterate), writes the results back as <name>.f64.
//
//   rx_driver <case_dir> <mode 0|1|2>
//   rx_driver <cfg_path> 3 <state_dir>: the case read natively from its cfg (include/rx_io.h rx_case_read: mesh,
//                                      library, rx_cfg, markers), the reference's iteration-start records from
//                                      <state_dir>, then one rx::Iterate; results written to <state_dir>.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "rx_io.h"
#include "rx_solver.hpp"

template <typename T>
static std::vector<T> load(const std::string& dir, const std::string& name, const char* ext) {
  std::ifstream f(dir + "/" + name + ext, std::ios::binary | std::ios::ate);
  if (!f) throw std::runtime_error("missing " + name + ext);
  const std::streamsize n = f.tellg();
  f.seekg(0);
  std::vector<T> v((size_t)n / sizeof(T));
  f.read(reinterpret_cast<char*>(v.data()), n);
  return v;
}
static std::vector<double> f64(const std::string& d, const std::string& n) { return load<double>(d, n, ".f64"); }
static std::vector<int64_t> i64(const std::string& d, const std::string& n) { return load<int64_t>(d, n, ".i64"); }
static std::vector<int32_t> i32(const std::string& d, const std::string& n) { return load<int32_t>(d, n, ".i32"); }
static void save(const std::string& dir, const std::string& name, const std::vector<double>& v) {
  std::ofstream f(dir + "/" + name + ".f64", std::ios::binary);
  f.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)(v.size() * sizeof(double)));
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "usage: rx_driver <case_dir> <implicit>\n";
    return 2;
  }
  const std::string d = argv[1];
  const int implicit = std::atoi(argv[2]);
  if (implicit == 3) {
    if (argc < 4) {
      std::cerr << "usage: rx_driver <cfg_path> 3 <state_dir>\n";
      return 2;
    }
    const std::string sd = argv[3];
    rx_case* cs = nullptr;
    if (int rc = rx_case_read(d.c_str(), &cs)) {
      std::printf("rx_case_read: %s (status %d)\n", rx_case_error(), rc);
      return 1;
    }
    try {
      rx_mesh_desc mesh{};
      rx_mech_desc mech{};
      rx_cfg fcfg{}, tcfg{};
      rx_bc_desc bc{};
      rx_mesh_describe(rx_case_mesh(cs), &mesh);
      rx_mech_describe(rx_case_mech(cs), &mech);
      rx_case_cfg(cs, &fcfg, &tcfg);
      rx_case_bc(cs, &bc);
      int32_t nrk = 0;
      const double* ark = nullptr;
      rx_case_rk(cs, &nrk, &ark);
      const std::vector<double> rk(ark, ark + nrk);
      const int nd = mesh.n_dim;
      const int64_t N = mesh.n_point;
      rx::ReactiveNSSolver flow(mesh, mech, fcfg, 0);
      flow.SetBoundaryConditions(bc);
      rx::TurbSSTSolver turb(mesh, flow, tcfg);
      const double* wd = rx_mesh_wall_distance(rx_case_mesh(cs), nullptr);
      auto T = f64(sd, "it_sst0");
      auto tg = f64(sd, "it_sstgrad0");
      std::vector<double> k(N), w(N), gk((size_t)N * nd);
      for (int64_t i = 0; i < N; ++i) {
        k[i] = T[2 * i];
        w[i] = T[2 * i + 1];
        for (int q = 0; q < nd; ++q) gk[(size_t)i * nd + q] = tg[(size_t)i * 2 * nd + q];  // grad k
      }
      flow.Upload(RX_F_V, f64(sd, "it_V0"));
      flow.Upload(RX_F_U, f64(sd, "it_U0"));
      flow.Upload(RX_F_TKE, k);
      flow.Upload(RX_F_OMEGA, w);
      flow.Upload(RX_F_MUT, f64(sd, "it_mut0"));
      flow.Upload(RX_F_SIGMAK, std::vector<double>(N, 0.85));
      flow.Upload(RX_F_GRADK, gk);
      turb.Upload(RX_F_U, T);
      turb.Upload(RX_F_WALLDIST, std::vector<double>(wd, wd + N));
      turb.Upload(RX_F_F1, f64(sd, "it_F1_0"));
      turb.Upload(RX_F_F2, f64(sd, "it_F2_0"));
      turb.Upload(RX_F_CDKW, f64(sd, "it_CDkw0"));
      std::vector<double> trms;
      auto rms = rx::Iterate(flow, turb, 0, &trms, rk);
      flow.Synchronize();
      save(sd, "out_u", flow.Download(RX_F_U));
      save(sd, "out_sst_u", turb.Download(RX_F_U));
      save(sd, "out_rms", rms);
      save(sd, "out_sst_rms", trms);
      std::printf("ok case iterate (%lld points)\n", (long long)N);
    } catch (const std::exception& e) {
      std::printf("exception: %s\n", e.what());
      rx_case_destroy(cs);
      return 1;
    }
    rx_case_destroy(cs);
    return 0;
  }
  try {
    // mesh
    auto edges = i64(d, "edges"), nbr_ptr = i64(d, "nbr_ptr"), nbr = i64(d, "nbr"), bvert = i64(d, "bvertex");
    auto normal = f64(d, "edge_normal"), coord = f64(d, "coord"), vol = f64(d, "volume"), bn = f64(d, "bvertex_normal");
    rx_mesh_desc mesh{};
    mesh.n_dim = 2;
    mesh.n_point = (int64_t)vol.size();
    mesh.n_edge = (int64_t)edges.size() / 2;
    mesh.n_bvert = (int64_t)bvert.size() / 2;
    mesh.edges = edges.data();
    mesh.edge_normal = normal.data();
    mesh.coord = coord.data();
    mesh.volume = vol.data();
    mesh.nbr_ptr = nbr_ptr.data();
    mesh.nbr = nbr.data();
    mesh.bvert = bvert.data();
    mesh.bvert_normal = bn.data();
    // mechanism
    auto mm = f64(d, "mech_mmass"), dv = f64(d, "mech_diff_vol"), sr = f64(d, "mech_stoich_reac"),
         sp = f64(d, "mech_stoich_prod"), er = f64(d, "mech_exp_reac"), ep = f64(d, "mech_exp_prod"), A = f64(d, "mech_A"),
         be = f64(d, "mech_beta"), Ta = f64(d, "mech_Ta"), Ab = f64(d, "mech_A_back"), beb = f64(d, "mech_beta_back"),
         Tab = f64(d, "mech_Ta_back"), tx = f64(d, "mech_tab_x"), ty = f64(d, "mech_tab_y"), ty2 = f64(d, "mech_tab_y2");
    auto rev = i32(d, "mech_reversible"), hb = i32(d, "mech_has_backward");
    rx_mech_desc mech{};
    mech.n_species = (int32_t)mm.size();
    mech.n_reactions = (int32_t)A.size();
    mech.n_tab = (int32_t)(tx.size() / (5 * mm.size()));
    mech.mmass = mm.data();
    mech.diff_vol = dv.data();
    mech.stoich_reac = sr.data();
    mech.stoich_prod = sp.data();
    mech.exp_reac = er.data();
    mech.exp_prod = ep.data();
    mech.A = A.data();
    mech.beta = be.data();
    mech.Ta = Ta.data();
    mech.A_back = Ab.data();
    mech.beta_back = beb.data();
    mech.Ta_back = Tab.data();
    mech.reversible = rev.data();
    mech.has_backward = hb.data();
    mech.tab_x = tx.data();
    mech.tab_y = ty.data();
    mech.tab_y2 = ty2.data();
    // configuration: [mach_inf, Pr_t, Le_t, c_mu, pasr_lb, cfl]
    auto c = f64(d, "cfg");
    rx_cfg cfg{};
    cfg.mach_inf = c[0];
    cfg.T_ref = cfg.E_ref = cfg.R_ref = cfg.rho_ref = cfg.t_ref = 1.0;
    cfg.prandtl_lam = 0.72;
    cfg.prandtl_turb = c[1];
    cfg.lewis_turb = c[2];
    cfg.c_mu = c[3];
    cfg.pasr_lb = c[4];
    cfg.cfl = c[5];
    cfg.max_delta_time = 1e6;
    cfg.ref_elem_length = 0.1;
    cfg.limiter_coeff = 0.5;
    cfg.lin_tol = 1e-6;
    cfg.relaxation = 1.0;
    cfg.implicit = implicit;
    cfg.rans = 1;
    cfg.lin_iter = 5;
    cfg.lin_prec = 1;
    cfg.t_min = 200.0;   // TEMPERATURE_MIN / MAX
    cfg.t_max = 6000.0;
    cfg.p_ref = cfg.visc_ref = cfg.cond_ref = cfg.vel_ref = cfg.len_ref = 1.0;  // DIMENSIONAL

    if (implicit == 2) {
      // CMeanFlowIteration::Iterate from the reference's records (cfg_it: mach, Pr_lam, Pr_t, Le_t, C_mu, PaSR_LB,
      // CFL, max dt, lin tol, lin iter, relax flow, T_min, T_max, relax turb, CFL reduction turb)
      auto ci = f64(d, "cfg_it");
      cfg.mach_inf = ci[0];
      cfg.prandtl_lam = ci[1];
      cfg.prandtl_turb = ci[2];
      cfg.lewis_turb = ci[3];
      cfg.c_mu = ci[4];
      cfg.pasr_lb = ci[5];
      cfg.cfl = ci[6];
      cfg.max_delta_time = ci[7];
      cfg.lin_tol = ci[8];
      cfg.lin_iter = (int32_t)ci[9];
      cfg.relaxation = ci[10];
      cfg.t_min = ci[11];
      cfg.t_max = ci[12];
      // cfg_scheme (optional): [flow implicit, SST lin_prec]; cfg_rk (optional): RK_ALPHA_COEFF
      std::vector<double> scheme{1.0, 1.0}, rk;
      if (std::ifstream(d + "/cfg_scheme.f64").good()) scheme = f64(d, "cfg_scheme");
      if (std::ifstream(d + "/cfg_rk.f64").good()) rk = f64(d, "cfg_rk");
      cfg.implicit = (int32_t)scheme[0];
      if (std::ifstream(d + "/cfg_laminar.f64").good()) cfg.rans = 0;
      rx::ReactiveNSSolver flow(mesh, mech, cfg, 0);
      auto pn = i64(d, "bvertex_pn");
      auto kind = i32(d, "bc_kind");
      auto bdata = f64(d, "bc_data"), bsc = f64(d, "bc_scalars");
      rx_bc_desc bc{};
      bc.n_marker = (int32_t)kind.size();
      bc.kind = kind.data();
      bc.data = bdata.data();
      bc.normal_neighbor = pn.data();
      bc.inlet_kind = (int32_t)bsc[0];
      bc.tke_inf = bsc[1];
      bc.kine_inf = bsc[2];
      bc.omega_inf = bsc[3];
      flow.SetBoundaryConditions(bc);
      if (std::ifstream(d + "/cfg_laminar.f64").good()) {
        // laminar REACTIVE_NAVIER_STOKES (round 6): no SST context, rx::IterateFlow
        flow.Upload(RX_F_V, f64(d, "it_V0"));
        flow.Upload(RX_F_U, f64(d, "it_U0"));
        auto rms = rx::IterateFlow(flow, 0, rk);
        flow.Synchronize();
        save(d, "out_u", flow.Download(RX_F_U));
        save(d, "out_rms", rms);
        std::printf("ok iterate (laminar)\n");
        return 0;
      }
      rx_cfg tcfg = cfg;
      tcfg.implicit = 1;
      tcfg.lin_prec = (int32_t)scheme[1];
      tcfg.relaxation = ci[13];
      tcfg.cfl = ci[14];
      rx::TurbSSTSolver turb(mesh, flow, tcfg);
      auto T = f64(d, "it_sst0");
      std::vector<double> k(T.size() / 2), w(T.size() / 2), gk(T.size());
      auto tg = f64(d, "it_sstgrad0");
      for (size_t i = 0; i < k.size(); ++i) {
        k[i] = T[2 * i];
        w[i] = T[2 * i + 1];
        gk[2 * i] = tg[4 * i];
        gk[2 * i + 1] = tg[4 * i + 1];
      }
      flow.Upload(RX_F_V, f64(d, "it_V0"));
      flow.Upload(RX_F_U, f64(d, "it_U0"));
      flow.Upload(RX_F_TKE, k);
      flow.Upload(RX_F_OMEGA, w);
      flow.Upload(RX_F_MUT, f64(d, "it_mut0"));
      flow.Upload(RX_F_SIGMAK, std::vector<double>(k.size(), 0.85));
      flow.Upload(RX_F_GRADK, gk);
      turb.Upload(RX_F_U, T);
      turb.Upload(RX_F_WALLDIST, f64(d, "wall_distance"));
      turb.Upload(RX_F_F1, f64(d, "it_F1_0"));
      turb.Upload(RX_F_F2, f64(d, "it_F2_0"));
      turb.Upload(RX_F_CDKW, f64(d, "it_CDkw0"));
      std::vector<double> trms;
      auto rms = rx::Iterate(flow, turb, 0, &trms, rk);
      flow.Synchronize();
      save(d, "out_u", flow.Download(RX_F_U));
      save(d, "out_sst_u", turb.Download(RX_F_U));
      save(d, "out_rms", rms);
      save(d, "out_sst_rms", trms);
      std::printf("ok iterate\n");
      return 0;
    }

    rx::ReactiveNSSolver solver(mesh, mech, cfg, 0);
    const struct {
      const char* name;
      rx_field f;
    } state[] = {{"U", RX_F_U},          {"V", RX_F_V},         {"dPdU", RX_F_DPDU},   {"dTdU", RX_F_DTDU},
                 {"mu", RX_F_MU},        {"kappa", RX_F_KAPPA}, {"Dij", RX_F_DIJ},     {"grad_prim", RX_F_GRAD},
                 {"turb_k", RX_F_TKE},   {"turb_omega", RX_F_OMEGA}, {"mu_t", RX_F_MUT}, {"sigma_k", RX_F_SIGMAK},
                 {"grad_k", RX_F_GRADK}, {"eddy_visc_flow", RX_F_EDDY}};
    for (const auto& s : state) solver.Upload(s.f, f64(d, s.name));

    // CReactiveNSSolver::Preprocessing tail (StrainMag from the gradient, solver_direct_reactive.cpp:4720-4735),
    // CIntegration::Space_Integration order (integration_structure.cpp:72-193), then Time_Integration
    solver.SetStrainMag();
    solver.SetTime_Step();
    solver.Preprocessing();
    solver.Upwind_Residual();
    solver.Viscous_Residual();
    solver.Source_Residual();
    save(d, "out_res", solver.Download(RX_F_RES));
    save(d, "out_dt", solver.Download(RX_F_DT));
    std::vector<double> rms;
    int lin_iters = 0;
    if (implicit) rms = solver.ImplicitEuler_Iteration(&lin_iters);
    else rms = solver.ExplicitEuler_Iteration();
    save(d, "out_u", solver.Download(RX_F_U));
    save(d, "out_rms", rms);
    std::printf("ok lin_iters=%d\n", lin_iters);
    if (implicit) {
      // CSingleGridIntegration::SingleGrid_Iteration for TURB_SOL (integration_time.cpp:777-810)
      rx_cfg tcfg = cfg;
      tcfg.relaxation = 1.0;  // RELAXATION_FACTOR_TURB
      tcfg.cfl = 1.0;         // CFL_REDUCTION_TURB
      auto wall = f64(d, "wall_distance");
      mesh.n_bvert = (int64_t)bvert.size() / 2;
      rx::TurbSSTSolver turb(mesh, solver, tcfg);
      turb.Upload(RX_F_U, f64(d, "sst_sol"));
      turb.Upload(RX_F_WALLDIST, wall);
      turb.Upload(RX_F_F1, f64(d, "sst_F1"));
      turb.Upload(RX_F_F2, f64(d, "sst_F2"));
      turb.Upload(RX_F_CDKW, f64(d, "sst_CDkw"));
      turb.Preprocessing();
      turb.Upwind_Residual();
      turb.Viscous_Residual();
      turb.Source_Residual();
      int tit = 0;
      auto trms = turb.ImplicitEuler_Iteration(&tit);
      turb.Postprocessing();
      save(d, "out_sst_u", turb.Download(RX_F_U));
      save(d, "out_sst_rms", trms);
      save(d, "out_sst_mut", turb.Download(RX_F_MUT));
      std::printf("ok sst lin_iters=%d\n", tit);
    }
  } catch (const std::exception& e) {
    std::printf("exception: %s\n", e.what());
    return 1;
  }
  return 0;
}
