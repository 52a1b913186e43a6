// Golden-vector harness: TEST INFRASTRUCTURE ONLY.
//
// Links against the reference SU2 reactive fork compiled from /root/reference by
// oracle/ref_build.mk (objects in oracle/_ref/, git-ignored). It builds the reference's own
// CFluidDriver on a cfg + mesh, overwrites the flow/turbulence solution with a supplied state,
// runs the reference's own preprocessing and then calls the reference's own operators
// (CNumerics::ComputeResidual / ComputeChemistry, CSolver loops, CSysMatrix/CSysSolve) and dumps
// their inputs and outputs as raw little-endian arrays + a manifest. oracle/make_golden.py packs
// them into tests/golden/*.npz. Nothing in here ships or is measured.
//
// Reference call sites reproduced (file:line relative to /root/reference):
//   per-edge AUSM setters/call       SU2_CFD/src/solver_direct_reactive.cpp:2546-2552,2731-2743
//   per-edge viscous setters/call    SU2_CFD/src/solver_direct_reactive.cpp:5312-5355
//   per-cell chemistry setters/call  SU2_CFD/src/solver_direct_reactive.cpp:2803-2817
//   ImplicitEuler system build       SU2_CFD/src/solver_direct_reactive.cpp:2350-2390
#include "../../SU2_CFD/include/driver_structure.hpp"
#include "../../SU2_CFD/include/solver_reactive.hpp"
#include "../../SU2_CFD/include/numerics_reactive.hpp"
#include "../../SU2_CFD/include/output_structure.hpp"

#include <chrono>
#include <cstdio>
#include <cstdint>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

std::string g_out;
std::ofstream g_manifest;

template <typename T>
void dump(const std::string& name, const std::vector<T>& v, const std::vector<long>& shape, const char* dtype) {
  std::string path = g_out + "/" + name + ".bin";
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) { std::perror(path.c_str()); std::exit(3); }
  if (!v.empty()) std::fwrite(v.data(), sizeof(T), v.size(), f);
  std::fclose(f);
  g_manifest << name << " " << dtype;
  for (long s : shape) g_manifest << " " << s;
  g_manifest << "\n";
  g_manifest.flush();
}
void dumpd(const std::string& n, const std::vector<double>& v, const std::vector<long>& s) { dump(n, v, s, "f8"); }
void dumpi(const std::string& n, const std::vector<int64_t>& v, const std::vector<long>& s) { dump(n, v, s, "i8"); }

// Expose the protected containers of the reference driver.
class HarnessDriver : public CFluidDriver {
 public:
  HarnessDriver(char* cfg, unsigned short nZone, unsigned short nDim, SU2_Comm comm)
      : CFluidDriver(cfg, nZone, nDim, comm) {}
  CGeometry* geo() { return geometry_container[ZONE_0][MESH_0]; }
  CSolver** sol() { return solver_container[ZONE_0][MESH_0]; }
  CNumerics* num(unsigned short s, unsigned short t) { return numerics_container[ZONE_0][MESH_0][s][t]; }
  CConfig* cfg() { return config_container[ZONE_0]; }
  CIntegration* integ(unsigned short s) { return integration_container[ZONE_0][s]; }
  CNumerics** nums(unsigned short s) { return numerics_container[ZONE_0][MESH_0][s]; }
  // one outer iteration of the reference (CMeanFlowIteration::Iterate, iteration_structure.cpp:486-560)
  void iterate() {
    iteration_container[ZONE_0]->Iterate(output, integration_container, geometry_container, solver_container,
                                         numerics_container, config_container, surface_movement, grid_movement,
                                         FFDBox, ZONE_0);
  }
};

// sigma_k is a protected CNumerics member; Set_Sigmak has no return statement (UB,
// SU2_CFD/include/numerics_structure.hpp:525-527), so set it through a derived accessor instead.
struct SigmaSetter : public CNumerics {
  static void set(CNumerics* n, double s) { static_cast<SigmaSetter*>(n)->sigma_k = s; }
};

double** alloc2(int n) {
  double** a = new double*[n];
  for (int i = 0; i < n; ++i) a[i] = new double[n]();
  return a;
}

// CTurbSSTSolver's kine_Inf / omega_Inf are private: recomputed with the constructor's own expressions
// (solver_direct_turbulent.cpp:2740-2752).
void sst_inf(CConfig* config, unsigned short nDim, double& kine, double& omega) {
  su2double rhoInf = config->GetDensity_FreeStreamND();
  su2double* VelInf = config->GetVelocity_FreeStreamND();
  su2double muLamInf = config->GetViscosity_FreeStreamND();
  su2double Intensity = config->GetTurbulenceIntensity_FreeStream();
  su2double viscRatio = config->GetTurb2LamViscRatio_FreeStream();
  su2double VelMag = 0;
  for (unsigned short iDim = 0; iDim < nDim; iDim++) VelMag += VelInf[iDim] * VelInf[iDim];
  VelMag = sqrt(VelMag);
  kine = 3.0 / 2.0 * (VelMag * VelMag * Intensity * Intensity);
  omega = rhoInf * kine / (muLamInf * viscRatio);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: harness <cfg> <state.txt> <outdir> [--bsr]\n");
    return 2;
  }
  char cfgname[MAX_STRING_SIZE];
  std::strcpy(cfgname, argv[1]);
  std::string state_file = argv[2];
  g_out = argv[3];
  bool do_bsr = (argc > 4 && std::string(argv[4]) == "--bsr");
  // --bc: boundary conditions of one Space_Integration (flow + SST); --iters K: K reference outer iterations
  const bool do_bc = (argc > 4 && std::string(argv[4]) == "--bc");
  const int n_iters = (argc > 5 && std::string(argv[4]) == "--iters") ? std::atoi(argv[5]) : 0;
  g_manifest.open(g_out + "/manifest.txt");

  SU2_Comm comm(0);
  CConfig* c0 = new CConfig(cfgname, SU2_CFD);
  unsigned short nZone = CConfig::GetnZone(c0->GetMesh_FileName(), c0->GetMesh_FileFormat(), c0);
  unsigned short nDim = CConfig::GetnDim(c0->GetMesh_FileName(), c0->GetMesh_FileFormat());
  delete c0;
  HarnessDriver drv(cfgname, nZone, nDim, comm);

  CGeometry* geo = drv.geo();
  CSolver** sc = drv.sol();
  CConfig* cfg = drv.cfg();
  CSolver* flow = sc[FLOW_SOL];
  CSolver* turb = sc[TURB_SOL];
  const bool rans = (turb != NULL);

  const unsigned long nPoint = geo->GetnPoint();
  const unsigned long nEdge = geo->GetnEdge();
  const unsigned short nVar = flow->GetnVar();
  const unsigned short nPrimVar = flow->GetnPrimVar();
  const unsigned short nPrimVarGrad = flow->GetnPrimVarGrad();
  const unsigned short nSpecies = nVar - nDim - 2;
  const unsigned short nPrimVarLim = nDim + 2;

  // ---- load the state: lines "global_index U[0..nVar) [k omega]"
  {
    std::map<unsigned long, unsigned long> g2l;
    for (unsigned long i = 0; i < nPoint; ++i) g2l[geo->node[i]->GetGlobalIndex()] = i;
    std::ifstream sf(state_file);
    std::string line;
    unsigned long nset = 0;
    while (std::getline(sf, line)) {
      if (line.empty()) continue;
      std::istringstream is(line);
      unsigned long gidx;
      is >> gidx;
      auto it = g2l.find(gidx);
      if (it == g2l.end()) continue;
      unsigned long i = it->second;
      for (unsigned short v = 0; v < nVar; ++v) {
        double u;
        is >> u;
        flow->node[i]->SetSolution(v, u);
        flow->node[i]->SetSolution_Old(v, u);
      }
      if (rans) {
        double k, w;
        is >> k >> w;
        turb->node[i]->SetSolution(0, k);
        turb->node[i]->SetSolution(1, w);
        turb->node[i]->SetSolution_Old(0, k);
        turb->node[i]->SetSolution_Old(1, w);
      }
      ++nset;
    }
    if (nset != nPoint) {
      std::fprintf(stderr, "state covers %lu of %lu points\n", nset, nPoint);
      return 4;
    }
  }

  // ---- the reference's own preprocessing (flow, then turbulence mu_t, then flow again)
  flow->Preprocessing(geo, sc, cfg, MESH_0, NO_RK_ITER, RUNTIME_FLOW_SYS, false);
  if (rans) {
    turb->Postprocessing(geo, sc, cfg, MESH_0);
    flow->Preprocessing(geo, sc, cfg, MESH_0, NO_RK_ITER, RUNTIME_FLOW_SYS, false);
    turb->Preprocessing(geo, sc, cfg, MESH_0, NO_RK_ITER, RUNTIME_TURB_SYS, false);
    turb->Postprocessing(geo, sc, cfg, MESH_0);
  }

  const bool implicit = (cfg->GetKind_TimeIntScheme_Flow() == EULER_IMPLICIT);

  // ---- geometry
  {
    std::vector<double> coord(nPoint * nDim), vol(nPoint);
    std::vector<int64_t> gidx(nPoint), nb_ptr(nPoint + 1, 0), nb;
    for (unsigned long i = 0; i < nPoint; ++i) {
      for (unsigned short d = 0; d < nDim; ++d) coord[i * nDim + d] = geo->node[i]->GetCoord(d);
      vol[i] = geo->node[i]->GetVolume();
      gidx[i] = geo->node[i]->GetGlobalIndex();
      for (unsigned short k = 0; k < geo->node[i]->GetnPoint(); ++k) nb.push_back(geo->node[i]->GetPoint(k));
      nb_ptr[i + 1] = nb.size();
    }
    dumpd("coord", coord, {(long)nPoint, nDim});
    dumpd("volume", vol, {(long)nPoint});
    dumpi("global_index", gidx, {(long)nPoint});
    dumpi("nbr_ptr", nb_ptr, {(long)nPoint + 1});
    dumpi("nbr", nb, {(long)nb.size()});
    std::vector<int64_t> edges(nEdge * 2);
    std::vector<double> normal(nEdge * nDim);
    for (unsigned long e = 0; e < nEdge; ++e) {
      edges[2 * e] = geo->edge[e]->GetNode(0);
      edges[2 * e + 1] = geo->edge[e]->GetNode(1);
      su2double* n = geo->edge[e]->GetNormal();
      for (unsigned short d = 0; d < nDim; ++d) normal[e * nDim + d] = n[d];
    }
    dumpi("edges", edges, {(long)nEdge, 2});
    dumpd("edge_normal", normal, {(long)nEdge, nDim});
    // boundary vertices: marker id, node, dual-face normal (geometry_structure.cpp SetBoundControlVolume)
    std::vector<int64_t> bv;
    std::vector<double> bn;
    for (unsigned short m = 0; m < geo->GetnMarker(); ++m)
      for (unsigned long v = 0; v < geo->GetnVertex(m); ++v) {
        bv.push_back(m);
        bv.push_back(geo->vertex[m][v]->GetNode());
        bv.push_back(cfg->GetMarker_All_KindBC(m));
        su2double* n = geo->vertex[m][v]->GetNormal();
        for (unsigned short d = 0; d < nDim; ++d) bn.push_back(n[d]);
      }
    dumpi("bvertex", bv, {(long)bv.size() / 3, 3});
    dumpd("bvertex_normal", bn, {(long)bn.size() / nDim, nDim});
    std::vector<double> wall(nPoint);
    for (unsigned long i = 0; i < nPoint; ++i) wall[i] = geo->node[i]->GetWall_Distance();
    dumpd("wall_distance", wall, {(long)nPoint});
  }

  // ---- node state after the reference's preprocessing
  {
    std::vector<double> U(nPoint * nVar), V(nPoint * nPrimVar), dPdU(nPoint * nVar), dTdU(nPoint * nVar);
    std::vector<double> mu(nPoint), kap(nPoint), cp(nPoint), Dij(nPoint * nSpecies * nSpecies);
    std::vector<double> grad(nPoint * nPrimVarGrad * nDim), lim(nPoint * nPrimVarLim);
    for (unsigned long i = 0; i < nPoint; ++i) {
      CVariable* n = flow->node[i];
      for (unsigned short v = 0; v < nVar; ++v) {
        U[i * nVar + v] = n->GetSolution(v);
        dPdU[i * nVar + v] = n->GetdPdU()[v];
        dTdU[i * nVar + v] = n->GetdTdU()[v];
      }
      for (unsigned short v = 0; v < nPrimVar; ++v) V[i * nPrimVar + v] = n->GetPrimitive(v);
      mu[i] = n->GetLaminarViscosity();
      kap[i] = n->GetThermalConductivity();
      cp[i] = n->GetSpecificHeatCp();
      double* d = n->GetDiffusionCoeff();
      for (int k = 0; k < nSpecies * nSpecies; ++k) Dij[i * nSpecies * nSpecies + k] = d[k];
      su2double** g = n->GetGradient_Primitive();
      for (unsigned short v = 0; v < nPrimVarGrad; ++v)
        for (unsigned short dd = 0; dd < nDim; ++dd) grad[(i * nPrimVarGrad + v) * nDim + dd] = g[v][dd];
      for (unsigned short v = 0; v < nPrimVarLim; ++v) lim[i * nPrimVarLim + v] = n->GetLimiter_Primitive(v);
    }
    dumpd("U", U, {(long)nPoint, nVar});
    dumpd("V", V, {(long)nPoint, nPrimVar});
    dumpd("dPdU", dPdU, {(long)nPoint, nVar});
    dumpd("dTdU", dTdU, {(long)nPoint, nVar});
    dumpd("mu", mu, {(long)nPoint});
    dumpd("kappa", kap, {(long)nPoint});
    dumpd("cp", cp, {(long)nPoint});
    dumpd("Dij", Dij, {(long)nPoint, nSpecies, nSpecies});
    dumpd("grad_prim", grad, {(long)nPoint, nPrimVarGrad, nDim});
    dumpd("limiter", lim, {(long)nPoint, nPrimVarLim});
    if (rans) {
      std::vector<double> tk(nPoint), tw(nPoint), mut(nPoint), sk(nPoint), gk(nPoint * nDim);
      for (unsigned long i = 0; i < nPoint; ++i) {
        tk[i] = turb->node[i]->GetSolution(0);
        tw[i] = turb->node[i]->GetSolution(1);
        mut[i] = turb->node[i]->GetmuT();
        sk[i] = turb->node[i]->Get_Sigmak();
        for (unsigned short d = 0; d < nDim; ++d) gk[i * nDim + d] = turb->node[i]->GetGradient()[0][d];
      }
      dumpd("turb_k", tk, {(long)nPoint});
      dumpd("turb_omega", tw, {(long)nPoint});
      dumpd("mu_t", mut, {(long)nPoint});
      dumpd("sigma_k", sk, {(long)nPoint});
      dumpd("grad_k", gk, {(long)nPoint, nDim});
      std::vector<double> ev(nPoint);
      for (unsigned long i = 0; i < nPoint; ++i) ev[i] = flow->node[i]->GetEddyViscosity();
      dumpd("eddy_visc_flow", ev, {(long)nPoint});
    }
  }

  // ---- boundary conditions (--bc) and whole reference iterations (--iters K)
  if (do_bc || n_iters > 0) {
    const unsigned short nMarker = geo->GetnMarker();
    const unsigned short kind_solver = cfg->GetKind_Solver();
    // per-vertex normal neighbour (CVertex::GetNormal_Neighbor), in bvertex order
    std::vector<int64_t> pn;
    for (unsigned short m = 0; m < nMarker; ++m)
      for (unsigned long v = 0; v < geo->GetnVertex(m); ++v) pn.push_back(geo->vertex[m][v]->GetNormal_Neighbor());
    dumpi("bvertex_pn", pn, {(long)pn.size()});
    // marker data rows [kind, a, b, dir0, dir1, dir2, Y_1..Y_Ns]: inlet (Ttotal, Ptotal, flow dir, mass fractions),
    // outlet (pressure), isothermal (wall temperature), heat flux (wall heat flux)
    const int W = 6 + nSpecies;
    std::vector<double> md((size_t)nMarker * W, 0.0);
    for (unsigned short m = 0; m < nMarker; ++m) {
      std::string tag = cfg->GetMarker_All_TagBound(m);
      const unsigned short kind = cfg->GetMarker_All_KindBC(m);
      double* r = md.data() + (size_t)m * W;
      r[0] = kind;
      if (kind == INLET_FLOW) {
        r[1] = cfg->GetInlet_Ttotal(tag);
        r[2] = cfg->GetInlet_Ptotal(tag);
        su2double* fd = cfg->GetInlet_FlowDir(tag);
        for (unsigned short d = 0; d < nDim; ++d) r[3 + d] = fd[d];
        const su2double* ys = cfg->GetInlet_MassFrac(tag);
        for (unsigned short s = 0; s < nSpecies; ++s) r[6 + s] = ys[s];
      } else if (kind == OUTLET_FLOW) {
        r[1] = cfg->GetOutlet_Pressure(tag);
      } else if (kind == ISOTHERMAL) {
        r[1] = cfg->GetIsothermal_Temperature(tag);
      } else if (kind == HEAT_FLUX) {
        r[1] = cfg->GetWall_HeatFlux(tag);
      } else if (kind == SUPERSONIC_INLET) {  // (T, P, velocity vector, mass fractions)
        r[1] = cfg->GetInlet_Temperature(tag);
        r[2] = cfg->GetInlet_Pressure(tag);
        su2double* vel = cfg->GetInlet_Velocity(tag);
        for (unsigned short d = 0; d < nDim; ++d) r[3 + d] = vel[d];
        const su2double* ys = cfg->GetInlet_MassFrac(tag);
        for (unsigned short s = 0; s < nSpecies; ++s) r[6 + s] = ys[s];
      }
    }
    dumpd("bc_marker", md, {(long)nMarker, W});
    double kine_inf = 0.0, omega_inf = 0.0;
    if (rans) sst_inf(cfg, nDim, kine_inf, omega_inf);
    std::vector<double> bp = {(double)cfg->GetKind_Inlet(), flow->GetTke_Inf(), kine_inf, omega_inf,
                              rans ? turb->GetConstants()[4] : 0.0,
                              cfg->GetPressure_Ref(), cfg->GetVelocity_Ref(), cfg->GetTemperature_Ref(),
                              cfg->GetEnergy_Ref(), cfg->GetGas_Constant_Ref(), cfg->GetDensity_Ref(),
                              (double)INLET_FLOW, (double)OUTLET_FLOW, (double)ISOTHERMAL, (double)HEAT_FLUX,
                              (double)TOTAL_CONDITIONS, (double)MASS_FLOW, (double)TEMPERATURE_IMPOSE,
                              cfg->GetCFL(MESH_0), cfg->GetLinear_Solver_Error(), (double)cfg->GetLinear_Solver_Iter(),
                              (double)cfg->GetKind_Linear_Solver_Prec(), cfg->GetRelaxation_Factor_Flow(),
                              cfg->GetRelaxation_Factor_Turb(), cfg->GetCFLRedCoeff_Turb(), cfg->GetMax_DeltaTime(),
                              (double)SYMMETRY_PLANE, (double)EULER_WALL, (double)SUPERSONIC_INLET,
                              (double)SUPERSONIC_OUTLET};
    dumpd("bc_params", bp, {(long)bp.size()});
    // the cfg values the other modes dump with their operators, same layouts
    dumpd("mach_inf", std::vector<double>{cfg->GetMach()}, {1});
    dumpd("visc_params", std::vector<double>{cfg->GetPrandtl_Lam(), cfg->GetPrandtl_Turb(), cfg->GetLewis_Turb()}, {3});
    dumpd("src_params", std::vector<double>{cfg->Get_Cmu(), cfg->Get_PaSR_LB(), cfg->GetDensity_Ref(), cfg->GetTime_Ref(),
                                            cfg->GetTemperature_Ref()}, {5});
    dumpd("dt_params", std::vector<double>{cfg->GetCFL(MESH_0), cfg->GetMax_DeltaTime(), cfg->GetPrandtl_Lam(),
                                           cfg->GetPrandtl_Turb()}, {4});
    dumpd("limiter_params", std::vector<double>{cfg->GetRefElemLength(), cfg->GetLimiterCoeff()}, {2});
    dumpd("p2v_params", std::vector<double>{0.0, cfg->GetTemperatureMin(), cfg->GetTemperatureMax(),
                                            cfg->GetTemperature_Ref(), cfg->GetEnergy_Ref(), cfg->GetGas_Constant_Ref(),
                                            cfg->GetPressure_Ref(), cfg->GetViscosity_Ref(), cfg->GetConductivity_Ref(),
                                            cfg->GetVelocity_Ref(), cfg->GetLength_Ref(), (double)cfg->GetExtIter()},
          {12});
    // sorted BSR pattern (neighbours + diagonal, matrix_structure.cpp:113-201)
    std::vector<int64_t> brp(nPoint + 1, 0), bcol;
    for (unsigned long i = 0; i < nPoint; ++i) {
      std::vector<unsigned long> cols;
      cols.push_back(i);
      for (unsigned short k = 0; k < geo->node[i]->GetnPoint(); ++k) cols.push_back(geo->node[i]->GetPoint(k));
      std::sort(cols.begin(), cols.end());
      for (auto c : cols) bcol.push_back(c);
      brp[i + 1] = bcol.size();
    }
    auto dump_mat = [&](CSysMatrix& A, int nb, const std::string& name) {
      std::vector<double> blocks(bcol.size() * nb * nb);
      for (unsigned long i = 0; i < nPoint; ++i)
        for (int64_t k = brp[i]; k < brp[i + 1]; ++k) {
          su2double* b = A.GetBlock(i, bcol[k]);
          for (int q = 0; q < nb * nb; ++q) blocks[k * nb * nb + q] = b[q];
        }
      dumpd(name, blocks, {(long)bcol.size(), nb, nb});
    };
    auto dump_vec = [&](CSysVector& R, int nb, const std::string& name) {
      std::vector<double> r(nPoint * nb);
      for (unsigned long i = 0; i < nPoint * nb; ++i) r[i] = R[i];
      dumpd(name, r, {(long)nPoint, nb});
    };
    auto dump_sol = [&](CSolver* s, int nb, bool old, const std::string& name) {
      std::vector<double> u(nPoint * nb);
      for (unsigned long i = 0; i < nPoint; ++i)
        for (int v = 0; v < nb; ++v) u[i * nb + v] = old ? s->node[i]->GetSolution_Old(v) : s->node[i]->GetSolution(v);
      dumpd(name, u, {(long)nPoint, nb});
    };
    dumpi("bsr_row_ptr", brp, {(long)nPoint + 1});
    dumpi("bsr_col", bcol, {(long)bcol.size()});

    if (do_bc) {
      if (rans) {  // SST node records after the reference's preprocessing
        std::vector<double> tg(nPoint * 2 * nDim), f1(nPoint), f2(nPoint), cd(nPoint), ts(nPoint * 2);
        for (unsigned long i = 0; i < nPoint; ++i) {
          for (unsigned short v = 0; v < 2; ++v)
            for (unsigned short d = 0; d < nDim; ++d) tg[(i * 2 + v) * nDim + d] = turb->node[i]->GetGradient()[v][d];
          f1[i] = turb->node[i]->GetF1blending();
          f2[i] = turb->node[i]->GetF2blending();
          cd[i] = turb->node[i]->GetCrossDiff();
          ts[2 * i] = turb->node[i]->GetSolution(0);
          ts[2 * i + 1] = turb->node[i]->GetSolution(1);
        }
        dumpd("sst_sol", ts, {(long)nPoint, 2});
        dumpd("sst_grad", tg, {(long)nPoint, 2, nDim});
        dumpd("sst_F1", f1, {(long)nPoint});
        dumpd("sst_F2", f2, {(long)nPoint});
        dumpd("sst_CDkw", cd, {(long)nPoint});
      }
      // flow: the interior loops alone, then the reference's whole Space_Integration (loops + weak and strong
      // BCs, integration_structure.cpp:72-193) from zero, after Set_OldSolution as in MultiGrid_Cycle (:162)
      CNumerics** fn = drv.nums(FLOW_SOL);
      cfg->SetGlobalParam(kind_solver, RUNTIME_REACTIVE_SYS, 0);
      flow->Set_OldSolution(geo);
      flow->LinSysRes.SetValZero();
      if (implicit) flow->Jacobian.SetValZero();
      flow->Upwind_Residual(geo, sc, fn[CONV_TERM], cfg, MESH_0);
      flow->Viscous_Residual(geo, sc, fn[VISC_TERM], cfg, MESH_0, NO_RK_ITER);
      flow->Source_Residual(geo, sc, fn[SOURCE_FIRST_TERM], fn[SOURCE_SECOND_TERM], cfg, MESH_0);
      dump_vec(flow->LinSysRes, nVar, "bc_pre_res");
      if (implicit) dump_mat(flow->Jacobian, nVar, "bc_pre_bsr");
      flow->LinSysRes.SetValZero();
      if (implicit) flow->Jacobian.SetValZero();
      drv.integ(FLOW_SOL)->Space_Integration(geo, sc, fn, cfg, MESH_0, NO_RK_ITER, RUNTIME_REACTIVE_SYS);
      dump_vec(flow->LinSysRes, nVar, "bc_res");
      if (implicit) dump_mat(flow->Jacobian, nVar, "bc_bsr");
      dump_sol(flow, nVar, true, "bc_sol_old");
      std::vector<double> ch;
      for (unsigned short m = 0; m < nMarker; ++m)
        for (unsigned long v = 0; v < geo->GetnVertex(m); ++v) {
          su2double* c = flow->GetCharacPrimVar(m, v);
          ch.insert(ch.end(), c, c + nPrimVar);
        }
      dumpd("bc_charac", ch, {(long)ch.size() / nPrimVar, nPrimVar});
      if (rans) {
        // SST: CTurbSSTSolver::Preprocessing (zero + gradient), Set_OldSolution, loops, then Space_Integration
        CNumerics** tn = drv.nums(TURB_SOL);
        cfg->SetGlobalParam(kind_solver, RUNTIME_TURB_SYS, 0);
        turb->Preprocessing(geo, sc, cfg, MESH_0, 0, RUNTIME_TURB_SYS, false);
        turb->Set_OldSolution(geo);
        turb->LinSysRes.SetValZero();
        if (implicit) turb->Jacobian.SetValZero();
        turb->Upwind_Residual(geo, sc, tn[CONV_TERM], cfg, MESH_0);
        turb->Viscous_Residual(geo, sc, tn[VISC_TERM], cfg, MESH_0, NO_RK_ITER);
        turb->Source_Residual(geo, sc, tn[SOURCE_FIRST_TERM], tn[SOURCE_SECOND_TERM], cfg, MESH_0);
        dump_vec(turb->LinSysRes, 2, "sst_bc_pre_res");
        if (implicit) dump_mat(turb->Jacobian, 2, "sst_bc_pre_bsr");
        turb->LinSysRes.SetValZero();
        if (implicit) turb->Jacobian.SetValZero();
        drv.integ(TURB_SOL)->Space_Integration(geo, sc, tn, cfg, MESH_0, NO_RK_ITER, RUNTIME_TURB_SYS);
        dump_vec(turb->LinSysRes, 2, "sst_bc_res");
        if (implicit) dump_mat(turb->Jacobian, 2, "sst_bc_bsr");
        dump_sol(turb, 2, false, "sst_bc_sol");
        dump_sol(turb, 2, true, "sst_bc_sol_old");
      }
    } else {
      // initial node records the first Iterate reads (flow U / V / Solution_Old, SST solution, mu_t, blending,
      // cross diffusion and gradient from the last Postprocessing)
      dump_sol(flow, nVar, false, "it_U0");
      dump_sol(flow, nVar, true, "it_Uold0");
      {
        std::vector<double> V0(nPoint * nPrimVar);
        for (unsigned long i = 0; i < nPoint; ++i)
          for (unsigned short v = 0; v < nPrimVar; ++v) V0[i * nPrimVar + v] = flow->node[i]->GetPrimitive(v);
        dumpd("it_V0", V0, {(long)nPoint, nPrimVar});
      }
      if (rans) {
        dump_sol(turb, 2, false, "it_sst0");
        std::vector<double> mt(nPoint), f1(nPoint), f2(nPoint), cd(nPoint), tg(nPoint * 2 * nDim);
        for (unsigned long i = 0; i < nPoint; ++i) {
          mt[i] = turb->node[i]->GetmuT();
          f1[i] = turb->node[i]->GetF1blending();
          f2[i] = turb->node[i]->GetF2blending();
          cd[i] = turb->node[i]->GetCrossDiff();
          for (unsigned short v = 0; v < 2; ++v)
            for (unsigned short d = 0; d < nDim; ++d) tg[(i * 2 + v) * nDim + d] = turb->node[i]->GetGradient()[v][d];
        }
        dumpd("it_mut0", mt, {(long)nPoint});
        dumpd("it_F1_0", f1, {(long)nPoint});
        dumpd("it_F2_0", f2, {(long)nPoint});
        dumpd("it_CDkw0", cd, {(long)nPoint});
        dumpd("it_sstgrad0", tg, {(long)nPoint, 2, nDim});
      }
      for (int k = 0; k < n_iters; ++k) {
        cfg->SetExtIter(k);
        const auto t0 = std::chrono::steady_clock::now();
        drv.iterate();
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const std::string p = "it" + std::to_string(k + 1) + "_";
        dumpd(p + "wall", std::vector<double>{wall}, {1});  // the reference's own time for this iteration
        dump_sol(flow, nVar, false, p + "U");
        std::vector<double> V(nPoint * nPrimVar), rms(nVar);
        for (unsigned long i = 0; i < nPoint; ++i)
          for (unsigned short v = 0; v < nPrimVar; ++v) V[i * nPrimVar + v] = flow->node[i]->GetPrimitive(v);
        dumpd(p + "V", V, {(long)nPoint, nPrimVar});
        for (unsigned short v = 0; v < nVar; ++v) rms[v] = flow->GetRes_RMS(v);
        dumpd(p + "rms", rms, {(long)nVar});
        dump_sol(flow, nVar, true, p + "Uold");
        if (rans) {
          dump_sol(turb, 2, false, p + "sst");
          std::vector<double> mt(nPoint), trms = {turb->GetRes_RMS(0), turb->GetRes_RMS(1)};
          std::vector<double> f1(nPoint), f2(nPoint), cd(nPoint), tg(nPoint * 2 * nDim);
          for (unsigned long i = 0; i < nPoint; ++i) {
            mt[i] = turb->node[i]->GetmuT();
            f1[i] = turb->node[i]->GetF1blending();
            f2[i] = turb->node[i]->GetF2blending();
            cd[i] = turb->node[i]->GetCrossDiff();
            for (unsigned short v = 0; v < 2; ++v)
              for (unsigned short d = 0; d < nDim; ++d) tg[(i * 2 + v) * nDim + d] = turb->node[i]->GetGradient()[v][d];
          }
          dumpd(p + "mut", mt, {(long)nPoint});
          dumpd(p + "sst_rms", trms, {2});
          dumpd(p + "F1", f1, {(long)nPoint});
          dumpd(p + "F2", f2, {(long)nPoint});
          dumpd(p + "CDkw", cd, {(long)nPoint});
          dumpd(p + "sstgrad", tg, {(long)nPoint, 2, nDim});
        }
      }
    }
    // --iters K --restart: the reference's own restart file of the final state, written by COutput as
    // CDriver's output step does it (SetResult_Files, output_structure.cpp:7478-7489: MergeCoordinates,
    // MergeSolution, SetRestart :3858-4060) into the work dir (RESTART_FLOW_FILENAME)
    if (n_iters > 0 && argc > 6 && std::string(argv[6]) == "--restart") {
      COutput out;
      out.MergeCoordinates(cfg, geo);
      out.MergeSolution(cfg, geo, sc, ZONE_0);
      out.SetRestart(cfg, geo, sc, ZONE_0);
    }
    std::vector<int64_t> dims = {nDim, nVar, nPrimVar, nPrimVarGrad, nSpecies, implicit ? 1 : 0, rans ? 1 : 0};
    dumpi("dims", dims, {7});
    g_manifest.close();
    std::fprintf(stderr, "harness: bc/iters done (%lu points)\n", nPoint);
    return 0;
  }

  // ---- Venkatakrishnan limiter computed by the reference from the gradients above
  //      (solver_direct_reactive.cpp:1328-1523). Forced on for the dump, independent of cfg.
  {
    flow->SetPrimitive_Limiter(geo, cfg);
    std::vector<double> lim(nPoint * nPrimVarLim);
    for (unsigned long i = 0; i < nPoint; ++i)
      for (unsigned short v = 0; v < nPrimVarLim; ++v) lim[i * nPrimVarLim + v] = flow->node[i]->GetLimiter_Primitive(v);
    dumpd("limiter_out", lim, {(long)nPoint, nPrimVarLim});
    std::vector<double> prm = {cfg->GetRefElemLength(), cfg->GetLimiterCoeff()};
    dumpd("limiter_params", prm, {2});
  }

  // ---- per-edge AUSM (1st order path, solver_direct_reactive.cpp:2731-2743)
  CNumerics* conv = drv.num(FLOW_SOL, CONV_TERM);
  double** Ji = alloc2(nVar);
  double** Jj = alloc2(nVar);
  {
    std::vector<double> res(nEdge * nVar), ji, jj;
    if (implicit) { ji.resize(nEdge * nVar * nVar); jj.resize(nEdge * nVar * nVar); }
    double r[64];
    for (unsigned long e = 0; e < nEdge; ++e) {
      unsigned long i = geo->edge[e]->GetNode(0), j = geo->edge[e]->GetNode(1);
      conv->SetNormal(geo->edge[e]->GetNormal());
      conv->SetPrimitive(flow->node[i]->GetPrimitive(), flow->node[j]->GetPrimitive());
      if (implicit) conv->SetSecondary(flow->node[i]->GetdPdU(), flow->node[j]->GetdPdU());
      conv->ComputeResidual(r, Ji, Jj, cfg);
      for (unsigned short v = 0; v < nVar; ++v) res[e * nVar + v] = r[v];
      if (implicit)
        for (unsigned short a = 0; a < nVar; ++a)
          for (unsigned short b = 0; b < nVar; ++b) {
            ji[(e * nVar + a) * nVar + b] = Ji[a][b];
            jj[(e * nVar + a) * nVar + b] = Jj[a][b];
          }
    }
    dumpd("conv_res", res, {(long)nEdge, nVar});
    if (implicit) {
      dumpd("conv_jac_i", ji, {(long)nEdge, nVar, nVar});
      dumpd("conv_jac_j", jj, {(long)nEdge, nVar, nVar});
    }
    std::vector<double> minf = {cfg->GetMach()};
    dumpd("mach_inf", minf, {1});
  }

  // ---- per-edge viscous flux (solver_direct_reactive.cpp:5312-5355)
  CNumerics* visc = drv.num(FLOW_SOL, VISC_TERM);
  {
    std::vector<double> res(nEdge * nVar), ji, jj;
    if (implicit) { ji.resize(nEdge * nVar * nVar); jj.resize(nEdge * nVar * nVar); }
    double r[64];
    for (unsigned long e = 0; e < nEdge; ++e) {
      unsigned long i = geo->edge[e]->GetNode(0), j = geo->edge[e]->GetNode(1);
      visc->SetCoord(geo->node[i]->GetCoord(), geo->node[j]->GetCoord());
      visc->SetNormal(geo->edge[e]->GetNormal());
      visc->SetPrimitive(flow->node[i]->GetPrimitive(), flow->node[j]->GetPrimitive());
      visc->SetPrimVarGradient(flow->node[i]->GetGradient_Primitive(), flow->node[j]->GetGradient_Primitive());
      if (implicit) visc->SetSecondary(flow->node[i]->GetdTdU(), flow->node[j]->GetdTdU());
      visc->SetLaminarViscosity(flow->node[i]->GetLaminarViscosity(), flow->node[j]->GetLaminarViscosity());
      visc->SetThermalConductivity(flow->node[i]->GetThermalConductivity(), flow->node[j]->GetThermalConductivity());
      visc->SetDiffusionCoeff(flow->node[i]->GetDiffusionCoeff(), flow->node[j]->GetDiffusionCoeff());
      if (rans) {
        visc->SetTurbKineticEnergy(turb->node[i]->GetSolution(0), turb->node[j]->GetSolution(0));
        visc->SetEddyViscosity(turb->node[i]->GetmuT(), turb->node[j]->GetmuT());
        SigmaSetter::set(visc, turb->node[i]->Get_Sigmak());
        visc->Set_GradTKE(turb->node[i]->GetGradient()[0], turb->node[j]->GetGradient()[0]);
      }
      visc->ComputeResidual(r, Ji, Jj, cfg);
      for (unsigned short v = 0; v < nVar; ++v) res[e * nVar + v] = r[v];
      if (implicit)
        for (unsigned short a = 0; a < nVar; ++a)
          for (unsigned short b = 0; b < nVar; ++b) {
            ji[(e * nVar + a) * nVar + b] = Ji[a][b];
            jj[(e * nVar + a) * nVar + b] = Jj[a][b];
          }
    }
    dumpd("visc_res", res, {(long)nEdge, nVar});
    if (implicit) {
      dumpd("visc_jac_i", ji, {(long)nEdge, nVar, nVar});
      dumpd("visc_jac_j", jj, {(long)nEdge, nVar, nVar});
    }
    std::vector<double> prm = {cfg->GetPrandtl_Lam(), cfg->GetPrandtl_Turb(), cfg->GetLewis_Turb()};
    dumpd("visc_params", prm, {3});
  }

  // ---- per-cell chemistry source (solver_direct_reactive.cpp:2803-2817)
  CNumerics* src = drv.num(FLOW_SOL, SOURCE_FIRST_TERM);
  {
    std::vector<double> res(nPoint * nVar), jac;
    if (implicit) jac.resize(nPoint * nVar * nVar);
    double r[64];
    for (unsigned long i = 0; i < nPoint; ++i) {
      src->SetPrimitive(flow->node[i]->GetPrimitive(), flow->node[i]->GetPrimitive());
      if (implicit) src->SetSecondary(flow->node[i]->GetdTdU(), flow->node[i]->GetdTdU());
      src->SetVolume(geo->node[i]->GetVolume());
      if (rans) src->SetOmegaParam(turb->node[i]->GetSolution(1));
      src->ComputeChemistry(r, Ji, cfg);
      for (unsigned short v = 0; v < nVar; ++v) res[i * nVar + v] = r[v];
      if (implicit)
        for (unsigned short a = 0; a < nVar; ++a)
          for (unsigned short b = 0; b < nVar; ++b) jac[(i * nVar + a) * nVar + b] = Ji[a][b];
    }
    dumpd("src_res", res, {(long)nPoint, nVar});
    if (implicit) dumpd("src_jac", jac, {(long)nPoint, nVar, nVar});
    std::vector<double> prm = {cfg->Get_Cmu(), cfg->Get_PaSR_LB(), cfg->GetDensity_Ref(), cfg->GetTime_Ref(),
                               cfg->GetTemperature_Ref()};
    dumpd("src_params", prm, {5});
  }

  // ---- SST turbulence operators (a14): the turbulent solver's own numerics on the same state.
  //      Per-edge setters as CTurbSolver::Upwind_Residual / Viscous_Residual
  //      (solver_direct_turbulent.cpp:429-600), per-node as CTurbSSTSolver::Source_Residual (:3018-3080).
  double** Ti = alloc2(2);
  double** Tj = alloc2(2);
  if (rans) {
    std::vector<double> tg(nPoint * 2 * nDim), f1(nPoint), f2(nPoint), cd(nPoint), sm(nPoint), ts(nPoint * 2);
    for (unsigned long i = 0; i < nPoint; ++i) {
      su2double** g = turb->node[i]->GetGradient();
      for (unsigned short v = 0; v < 2; ++v)
        for (unsigned short d = 0; d < nDim; ++d) tg[(i * 2 + v) * nDim + d] = g[v][d];
      f1[i] = turb->node[i]->GetF1blending();
      f2[i] = turb->node[i]->GetF2blending();
      cd[i] = turb->node[i]->GetCrossDiff();
      sm[i] = flow->node[i]->GetStrainMag();
      ts[2 * i] = turb->node[i]->GetSolution(0);
      ts[2 * i + 1] = turb->node[i]->GetSolution(1);
    }
    dumpd("sst_sol", ts, {(long)nPoint, 2});
    dumpd("sst_grad", tg, {(long)nPoint, 2, nDim});
    dumpd("sst_F1", f1, {(long)nPoint});
    dumpd("sst_F2", f2, {(long)nPoint});
    dumpd("sst_CDkw", cd, {(long)nPoint});
    dumpd("strain_mag", sm, {(long)nPoint});

    CNumerics* tconv = drv.num(TURB_SOL, CONV_TERM);
    CNumerics* tvisc = drv.num(TURB_SOL, VISC_TERM);
    CNumerics* tsrc = drv.num(TURB_SOL, SOURCE_FIRST_TERM);
    std::vector<double> ur(nEdge * 2), uji(nEdge * 4), ujj(nEdge * 4), vr(nEdge * 2), vji(nEdge * 4), vjj(nEdge * 4);
    double r[8];
    auto put = [&](std::vector<double>& dst, size_t at, double** J) {
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) dst[at * 4 + a * 2 + b] = J[a][b];
    };
    for (unsigned long e = 0; e < nEdge; ++e) {
      unsigned long i = geo->edge[e]->GetNode(0), j = geo->edge[e]->GetNode(1);
      tconv->SetNormal(geo->edge[e]->GetNormal());
      tconv->SetPrimitive(flow->node[i]->GetPrimitive(), flow->node[j]->GetPrimitive());
      tconv->SetTurbVar(turb->node[i]->GetSolution(), turb->node[j]->GetSolution());
      tconv->ComputeResidual(r, Ti, Tj, cfg);
      ur[2 * e] = r[0];
      ur[2 * e + 1] = r[1];
      put(uji, e, Ti);
      put(ujj, e, Tj);
      tvisc->SetCoord(geo->node[i]->GetCoord(), geo->node[j]->GetCoord());
      tvisc->SetNormal(geo->edge[e]->GetNormal());
      tvisc->SetPrimitive(flow->node[i]->GetPrimitive(), flow->node[j]->GetPrimitive());
      tvisc->SetTurbVar(turb->node[i]->GetSolution(), turb->node[j]->GetSolution());
      tvisc->SetTurbVarGradient(turb->node[i]->GetGradient(), turb->node[j]->GetGradient());
      tvisc->SetF1blending(turb->node[i]->GetF1blending(), turb->node[j]->GetF1blending());
      tvisc->SetLaminarViscosity(flow->node[i]->GetLaminarViscosity(), flow->node[j]->GetLaminarViscosity());
      tvisc->SetEddyViscosity(flow->node[i]->GetEddyViscosity(), flow->node[j]->GetEddyViscosity());
      tvisc->ComputeResidual(r, Ti, Tj, cfg);
      vr[2 * e] = r[0];
      vr[2 * e + 1] = r[1];
      put(vji, e, Ti);
      put(vjj, e, Tj);
    }
    dumpd("sst_upw_res", ur, {(long)nEdge, 2});
    dumpd("sst_upw_jac_i", uji, {(long)nEdge, 2, 2});
    dumpd("sst_upw_jac_j", ujj, {(long)nEdge, 2, 2});
    dumpd("sst_visc_res", vr, {(long)nEdge, 2});
    dumpd("sst_visc_jac_i", vji, {(long)nEdge, 2, 2});
    dumpd("sst_visc_jac_j", vjj, {(long)nEdge, 2, 2});
    std::vector<double> sr(nPoint * 2), sj(nPoint * 4);
    for (unsigned long i = 0; i < nPoint; ++i) {
      tsrc->SetPrimitive(flow->node[i]->GetPrimitive(), NULL);
      tsrc->SetPrimVarGradient(flow->node[i]->GetGradient_Primitive(), NULL);
      tsrc->SetTurbVar(turb->node[i]->GetSolution(), NULL);
      tsrc->SetTurbVarGradient(turb->node[i]->GetGradient(), NULL);
      tsrc->SetVolume(geo->node[i]->GetVolume());
      tsrc->SetDistance(geo->node[i]->GetWall_Distance(), 0.0);
      tsrc->SetF1blending(turb->node[i]->GetF1blending(), 0.0);
      tsrc->SetF2blending(turb->node[i]->GetF2blending(), 0.0);
      tsrc->SetVorticity(flow->node[i]->GetVorticity(), NULL);
      tsrc->SetStrainMag(flow->node[i]->GetStrainMag(), 0.0);
      tsrc->SetCrossDiff(turb->node[i]->GetCrossDiff(), 0.0);
      tsrc->SetLaminarViscosity(flow->node[i]->GetLaminarViscosity(), flow->node[i]->GetLaminarViscosity());
      tsrc->SetEddyViscosity(flow->node[i]->GetEddyViscosity(), flow->node[i]->GetEddyViscosity());
      tsrc->ComputeResidual(r, Ti, NULL, cfg);
      sr[2 * i] = r[0];
      sr[2 * i + 1] = r[1];
      put(sj, i, Ti);
    }
    dumpd("sst_src_res", sr, {(long)nPoint, 2});
    dumpd("sst_src_jac", sj, {(long)nPoint, 2, 2});
  }

  // ---- LSQ gradient recomputed by the reference (solver_direct_reactive.cpp:4887-5050)
  {
    CReactiveNSSolver* ns = dynamic_cast<CReactiveNSSolver*>(flow);
    ns->SetPrimitive_Gradient_LS(geo, cfg);
    std::vector<double> grad(nPoint * nPrimVarGrad * nDim);
    for (unsigned long i = 0; i < nPoint; ++i) {
      su2double** g = flow->node[i]->GetGradient_Primitive();
      for (unsigned short v = 0; v < nPrimVarGrad; ++v)
        for (unsigned short dd = 0; dd < nDim; ++dd) grad[(i * nPrimVarGrad + v) * nDim + dd] = g[v][dd];
    }
    dumpd("grad_lsq_out", grad, {(long)nPoint, nPrimVarGrad, nDim});
  }

  // ---- whole loops (solver_direct_reactive.cpp Upwind/Viscous/Source) and the time step
  if (do_bsr) {
    CNumerics* visc_n = drv.num(FLOW_SOL, VISC_TERM);
    CNumerics* conv_n = drv.num(FLOW_SOL, CONV_TERM);
    CNumerics* src_n = drv.num(FLOW_SOL, SOURCE_FIRST_TERM);
    CNumerics* src2_n = drv.num(FLOW_SOL, SOURCE_SECOND_TERM);
    CSysVector& R = flow->LinSysRes;
    auto dump_res = [&](const std::string& name) {
      std::vector<double> r(nPoint * nVar);
      for (unsigned long i = 0; i < nPoint * nVar; ++i) r[i] = R[i];
      dumpd(name, r, {(long)nPoint, nVar});
    };
    R.SetValZero();
    if (implicit) flow->Jacobian.SetValZero();
    flow->Upwind_Residual(geo, sc, conv_n, cfg, MESH_0);
    dump_res("loop_upwind_res");
    flow->Viscous_Residual(geo, sc, visc_n, cfg, MESH_0, NO_RK_ITER);
    dump_res("loop_upwind_visc_res");
    flow->Source_Residual(geo, sc, src_n, src2_n, cfg, MESH_0);
    dump_res("loop_total_res");

    flow->SetTime_Step(geo, sc, cfg, MESH_0, 0);
    std::vector<double> dt(nPoint), li(nPoint), lv(nPoint);
    for (unsigned long i = 0; i < nPoint; ++i) {
      dt[i] = flow->node[i]->GetDelta_Time();
      li[i] = flow->node[i]->GetMax_Lambda_Inv();
      lv[i] = flow->node[i]->GetMax_Lambda_Visc();
    }
    dumpd("dt", dt, {(long)nPoint});
    dumpd("lambda_inv", li, {(long)nPoint});
    dumpd("lambda_visc", lv, {(long)nPoint});
    std::vector<double> tprm = {cfg->GetCFL(MESH_0), cfg->GetMax_DeltaTime(), cfg->GetPrandtl_Lam(), cfg->GetPrandtl_Turb()};
    dumpd("dt_params", tprm, {4});

    if (implicit) {
      CSysMatrix& A = flow->Jacobian;
      // BSR of the assembled Jacobian (sorted neighbours + diagonal, matrix_structure.cpp:113-201)
      std::vector<int64_t> row_ptr(nPoint + 1, 0), col;
      for (unsigned long i = 0; i < nPoint; ++i) {
        std::vector<unsigned long> cols;
        cols.push_back(i);
        for (unsigned short k = 0; k < geo->node[i]->GetnPoint(); ++k) cols.push_back(geo->node[i]->GetPoint(k));
        std::sort(cols.begin(), cols.end());
        for (auto c : cols) col.push_back(c);
        row_ptr[i + 1] = col.size();
      }
      auto dump_bsr = [&](const std::string& name) {
        std::vector<double> blocks(col.size() * nVar * nVar);
        for (unsigned long i = 0; i < nPoint; ++i)
          for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
            su2double* b = A.GetBlock(i, col[k]);
            for (int q = 0; q < nVar * nVar; ++q) blocks[k * nVar * nVar + q] = b[q];
          }
        dumpd(name, blocks, {(long)col.size(), nVar, nVar});
      };
      dumpi("bsr_row_ptr", row_ptr, {(long)nPoint + 1});
      dumpi("bsr_col", col, {(long)col.size()});
      dump_bsr("bsr_jac_residual");

      // ImplicitEuler system build (solver_direct_reactive.cpp:2350-2377), truncation error is zero here
      CSysVector rhs(nPoint, nPoint, nVar, 0.0), x(nPoint, nPoint, nVar, 0.0);
      for (unsigned long i = 0; i < nPoint; ++i) {
        double Vol = geo->node[i]->GetVolume();
        double Dt = flow->node[i]->GetDelta_Time();
        if (Dt > EPS) A.AddVal2Diag(i, Vol / Dt);
        else A.SetVal2Diag(i, 1.0);
        for (unsigned short v = 0; v < nVar; ++v) rhs[i * nVar + v] = (Dt > EPS) ? -R[i * nVar + v] : -0.0;
      }
      dump_bsr("bsr_system");
      std::vector<double> b(nPoint * nVar);
      for (unsigned long i = 0; i < nPoint * nVar; ++i) b[i] = rhs[i];
      dumpd("sys_rhs", b, {(long)nPoint, nVar});

      CSysMatrixVectorProduct mv(A, geo, cfg);
      CSysVector y(nPoint, nPoint, nVar, 0.0);
      mv(rhs, y);
      std::vector<double> yy(nPoint * nVar);
      for (unsigned long i = 0; i < nPoint * nVar; ++i) yy[i] = y[i];
      dumpd("spmv_rhs", yy, {(long)nPoint, nVar});

      CSysVector z(nPoint, nPoint, nVar, 0.0);
      CSysSolve solver;
      double resid = 0.0;
      const unsigned long m = cfg->GetLinear_Solver_Iter();
      const double tol = cfg->GetLinear_Solver_Error();
      if (cfg->GetKind_Linear_Solver_Prec() != ILU) {
      CLU_SGSPreconditioner lusgs(A, geo, cfg);
      lusgs(rhs, z);
      for (unsigned long i = 0; i < nPoint * nVar; ++i) yy[i] = z[i];
      dumpd("lusgs_rhs", yy, {(long)nPoint, nVar});

      x.SetValZero();
      unsigned long it1 = solver.FGMRES_LinSolver(rhs, x, mv, lusgs, tol, m, &resid, false);
      for (unsigned long i = 0; i < nPoint * nVar; ++i) yy[i] = x[i];
      dumpd("fgmres_lusgs_x", yy, {(long)nPoint, nVar});
      std::vector<double> info = {(double)it1, resid, tol, (double)m};
      dumpd("fgmres_lusgs_info", info, {4});
      } else {

      A.BuildILUPreconditioner();
      std::vector<double> ilu(col.size() * nVar * nVar);
      for (unsigned long i = 0; i < nPoint; ++i)
        for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
          su2double* bb = A.GetBlock_ILUMatrix(i, col[k]);
          for (int q = 0; q < nVar * nVar; ++q) ilu[k * nVar * nVar + q] = bb[q];
        }
      dumpd("ilu_factor", ilu, {(long)col.size(), nVar, nVar});
      CILUPreconditioner ilup(A, geo, cfg);
      ilup(rhs, z);
      for (unsigned long i = 0; i < nPoint * nVar; ++i) yy[i] = z[i];
      dumpd("ilu_rhs", yy, {(long)nPoint, nVar});
      x.SetValZero();
      unsigned long it2 = solver.FGMRES_LinSolver(rhs, x, mv, ilup, tol, m, &resid, false);
      for (unsigned long i = 0; i < nPoint * nVar; ++i) yy[i] = x[i];
      dumpd("fgmres_ilu_x", yy, {(long)nPoint, nVar});
      std::vector<double> info = {(double)it2, resid, tol, (double)m};
      dumpd("fgmres_ilu_info", info, {4});
      }
      // ---- one MPI rank of the same system. RX_RANK_SPLIT=P: a CSysMatrix whose domain is the
      // points [0, P) and whose halo is [P, nPoint) — the reference's own per-rank layout, domain points first with
      // the halo columns present (CSysMatrix::Initialize with nPointDomain = P, matrix_structure.cpp:113-201) —
      // holding the same blocks; then the reference's BuildILUPreconditioner (:1368-1451, needs the ILU0 cfg: the
      // ILU matrix is allocated for it, :236-247), ComputeILUPreconditioner (:1453-1515) and
      // ComputeLU_SGSPreconditioner (:1673-1709) on it. The LU-SGS product's halo entries are preset from
      // halo_x.bin: what the neighbour ranks' forward sweeps would deliver through SendReceive_Solution (:1687), a
      // no-op on this serial mesh (no SEND_RECEIVE marker, :794-880), which therefore leaves the preset in place.
      if (const char* sp = std::getenv("RX_RANK_SPLIT")) {
        const unsigned long P = std::strtoul(sp, nullptr, 10);
        CSysMatrix Rk;
        Rk.Initialize(nPoint, P, nVar, nVar, true, geo, cfg);
        for (unsigned long i = 0; i < nPoint; ++i)
          for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) Rk.SetBlock(i, col[k], A.GetBlock(i, col[k]));
        std::vector<double> zz(P * nVar);
        if (cfg->GetKind_Linear_Solver_Prec() == ILU) {
          Rk.BuildILUPreconditioner();
          std::vector<double> f((size_t)row_ptr[P] * nVar * nVar);
          for (unsigned long i = 0; i < P; ++i)
            for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
              su2double* bb = Rk.GetBlock_ILUMatrix(i, col[k]);
              for (int q = 0; q < nVar * nVar; ++q) f[k * nVar * nVar + q] = bb[q];
            }
          dumpd("rank_ilu_factor", f, {(long)row_ptr[P], nVar, nVar});
          CSysVector zr(nPoint, P, nVar, 0.0);
          Rk.ComputeILUPreconditioner(rhs, zr, geo, cfg);
          for (unsigned long q = 0; q < P * nVar; ++q) zz[q] = zr[q];
          dumpd("rank_ilu_rhs", zz, {(long)P, nVar});
        }
        std::vector<double> hx(nPoint * nVar, 0.0);
        {
          FILE* hf = std::fopen("halo_x.bin", "rb");
          if (!hf || std::fread(hx.data(), sizeof(double), hx.size(), hf) != hx.size()) {
            std::fprintf(stderr, "RX_RANK_SPLIT needs halo_x.bin (%lu x %d doubles)\n", nPoint, nVar);
            std::exit(4);
          }
          std::fclose(hf);
        }
        CSysVector zl(nPoint, P, nVar, 0.0);
        for (unsigned long q = P * nVar; q < nPoint * nVar; ++q) zl[q] = hx[q];
        Rk.ComputeLU_SGSPreconditioner(rhs, zl, geo, cfg);
        for (unsigned long q = 0; q < P * nVar; ++q) zz[q] = zl[q];
        dumpd("rank_lusgs_rhs", zz, {(long)P, nVar});
        std::vector<double> ps = {(double)P};
        dumpd("rank_split", ps, {1});
      }
    }
    // ---- SST loops and the turbulent implicit step (CTurbSSTSolver::Preprocessing :2923-2946,
    //      CTurbSolver::Upwind/Viscous_Residual :429-600, Source_Residual :3018-3080,
    //      CTurbSolver::ImplicitEuler_Iteration :615-728, CTurbSSTSolver::Postprocessing :2948-3016)
    if (rans) {
      CNumerics* tconv = drv.num(TURB_SOL, CONV_TERM);
      CNumerics* tvisc = drv.num(TURB_SOL, VISC_TERM);
      CNumerics* tsrc = drv.num(TURB_SOL, SOURCE_FIRST_TERM);
      CNumerics* tsrc2 = drv.num(TURB_SOL, SOURCE_SECOND_TERM);
      CSysVector& TR = turb->LinSysRes;
      auto dump_tres = [&](const std::string& name) {
        std::vector<double> rr(nPoint * 2);
        for (unsigned long i = 0; i < nPoint * 2; ++i) rr[i] = TR[i];
        dumpd(name, rr, {(long)nPoint, 2});
      };
      turb->Preprocessing(geo, sc, cfg, MESH_0, 0, RUNTIME_TURB_SYS, false);
      {
        std::vector<double> tg(nPoint * 2 * nDim);
        for (unsigned long i = 0; i < nPoint; ++i)
          for (unsigned short v = 0; v < 2; ++v)
            for (unsigned short d = 0; d < nDim; ++d) tg[(i * 2 + v) * nDim + d] = turb->node[i]->GetGradient()[v][d];
        dumpd("sst_grad_ls", tg, {(long)nPoint, 2, nDim});
      }
      turb->Upwind_Residual(geo, sc, tconv, cfg, MESH_0);
      dump_tres("sst_loop_upw_res");
      turb->Viscous_Residual(geo, sc, tvisc, cfg, MESH_0, NO_RK_ITER);
      dump_tres("sst_loop_upw_visc_res");
      turb->Source_Residual(geo, sc, tsrc, tsrc2, cfg, MESH_0);
      dump_tres("sst_loop_total_res");
      if (implicit) {
        CSysMatrix& TA = turb->Jacobian;
        std::vector<int64_t> trp(nPoint + 1, 0), tcol;
        for (unsigned long i = 0; i < nPoint; ++i) {
          std::vector<unsigned long> cols;
          cols.push_back(i);
          for (unsigned short k = 0; k < geo->node[i]->GetnPoint(); ++k) cols.push_back(geo->node[i]->GetPoint(k));
          std::sort(cols.begin(), cols.end());
          for (auto c : cols) tcol.push_back(c);
          trp[i + 1] = tcol.size();
        }
        auto dump_tbsr = [&](const std::string& name) {
          std::vector<double> blocks(tcol.size() * 4);
          for (unsigned long i = 0; i < nPoint; ++i)
            for (int64_t k = trp[i]; k < trp[i + 1]; ++k) {
              su2double* b = TA.GetBlock(i, tcol[k]);
              for (int q = 0; q < 4; ++q) blocks[k * 4 + q] = b[q];
            }
          dumpd(name, blocks, {(long)tcol.size(), 2, 2});
        };
        dump_tbsr("sst_bsr_jac_residual");
        turb->ImplicitEuler_Iteration(geo, sc, cfg);
        dump_tbsr("sst_bsr_system");
        dump_tres("sst_sys_rhs");
        std::vector<double> xs(nPoint * 2), ns2(nPoint * 2);
        for (unsigned long i = 0; i < nPoint * 2; ++i) xs[i] = turb->LinSysSol[i];
        for (unsigned long i = 0; i < nPoint; ++i) {
          ns2[2 * i] = turb->node[i]->GetSolution(0);
          ns2[2 * i + 1] = turb->node[i]->GetSolution(1);
        }
        dumpd("sst_lin_sol", xs, {(long)nPoint, 2});
        dumpd("sst_new_sol", ns2, {(long)nPoint, 2});
        std::vector<double> rms = {turb->GetRes_RMS(0), turb->GetRes_RMS(1)};
        dumpd("sst_rms", rms, {2});
        turb->Postprocessing(geo, sc, cfg, MESH_0);
        std::vector<double> mt(nPoint), f1(nPoint), f2(nPoint), cd(nPoint), tg(nPoint * 2 * nDim);
        for (unsigned long i = 0; i < nPoint; ++i) {
          mt[i] = turb->node[i]->GetmuT();
          f1[i] = turb->node[i]->GetF1blending();
          f2[i] = turb->node[i]->GetF2blending();
          cd[i] = turb->node[i]->GetCrossDiff();
          for (unsigned short v = 0; v < 2; ++v)
            for (unsigned short d = 0; d < nDim; ++d) tg[(i * 2 + v) * nDim + d] = turb->node[i]->GetGradient()[v][d];
        }
        dumpd("sst_post_mut", mt, {(long)nPoint});
        dumpd("sst_post_F1", f1, {(long)nPoint});
        dumpd("sst_post_F2", f2, {(long)nPoint});
        dumpd("sst_post_CDkw", cd, {(long)nPoint});
        dumpd("sst_post_grad", tg, {(long)nPoint, 2, nDim});
      }
    }
  }

  // ---- a2 second-order branch: Upwind_Residual with the MUSCL reconstruction on the cfg's spatial
  //      order (jet9: 2ND_ORDER_LIMITER), solver_direct_reactive.cpp:2554-2729. Whole residual and the
  //      BSR Jacobian it assembles (make_golden keeps a window / a row sample).
  if (!do_bsr) {
    CNumerics* conv_n = drv.num(FLOW_SOL, CONV_TERM);
    flow->LinSysRes.SetValZero();
    if (implicit) flow->Jacobian.SetValZero();
    flow->Upwind_Residual(geo, sc, conv_n, cfg, MESH_0);
    std::vector<double> r(nPoint * nVar);
    for (unsigned long i = 0; i < nPoint * nVar; ++i) r[i] = flow->LinSysRes[i];
    dumpd("muscl_loop_res", r, {(long)nPoint, nVar});
    if (implicit) {
      std::vector<int64_t> rp(nPoint + 1, 0), cl;
      std::vector<double> blocks;
      for (unsigned long i = 0; i < nPoint; ++i) {
        std::vector<unsigned long> cols;
        cols.push_back(i);
        for (unsigned short k = 0; k < geo->node[i]->GetnPoint(); ++k) cols.push_back(geo->node[i]->GetPoint(k));
        std::sort(cols.begin(), cols.end());
        for (auto c : cols) {
          cl.push_back(c);
          su2double* b = flow->Jacobian.GetBlock(i, c);
          blocks.insert(blocks.end(), b, b + nVar * nVar);
        }
        rp[i + 1] = cl.size();
      }
      dumpi("muscl_bsr_row_ptr", rp, {(long)nPoint + 1});
      dumpi("muscl_bsr_col", cl, {(long)cl.size()});
      dumpd("muscl_bsr", blocks, {(long)cl.size(), nVar, nVar});
    }
    std::vector<double> prm = {(double)cfg->GetSpatialOrder_Flow(), cfg->GetTemperature_Ref(), cfg->GetEnergy_Ref(),
                               cfg->GetGas_Constant_Ref()};
    dumpd("muscl_params", prm, {4});
  }

  // ---- next-1: one reference update (residual loops, time step, Euler update) followed by
  //      CReactiveEulerSolver::SetPrimitive_Variables (solver_direct_reactive.cpp:985-1040):
  //      Cons2PrimVar from the updated U with the previous T as the secant's start, Cp, dT/dU, dP/dU,
  //      mu, kappa, Dij, eddy viscosity (variable_direct_reactive.cpp:550-853, 1188-1228).
  {
    CNumerics* conv_n = drv.num(FLOW_SOL, CONV_TERM);
    CNumerics* visc_n = drv.num(FLOW_SOL, VISC_TERM);
    CNumerics* src_n = drv.num(FLOW_SOL, SOURCE_FIRST_TERM);
    CNumerics* src2_n = drv.num(FLOW_SOL, SOURCE_SECOND_TERM);
    flow->LinSysRes.SetValZero();
    if (implicit) flow->Jacobian.SetValZero();
    flow->Upwind_Residual(geo, sc, conv_n, cfg, MESH_0);
    flow->Viscous_Residual(geo, sc, visc_n, cfg, MESH_0, NO_RK_ITER);
    flow->Source_Residual(geo, sc, src_n, src2_n, cfg, MESH_0);
    flow->SetTime_Step(geo, sc, cfg, MESH_0, 0);
    std::vector<double> Uprev(nPoint * nVar);
    for (unsigned long i = 0; i < nPoint; ++i)
      for (unsigned short v = 0; v < nVar; ++v) Uprev[i * nVar + v] = flow->node[i]->GetSolution(v);
    if (implicit) flow->ImplicitEuler_Iteration(geo, sc, cfg);
    else flow->ExplicitEuler_Iteration(geo, sc, cfg);
    // mini9 (CFL 5 on a 21x11 mesh without boundary conditions): a fraction of the reference's update
    // keeps every point inside the property tables; jet9 takes the whole update.
    const double frac = do_bsr ? 0.05 : 1.0;
    if (frac != 1.0)
      for (unsigned long i = 0; i < nPoint; ++i)
        for (unsigned short v = 0; v < nVar; ++v) {
          const double u0 = Uprev[i * nVar + v];
          flow->node[i]->SetSolution(v, u0 + frac * (flow->node[i]->GetSolution(v) - u0));
        }
    std::vector<double> U(nPoint * nVar), V0(nPoint * nPrimVar), tk(nPoint), mt(nPoint);
    for (unsigned long i = 0; i < nPoint; ++i) {
      for (unsigned short v = 0; v < nVar; ++v) U[i * nVar + v] = flow->node[i]->GetSolution(v);
      for (unsigned short v = 0; v < nPrimVar; ++v) V0[i * nPrimVar + v] = flow->node[i]->GetPrimitive(v);
      tk[i] = rans ? turb->node[i]->GetSolution(0) : 0.0;
      mt[i] = rans ? turb->node[i]->GetmuT() : 0.0;
    }
    dumpd("p2v_U", U, {(long)nPoint, nVar});
    dumpd("p2v_V_before", V0, {(long)nPoint, nPrimVar});
    dumpd("p2v_tke", tk, {(long)nPoint});
    dumpd("p2v_mut", mt, {(long)nPoint});
    const unsigned long nerr = flow->SetPrimitive_Variables(sc, cfg, false);
    std::vector<double> U1(nPoint * nVar), V(nPoint * nPrimVar), dPdU(nPoint * nVar), dTdU(nPoint * nVar);
    std::vector<double> mu(nPoint), kap(nPoint), cp(nPoint), ed(nPoint), Dij(nPoint * nSpecies * nSpecies);
    for (unsigned long i = 0; i < nPoint; ++i) {
      CVariable* n = flow->node[i];
      for (unsigned short v = 0; v < nVar; ++v) {
        U1[i * nVar + v] = n->GetSolution(v);
        dPdU[i * nVar + v] = n->GetdPdU()[v];
        dTdU[i * nVar + v] = n->GetdTdU()[v];
      }
      for (unsigned short v = 0; v < nPrimVar; ++v) V[i * nPrimVar + v] = n->GetPrimitive(v);
      mu[i] = n->GetLaminarViscosity();
      kap[i] = n->GetThermalConductivity();
      cp[i] = n->GetSpecificHeatCp();
      ed[i] = n->GetEddyViscosity();
      double* d = n->GetDiffusionCoeff();
      for (int k = 0; k < nSpecies * nSpecies; ++k) Dij[i * nSpecies * nSpecies + k] = d[k];
    }
    dumpd("p2v_U_after", U1, {(long)nPoint, nVar});
    dumpd("p2v_V", V, {(long)nPoint, nPrimVar});
    dumpd("p2v_dPdU", dPdU, {(long)nPoint, nVar});
    dumpd("p2v_dTdU", dTdU, {(long)nPoint, nVar});
    dumpd("p2v_mu", mu, {(long)nPoint});
    dumpd("p2v_kappa", kap, {(long)nPoint});
    dumpd("p2v_cp", cp, {(long)nPoint});
    dumpd("p2v_eddy", ed, {(long)nPoint});
    dumpd("p2v_Dij", Dij, {(long)nPoint, nSpecies, nSpecies});
    std::vector<double> prm = {(double)nerr, cfg->GetTemperatureMin(), cfg->GetTemperatureMax(),
                               cfg->GetTemperature_Ref(), cfg->GetEnergy_Ref(), cfg->GetGas_Constant_Ref(),
                               cfg->GetPressure_Ref(), cfg->GetViscosity_Ref(), cfg->GetConductivity_Ref(),
                               cfg->GetVelocity_Ref(), cfg->GetLength_Ref(), (double)cfg->GetExtIter()};
    dumpd("p2v_params", prm, {(long)prm.size()});
  }

  std::vector<int64_t> dims = {nDim, nVar, nPrimVar, nPrimVarGrad, nSpecies, implicit ? 1 : 0, rans ? 1 : 0};
  dumpi("dims", dims, {7});
  g_manifest.close();
  std::fprintf(stderr, "harness: done (%lu points, %lu edges)\n", nPoint, nEdge);
  return 0;
}
