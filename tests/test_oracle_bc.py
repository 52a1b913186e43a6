"""next-3 + a8: the CPU oracle's boundary conditions and whole outer iteration against the reference's own
(golden bc9 / it9 from oracle/ref_harness --bc / --iters, see oracle/make_golden.py).

bc9: one Space_Integration of the reference (integration_structure.cpp:72-193) on the mini9 jet — interior loops,
then the weak BCs (BC_Inlet TEMPERATURE_IMPOSE, BC_Outlet with the boundary viscous numerics
CAvgGradReactive_Boundary) and the strong BC_Isothermal_Wall, for the flow and the SST solver.
it9: three whole reference outer iterations (CMeanFlowIteration::Iterate) from the mini9 state.
bc3d / it3d: the same on the 3-D extruded jet (symmetry planes in z: CSolver::BC_Sym_Plane is a no-op for the
reactive solvers, solver_structure.inl:731-732, and CTurbSolver::BC_Sym_Plane, solver_direct_turbulent.cpp:602-606),
two iterations.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def golden(case):
    return dict(np.load(os.path.join(GOLD, case + ".npz")))


def bc_case(name):
    """bc9 (INLET_TYPE = TEMPERATURE_IMPOSE, the shipped jet cfgs), bc9t (TOTAL_CONDITIONS), bc9m (MASS_FLOW): the
    variants hold only the outputs their inlet kind changes, over bc9's mesh and state."""
    if name == "bc3d":
        return golden(name)
    g = golden("bc9")
    if name != "bc9":
        g.update(golden(name))
    return g


@pytest.fixture(scope="module", params=["bc9", "bc9t", "bc9m", "bc3d"])
def bc9(request):
    return bc_case(request.param)


# ls*: CSysSolve::Solve's other branches (oracle/make_golden.py LIN_CASES): BCGSTAB with ILU0 / JACOBI, FGMRES with
# JACOBI, RESTARTED_FGMRES, the LU_SGS / Jacobi / ILU0 smoothers
LIN_GOLDENS = ["lsbc", "lsbj", "lsfj", "lsrs", "lssl", "lssj", "lssi"]
# it5s / it6s / it8s: the species counts the device instantiates beside 3 / 4 / 7 / 9 (csrc/rx_species.h)
NS_GOLDENS = ["it5s", "it6s", "it8s"]


@pytest.fixture(scope="module", params=["it9", "it3d", "it7", "itx9", "itx4", "ig9", "fpit", "gg9", "mix3d", "fpit2",
                                        "fpit2l", "it4t"] + LIN_GOLDENS + NS_GOLDENS)
def it9(request):
    return golden(request.param)


def n_iters(g):
    return sum(1 for k in g if k.startswith("it") and k.endswith("_U") and k[2:-2].isdigit())


def _bc_setup(g):
    nDim, nVar = int(g["dims"][0]), int(g["dims"][1])
    rp, col = g["bsr_row_ptr"], g["bsr_col"]
    prm = O.bc_prm(g["bc_params"], g["mach_inf"][0], g["visc_params"][1], g["visc_params"][2])
    return nDim, nVar, rp, col, prm


def test_flow_bc_vs_reference(bc9):
    g = bc9
    nDim, nVar, rp, col, prm = _bc_setup(g)
    m = O.Mechanism(g)
    R = g["bc_pre_res"].copy()
    A = np.zeros((int(rp[-1]), nVar, nVar))
    A[g["bc_blk"]] = g["bc_pre_bsr"]
    Uold = g["U"].copy()
    ch = O.bc_flow(m, nDim, g, g["bc_marker"], prm, g, rp, col, R, A, Uold, True, True)
    if nDim == 3:  # the symmetry planes are markers with no action
        assert int(g["bc_params"][26]) in g["bc_marker"][:, 0]
    # ghost states (CharacPrimVar), Jacobian rows, Solution_Old (SetVelocity_Old at the walls): bitwise
    assert np.array_equal(ch, g["bc_charac"])
    assert np.array_equal(A[g["bc_blk"]], g["bc_bsr"])
    assert np.array_equal(Uold, g["bc_sol_old"])
    # residual: bitwise except the Stefan-Maxwell BiCGSTAB rounding of the boundary viscous flux
    ref = g["bc_res"]
    scale = np.maximum(np.abs(ref).max(axis=0), 1e-300)
    assert (np.abs(R - ref).max(axis=0) / scale).max() < 1e-13
    flow_rows = np.abs(R[:, :3] - ref[:, :3]).max()
    assert flow_rows == 0.0


def test_sst_bc_vs_reference(bc9):
    g = bc9
    nDim, nVar, rp, col, prm = _bc_setup(g)
    charac = g["bc_charac"]
    T = g["sst_sol"].copy()
    R = g["sst_bc_pre_res"].copy()
    A = np.zeros((int(rp[-1]), 2, 2))
    A[g["bc_blk"]] = g["sst_bc_pre_bsr"]
    O.bc_sst(nDim, g, g["bc_marker"], prm, g["V"], g["mu"], g["eddy_visc_flow"], charac, g["sst_grad"], g["sst_F1"],
             rp, col, T, R, A, True)
    assert np.array_equal(R, g["sst_bc_res"])
    assert np.array_equal(A[g["bc_blk"]], g["sst_bc_bsr"])
    assert np.array_equal(T, g["sst_bc_sol"])


def iteration_cfg(g):
    bp = g["bc_params"]
    cfg = dict(p2v=O.p2v_params(g), cfl=g["dt_params"][0], max_delta_time=g["dt_params"][1],
               prandtl_lam=g["dt_params"][2], prandtl_turb=g["dt_params"][3], lewis_turb=g["visc_params"][2],
               mach_inf=g["mach_inf"][0], c_mu=g["src_params"][0], pasr_lb=g["src_params"][1], lin_tol=bp[19],
               lin_iter=int(bp[20]), relaxation=bp[22], relaxation_turb=bp[23], cfl_red_turb=bp[24])
    # TIME_DISCRE_FLOW / RK_ALPHA_COEFF / LINEAR_SOLVER_PREC of the golden's cfg (it9 / it3d: implicit, ILU0)
    tf = str(g["time_flow"]) if "time_flow" in g else "EULER_IMPLICIT"
    cfg["time"] = {"EULER_IMPLICIT": "implicit", "EULER_EXPLICIT": "euler_explicit", "RUNGE-KUTTA_EXPLICIT": "rk"}[tf]
    if "rk_alpha" in g:
        cfg["rk_alpha"] = [float(x) for x in g["rk_alpha"]]
    cfg["sst_prec"] = {"LU_SGS": "lusgs", "JACOBI": "jacobi"}.get(str(g["lin_prec"]), "ilu") if "lin_prec" in g else "ilu"
    cfg["flow_prec"] = cfg["sst_prec"]  # LINEAR_SOLVER_PREC serves both solvers
    if "lin_solver" in g:  # LINEAR_SOLVER, LINEAR_SOLVER_RESTART_FREQUENCY (ls*)
        cfg.update(lin_solver=str(g["lin_solver"]), lin_restart=int(g["lin_restart"]))
    cfg["spatial_order"] = int(g["spatial_order"]) if "spatial_order" in g else 0
    if "limiter_params" in g:  # REF_ELEM_LENGTH, LIMITER_COEFF
        cfg.update(ref_elem_length=float(g["limiter_params"][0]), limiter_coeff=float(g["limiter_params"][1]))
    if "sst_spatial_order" in g:  # SPATIAL_ORDER_TURB (fpit2 / fpit2l), SLOPE_LIMITER_TURB VENKATAKRISHNAN
        cfg["sst_order"] = int(g["sst_spatial_order"])
    if "grad_method" in g and str(g["grad_method"]) == "GREEN_GAUSS":  # NUM_METHOD_GRAD (gg9)
        cfg["grad"] = "gg"
    if "ignition" in g:  # IGNITION, IGNITION_ITER, IGNITION_TEMPERATURE, FUEL_INDEX, OXIDIZER_INDEX (ig9)
        cfg["p2v"] = list(cfg["p2v"]) + [float(x) for x in g["ignition"]]
    bc = dict(marker=g["bc_marker"], prm=O.bc_prm(bp, g["mach_inf"][0], g["visc_params"][1], g["visc_params"][2]))
    if "laminar" in g:  # KIND_TURB_MODEL= NONE (lam4): no SST records
        cfg["rans"] = False
        return cfg, bc, dict(U=g["it_U0"], V=g["it_V0"], Uold=g["it_Uold0"])
    state = dict(U=g["it_U0"], V=g["it_V0"], Uold=g["it_Uold0"], T=g["it_sst0"], TG=g["it_sstgrad0"],
                 F1=g["it_F1_0"], F2=g["it_F2_0"], CDkw=g["it_CDkw0"], mut=g["it_mut0"])
    return cfg, bc, state


def colrel(a, ref):
    return (np.abs(a - ref).max(axis=0) / np.maximum(np.abs(ref).max(axis=0), 1e-300)).max()


# chained iterations: last-bit differences of the Stefan-Maxwell solve grow through FGMRES
ITER_TOL = {1: 1e-13, 2: 1e-11, 3: 1e-9}
# 3-D: the small spanwise / wall-normal momentum columns carry the FGMRES-amplified rounding of the large ones.
# Chained, the second 3-D iteration already crosses the Ds discontinuity of the viscous Jacobian (DESIGN.md §2:
# an energy-row species entry moves by 8e-7 relative for a 4e-12 state difference), so only the first is chained;
# every iteration is checked from the reference's own state in test_each_iteration_from_reference_state.
ITER_TOL3 = {1: 1e-11}


def test_each_iteration_from_reference_state(it9):
    """Every iteration restarted from the reference's own records after the previous one."""
    g = it9
    nDim = int(g["dims"][0])
    m = O.Mechanism(g)
    cfg, bc, s0 = iteration_cfg(g)
    pat = (g["bsr_row_ptr"], g["bsr_col"])
    for k in range(n_iters(g)):
        if k == 0:
            s = s0
        else:
            p = f"it{k}_"
            s = dict(U=g[p + "U"], V=g[p + "V"], Uold=g[p + "Uold"], T=g[p + "sst"], TG=g[p + "sstgrad"], F1=g[p + "F1"],
                     F2=g[p + "F2"], CDkw=g[p + "CDkw"], mut=g[p + "mut"])
        s = O.outer_iteration(m, nDim, g, s, bc, cfg, k, pat)
        p = f"it{k + 1}_"
        for key, ref in (("U", "U"), ("V", "V"), ("T", "sst")):
            assert colrel(s[key], g[p + ref]) < (1e-12 if nDim == 2 else 1e-10), (k, key)
        np.testing.assert_allclose(s["rms"], g[p + "rms"], rtol=1e-12)


def test_outer_iterations_vs_reference(it9):
    g = it9
    nDim = int(g["dims"][0])
    m = O.Mechanism(g)
    cfg, bc, s = iteration_cfg(g)
    pat = (g["bsr_row_ptr"], g["bsr_col"])
    for k in range(n_iters(g) if nDim == 2 else len(ITER_TOL3)):
        s = O.outer_iteration(m, nDim, g, s, bc, cfg, k, pat)
        p, tol = f"it{k + 1}_", (ITER_TOL if nDim == 2 else ITER_TOL3)[k + 1]
        assert colrel(s["U"], g[p + "U"]) < tol, k
        assert colrel(s["V"], g[p + "V"]) < tol, k
        assert colrel(s["T"], g[p + "sst"]) < tol, k
        assert np.abs(s["mut"] - g[p + "mut"]).max() / np.abs(g[p + "mut"]).max() < tol * 100
        np.testing.assert_allclose(s["rms"], g[p + "rms"], rtol=tol * 100)
        np.testing.assert_allclose(s["sst_rms"], g[p + "sst_rms"], rtol=tol * 100)


def test_ignition_branch_of_set_primitive():
    """SetPrimitive_Variables' ignition branch (solver_direct_reactive.cpp:1013-1024) on the reference's stage-1
    start (golden ig9: no_chem.dat under my_combustion_first_chem_PaSR.cfg): while ExtIter < IGNITION_ITER every
    point with Y_fuel > 0.4, Y_O2 > 0.2 and T < 1700 K gets T = 1700 K in its record, and only T (pressure, enthalpy,
    sound speed, derivatives and transport keep the secant's temperature: the reference record it_V0 bitwise);
    from IGNITION_ITER on nothing changes."""
    g = golden("ig9")
    m = O.Mechanism(g)
    nDim = int(g["dims"][0])
    cfg, _, st = iteration_cfg(g)
    V0 = g["it_V0"]
    hot = V0[:, 0] == 1700.0
    assert hot.sum() == 1283
    prm = list(cfg["p2v"])
    o = O.set_primitive(m, nDim, g["it_U0"], V0, g["it_sst0"][:, 0].copy(), g["it_mut0"], prm)
    assert np.array_equal(o["V"], V0)
    prm_late = list(prm)
    prm_late[10] = 8000.0  # ExtIter == IGNITION_ITER: branch off
    o2 = O.set_primitive(m, nDim, g["it_U0"], V0, g["it_sst0"][:, 0].copy(), g["it_mut0"], prm_late)
    assert np.array_equal(o2["V"][~hot], V0[~hot]) and np.all(o2["V"][hot, 0] != 1700.0)
    assert np.array_equal(o2["V"][hot, 1:], V0[hot, 1:]) and np.array_equal(o2["dPdU"], o["dPdU"])


@pytest.mark.parametrize("case", ["lam4", "sup4"])
def test_laminar_outer_iterations_vs_reference(case):
    """Round 6: the laminar REACTIVE_NAVIER_STOKES outer iteration (KIND_TURB_MODEL= NONE, golden lam4: the flow's
    MultiGrid_Iteration alone, iteration_structure.cpp:531-534) restated: each reference iteration from its own state,
    then both chained. sup4: both jet inlets MARKER_SUPERSONIC_INLET and the outlet MARKER_SUPERSONIC_OUTLET
    (BC_Supersonic_Inlet / BC_Supersonic_Outlet, solver_direct_reactive.cpp:2998-3206 / :3681-3800)."""
    g = golden(case)
    nDim = int(g["dims"][0])
    m = O.Mechanism(g)
    cfg, bc, s0 = iteration_cfg(g)
    assert cfg["rans"] is False
    pat = (g["bsr_row_ptr"], g["bsr_col"])
    for chained in (False, True):
        s = s0
        for k in range(2):
            if not chained and k > 0:
                p = f"it{k}_"
                s = dict(U=g[p + "U"], V=g[p + "V"], Uold=g[p + "Uold"])
            s = O.outer_iteration(m, nDim, g, s, bc, cfg, k, pat)
            p = f"it{k + 1}_"
            assert colrel(s["U"], g[p + "U"]) < (1e-12 if not chained else ITER_TOL[k + 1]), (chained, k)
            assert colrel(s["V"], g[p + "V"]) < (1e-12 if not chained else ITER_TOL[k + 1]), (chained, k)
            np.testing.assert_allclose(s["rms"], g[p + "rms"], rtol=1e-12)
            assert "T" not in s
