"""Pin the CPU oracle's SST turbulence restatement (SURVEY §8 a14 + next-2) against golden vectors from
the compiled reference (oracle/ref_harness: CUpwSca_TurbSST, CAvgGradCorrected_TurbSST,
CSourcePieceWise_TurbSST on the turbulent solver's own numerics; CTurbSolver loops,
ImplicitEuler_Iteration and CTurbSSTSolver::Postprocessing on mini9). CPU only."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(case):
    g = dict(np.load(os.path.join(GOLD, case + ".npz")))
    return g, [int(x) for x in g["dims"]]


@pytest.fixture(scope="module", params=["mini9", "jet9w", "mini3d", "fp3"])
def case(request):
    g, dims = load(request.param)
    return request.param, g, dims


def test_strain_mag(case):
    name, g, (nDim, *_r) = case
    assert np.array_equal(O.strain_mag(nDim, g["grad_prim"]), g["strain_mag"])


def test_sst_upwind(case):
    name, g, (nDim, *_r) = case
    r, Ji, Jj = O.sst_upwind(nDim, g["edges"], g["edge_normal"], g["V"], g["sst_sol"])
    assert np.array_equal(r, g["sst_upw_res"])
    assert np.array_equal(Ji, g["sst_upw_jac_i"]) and np.array_equal(Jj, g["sst_upw_jac_j"])


def test_sst_visc(case):
    name, g, (nDim, *_r) = case
    r, Ji, Jj = O.sst_visc(nDim, g["edges"], g["edge_normal"], g["coord"], g["V"], g["sst_sol"], g["sst_grad"],
                           g["sst_F1"], g["mu"], g["eddy_visc_flow"])
    assert np.array_equal(r, g["sst_visc_res"])
    assert np.array_equal(Ji, g["sst_visc_jac_i"]) and np.array_equal(Jj, g["sst_visc_jac_j"])


def test_sst_source(case):
    name, g, (nDim, *_r) = case
    r, J = O.sst_source(nDim, g["V"], g["grad_prim"], g["sst_sol"], g["volume"], g["wall_distance"], g["sst_F1"],
                        g["sst_F2"], g["sst_CDkw"], g["strain_mag"], g["eddy_visc_flow"])
    assert np.array_equal(r, g["sst_src_res"]) and np.array_equal(J, g["sst_src_jac"])


@pytest.mark.parametrize("name", ["mini9", "mini3d"])
def test_sst_gradient_and_blending(name):
    g, (nDim, *_r) = load(name)
    TG = O.sol_grad_ls(nDim, g["coord"], g["sst_sol"], g["nbr_ptr"], g["nbr"])
    assert np.array_equal(TG, g["sst_grad_ls"])
    assert np.array_equal(TG, g["sst_grad"])
    rho = g["V"][:, nDim + 2]
    F1, F2, CD, mt = O.sst_blending(nDim, g["sst_sol"], TG, rho, g["mu"], g["wall_distance"], g["strain_mag"])
    for a, k in ((F1, "sst_F1"), (F2, "sst_F2"), (CD, "sst_CDkw"), (mt, "mu_t")):
        assert np.array_equal(a, g[k]), k


@pytest.mark.parametrize("name", ["mini9", "mini3d"])
@pytest.mark.parametrize("prec", ["lusgs", "ilu"])
def test_sst_implicit_step(prec, name):
    """Loops, system and the whole turbulent implicit step + Postprocessing against the reference."""
    g, (nDim, *_r) = load(name)
    mesh = {k: g[k] for k in ("edges", "edge_normal", "coord", "volume", "nbr_ptr", "nbr", "wall_distance")}
    flow = dict(V=g["V"], grad=g["grad_prim"], mu=g["mu"], eddy=g["eddy_visc_flow"], strain=g["strain_mag"])
    cfg = dict(lin_tol=1e-6, lin_iter=5)
    T, info = O.sst_step(nDim, mesh, flow, g["sst_sol"], g["sst_grad"], g["sst_F1"], g["sst_F2"], g["sst_CDkw"],
                         g["dt"], cfg, prec=prec)
    # bitwise: residual loops (the golden loops exclude boundary conditions, as the device path), system,
    # rhs, FGMRES solution, updated (k, omega), RMS and the Postprocessing outputs
    sfx = "_ilu" if prec == "ilu" else ""
    for a, k in ((info["res"], "sst_loop_total_res"), (info["jac"], "sst_bsr_system"), (info["rhs"], "sst_sys_rhs"),
                 (info["sol"].reshape(-1, 2), "sst_lin_sol" + sfx), (T, "sst_new_sol" + sfx),
                 (info["rms"], "sst_rms" + sfx), (info["mut"], "sst_post_mut" + sfx), (info["F1"], "sst_post_F1" + sfx),
                 (info["F2"], "sst_post_F2" + sfx), (info["CDkw"], "sst_post_CDkw" + sfx),
                 (info["grad"], "sst_post_grad" + sfx)):
        assert np.array_equal(a, g[k]), k
