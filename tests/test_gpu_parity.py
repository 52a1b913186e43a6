"""HIP path (librx.so through the C ABI) against the golden vectors of the compiled reference and
against the CPU oracle on larger synthetic meshes. Requires an MI355X.

Tolerance: 1e-10 relative (north star), see tests/parity.py for the block-relative metric used on
components that cancel to solver tolerance.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.parity import assert_close, per_column_close
from tests.rxpkg import rx, synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def golden(case):
    g = dict(np.load(os.path.join(GOLD, case + ".npz")))
    g.setdefault("eddy_visc_flow", g["mu_t"])
    return g


def make_solver(g, implicit, lin_prec=1, cfl=None, spatial_order=0, slope_limiter=0):
    nDim, nVar, nPV, nG, ns, imp, rans = [int(x) for x in g["dims"]]
    mesh = {k: g[k] for k in ("edges", "edge_normal", "coord", "volume", "nbr_ptr", "nbr")}
    mesh["bvertex"] = g.get("bvertex", np.zeros((0, 3), dtype=np.int64))
    mesh["bvertex_normal"] = g.get("bvertex_normal", np.zeros((0, 2)))
    mech = rx.Mechanism(g)
    kw = dict(mach_inf=float(g["mach_inf"][0]), prandtl_turb=float(g["visc_params"][1]),
              lewis_turb=float(g["visc_params"][2]), c_mu=float(g["src_params"][0]),
              pasr_lb=float(g["src_params"][1]), implicit=int(implicit), lin_prec=lin_prec,
              spatial_order=spatial_order, slope_limiter=slope_limiter)
    if "limiter_params" in g:
        kw.update(ref_elem_length=float(g["limiter_params"][0]), limiter_coeff=float(g["limiter_params"][1]))
    if "dt_params" in g:
        kw.update(cfl=float(g["dt_params"][0]), max_delta_time=float(g["dt_params"][1]),
                  prandtl_lam=float(g["dt_params"][2]))
    if cfl is not None:
        kw["cfl"] = cfl
    s = rx.ReactiveNSSolver(mesh, mech, rx.default_cfg(**kw))
    s.set_state(g)
    return s, (nDim, nVar, nPV, nG, ns)


@pytest.mark.parametrize("case", ["mini9", "jet9w", "mini3d", "muscl3d", "fp3"])
def test_gradient_and_limiter(case):
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=False)
    s.SetPrimitive_Gradient_LS()
    s.sync()
    G = s.download("GRAD").reshape(len(g["V"]), nG, nDim)
    pts = np.nonzero(g["interior"])[0] if "interior" in g else np.arange(len(g["V"]))
    if "grad_lsq_out" in g:
        assert_close(G[pts], g["grad_lsq_out"][pts], what="LSQ gradient (HIP vs reference)")
    else:
        assert_close(G[pts], g["grad_prim"][pts], what="LSQ gradient (HIP vs reference)")
    if case in ("jet9w", "muscl3d"):  # 2ND_ORDER_LIMITER runs (the 1st-order dumps carry no limiter state)
        s.upload("GRAD", g["grad_prim"])
        s.SetPrimitive_Limiter()
        s.sync()
        L = s.download("LIMITER").reshape(-1, nDim + 2)
        it = g["interior"] if "interior" in g else slice(None)
        assert_close(L[it], g["limiter_out"][it], what="Venkatakrishnan limiter (HIP vs reference)")
    s.close()


@pytest.mark.parametrize("case", ["mini9", "mini3d"])
def test_gradient_green_gauss(case):
    """NUM_METHOD_GRAD= GREEN_GAUSS: CReactiveNSSolver::SetPrimitive_Gradient_GG (solver_direct_reactive.cpp:
    4784-4880, node 0's species on both sides of an edge, / Volume) against the oracle's edge-loop restatement
    (the device accumulates each point's edges in edge order, then its boundary vertices in marker order), and
    the SST's SetSolution_Gradient_GG (solver_structure.cpp:519-578, / (Volume + EPS)) of (k, omega)."""
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=False)
    N = len(g["V"])
    s.SetPrimitive_Gradient_GG()
    s.sync()
    G = s.download("GRAD").reshape(N, nG, nDim)
    ref = O.grad_gg(O.Mechanism(g), nDim, g, g["V"])
    per_column_close(G.reshape(N, -1), ref.reshape(N, -1), rtol=1e-13, what="Green-Gauss gradient (HIP vs oracle)")
    s.close()


@pytest.mark.parametrize("case", ["bj9", "muscl3d", "jet9w"])
def test_limiter_barth(case):
    """a13 Barth-Jespersen branch on the device: bitwise against the reference's own limiter (bj9, 2-D,
    SLOPE_LIMITER_FLOW= BARTH_JESPERSEN) and against the oracle's restatement on the 3-D / jet-window records."""
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=False, spatial_order=2, slope_limiter=1)
    s.upload("GRAD", g["grad_prim"])
    s.SetPrimitive_Limiter()
    s.sync()
    L = s.download("LIMITER").reshape(-1, nDim + 2)
    ref = g["limiter_out"] if case == "bj9" else O.limiter_barth(nDim, ns, g["edges"], g["coord"], g["V"],
                                                                 g["grad_prim"])
    assert np.array_equal(L, ref)
    if case == "bj9":  # the MUSCL loop on the device limiter against the reference's residual
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.sync()
        assert np.array_equal(s.download("RES").reshape(-1, nVar), g["muscl_loop_res"])
    s.close()


@pytest.mark.parametrize("case", ["mini9", "mini3d"])
def test_explicit_residual_loops_and_time_step(case):
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=False)
    F = nDim + 2  # flow rows rho, rho u.., rho E; species rows after
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    assert_close(s.download("RES").reshape(-1, nVar), g["loop_upwind_res"], what="Upwind_Residual (HIP)")
    s.Viscous_Residual()
    s.sync()
    R = s.download("RES").reshape(-1, nVar)
    ref = g["loop_upwind_visc_res"]
    assert_close(R[:, :F], ref[:, :F], what="Upwind+Viscous (HIP) flow rows")
    blk = np.abs(ref[:, F:]).max()
    assert np.max(np.abs(R[:, F:] - ref[:, F:])) <= 1e-10 * blk
    s.Source_Residual()
    s.sync()
    R = s.download("RES").reshape(-1, nVar)
    ref = g["loop_total_res"]
    assert_close(R[:, :F], ref[:, :F], what="total residual (HIP) flow rows")
    assert np.max(np.abs(R[:, F:] - ref[:, F:])) <= 1e-10 * np.abs(ref[:, F:]).max()
    s.SetTime_Step()
    s.sync()
    assert_close(s.download("DT"), g["dt"], what="SetTime_Step dt (HIP)")
    assert_close(s.download("LAMBDA_VISC"), g["lambda_visc"], what="viscous spectral radius (HIP)")
    s.close()


@pytest.mark.parametrize("case", ["jet9w", "fp3"])
def test_jet_window_edge_fluxes_vs_reference(case):
    """Per-edge AUSM / viscous fluxes of the reference jet window (and of the flat-plate boundary-layer window),
    gathered per node by the HIP path, against the same gather of the reference's own per-edge fluxes."""
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=False)
    N = len(g["V"])
    ref_c = np.zeros((N, nVar))
    ref_v = np.zeros((N, nVar))
    for e, (i, j) in enumerate(g["edges"]):
        ref_c[i] += g["conv_res"][e]
        ref_c[j] -= g["conv_res"][e]
        ref_v[i] -= g["visc_res"][e]
        ref_v[j] += g["visc_res"][e]
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    assert_close(s.download("RES").reshape(-1, nVar), ref_c, floor=1e-9, what="AUSM gather, jet window")
    s.Preprocessing_zero()
    s.Viscous_Residual()
    s.sync()
    R = s.download("RES").reshape(-1, nVar)
    assert_close(R[:, 1:4], ref_v[:, 1:4], floor=1e-9, what="viscous gather, jet window (flow rows)")
    sc = np.abs(ref_v[:, 4:]).max(axis=1, keepdims=True)
    sc = np.where(sc == 0.0, 1.0, sc)
    assert np.max(np.abs(R[:, 4:] - ref_v[:, 4:]) / sc) <= 1e-10
    s.close()


@pytest.mark.parametrize("case", ["mini9", "mini3d"])
def test_implicit_assembly_matches_reference_jacobian(case):
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=True)
    F = nDim + 2
    s.upload("DT", g["dt"])
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    s.sync()
    R = s.download("RES").reshape(-1, nVar)
    ref = g["loop_total_res"]
    assert_close(R[:, :F], ref[:, :F], what="implicit-path residual flow rows")
    assert np.max(np.abs(R[:, F:] - ref[:, F:])) <= 1e-10 * np.abs(ref[:, F:]).max()
    rp, col = s.bsr_pattern()
    assert np.array_equal(rp, g["bsr_row_ptr"]) and np.array_equal(col, g["bsr_col"])
    A = s.download("JAC").reshape(-1, nVar, nVar)
    Aref = g["bsr_system"].copy()
    diag = np.array([rp[i] + np.nonzero(col[rp[i]:rp[i + 1]] == i)[0][0] for i in range(len(rp) - 1)])
    Aref[diag] -= np.einsum("i,ab->iab", g["volume"] / g["dt"], np.eye(nVar))
    scale = np.abs(Aref).max(axis=(1, 2), keepdims=True)
    err = np.abs(A - Aref) / np.where(scale == 0, 1, scale)
    assert err.max() <= 1e-10, f"Jacobian block err {err.max():.3e}"
    s.close()


@pytest.mark.parametrize("case", ["mini9", "mini3d"])
@pytest.mark.parametrize("prec", ["lusgs", "ilu"])
def test_linear_algebra_matches_reference(prec, case):
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=True, lin_prec=(1 if prec == "ilu" else 0))
    # run the residual phases once so the context's Jacobian is marked assembled, then overwrite it
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    s.download("RES")
    s.upload("JAC", g["bsr_system"])
    s.upload("RHS", g["sys_rhs"])
    s.spmv("RHS", "SOL")
    s.sync()
    assert_close(s.download("SOL").reshape(-1, nVar), g["spmv_rhs"], what="BSR SpMV (HIP)")
    if prec == "lusgs":
        s.lusgs_apply("RHS", "SOL")
        s.sync()
        assert_close(s.download("SOL").reshape(-1, nVar), g["lusgs_rhs"], what="LU-SGS (HIP)")
        ref_x, info = g["fgmres_lusgs_x"], g["fgmres_lusgs_info"]
    else:
        s.ilu0_build()
        s.sync()
        F = s.download("ILU").reshape(-1, nVar, nVar)
        assert_close(F, g["ilu_factor"], floor=1e-9, what="ILU(0) factor (HIP)")
        s.ilu0_apply("RHS", "SOL")
        s.sync()
        assert_close(s.download("SOL").reshape(-1, nVar), g["ilu_rhs"], what="ILU(0) apply (HIP)")
        ref_x, info = g["fgmres_ilu_x"], g["fgmres_ilu_info"]
    s.upload("SOL", np.zeros_like(g["sys_rhs"]))
    it, res = s.fgmres(tol=float(info[2]), m=int(info[3]))
    assert it == int(info[0])
    x = s.download("SOL").reshape(-1, nVar)
    # Inner products are tree-reduced on the device and summed sequentially by the reference; the
    # Krylov basis amplifies that ULP-level difference, so the solution is compared normwise per
    # variable (|dx| <= 1e-10 * max|x_var|) and elementwise at 1e-8.
    per_column_close(x, ref_x, floor=1.0, what=f"FGMRES({prec}) (HIP), normwise")
    assert_close(x, ref_x, rtol=1e-8, what=f"FGMRES({prec}) (HIP), elementwise")
    s.close()


def test_ilu_field_needs_a_factor():
    """the per-edge viscous Jacobians share the ILU buffer, so after a new viscous sweep the
    field holds scratch, not a factor. rx_ilu0_apply and rx_download(ILU) then refuse with RX_ERR_STATE instead of
    sweeping over scratch; after the next ILU build both work again and give the same factor and apply."""
    g = golden("mini9")
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=True, lin_prec=1)
    s.upload("DT", g["dt"])

    def residual():
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.Viscous_Residual()
        s.Source_Residual()
        s.sync()

    residual()
    s.upload("RHS", g["sys_rhs"])
    with pytest.raises(rx.RxError, match="status 7"):  # never built
        s.ilu0_apply("RHS", "SOL")
    s.ilu0_build()
    F0 = s.download("ILU")
    s.ilu0_apply("RHS", "SOL")
    x0 = s.download("SOL")
    residual()  # a new residual: the viscous sweep writes its scratch into the ILU buffer
    with pytest.raises(rx.RxError, match="status 7"):
        s.ilu0_apply("RHS", "SOL")
    with pytest.raises(rx.RxError, match="status 7"):
        s.download("ILU")
    s.ilu0_build()
    assert np.array_equal(s.download("ILU"), F0)
    s.upload("SOL", np.zeros_like(x0))
    s.ilu0_apply("RHS", "SOL")
    assert np.array_equal(s.download("SOL"), x0)
    s.close()


@pytest.mark.parametrize("nx,ny", [(120, 40)])
def test_synthetic_jet_vs_oracle(nx, ny):
    """Larger mesh (resampled reacting records): HIP vs CPU oracle for every residual phase."""
    mesh, st, mech_arrays, kw = synth.jet_case(nx, ny)
    mech = rx.Mechanism(mech_arrays)
    omech = O.Mechanism(mech_arrays)
    ns, nDim = mech.ns, 2
    nVar, nG = ns + nDim + 2, ns + nDim + 2
    s = rx.ReactiveNSSolver(mesh, mech, rx.default_cfg(implicit=0, **kw))
    s.set_state(st)
    s.SetPrimitive_Gradient_LS()
    s.sync()
    G = s.download("GRAD").reshape(-1, nG, nDim)
    Go = O.grad_lsq(omech, nDim, np.arange(len(st["V"])), mesh["coord"], st["V"], mesh["nbr_ptr"], mesh["nbr"])
    assert_close(G, Go, floor=1e-9, what="LSQ gradient (HIP vs oracle)")
    s.upload("GRAD", Go)
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    s.sync()
    R = s.download("RES").reshape(-1, nVar)
    rc, _, _ = O.ausm_edges(nDim, ns, mesh["edges"], mesh["edge_normal"], st["V"], st["dPdU"], kw["mach_inf"], False)
    rv, _, _ = O.visc_edges(omech, nDim, mesh["edges"], mesh["edge_normal"], mesh["coord"], st["V"], Go, st["mu"],
                            st["kappa"], st["Dij"], st["dTdU"], st["turb_k"], st["mu_t"], st["sigma_k"],
                            st["grad_k"], True, False, [1, 1, 1, kw["prandtl_turb"], kw["lewis_turb"]])
    rs, _ = O.source_cells(omech, nDim, st["V"], st["dTdU"], mesh["volume"], st["turb_omega"], True, False,
                           [kw["c_mu"], kw["pasr_lb"], 1, 1, 1])
    Ro = np.zeros_like(R)
    for e, (i, j) in enumerate(mesh["edges"]):
        Ro[i] += rc[e]
        Ro[j] -= rc[e]
    for e, (i, j) in enumerate(mesh["edges"]):
        Ro[i] -= rv[e]
        Ro[j] += rv[e]
    Ro += rs
    assert_close(R[:, :4], Ro[:, :4], floor=1e-9, what="residual flow rows (HIP vs oracle)")
    sc = np.abs(Ro[:, 4:]).max()
    assert np.max(np.abs(R[:, 4:] - Ro[:, 4:])) <= 1e-10 * sc
    s.close()
