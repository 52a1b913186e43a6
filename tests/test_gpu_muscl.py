"""a2 second-order branch on the device (k_muscl_edge + the AUSM kernels on reconstructed edge states)
against the reference's own Upwind_Residual loop (jet9w: 2ND_ORDER_LIMITER, implicit) and the CPU
oracle on a synthetic jet. Requires an MI355X. Bar: bitwise (same IEEE operations, splines included)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.rxpkg import rx, synth
from tests.test_gpu_parity import golden, make_solver
from tests.test_oracle_muscl import muscl_loop

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["jet9w", "muscl3d", "fp3"])
@pytest.mark.parametrize("implicit", [1, 0])
def test_muscl_loop_vs_reference(implicit, case):
    """jet9w / muscl3d: SECOND_ORDER_LIMITER; fp3 (the flat plate): SECOND_ORDER, no limiter."""
    g = golden(case)
    order = int(g["muscl_params"][0])
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=implicit, spatial_order=order)
    s.upload("GRAD", g["grad_prim"])
    if order == 2:
        s.upload("LIMITER", g["limiter_out"])
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    R = s.download("RES").reshape(-1, nVar)
    ii = np.nonzero(g["interior"])[0] if "interior" in g else np.arange(len(g["V"]))
    assert np.array_equal(R[ii], g["muscl_loop_res"][ii])
    if implicit:
        rp, col = s.bsr_pattern()
        A = s.download("JAC").reshape(-1, nVar, nVar)
        for q, r in enumerate(g["muscl_jac_rows"]):
            for k, c in enumerate(g["muscl_jac_cols"][q]):
                if c < 0:
                    continue
                b = rp[r] + int(np.nonzero(col[rp[r]:rp[r + 1]] == c)[0][0])
                assert np.array_equal(A[b], g["muscl_jac"][q, k]), (r, c)
    s.close()


@pytest.mark.parametrize("order", [1, 2])
def test_muscl_vs_oracle_synthetic(order):
    mesh, st, mech_arrays, kw = synth.jet_case(48, 20, n_species=7)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays),
                            rx.default_cfg(implicit=1, spatial_order=order, **kw))
    s.set_state(st)
    s.SetPrimitive_Gradient_LS()
    s.SetPrimitive_Limiter()
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    N = len(st["V"])
    G = s.download("GRAD").reshape(N, -1, 2)
    L = s.download("LIMITER").reshape(N, -1)
    om = O.Mechanism(mech_arrays)
    r, Ji, Jj = O.muscl_edges(om, 2, mesh["edges"], mesh["edge_normal"], mesh["coord"], st["V"], st["dPdU"], G,
                              L if order == 2 else None, [1.0, 1.0, 1.0], kw["mach_inf"], True)
    rp, col = O.bsr_pattern(N, mesh["edges"])
    nVar = r.shape[1]
    R, A, _ = O.assemble(rp, col, mesh["edges"], r, Ji, Jj, None, None, None, None, None, mesh["volume"],
                         np.ones(N), nVar)
    assert np.array_equal(s.download("RES").reshape(N, nVar), R)
    s.close()


def test_explicit_rk_stages_vs_oracle():
    """ExplicitRK_Iteration (a18): three stages from the same Solution_Old (RK_ALPHA_COEFF 0.66667,
    0.66667, 1.0), residual re-evaluated between stages from the fixed node records."""
    g = golden("mini9")
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=False)
    s.upload("DT", g["dt"])
    U0 = g["U"].copy()
    for stage, alpha in enumerate((0.66667, 0.66667, 1.0)):
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.Viscous_Residual()
        s.Source_Residual()
        s.sync()
        R = s.download("RES").reshape(-1, nVar)
        rms = s.ExplicitRK_Iteration(stage, alpha)
        U = s.download("U").reshape(-1, nVar)
        assert np.array_equal(U, O.update_rk(U0, R, nDim, alpha, g["volume"], g["dt"])), f"stage {stage}"
        ref_rms = np.maximum(1e-32, np.sqrt((R ** 2).sum(axis=0) / len(R)))
        assert np.allclose(rms, ref_rms, rtol=1e-12, atol=0)
    s.close()
