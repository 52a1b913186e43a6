"""a2 second-order branch (MUSCL reconstruction + limiter, solver_direct_reactive.cpp:2554-2729): the CPU
oracle against the reference's own Upwind_Residual loop on its jet mesh with the converged PaSR state
(jet9w window, cfg 2ND_ORDER_LIMITER, implicit). CPU only."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def muscl_loop(g, edge_res, Ji, Jj):
    """Reference scatter of the upwind loop (:2759-2772) for a window: residual + sampled Jacobian rows."""
    N, nVar = g["V"].shape[0], edge_res.shape[1]
    R = np.zeros((N, nVar))
    rows = {int(r): q for q, r in enumerate(g["muscl_jac_rows"])}
    cols = g["muscl_jac_cols"]
    J = np.zeros_like(g["muscl_jac"])

    def add(r, c, blk, sgn):
        if r in rows:
            q = rows[r]
            k = int(np.nonzero(cols[q] == c)[0][0])
            J[q, k] = J[q, k] + blk if sgn > 0 else J[q, k] - blk

    for e, (i, j) in enumerate(g["edges"]):
        R[i] += edge_res[e]
        R[j] -= edge_res[e]
        add(i, i, Ji[e], 1)
        add(i, j, Jj[e], 1)
        add(j, i, Ji[e], -1)
        add(j, j, Jj[e], -1)
    return R, J


@pytest.mark.parametrize("case", ["jet9w", "muscl3d", "fp3"])
def test_muscl_upwind_loop_bitwise(case):
    """jet9w: the reference's 2-D jet window (2ND_ORDER_LIMITER); muscl3d: the 3-D extruded jet, every point;
    fp3: the flat-plate window, 2ND_ORDER (no limiter)."""
    g = dict(np.load(os.path.join(GOLD, case + ".npz")))
    nDim, ns = int(g["dims"][0]), int(g["dims"][4])
    limited = int(g["muscl_params"][0]) == 2  # SECOND_ORDER_LIMITER (1: SECOND_ORDER)
    m = O.Mechanism(g)
    r, Ji, Jj = O.muscl_edges(m, nDim, g["edges"], g["edge_normal"], g["coord"], g["V"], g["dPdU"], g["grad_prim"],
                              g["limiter_out"] if limited else None, g["muscl_params"][1:], g["mach_inf"][0], True)
    R, J = muscl_loop(g, r, Ji, Jj)
    ii = np.nonzero(g["interior"])[0] if "interior" in g else np.arange(len(g["V"]))
    assert np.array_equal(R[ii], g["muscl_loop_res"][ii])
    assert np.array_equal(J, g["muscl_jac"])
    # the reconstruction changes the flux (the check is not vacuous)
    r1, _, _ = O.ausm_edges(nDim, ns, g["edges"], g["edge_normal"], g["V"], g["dPdU"], g["mach_inf"][0], False)
    assert np.abs(r1 - r).max() > 1e-6 * np.abs(r).max()


def test_muscl_upwind_loop_barth_bitwise():
    """bj9: the 2-D mini jet with 2ND_ORDER_LIMITER + BARTH_JESPERSEN; the reconstruction reads the oracle's own
    Barth-Jespersen limiter, so this pins limiter and loop together against the reference's residual."""
    g = dict(np.load(os.path.join(GOLD, "bj9.npz")))
    nDim, ns = int(g["dims"][0]), int(g["dims"][4])
    m = O.Mechanism(g)
    L = O.limiter_barth(nDim, ns, g["edges"], g["coord"], g["V"], g["grad_prim"])
    r, _, _ = O.muscl_edges(m, nDim, g["edges"], g["edge_normal"], g["coord"], g["V"], g["dPdU"], g["grad_prim"], L,
                            g["muscl_params"][1:], g["mach_inf"][0], True)
    R = np.zeros_like(g["muscl_loop_res"])
    for e, (i, j) in enumerate(g["edges"]):
        R[i] += r[e]
        R[j] -= r[e]
    assert np.array_equal(R, g["muscl_loop_res"])
