"""next-1: CReactiveEulerSolver::SetPrimitive_Variables (Cons2PrimVar secant/bisection from the previous T,
Cp, dT/dU, dP/dU, mu, kappa, Dij, eddy viscosity) — the CPU oracle against the reference's own call after
one reference update (mini9: a fraction of the implicit update; jet9w: the whole update). CPU only."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KEYS = (("V", "p2v_V"), ("dPdU", "p2v_dPdU"), ("dTdU", "p2v_dTdU"), ("mu", "p2v_mu"), ("kappa", "p2v_kappa"),
        ("Dij", "p2v_Dij"), ("eddy", "p2v_eddy"), ("cp", "p2v_cp"), ("U", "p2v_U_after"))


@pytest.mark.parametrize("case", ["mini9", "jet9w", "mini3d", "fp3"])
def test_set_primitive_bitwise(case):
    g = dict(np.load(os.path.join(GOLD, case + ".npz")))
    m = O.Mechanism(g)
    o = O.set_primitive(m, int(g["dims"][0]), g["p2v_U"], g["p2v_V_before"], g["p2v_tke"], g["p2v_mut"], O.p2v_params(g))
    assert o["nonphys"] == int(g["p2v_params"][0])
    for k, gk in KEYS:
        assert np.array_equal(o[k], g[gk]), k
    # the secant started from the previous temperature and moved (history dependence is exercised)
    assert np.abs(g["p2v_V"][:, 0] - g["p2v_V_before"][:, 0]).max() > 1e-3


def test_set_primitive_edge_cases():
    """Negative partial density -> clamped to 1e-30 and counted non-physical; a start outside the property
    tables -> the bisection fallback still lands on the reference's temperature."""
    g = dict(np.load(os.path.join(GOLD, "mini9.npz")))
    m = O.Mechanism(g)
    U = g["p2v_U"][:4].copy()
    V0 = g["p2v_V_before"][:4].copy()
    U[0, 7] = -1e-12
    V0[1, 0] = 7000.0  # secant start above TEMPERATURE_MAX: ComputeEnthalpy throws out_of_range
    o = O.set_primitive(m, 2, U, V0, g["p2v_tke"][:4], g["p2v_mut"][:4], O.p2v_params(g))
    assert o["nonphys"] >= 1 and o["U"][0, 7] == 1e-30
    assert abs(o["V"][1, 0] - g["p2v_V"][1, 0]) < 1e-2  # bisection tolerance (Btol = 1e-4 on f)
