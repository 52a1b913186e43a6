"""next-1 on the device: SetPrimitive_Variables (k_set_primitive) against the reference's own call after a
reference update (golden p2v_* arrays), and a device-resident outer iteration (update -> primitives ->
residual) against the oracle. Requires an MI355X.

Bars: the primitive record, dP/dU, dT/dU, mu, kappa, eddy viscosity and the clamped U bitwise (same IEEE
operations; the mechanism's pow/sqrt/cbrt constants are evaluated on the host with the reference's libm);
Dij within 1e-14 and bitwise at >= 99 % of the points (the device's correctly rounded T^1.75 against the host
libm's pow, itself misrounded at ~0.07 % of temperatures)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.parity import assert_close
from tests.rxpkg import rx, synth
from tests.test_gpu_parity import golden, make_solver

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["mini9", "jet9w", "mini3d", "fp3"])
def test_set_primitive_vs_reference(case):
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=True)
    s.upload("U", g["p2v_U"])
    s.upload("V", g["p2v_V_before"])
    s.upload("TKE", g["p2v_tke"])
    s.upload("MUT", g["p2v_mut"])
    n = s.SetPrimitive_Variables(count=True)
    assert n == int(g["p2v_params"][0])
    N = len(g["p2v_U"])
    for f, k, shape in (("V", "p2v_V", (N, nPV)), ("DPDU", "p2v_dPdU", (N, nVar)), ("DTDU", "p2v_dTdU", (N, nVar)),
                        ("MU", "p2v_mu", (N,)), ("KAPPA", "p2v_kappa", (N,)), ("EDDY", "p2v_eddy", (N,)),
                        ("U", "p2v_U_after", (N, nVar))):
        assert np.array_equal(s.download(f).reshape(shape), g[k]), f
    D = s.download("DIJ").reshape(N, ns, ns)
    assert_close(D, g["p2v_Dij"], rtol=1e-14, what="Dij")
    assert np.mean(np.all(D == g["p2v_Dij"], axis=(1, 2))) >= 0.99, "Dij bitwise"
    s.close()


def test_device_resident_iteration_vs_oracle():
    """Implicit update -> SetPrimitive_Variables -> next residual, all on the device, against the oracle."""
    mesh, st, mech_arrays, kw = synth.jet_case(40, 16, n_species=7)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays), rx.default_cfg(implicit=1, lin_prec=1, cfl=0.5, **kw))
    s.set_state(st)
    s.SetPrimitive_Gradient_LS()
    s.SetTime_Step()
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    s.ImplicitEuler_Iteration()
    U1 = s.download("U").reshape(len(st["V"]), -1)
    s.SetPrimitive_Variables()
    s.sync()
    om = O.Mechanism(mech_arrays)
    prm = [200.0, 6000.0, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0]
    o = O.set_primitive(om, 2, U1, st["V"], st["turb_k"], st["mu_t"], prm)
    assert o["nonphys"] >= 0
    N = len(st["V"])
    assert np.array_equal(s.download("V").reshape(N, -1), o["V"])
    assert np.array_equal(s.download("DTDU").reshape(N, -1), o["dTdU"])
    assert np.array_equal(s.download("MU"), o["mu"])
    # the next residual evaluation reads the refreshed records
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    r, _, _ = O.ausm_edges(2, 7, mesh["edges"], mesh["edge_normal"], o["V"], o["dPdU"], kw["mach_inf"], False)
    R = np.zeros((N, r.shape[1]))
    for e, (i, j) in enumerate(mesh["edges"]):
        R[i] += r[e]
        R[j] -= r[e]
    assert np.array_equal(s.download("RES").reshape(N, -1), R)
    s.close()


def _iteration_fields(shared, monkeypatch):
    monkeypatch.setenv("RX_SPLINE_SHARED", "1" if shared else "0")  # read when the mechanism is uploaded
    mesh, st, mech_arrays, kw = synth.jet_case(40, 16, n_species=7)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays), rx.default_cfg(implicit=1, lin_prec=1, cfl=0.5, **kw))
    s.set_state(st)
    s.SetPrimitive_Gradient_LS()
    s.SetTime_Step()
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    out = {"RES": s.download("RES")}
    s.ImplicitEuler_Iteration()
    s.SetPrimitive_Variables()
    s.sync()
    for f in ("U", "V", "DPDU", "DTDU", "MU", "KAPPA", "DIJ"):
        out[f] = s.download(f)
    s.close()
    return out


def test_shared_grid_spline_matches_per_row(monkeypatch):
    """The spline interval searched once per temperature (every table on one grid: DevMech::xshared, rx_device.h
    spline_at / spline_k) against the per-row search (RX_SPLINE_SHARED=0): the secant's enthalpies, Cp, H, mu,
    kappa, the viscous flux's H and Cp rows and the source's Gibbs energies, through one implicit outer iteration
    (residual, solve, primitives), bitwise."""
    a = _iteration_fields(True, monkeypatch)
    b = _iteration_fields(False, monkeypatch)
    for f in a:
        assert np.array_equal(a[f], b[f]), f
