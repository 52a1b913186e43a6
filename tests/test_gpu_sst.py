"""SST turbulence solver on the device (SURVEY §8 a14 + next-2): librx.so through the C ABI against the
reference's own outputs (golden mini9: the turbulent solver's loops, implicit step and Postprocessing)
and against the CPU oracle on larger partitioned synthetic jets. Requires an MI355X.

Bars: gradient, residual loops, Jacobian and system are bitwise the reference's (no transcendental on
that path); StrainMag and the blending functions (tanh, pow) within 1e-12 relative; FGMRES bitwise the
oracle in the device's inner-product order and within 1e-10 of the reference's solution normwise."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.parity import assert_close, per_column_close
from tests.rxpkg import rx, synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
MESH_KEYS = ("edges", "edge_normal", "coord", "volume", "nbr_ptr", "nbr", "bvertex", "bvertex_normal",
             "wall_distance")


def golden_solvers(prec, case="mini9"):
    g = dict(np.load(os.path.join(GOLD, case + ".npz")))
    mesh = {k: g[k] for k in MESH_KEYS}
    kw = dict(mach_inf=float(g["mach_inf"][0]), prandtl_turb=float(g["visc_params"][1]),
              lewis_turb=float(g["visc_params"][2]), c_mu=float(g["src_params"][0]), pasr_lb=float(g["src_params"][1]))
    lp = 1 if prec == "ilu" else 0
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(g), rx.default_cfg(implicit=1, lin_prec=lp, **kw))
    s.set_state(g)
    s.upload("DT", g["dt"])
    t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg(lin_prec=lp))
    t.set_state(g["sst_sol"], g["wall_distance"], g["sst_F1"], g["sst_F2"], g["sst_CDkw"])
    return g, s, t


@pytest.mark.parametrize("case", ["mini9", "mini3d"])
@pytest.mark.parametrize("prec", ["lusgs", "ilu"])
def test_sst_iteration_vs_reference(prec, case):
    g, s, t = golden_solvers(prec, case)
    N = len(g["V"])
    nDim = int(g["dims"][0])
    s.SetStrainMag()
    s.sync()
    assert_close(s.download("STRAIN"), g["strain_mag"], rtol=1e-14, what="StrainMag")
    t.Preprocessing()
    t.sync()
    assert np.array_equal(t.download("GRAD").reshape(N, 2, nDim), g["sst_grad_ls"]), "LS gradient of (k, omega)"
    t.Upwind_Residual()
    t.sync()
    assert np.array_equal(t.download("RES").reshape(N, 2), g["sst_loop_upw_res"]), "upwind loop"
    t.Viscous_Residual()
    t.sync()
    assert np.array_equal(t.download("RES").reshape(N, 2), g["sst_loop_upw_visc_res"]), "viscous loop"
    t.Source_Residual()
    t.sync()
    R = t.download("RES").reshape(N, 2)
    per_column_close(R, g["sst_loop_total_res"], rtol=1e-13, what="source loop")
    J = t.download("JAC").reshape(-1, 2, 2)
    assert_close(J, g["sst_bsr_jac_residual"], rtol=1e-13, floor=1e-12, what="SST Jacobian")
    rms, it = t.ImplicitEuler_Iteration()
    sfx = "_ilu" if prec == "ilu" else ""
    assert_close(t.download("JAC").reshape(-1, 2, 2), g["sst_bsr_system"], rtol=1e-13, floor=1e-12,
                 what="SST system")
    per_column_close(t.download("RHS").reshape(N, 2), g["sst_sys_rhs"], rtol=1e-13, what="SST rhs")
    per_column_close(t.download("SOL").reshape(N, 2), g["sst_lin_sol" + sfx], floor=1e-3, what="SST dU")
    per_column_close(t.download("U").reshape(N, 2), g["sst_new_sol" + sfx], what="SST (k, omega)")
    assert_close(rms, g["sst_rms" + sfx], what="SST RMS")
    t.Postprocessing()
    t.sync()
    assert_close(t.download("MUT"), g["sst_post_mut" + sfx], what="post mu_t")
    assert_close(t.download("F1"), g["sst_post_F1" + sfx], what="post F1")
    assert_close(t.download("F2"), g["sst_post_F2" + sfx], what="post F2")
    assert_close(t.download("CDKW"), g["sst_post_CDkw" + sfx], what="post CDkw")
    # the flow context now reads the turbulent fields the SST solver produced (MANGOTURB coupling)
    T = t.download("U").reshape(N, 2)
    assert np.array_equal(s.download("TKE"), T[:, 0]) and np.array_equal(s.download("OMEGA"), T[:, 1])
    assert np.array_equal(s.download("MUT"), t.download("MUT"))
    assert np.array_equal(s.download("EDDY"), t.download("MUT"))
    assert np.array_equal(s.download("GRADK").reshape(N, nDim), t.download("GRAD").reshape(N, 2, nDim)[:, 0])
    s.close()


@pytest.mark.parametrize("n_part", [1, 8])
@pytest.mark.parametrize("prec", ["ilu", "lusgs"])
def test_sst_step_vs_oracle(n_part, prec):
    """Whole SST iteration on a partitioned synthetic jet against the oracle's restatement."""
    mesh, st, mech_arrays, kw = synth.jet_case(48, 20, n_species=7, n_part=n_part)
    lp = 1 if prec == "ilu" else 0
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays), rx.default_cfg(implicit=1, lin_prec=lp, **kw))
    s.set_state(st)
    s.SetPrimitive_Gradient_LS()
    s.SetStrainMag()
    s.SetTime_Step()
    s.sync()
    G, strain, dt = s.download("GRAD").reshape(len(st["V"]), -1, 2), s.download("STRAIN"), s.download("DT")
    t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg(lin_prec=lp))
    t.set_state(st["sst_sol"], mesh["wall_distance"], st["sst_F1"], st["sst_F2"], st["sst_CDkw"])
    t.Preprocessing()
    t.Upwind_Residual()
    t.Viscous_Residual()
    t.Source_Residual()
    rms, it = t.ImplicitEuler_Iteration()
    t.Postprocessing()
    t.sync()
    flow = dict(V=st["V"], grad=G, mu=st["mu"], eddy=st["eddy_visc_flow"], strain=strain)
    pattern = O.bsr_pattern(len(st["V"]), mesh["edges"])
    pp = mesh["part_ptr"]
    with O.dot_order("device"):
        Td, info = O.sst_step(2, mesh, flow, st["sst_sol"], None, st["sst_F1"], st["sst_F2"], st["sst_CDkw"], dt,
                              dict(lin_tol=1e-6, lin_iter=5), pattern=pattern, part_ptr=pp, prec=prec)
    Tr, info_r = O.sst_step(2, mesh, flow, st["sst_sol"], None, st["sst_F1"], st["sst_F2"], st["sst_CDkw"], dt,
                            dict(lin_tol=1e-6, lin_iter=5), pattern=pattern, part_ptr=pp, prec=prec)
    N = len(st["V"])
    assert it == info["lin_iters"]
    assert np.array_equal(t.download("RHS").reshape(N, 2), info["rhs"])
    assert np.array_equal(t.download("JAC").reshape(-1, 2, 2), info["jac"])
    assert np.array_equal(t.download("SOL").reshape(N, 2), info["sol"].reshape(N, 2)), "FGMRES (device dot order)"
    assert np.array_equal(t.download("U").reshape(N, 2), Td)
    per_column_close(t.download("U").reshape(N, 2), Tr, rtol=1e-8, what="(k, omega) vs reference dot order")
    assert_close(rms, info["rms"], what="RMS")
    assert_close(t.download("MUT"), info["mut"], what="mu_t")
    assert_close(t.download("F1"), info["F1"], what="F1")
    s.close()


def _split_run(split, monkeypatch):
    if split is None:
        monkeypatch.delenv("RX_FG_SPLIT", raising=False)
    else:
        monkeypatch.setenv("RX_FG_SPLIT", str(split))
    mesh, st, mech_arrays, kw = synth.jet_case(48, 20, n_species=7, n_part=8)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays), rx.default_cfg(implicit=1, lin_prec=1, **kw))
    s.set_state(st)
    t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg(lin_prec=1))
    t.set_state(st["sst_sol"], mesh["wall_distance"], st["sst_F1"], st["sst_F2"], st["sst_CDkw"])
    out = []
    for _ in range(3):
        s.SetPrimitive_Gradient_LS()
        s.SetStrainMag()
        s.SetTime_Step()
        t.Preprocessing()
        t.Upwind_Residual()
        t.Viscous_Residual()
        t.Source_Residual()
        rms_t, it_t = t.ImplicitEuler_Iteration()
        t.Postprocessing()
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.Viscous_Residual()
        s.Source_Residual()
        rms_f, it_f = s.ImplicitEuler_Iteration()
        s.SetPrimitive_Variables()
        s.sync()
        out.append((it_t, it_f, list(rms_t), list(rms_f), t.download("U"), t.download("SOL"), s.download("U"),
                    s.download("SOL")))
    s.close()
    return out


def test_fgmres_split_solve_bitwise(monkeypatch):
    """The FGMRES solve enqueued in two parts with the host's stop check between them (implicit_solve: the split at
    the previous solve's iteration count, RX_FG_SPLIT=c fixed, 0 off) runs the kernels of the whole solve or skips
    only launches that would return at once: three flow + SST outer iterations bitwise equal for the whole solve,
    the adaptive split, a split after 1 iteration (the continuing tail) and after 2."""
    ref = _split_run(0, monkeypatch)
    assert any(r[0] < 5 for r in ref), "the SST solve stops early (the split is exercised)"
    for split in (None, 1, 2):
        got = _split_run(split, monkeypatch)
        for a, b in zip(ref, got):
            assert a[0] == b[0] and a[1] == b[1], (split, a[:2], b[:2])
            assert a[2] == b[2] and a[3] == b[3], split
            for x, y in zip(a[4:], b[4:]):
                assert np.array_equal(x, y), split
