"""CSysSolve::Solve's branches on the device (rx_linear_solve): BCGSTAB_LinSolver, RESTARTED_FGMRES, the JACOBI
preconditioner and the LU_SGS / Jacobi / ILU0 smoothers (Common/src/linear_solvers_structure.cpp:465-708,
matrix_structure.cpp:1230-1366, 1517-1835) against the CPU oracle on the implicit system of a partitioned synthetic
jet. Requires an MI355X.

Bars: bitwise equal to the oracle run with the device's inner-product order (O.dot_order("device")): solution,
iteration count and residual norm; the preconditioner sweeps and the vector updates are the reference's operations in
its order, only the inner products' summation order differs from the reference's sequential sums (the same bar as
test_gpu_partitions.test_partitioned_preconditioners_vs_oracle for FGMRES). Whole reference iterations with these
solvers against the reference itself: tests/test_gpu_bc.py (goldens ls*).
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.parity import assert_close
from tests.rxpkg import rx, synth
from tests.test_gpu_partitions import case, oracle_system

pytestmark = pytest.mark.gpu

PREC = {"lusgs": rx.PREC_LU_SGS, "ilu": rx.PREC_ILU, "jacobi": rx.PREC_JACOBI}
SOLVER = {"FGMRES": rx.LIN_FGMRES, "BCGSTAB": rx.LIN_BCGSTAB, "RESTARTED_FGMRES": rx.LIN_RESTARTED_FGMRES,
          "SMOOTHER_LUSGS": rx.LIN_SMOOTHER_LUSGS, "SMOOTHER_JACOBI": rx.LIN_SMOOTHER_JACOBI,
          "SMOOTHER_ILU0": rx.LIN_SMOOTHER_ILU}

CASES = [("BCGSTAB", "ilu"), ("BCGSTAB", "lusgs"), ("BCGSTAB", "jacobi"), ("FGMRES", "jacobi"),
         ("RESTARTED_FGMRES", "ilu"), ("RESTARTED_FGMRES", "jacobi"), ("SMOOTHER_LUSGS", "lusgs"),
         ("SMOOTHER_JACOBI", "lusgs"), ("SMOOTHER_ILU0", "lusgs")]


def system(n_part):
    ns = 7
    mesh, st, mech_arrays, kw, cfg = case(48, 20, n_part, ns)
    (rp, col), info, _ = oracle_system(mesh, st, mech_arrays, cfg, ns)
    return mesh, st, mech_arrays, kw, rp, col, info["jac"], info["rhs"].ravel()


@pytest.mark.parametrize("n_part", [1, 5])
@pytest.mark.parametrize("solver,prec", CASES)
def test_linear_solver_vs_oracle(solver, prec, n_part):
    mesh, st, mech_arrays, kw, rp, col, A, b = system(n_part)
    pp = mesh["part_ptr"]
    # RESTARTED_FGMRES: a loose tolerance, so the cycles stop early and the restart loop runs several
    tol, iters, restart = (0.05, 8, 2) if solver == "RESTARTED_FGMRES" else (1e-6, 5, 10)
    kw.update(lin_tol=tol, lin_iter=iters)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays),
                            rx.default_cfg(implicit=1, lin_prec=PREC[prec], lin_solver=SOLVER[solver],
                                           lin_restart=restart, **kw))
    s.set_state(st)
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    s.download("RES")  # mark the system assembled, then overwrite it with the oracle's
    s.upload("JAC", A)
    s.upload("RHS", b)
    s.upload("SOL", np.zeros_like(b))
    it, res = s.linear_solve()
    with O.dot_order("device"):
        x_o, it_o, res_o = O.lin_solve(rp, col, A, b, solver, prec, tol=tol, m=iters, restart=restart, part_ptr=pp)
    x = s.download("SOL").reshape(x_o.shape)
    assert it == it_o, (it, it_o)
    assert_close(x, x_o, rtol=0.0, what=f"{solver}({prec}) P={n_part} vs oracle in device dot order")
    assert res == res_o, (res, res_o)
    if solver == "RESTARTED_FGMRES":
        assert it > 5, it  # more than one cycle ran
    s.close()


@pytest.mark.parametrize("solver,prec", [("BCGSTAB", "ilu"), ("SMOOTHER_JACOBI", "lusgs"),
                                         ("RESTARTED_FGMRES", "lusgs")])
def test_implicit_step_with_solver_vs_oracle(solver, prec):
    """rx_implicit_euler with the branch (BCGSTAB / the smoothers replayed as a hipGraph, RESTARTED_FGMRES eagerly):
    the device's own assembled system (JAC with V/dt on the diagonal, RHS = -R) solved by the oracle's restatement of
    the same branch in the device's inner-product order gives the device's solution bitwise (the system itself is the
    device's: the oracle's assembly differs from it by the Stefan-Maxwell rounding, which BCGSTAB at CFL 5 amplifies
    to 1e-2); then a second step on the same state: the same solution bitwise."""
    mesh, st, mech_arrays, kw, rp, col, A, b = system(4)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays),
                            rx.default_cfg(implicit=1, lin_prec=PREC[prec], lin_solver=SOLVER[solver], **kw))
    s.set_state(st)
    out = []
    for _ in range(2):
        s.SetPrimitive_Gradient_LS()
        s.SetTime_Step()
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.Viscous_Residual()
        s.Source_Residual()
        rms, it = s.ImplicitEuler_Iteration()
        out.append((rms, it, s.download("SOL"), s.download("JAC"), s.download("RHS")))
    nv = s.nVar
    Ad = out[0][3].reshape(-1, nv, nv)
    with O.dot_order("device"):
        x_o, it_o, _ = O.lin_solve(rp, col, Ad, out[0][4], solver, prec, tol=kw.get("lin_tol", 1e-6),
                                   m=kw.get("lin_iter", 5), part_ptr=mesh["part_ptr"])
    assert out[0][1] == it_o
    assert_close(out[0][2], x_o.ravel(), rtol=0.0, what=f"{solver} step solution vs oracle on the device system")
    assert out[1][1] == out[0][1] and np.array_equal(out[1][0], out[0][0]) and np.array_equal(out[1][2], out[0][2])
    s.close()


def test_restarted_fgmres_stops_when_a_cycle_starts_converged():
    """a RESTARTED_FGMRES cycle that returns 0 iterations (FGMRES's start test, |r| < eps,
    linear_solvers_structure.cpp:367-370) leaves x unchanged, so the reference's cycle loop would spin (|b| >= 1: its
    tolerance only shrinks); the device stops there with RX_OK, x untouched, 0 iterations — it used to spin 4096
    host-synchronous cycles and report RX_ERR_DIVERGED. System: identity blocks, x0 = b (r = 0 exactly), |b| >> 1."""
    mesh, st, mech_arrays, kw, rp, col, A, b = system(1)
    nv = A.shape[1]
    eye = np.zeros_like(A)
    for i in range(len(rp) - 1):
        d = rp[i] + int(np.nonzero(col[rp[i]:rp[i + 1]] == i)[0][0])
        eye[d] = np.eye(nv)
    bb = 3.0 + np.arange(b.size, dtype=np.float64) % 7
    kw.update(lin_tol=1e-6, lin_iter=8)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays),
                            rx.default_cfg(implicit=1, lin_prec=rx.PREC_ILU, lin_solver=rx.LIN_RESTARTED_FGMRES,
                                           lin_restart=2, **kw))
    s.set_state(st)
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    s.download("RES")
    s.upload("JAC", eye)
    s.upload("RHS", bb)
    s.upload("SOL", bb)
    it, res = s.linear_solve()
    assert it == 0 and res == 0.0, (it, res)
    assert np.array_equal(s.download("SOL"), bb)
    s.close()
