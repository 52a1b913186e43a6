"""Partitioned preconditioners and the whole implicit step: HIP path (librx.so through the C ABI)
against the CPU oracle on synthetic reacting jets. Requires an MI355X.

Partitions stand for the reference's MPI ranks (include/rx.h, rx_mesh_desc.part_ptr): ILU(0) is
per rank (halo columns skipped), LU-SGS's backward sweep reads halo x* values.

Bars: the triangular work is bitwise equal to the oracle. FGMRES is bitwise equal to the oracle run
with the device's inner-product summation order (O.dot_order("device")); against the reference's
sequential sums the solution agrees normwise per variable to 1e-8 (Krylov amplification of
last-bit differences of the inner products; measured 2e-10 on these cases).
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.parity import assert_close, per_column_close
from tests.rxpkg import rx, synth

pytestmark = pytest.mark.gpu


def case(nx, ny, n_part, ns=7):
    mesh, st, mech_arrays, kw = synth.jet_case(nx, ny, n_species=ns, n_part=n_part)
    cfg = dict(cfl=5.0, max_delta_time=1e6, prandtl_lam=0.72, prandtl_turb=kw["prandtl_turb"],
               lewis_turb=kw["lewis_turb"], mach_inf=kw["mach_inf"], c_mu=kw["c_mu"], pasr_lb=kw["pasr_lb"],
               lin_tol=1e-6, lin_iter=5, relaxation=1.0)
    kw["cfl"] = cfg["cfl"]  # the device cfg's CFL is the oracle's (default_cfg's is the bench's, rx.BENCH_CFL)
    return mesh, st, mech_arrays, kw, cfg


def oracle_system(mesh, st, mech_arrays, cfg, ns, order="reference"):
    """One implicit iteration restated by the oracle (reference-order Jacobian, rhs, solve)."""
    om = O.Mechanism(mech_arrays)
    N = len(st["V"])
    pattern = O.bsr_pattern(N, mesh["edges"])
    with O.dot_order(order):
        U, info = O.implicit_step(om, 2, ns, mesh, st, cfg, pattern=pattern, part_ptr=mesh["part_ptr"])
    return pattern, info, U


@pytest.mark.parametrize("nx,ny,n_part", [(48, 20, 1), (48, 20, 5), (48, 20, 16), (100, 40, 1), (100, 40, 3)])
@pytest.mark.parametrize("prec", ["ilu", "lusgs"])
def test_partitioned_preconditioners_vs_oracle(nx, ny, n_part, prec):
    ns = 7
    mesh, st, mech_arrays, kw, cfg = case(nx, ny, n_part, ns)
    (rp, col), info, _ = oracle_system(mesh, st, mech_arrays, cfg, ns)
    A, b = info["jac"], info["rhs"].ravel()
    pp = mesh["part_ptr"]
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays),
                            rx.default_cfg(implicit=1, lin_prec=(1 if prec == "ilu" else 0), **kw))
    s.set_state(st)
    grp, gcol = s.bsr_pattern()
    assert np.array_equal(grp, rp) and np.array_equal(gcol, col)
    # mark the Jacobian assembled, then overwrite it with the oracle's
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    s.download("RES")
    s.upload("JAC", A)
    s.upload("RHS", b)
    if prec == "ilu":
        s.ilu0_build()
        s.sync()
        F = O.ilu_build(rp, col, A, part_ptr=pp)
        assert_close(s.download("ILU").reshape(F.shape), F, rtol=0.0, what=f"ILU(0) factor P={n_part}")
        s.ilu0_apply("RHS", "SOL")
        s.sync()
        assert_close(s.download("SOL"), O.ilu_apply(rp, col, F, b, part_ptr=pp).ravel(), rtol=0.0,
                     what=f"ILU(0) apply P={n_part}")
        kw_ = dict(prec="ilu", F=F)
    else:
        s.lusgs_apply("RHS", "SOL")
        s.sync()
        assert_close(s.download("SOL"), O.lusgs(rp, col, A, b, part_ptr=pp).ravel(), rtol=0.0,
                     what=f"LU-SGS apply P={n_part}")
        kw_ = dict(prec="lusgs")
    with O.dot_order("device"):
        dev_x, it_dev, res_dev = O.fgmres(rp, col, A, b, tol=1e-6, m=5, part_ptr=pp, **kw_)
    ref_x, it_ref, _ = O.fgmres(rp, col, A, b, tol=1e-6, m=5, part_ptr=pp, **kw_)
    s.upload("SOL", np.zeros_like(b))
    it, res = s.fgmres(tol=1e-6, m=5)
    assert it == it_dev == it_ref
    x = s.download("SOL").reshape(ref_x.shape)
    assert_close(x, dev_x, rtol=0.0, what=f"FGMRES({prec}) P={n_part} vs oracle in device dot order")
    assert res == res_dev
    per_column_close(x, ref_x, rtol=1e-8, floor=1.0, what=f"FGMRES({prec}) P={n_part} vs reference dot order")
    s.close()


@pytest.mark.parametrize("n_part", [1, 8])
def test_implicit_step_vs_oracle(n_part):
    """One whole outer iteration on the device (gradient, dt, AUSM/viscous/PaSR with Jacobians,
    assembly, ILU(0), FGMRES(5), clipped update) against the oracle's restatement."""
    ns = 7
    mesh, st, mech_arrays, kw, cfg = case(40, 16, n_part, ns)
    _, info, U_ref = oracle_system(mesh, st, mech_arrays, cfg, ns, order="device")
    _, info_r, U_seq = oracle_system(mesh, st, mech_arrays, cfg, ns)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays), rx.default_cfg(implicit=1, lin_prec=1, **kw))
    s.set_state(st)
    s.SetPrimitive_Gradient_LS()
    s.SetTime_Step()
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    rms, it = s.ImplicitEuler_Iteration()
    assert it == info["lin_iters"]
    assert_close(s.download("DT"), info["dt"], what="dt")
    rhs = s.download("RHS").reshape(info["rhs"].shape)
    assert_close(rhs[:, :4], info["rhs"][:, :4], floor=1e-9, what="rhs flow rows")
    per_column_close(rhs, info["rhs"], floor=1.0, what="rhs")
    sol = s.download("SOL").reshape(info["rhs"].shape)
    per_column_close(sol, info["sol"].reshape(sol.shape), floor=1.0, what="FGMRES solution (device dot order)")
    per_column_close(sol, info_r["sol"].reshape(sol.shape), rtol=1e-8, floor=1.0,
                     what="FGMRES solution (reference dot order)")
    U = s.download("U").reshape(U_ref.shape)
    per_column_close(U, U_ref, floor=1.0, what="updated U")
    per_column_close(U, U_seq, floor=1.0, what="updated U (reference dot order)")
    ref_rms = np.maximum(1e-32, np.sqrt((info["rhs"] ** 2).sum(axis=0) / len(U_ref)))
    assert_close(rms, ref_rms, what="RMS residual")
    # a second step replays the captured solve graph
    s.SetPrimitive_Gradient_LS()
    s.SetTime_Step()
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    rms2, it2 = s.ImplicitEuler_Iteration()
    assert it2 == it and np.all(np.isfinite(rms2))
    # the node records did not change, so the replayed solve is the same linear system: same
    # solution bitwise (no state may leak from one solve into the next)
    assert np.array_equal(rms2, rms)
    assert np.array_equal(s.download("SOL"), sol.ravel())
    s.close()


@pytest.mark.parametrize("nx,ny,nz,n_part", [(20, 8, 6, 1), (20, 8, 6, 4), (50, 10, 10, 32), (40, 10, 8, 1),
                                             (40, 10, 8, 2)])
def test_ilu_factor_3d_vs_oracle(nx, ny, nz, n_part):
    """The grouped ILU(0) build on 3-D hexahedral jets (7-point stencil: up to six lower blocks per row under the
    partitions' RCM orderings; 50x10x10 in 32 partitions has 72 rows with four, like 22 272 rows of C5), on a
    diagonally dominant random matrix of the mesh's pattern: factor and apply bitwise equal to the oracle
    (BuildILUPreconditioner / ComputeILUPreconditioner, matrix_structure.cpp:1368-1515). 40x10x8 in 1 / 2 partitions
    (3 200 / 1 600 rows, levels up to 80 rows wide): partitions too large for the LDS-resident apply, so the apply is
    the LDS-ring sweep (k_ilu_apply_ring); 2-D ring cases with far rows (dependencies more than kIluRing - 1 levels
    back): test_partitioned_preconditioners_vs_oracle's 100x40 in 3 partitions."""
    mesh, st, mech_arrays, kw = synth.jet_case(nx, ny, n_species=7, n_part=n_part, nz=nz)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays), rx.default_cfg(implicit=1, lin_prec=1, **kw))
    s.set_state(st)
    rp, col = s.bsr_pattern()
    N, nv = len(rp) - 1, s.nVar
    rng = np.random.default_rng(nz * 100 + n_part)
    A = rng.standard_normal((len(col), nv, nv))
    for i in range(N):
        k = rp[i] + np.searchsorted(col[rp[i]:rp[i + 1]], i)
        A[k] += 8.0 * nv * np.eye(nv)
    b = rng.standard_normal(N * nv)
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.sync()
    s.download("RES")
    s.upload("JAC", A.ravel())
    s.upload("RHS", b)
    s.ilu0_build()
    s.sync()
    pp = mesh["part_ptr"]
    F = O.ilu_build(rp, col, A, part_ptr=pp)
    assert_close(s.download("ILU").reshape(F.shape), F, rtol=0.0, what=f"3-D ILU(0) factor nz={nz} P={n_part}")
    s.ilu0_apply("RHS", "SOL")
    s.sync()
    assert_close(s.download("SOL"), O.ilu_apply(rp, col, F, b, part_ptr=pp).ravel(), rtol=0.0,
                 what=f"3-D ILU(0) apply nz={nz} P={n_part}")
    # the SST context's 2x2 factor (k_ilu_build_2; rows with more than three lower blocks take the grouped plan)
    t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
    A2 = rng.standard_normal((len(col), 2, 2))
    for i in range(N):
        A2[rp[i] + np.searchsorted(col[rp[i]:rp[i + 1]], i)] += 16.0 * np.eye(2)
    b2 = rng.standard_normal(N * 2)
    t.upload("JAC", A2.ravel())
    t.upload("RHS", b2)
    t.ilu0_build()
    t.sync()
    F2 = O.ilu_build(rp, col, A2, part_ptr=pp)
    assert_close(t.download("ILU")[:F2.size].reshape(F2.shape), F2, rtol=0.0, what=f"3-D SST ILU(0) nz={nz} P={n_part}")
    t.ilu0_apply("RHS", "SOL")
    t.sync()
    assert_close(t.download("SOL"), O.ilu_apply(rp, col, F2, b2, part_ptr=pp).ravel(), rtol=0.0,
                 what=f"3-D SST ILU(0) apply nz={nz} P={n_part}")
    s.close()


def test_rank_preconditioners_vs_reference_rank():
    """the device's partition semantics against the reference's own one-rank computation (golden
    rank9: the reference's CSysMatrix with domain [0, P) and halo columns [P, N), mini9's system; its ILU(0) factor,
    ILU apply and LU-SGS apply with the halo preset to the other rank's forward sweep). The device runs mini9's mesh
    cut into the partitions [0, P) and [P, N): rows [0, P) of its factor, ILU apply and LU-SGS apply equal the
    reference's bitwise (the device's partition [P, N) computes the very forward result the preset holds)."""
    import os

    import tests.test_gpu_parity as tp
    g = dict(np.load(os.path.join(tp.GOLD, "rank9.npz")))
    m = tp.golden("mini9")
    rp, col, A, b = g["bsr_row_ptr"], g["bsr_col"], g["bsr_system"], g["sys_rhs"].ravel()
    N, P = len(rp) - 1, int(g["rank_split"][0])
    nDim, nVar = int(m["dims"][0]), int(m["dims"][1])
    mesh = {k: m[k] for k in ("edges", "edge_normal", "coord", "volume", "nbr_ptr", "nbr")}
    mesh["bvertex"] = m.get("bvertex", np.zeros((0, 3), dtype=np.int64))
    mesh["bvertex_normal"] = m.get("bvertex_normal", np.zeros((0, 2)))
    mesh["part_ptr"] = np.array([0, P, N], dtype=np.int64)
    kw = dict(mach_inf=float(m["mach_inf"][0]), prandtl_turb=float(m["visc_params"][1]),
              lewis_turb=float(m["visc_params"][2]), c_mu=float(m["src_params"][0]),
              pasr_lb=float(m["src_params"][1]))
    for prec in ("ilu", "lusgs"):
        s = rx.ReactiveNSSolver(mesh, rx.Mechanism(m), rx.default_cfg(implicit=1, lin_prec=(1 if prec == "ilu" else 0),
                                                                      **kw))
        s.set_state(m)
        grp, gcol = s.bsr_pattern()
        assert np.array_equal(grp, rp) and np.array_equal(gcol, col)
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.sync()
        s.download("RES")  # the system counts as assembled; then the golden's system replaces it
        s.upload("JAC", A)
        s.upload("RHS", b)
        if prec == "ilu":
            s.ilu0_build()
            s.sync()
            F = s.download("ILU").reshape(-1, nVar, nVar)
            assert np.array_equal(F[:rp[P]], g["rank_ilu_factor"]), "ILU(0) factor of the rank vs reference"
            s.ilu0_apply("RHS", "SOL")
            s.sync()
            assert np.array_equal(s.download("SOL").reshape(N, nVar)[:P], g["rank_ilu_rhs"]), "ILU apply vs reference"
        else:
            s.lusgs_apply("RHS", "SOL")
            s.sync()
            assert np.array_equal(s.download("SOL").reshape(N, nVar)[:P], g["rank_lusgs_rhs"]), "LU-SGS vs reference"
        s.close()
