#!/usr/bin/env python3
"""Where the reference and the restatement part on the c2b calibration case (TEST INFRASTRUCTURE; runs only where
/root/reference exists — the reference is compiled here by oracle/ref_build.mk and driven by oracle/ref_harness).

c2b (oracle/calibrate.py): the bench's own state on a 500 x 200 = 100 000-point jet, 7 species every one floored at
1e-6 of rho, EULER_IMPLICIT CFL 5, serial ILU(0) FGMRES(5) (the reference's one rank). Round 3 measured
reference <-> restatement 1.5e-2 column-relative in U after one outer iteration (profiles/r03_calibration_c2b.json).
VERDICT r03 asked for the error relative to rho and elementwise, the worst points, and the discrete branch or the
conditioning that makes it. This script answers with:

1. the reference's iteration (harness --iters 1) against the restatement's O.outer_iteration (the reference's
   sequential inner products): per-variable error relative to rho (species) / to each column's max, elementwise
   relative error, the worst points with their coordinates and species mass fractions;
2. the restatement's flow system at the same state solved twice by FGMRES(5)+ILU(0), once with the reference's
   sequential inner products and once with another summation order (the device's), everything else bitwise equal;
   then an instrumented replica of orc_fgmres_p (validated bitwise against it in both orders) that records the
   Hessenberg matrix, Givens coefficients, the least-squares coefficients y, the MGS re-orthogonalisation decisions
   and the stop test of each run, so the amplification can be attributed:
     * discrete branches: the iteration count (FGMRES's stop test / early return, linear_solvers_structure.cpp:
       309-463), MGS's re-orthogonalisation test (:87-186), AddClippedSolution's clipping (solver_direct_reactive.cpp:
       2390-2398) of the update, and the viscous Jacobian's Ds_i switch (numerics_direct_reactive.cpp:1578-1588)
       — present only at a pure-species point, X_s -> 1; the bench state has none (every species >= 1e-6 rho);
     * conditioning: the relative change of y against that of H (the triangular solve's amplification), the
       condition number of the rotated R, and how much of the solution difference the system maps to the residual
       (|A dx| / |A x| against |dx| / |x|: an update difference in a near-null direction of the preconditioned
       operator changes x without changing the residual FGMRES minimises).
Writes profiles/r04_calibration_c2b.json."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path = [REPO] + [q for q in sys.path if os.path.abspath(q or ".") != HERE]

from oracle import calibrate as CAL  # noqa: E402
from oracle import oracle as O  # noqa: E402

CACHE = "/tmp/rx_calib_c2b.npz"


def harness_case():
    if os.path.exists(CACHE):
        return dict(np.load(CACHE, allow_pickle=False))
    CAL.subprocess_make()
    g, _ = CAL.run_case("c2b")
    np.savez(CACHE, **{k: np.asarray(v) for k, v in g.items()})
    return g


def fgmres_traced(rp, col, A, F, b, tol, m):
    """orc_fgmres_p (prec ILU0, one rank, x0 = 0) restated in numpy with orc_dot for every inner product; returns x
    and the trace (H, g, cs, sn, y, the re-orthogonalisation decisions, beta after each iteration, iterations)."""
    L = O.lib()
    N, nb = len(rp) - 1, A.shape[1]
    n = N * nb

    def dot(a, c):
        return L.orc_dot(O.C.c_int64(n), O._p(a), O._p(c))

    x = np.zeros(n)
    w = [None] * (m + 1)
    z = [None] * (m + 1)
    H = np.zeros((m + 1, m))
    g = np.zeros(m + 1)
    sn = np.zeros(m + 1)
    cs = np.zeros(m + 1)
    reo = np.zeros((m, m), dtype=bool)
    betas = []
    norm0 = np.sqrt(dot(b, b))
    w[0] = O.bsr_spmv(rp, col, A, x).ravel() - b
    beta = np.sqrt(dot(w[0], w[0]))
    if beta < tol * norm0 or beta < np.finfo(float).eps:
        return x, dict(iters=0, early=True)
    w[0] = w[0] / -beta
    g[0] = beta
    norm0 = beta
    i = 0
    for i in range(m):
        if beta < tol * norm0:
            break
        z[i] = O.ilu_apply(rp, col, F, w[i]).ravel()
        w[i + 1] = O.bsr_spmv(rp, col, A, z[i]).ravel()
        nrm = dot(w[i + 1], w[i + 1])
        thr = nrm * 0.98
        for k in range(i + 1):
            prod = dot(w[i + 1], w[k])
            H[k, i] = prod
            w[i + 1] = w[i + 1] + (-prod) * w[k]
            if prod * prod > thr:
                reo[k, i] = True
                prod = dot(w[i + 1], w[k])
                H[k, i] += prod
                w[i + 1] = w[i + 1] + (-prod) * w[k]
            nrm -= H[k, i] * H[k, i]
            nrm = max(nrm, 0.0)
            thr = nrm * 0.98
        nrm = np.sqrt(dot(w[i + 1], w[i + 1]))
        H[i + 1, i] = nrm
        w[i + 1] = w[i + 1] / nrm
        for k in range(i):
            t = cs[k] * H[k, i] + sn[k] * H[k + 1, i]
            H[k + 1, i] = cs[k] * H[k + 1, i] - sn[k] * H[k, i]
            H[k, i] = t
        dx, dy = H[i, i], H[i + 1, i]
        sgn = lambda a, bb: 0.0 if bb == 0.0 else (-abs(a) if bb < 0 else abs(a))
        if dx == 0.0 and dy == 0.0:
            cs[i], sn[i] = 1.0, 0.0
        elif abs(dy) > abs(dx):
            tmp = dx / dy
            dx = np.sqrt(1.0 + tmp * tmp)
            sn[i] = sgn(1.0 / dx, dy)
            cs[i] = tmp * sn[i]
        else:
            tmp = dy / dx
            dy = np.sqrt(1.0 + tmp * tmp)
            cs[i] = sgn(1.0 / dy, dx)
            sn[i] = tmp * cs[i]
        H[i, i], H[i + 1, i] = abs(dx * dy), 0.0
        t = cs[i] * g[i] + sn[i] * g[i + 1]
        g[i + 1] = cs[i] * g[i + 1] - sn[i] * g[i]
        g[i] = t
        beta = abs(g[i + 1])
        betas.append(beta)
    else:
        i = m
    y = g[:i].copy()
    for k in range(i - 1, -1, -1):
        y[k] /= H[k, k]
        for j in range(k - 1, -1, -1):
            y[j] -= H[j, k] * y[k]
    for k in range(i):
        x = x + y[k] * z[k]
    return x, dict(iters=i, H=H, g=g, y=y, reo=reo, betas=np.array(betas), norm0=norm0, z=z)


def rel_report(U, Uref, nDim, coord, names):
    """Per variable: max |dU| / rho (species) or / the column max, elementwise max |dU| / |U| (floor 1e-300), and
    the five worst points of the species error relative to rho."""
    rho = np.abs(Uref[:, 0])
    out = {}
    fl = nDim + 2
    for v in range(U.shape[1]):
        d = np.abs(U[:, v] - Uref[:, v])
        el = d / np.maximum(np.abs(Uref[:, v]), 1e-300)
        rec = dict(colrel=float(d.max() / max(np.abs(Uref[:, v]).max(), 1e-300)), elementwise=float(el.max()))
        if v >= fl:
            rec["rel_to_rho"] = float((d / rho).max())
            rec["column_max_over_rho"] = float((np.abs(Uref[:, v]) / rho).max())
            k = np.argsort(d / rho)[::-1][:5]
            rec["worst_points"] = [dict(point=int(p), x=float(coord[p, 0]), y=float(coord[p, 1]),
                                        Y=float(Uref[p, v] / rho[p]), dU_over_rho=float(d[p] / rho[p]),
                                        elementwise=float(el[p])) for p in k]
        out[names[v]] = rec
    return out


def main():
    g = harness_case()
    from tests.test_oracle_bc import iteration_cfg
    nDim = int(g["dims"][0])
    m = O.Mechanism(g)
    cfg, bc, s0 = iteration_cfg(g)
    pat = (g["bsr_row_ptr"], g["bsr_col"])
    coord = np.asarray(g["coord"])
    ns = int(g["dims"][4])
    names = ["rho", "rho_u", "rho_v", "rho_E"] + [f"rho_Y{s}" for s in range(ns)]
    out = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "points": int(len(coord))}
    o = O.outer_iteration(m, nDim, g, s0, bc, cfg, 0, pat, keep=True)
    out["reference_vs_restatement"] = rel_report(o["U"], g["it1_U"], nDim, coord, names)
    out["reference_vs_restatement"]["k_omega_colrel"] = CAL.colrel(o["T"], g["it1_sst"])
    out["reference_vs_restatement"]["rms_rel"] = float(np.max(np.abs(o["rms"] - g["it1_rms"]) / np.abs(g["it1_rms"])))
    with O.dot_order("device"):
        od = O.outer_iteration(m, nDim, g, s0, bc, cfg, 0, pat, keep=True)
    out["restatement_dot_order_perturbation"] = rel_report(od["U"], o["U"], nDim, coord, names)
    # 2. the flow system: identical A and rhs (both runs assemble them before any inner product)
    A, rhs = o["sys"], o["rhs"]
    assert np.array_equal(A, od["sys"]) and np.array_equal(rhs, od["rhs"]), "systems differ before the solve"
    rp, col = pat
    F = O.ilu_build(rp, col, A)
    b = rhs.ravel()
    tol, mm = cfg["lin_tol"], cfg["lin_iter"]
    xs, its, _ = O.fgmres(rp, col, A, b, "ilu", F=F, tol=tol, m=mm)
    with O.dot_order("device"):
        xd, itd, _ = O.fgmres(rp, col, A, b, "ilu", F=F, tol=tol, m=mm)
    xs_t, trs = fgmres_traced(rp, col, A, F, b, tol, mm)
    with O.dot_order("device"):
        xd_t, trd = fgmres_traced(rp, col, A, F, b, tol, mm)
    out["replica_bitwise"] = bool(np.array_equal(xs_t, xs.ravel()) and np.array_equal(xd_t, xd.ravel()))
    assert np.array_equal(xs.ravel(), o["sol"].ravel())
    nb = A.shape[1]
    X, Xd = xs.reshape(-1, nb), xd.reshape(-1, nb)
    dx = X - Xd
    Adx = O.bsr_spmv(rp, col, A, dx.ravel())
    Ax = O.bsr_spmv(rp, col, A, X.ravel())
    H1, H2 = trs["H"], trd["H"]
    R = H1[:trs["iters"], :trs["iters"]]
    out["solve"] = dict(
        iterations=[int(its), int(itd)], betas_sequential=trs["betas"].tolist(), betas_device=trd["betas"].tolist(),
        norm0=[trs["norm0"], trd["norm0"]],
        reorth_decisions_sequential=trs["reo"].astype(int).tolist(), reorth_decisions_device=trd["reo"].astype(int).tolist(),
        H_relchange=float(np.abs(H1 - H2).max() / np.abs(H1).max()),
        y_sequential=trs["y"].tolist(), y_device=trd["y"].tolist(),
        y_relchange=float(np.abs(trs["y"] - trd["y"]).max() / np.abs(trs["y"]).max()),
        cond_R=float(np.linalg.cond(R)),
        x_colrel=[float(np.abs(dx[:, v]).max() / max(np.abs(X[:, v]).max(), 1e-300)) for v in range(nb)],
        x_rel=float(np.linalg.norm(dx) / np.linalg.norm(X)),
        residual_image_rel=float(np.linalg.norm(Adx) / np.linalg.norm(Ax)),
        basis_gram_offdiag=None)
    # the preconditioned Krylov directions z_k: how close to dependent (the y solve's sensitivity)
    Z = np.stack([v for v in trs["z"][:trs["iters"]]], axis=1)
    Zn = Z / np.linalg.norm(Z, axis=0)
    out["solve"]["z_gram_cond"] = float(np.linalg.cond(Zn.T @ Zn))
    out["solve"]["z_singular_values"] = np.linalg.svd(Zn, compute_uv=False).tolist()
    # the clipped update (AddClippedSolution): entries that hit a bound, and whether the two runs clip differently
    Uold = np.asarray(s0["U"])
    for tag, xx in (("sequential", X), ("device", Xd)):
        Un = Uold + cfg["relaxation"] * xx
        out["solve"][f"clipped_{tag}"] = int(np.sum(Un[:, nDim + 2:] < 0.0) + np.sum(Un[:, 0] < 0.0))
    # 3. the preconditioner: power iteration on M^-1 = (L U)^-1 and on its two triangular factors alone (the oracle's
    # ILU apply on the factor with the other triangle removed), the support of the dominant direction, and the
    # smallest pivot block relative to its matrix block
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    cols = np.asarray(col)
    low, up, dg = cols < rows, cols > rows, cols == rows
    FU = F.copy()
    FU[low] = 0.0
    FL = F.copy()
    FL[up] = 0.0
    FL[dg] = np.eye(nb)

    def power(Fx, its=25):
        rng = np.random.default_rng(1)
        v = rng.normal(size=b.size)
        v /= np.linalg.norm(v)
        gr = 0.0
        for _ in range(its):
            w_ = O.ilu_apply(rp, col, Fx, v).ravel()
            gr = float(np.linalg.norm(w_))
            v = w_ / gr
        mag = np.linalg.norm(v.reshape(-1, nb), axis=1)
        k = np.argsort(mag)[::-1][:8]
        return dict(growth=gr, support=[dict(point=int(p), x=float(coord[p, 0]), y=float(coord[p, 1]),
                                             weight=float(mag[p])) for p in k],
                    support_energy_top8=float(np.sum(mag[k] ** 2)))
    sD = np.linalg.svd(F[dg], compute_uv=False)
    sA = np.linalg.svd(A[dg], compute_uv=False)
    piv = sD[:, -1] / sA[:, -1]
    worst_sol = np.argsort(np.abs(dx).max(axis=1) / np.maximum(np.abs(X).max(axis=0).max(), 1e-300))[::-1][:8]
    out["preconditioner"] = dict(
        M_inverse=power(F), L_inverse=power(FL), U_inverse=power(FU),
        A_norm_max_block=float(np.abs(A).max()),
        min_pivot_sigma_ratio=float(piv.min()),
        min_pivot_point=dict(point=int(np.argmin(piv)), x=float(coord[np.argmin(piv), 0]),
                             y=float(coord[np.argmin(piv), 1])),
        solution_difference_worst_points=[int(p) for p in worst_sol])
    print(json.dumps(out["solve"], indent=1)[:3000])
    print(json.dumps(out["preconditioner"], indent=1)[:3000])
    fn = os.path.join(REPO, "profiles", "r04_calibration_c2b.json")
    with open(fn, "w") as f:
        json.dump(out, f, indent=1)
    print("->", fn)


if __name__ == "__main__":
    main()
