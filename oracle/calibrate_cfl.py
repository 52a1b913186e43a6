#!/usr/bin/env python3
"""Which flow CFL the bench's implicit step can be pinned against the reference at (TEST INFRASTRUCTURE; runs only
where /root/reference exists — the reference is compiled here by oracle/ref_build.mk and driven by
oracle/ref_harness; never on the GPU box).

VERDICT r04 #1: at the bench's former CFL 5 the serial ILU(0) of the bench state is numerically singular
(|lambda_max(M^-1)| = 3.3e21, profiles/r04_calibration_c2b.json), FGMRES(5) reduces the residual by 7e-7 relative,
and no two implementations of that step agree beyond 1e-4 — the reference against itself with another summation
order included. The reference's own PaSR cfg runs CFL_NUMBER= 0.1
(Test_Cases/TURBOLENT/TURBOLENT_COMBUSTION/my_combustion_second_chem_PaSR.cfg:120).

For each CFL this runs the c2b case of oracle/calibrate.py — the bench's own state on the 500 x 200 = 100 000-point
jet (7 species, every one floored at 1e-6 of rho), EULER_IMPLICIT flow with serial ILU(0) FGMRES(5) (the reference's
one rank, LINEAR_SOLVER_ERROR 1e-6), jet boundary conditions, then the SST step — once by the reference itself
(harness --iters 1) and once by the restatement (O.outer_iteration, the reference's sequential inner products), and
records:
  * reference <-> restatement after the outer iteration: every species partial density elementwise relative to the
    point's rho (tests/parity.py:species_close's measure), rho / rho E / (k, omega) column-relative, both RMS vectors;
  * the same against the restatement rerun with the device's inner-product order (the rounding sensitivity of the
    step: what any other implementation, the device included, can at best agree to);
  * how much the flow's FGMRES(5) actually solves: the true relative residual |b - A x| / |b| of the restatement's
    update (bsr_spmv, not FGMRES's own estimate), its own beta / |b|, and the iteration count.
Writes profiles/r05_calibration_c2.json. The bench adopts the largest CFL at which reference <-> restatement is
<= 1e-10 and the solve reduces the residual (|b - A x| / |b| well below 1)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path = [REPO] + [q for q in sys.path if os.path.abspath(q or ".") != HERE]

from oracle import calibrate as CAL  # noqa: E402
from oracle import oracle as O  # noqa: E402


def compare(a, b, nDim, ns):
    """a, b: outer_iteration-shaped dicts (U, T, rms, sst_rms); b is the reference side."""
    Ua, Ub = np.asarray(a["U"]), np.asarray(b["U"])
    rho = np.abs(Ub[:, 0])
    sp = slice(nDim + 2, nDim + 2 + ns)
    species = float((np.abs(Ua[:, sp] - Ub[:, sp]) / rho[:, None]).max())
    col = lambda q: float(np.abs(Ua[:, q] - Ub[:, q]).max() / max(np.abs(Ub[:, q]).max(), 1e-300))
    mom = float(np.linalg.norm(Ua[:, 1:nDim + 1] - Ub[:, 1:nDim + 1], axis=1).max() /
                max(np.linalg.norm(Ub[:, 1:nDim + 1], axis=1).max(), 1e-300))
    Ta, Tb = np.asarray(a["T"]), np.asarray(b["T"])
    kw = float((np.abs(Ta - Tb).max(axis=0) / np.maximum(np.abs(Tb).max(axis=0), 1e-300)).max())
    rr = lambda x, y: float(np.max(np.abs(np.asarray(x) - np.asarray(y)) / np.abs(np.asarray(y))))
    out = dict(species_rel_rho_elementwise=species, rho_colrel=col(0), momentum_rel=mom, rhoE_colrel=col(nDim + 1),
               k_omega_colrel=kw, rms_rel=rr(a["rms"], b["rms"]), sst_rms_rel=rr(a["sst_rms"], b["sst_rms"]))
    out["max"] = max(out.values())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfl", default="0.1,1,2,5")
    ap.add_argument("--case", default="c2b", help="c2b (500 x 200) or c3b (2000 x 500: the bench mesh, serial ILU)")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05_calibration_c2.json"))
    a = ap.parse_args()
    CAL.subprocess_make()
    from tests.test_oracle_bc import iteration_cfg
    out = {"what": __doc__.split("\n\n")[0].replace("\n", " "), "host": os.uname().nodename, "cases": {}}
    for cfl in [float(c) for c in a.cfl.split(",")]:
        t0 = time.perf_counter()
        g, harness_s = CAL.run_case(a.case, cfl=cfl)
        nDim, ns = int(g["dims"][0]), int(g["dims"][4])
        m = O.Mechanism(g)
        cfg, bc, s0 = iteration_cfg(g)
        assert abs(cfg["cfl"] - cfl) < 1e-12, (cfg["cfl"], cfl)
        pat = (g["bsr_row_ptr"], g["bsr_col"])
        o = O.outer_iteration(m, nDim, g, s0, bc, cfg, 0, pat, keep=False)
        with O.dot_order("device"):
            od = O.outer_iteration(m, nDim, g, s0, bc, cfg, 0, pat, keep=False)
        ref = dict(U=g["it1_U"], T=g["it1_sst"], rms=g["it1_rms"], sst_rms=g["it1_sst_rms"])
        A, b, x = o["sys"], np.asarray(o["rhs"]).ravel(), np.asarray(o["sol"]).ravel()
        r = O.bsr_spmv(pat[0], pat[1], A, x).ravel() - b
        nb = float(np.linalg.norm(b))
        rec = dict(
            cfl=cfl, points=int(len(g["it_U0"])), species=ns,
            reference_vs_restatement=compare(o, ref, nDim, ns),
            restatement_device_dot_order_vs_restatement=compare(od, o, nDim, ns),
            flow_solve=dict(lin_iters=int(o["lin_iters"]), lin_tol=float(cfg["lin_tol"]),
                            true_rel_residual=float(np.linalg.norm(r)) / nb,
                            fgmres_beta_rel=float(o["lin_resid"]) / nb,
                            rhs_norm=nb, update_norm=float(np.linalg.norm(x))),
            sst_lin_iters=int(o["sst_lin_iters"]),
            reference_s_per_iter=float(g["it1_wall"][0]), harness_total_s=harness_s,
            wall_s=time.perf_counter() - t0)
        out["cases"][f"{a.case}_cfl{cfl:g}"] = rec
        print(json.dumps(rec), flush=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print("->", a.out)


if __name__ == "__main__":
    main()
