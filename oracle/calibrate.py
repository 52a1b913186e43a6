#!/usr/bin/env python3
"""Reference-vs-restatement calibration and size-true parity (TEST INFRASTRUCTURE; runs only where
/root/reference exists, i.e. in the build container, never on the GPU box).

BASELINE.md "CPU-baseline plan" steps 1-3: the reference itself (compiled from /root/reference by
oracle/ref_build.mk, driven by oracle/ref_harness --iters) and our CPU restatement (oracle/rx_oracle.cpp) run the
same whole outer iteration (CMeanFlowIteration::Iterate: flow implicit FGMRES(5)+ILU0 step with the jet's
boundary conditions, then the SST step) on identical meshes and states here:

  c1  the reference's own 9 000-point jet (mesh_stretched.su2) with its converged PaSR state
      (PLOT/flow_second_chem.dat), 9 species
  c2  a 500 x 200 = 100 000-point synthetic jet (meshgen, read by the reference's SU2 reader, its dual grid), the
      bench's initial field on it (synth.field_at: the converged jet interpolated, species floored at 1e-10),
      9 species
  c2b the same mesh with the bench's own state: 7 species (the subset library files), every species floored at
      1e-6 of rho (synth.field_at's default, the state bench.py runs), serial ILU(0) (the reference's one rank)
  c2e the c2b mesh and state under the shipped cfgs' scheme: EULER_EXPLICIT flow at CFL 0.5 (no flow linear
      solve), SST with FGMRES(5) + LU_SGS

Outputs (profiles/r02_calibration.json): the reference's wall time per iteration (1 core; the serial reference
build has no MPI), the restatement's wall time on 1 thread and on all threads, their ratio (the factor that turns
the restatement's throughput on the GPU box's host cores into reference-equivalent throughput), and the
restatement's agreement with the reference after the iteration (column-relative, U / (k, omega) / RMS) at these
sizes, next to the iteration's sensitivity to rounding alone (the restatement rerun with another inner-product
summation order): where that sensitivity is O(1) — a serial (one-rank) ILU(0)-preconditioned FGMRES(5) on a 100k-point
system is chaotic — no 1e-10 parity exists between any two implementations, the reference included. The reference's solver TU is built at -O0 (the Set_Sigmak UB workaround); the ratio is
quoted for that build.
"""
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

from oracle import make_golden as MG  # noqa: E402
from oracle import oracle as O  # noqa: E402


def colrel(a, ref):
    return float((np.abs(a - ref).max(axis=0) / np.maximum(np.abs(ref).max(axis=0), 1e-300)).max())


def run_case(name, cfl=None):
    """cfl: the flow CFL of c2b (default 5.0, the round-2..4 bench value); c2e keeps 0.5."""
    if name == "c1":
        def writer(wd):
            os.symlink(os.path.join(MG.CASE_DIR, "mesh_stretched.su2"), os.path.join(wd, "mesh.su2"))
            return "mesh.su2"
        _, U = MG.read_plot(os.path.join(MG.CASE_DIR, "PLOT/flow_second_chem.dat"))
    else:
        nx, ny = {"c2": (500, 200), "c2b": (500, 200), "c2e": (500, 200), "c3b": (2000, 500)}[name]
        ns = 7 if name in ("c2b", "c2e", "c3b") else 9
        pts, quads, bnd = MG.meshgen.jet_mesh(nx, ny)
        from tests.rxpkg import synth
        # c2b: the bench's own state (7 species, every species floored at 1e-6 of rho: synth.field_at's default)
        _, Uc, k, om, _, _ = synth.field_at(pts, ns, y_floor=1e-6 if name in ("c2b", "c2e", "c3b") else 1e-10)
        U = np.concatenate([Uc, k[:, None], om[:, None]], axis=1)

        def writer(wd):
            MG.meshgen.write_su2(os.path.join(wd, "mesh.su2"), pts, quads, bnd)
            return "mesh.su2"
    ns = 7 if name in ("c2b", "c2e", "c3b") else 9
    if name == "c2e":  # the shipped cfgs' scheme: EULER_EXPLICIT flow (no flow linear solve), LU_SGS SST
        wd = MG.make_workdir("calib_" + name, writer, cfl=0.5, order="1ST_ORDER", prec="LU_SGS", ns=ns,
                             time_flow="EULER_EXPLICIT")
    else:
        wd = MG.make_workdir("calib_" + name + ("" if cfl is None else f"_cfl{cfl:g}"), writer,
                             cfl=5.0 if cfl is None else cfl, order="1ST_ORDER", prec="ILU0", ns=ns)
    MG.write_state(wd, U)
    t0 = time.perf_counter()
    g = MG.run_harness(wd, bsr=False, extra=["--iters", "1"])
    harness_s = time.perf_counter() - t0
    g.update(MG.mech_arrays(wd, "test_chem_second.txt") if ns != 9 else MG.mech_arrays())
    # the cfg's scheme for iteration_cfg (as make_golden.iteration_case records it)
    g["time_flow"] = np.array("EULER_EXPLICIT" if name == "c2e" else "EULER_IMPLICIT")
    g["lin_prec"] = np.array("LU_SGS" if name == "c2e" else "ILU0")
    return g, harness_s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c1,c2")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r02_calibration.json"))
    a = ap.parse_args()
    subprocess_make()
    from tests.test_oracle_bc import iteration_cfg
    out = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "host": os.uname().nodename,
           "host_cpus": os.cpu_count(), "cases": {}}
    for name in a.cases.split(","):
        g, harness_s = run_case(name)
        N = len(g["it_U0"])
        nDim = int(g["dims"][0])
        m = O.Mechanism(g)
        cfg, bc, s0 = iteration_cfg(g)
        pat = (g["bsr_row_ptr"], g["bsr_col"])
        times = {}
        res = None
        for th in (1, a.threads):
            O.lib().orc_set_num_threads(th)
            t0 = time.perf_counter()
            o = O.outer_iteration(m, nDim, g, s0, bc, cfg, 0, pat, keep=False)
            times[th] = time.perf_counter() - t0
            if res is None:
                res = o
            else:  # the OpenMP restatement is thread-count independent
                assert np.array_equal(o["U"], res["U"]) and np.array_equal(o["T"], res["T"])
        # sensitivity of the iteration to rounding alone: the same restatement with the device's inner-product
        # summation order (a last-bit perturbation of every FGMRES dot product)
        with O.dot_order("device"):
            od = O.outer_iteration(m, nDim, g, s0, bc, cfg, 0, pat, keep=False)
        ref_s = float(g["it1_wall"][0])
        rec = dict(points=N, edges=int(len(g["edges"])), species=int(g["dims"][4]),
                   reference_s_per_iter=ref_s, restatement_s_per_iter_1thread=times[1],
                   restatement_s_per_iter_all=times[a.threads], threads_all=a.threads,
                   ratio_reference_over_restatement_1thread=ref_s / times[1],
                   reference_mcells_iters_per_s=N / ref_s / 1e6,
                   parity_vs_reference=dict(
                       U_colrel=colrel(res["U"], g["it1_U"]), V_colrel=colrel(res["V"], g["it1_V"]),
                       k_omega_colrel=colrel(res["T"], g["it1_sst"]),
                       mut_rel=colrel(res["mut"][:, None], g["it1_mut"][:, None]),
                       rms_rel=float(np.max(np.abs(res["rms"] - g["it1_rms"]) / np.abs(g["it1_rms"]))),
                       sst_rms_rel=float(np.max(np.abs(res["sst_rms"] - g["it1_sst_rms"]) / np.abs(g["it1_sst_rms"]))),
                       lin_iters=int(res["lin_iters"])),
                   rounding_sensitivity_U_colrel=colrel(od["U"], res["U"]),
                   harness_total_s=harness_s)
        out["cases"][name] = rec
        print(name, json.dumps(rec), flush=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("->", a.out)


def subprocess_make():
    import subprocess
    subprocess.run(["make", "-s", "-f", os.path.join(HERE, "ref_build.mk"), "-j8", "all", "harness"], check=True,
                   cwd=REPO)
    subprocess.run(["make", "-s", "-C", HERE], check=True)


if __name__ == "__main__":
    main()
