#!/usr/bin/env python3
"""Generate golden vectors from the compiled reference (TEST INFRASTRUCTURE, runs only where
/root/reference exists).

Steps per case:
  1. build oracle/_ref/harness (oracle/ref_build.mk: reference sources compiled as they lie);
  2. lay out a work dir with a cfg written here, the mesh and the reference's own library data
     files (Test_Cases/TURBOLENT/TURBOLENT_COMBUSTION/{Mixture,Chemistry,Thermo,Transp}, read in
     place through symlinks, never copied into the repo);
  3. write the state (conservatives + SST k, omega) from the reference's converged PaSR field
     `PLOT/flow_second_chem.dat` (nearest-point sampling for coarser synthetic meshes);
  4. run the harness, which drives the reference's own preprocessing and operators;
  5. pack the dumped arrays into tests/golden/<case>.npz (+ the mechanism tables the oracle and the
     HIP path need, parsed here by oracle/mech.py from the same files).

Cases:
  mini9 : 21 x 11 synthetic jet (same markers), 9 species, SST, implicit, full loops + BSR +
          LU-SGS / ILU0 / FGMRES dumps.
  jet9w : the reference's 9000-point mesh_stretched.su2 with the converged PaSR state, 2nd order
          + Venkatakrishnan limiter enabled, implicit; a window of ~700 points around the flame
          is kept (all inputs, per-edge residuals, sampled Jacobians).
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("RX_REFERENCE", "/root/reference")
CASE_DIR = os.path.join(REF, "Test_Cases/TURBOLENT/TURBOLENT_COMBUSTION")
PKG = os.path.join(REPO, "development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


meshgen = _load("rx_meshgen", os.path.join(PKG, "meshgen.py"))

CFG_TEMPLATE = """\
% golden-vector cfg written by oracle/make_golden.py (keys of the reference's cfg grammar)
CONFIG_LIB_FILE = test_chem_second.txt
FREESTREAM_MASS_FRAC = (0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
SPECIES_ORDER = (C4H6, H2O, O2, CO, CO2, H2, O, OH, H)
PHYSICAL_PROBLEM= REACTIVE_NAVIER_STOKES
KIND_TURB_MODEL= SST
MATH_PROBLEM= DIRECT
RESTART_SOL= NO
IGNITION = NO
MACH_NUMBER= 0.01819
FREESTREAM_TEMPERATURE= 300.0
FREESTREAM_VELOCITY= (6.0, 0.0, 0.0)
FREESTREAM_PRESSURE= 130000.0
REYNOLDS_LENGTH= 0.125
REF_DIMENSIONALIZATION= DIMENSIONAL
REF_LENGTH= 0.125
REF_AREA= 0
MARKER_ISOTHERMAL = (upper_wall, 300.0, lower_wall_pre, 300.0, lower_wall_post, 600.0)
INLET_TYPE = {inlet_type}
MARKER_INLET= ( Oxidizer_Inlet, {inlet_ox}, 1.0, 0.0, 0.0, Fuel_Inlet, {inlet_fuel}, 0.0, 1.0, 0.0)
INLET_MASS_FRAC = (Oxidizer_Inlet, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0; Fuel_Inlet, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
MARKER_OUTLET= ( Outlet, 101325.0)
{extra}NUM_METHOD_GRAD= WEIGHTED_LEAST_SQUARES
CFL_NUMBER= {cfl}
CFL_ADAPT= NO
EXT_ITER= 1
LINEAR_SOLVER= FGMRES
LINEAR_SOLVER_PREC= {prec}
LINEAR_SOLVER_ERROR= 1E-6
LINEAR_SOLVER_ITER= 5
MGLEVEL= 0
CONV_NUM_METHOD_FLOW= AUSM
SPATIAL_ORDER_FLOW= {order}
SLOPE_LIMITER_FLOW= VENKATAKRISHNAN
TIME_DISCRE_FLOW= {time_flow}
CONV_NUM_METHOD_TURB= SCALAR_UPWIND
SLOPE_LIMITER_TURB= VENKATAKRISHNAN
TIME_DISCRE_TURB= EULER_IMPLICIT
PASR_LB = 0.2
CONV_CRITERIA= RESIDUAL
RESIDUAL_REDUCTION= 6
RESIDUAL_MINVAL= -4
MESH_FILENAME= {mesh}
MESH_FORMAT= SU2
OUTPUT_FORMAT= TECPLOT
CONV_FILENAME= history
WRT_SOL_FREQ= 100000
WRT_CON_FREQ= 1
"""


def read_plot(path, ncons=15):
    """(coords, conservatives + k + omega) per node of a Tecplot POINT file (ncons columns after x, y)."""
    rows = []
    with open(path) as f:
        for line in f:
            t = line.split()
            if not t:
                continue
            try:
                vals = [float(x) for x in t]
            except ValueError:
                continue
            if len(vals) >= 2 + ncons:
                rows.append(vals)
    a = np.array(rows)
    return a[:, :2], a[:, 2:2 + ncons]


# INLET_TYPE variants: (a, b) of MARKER_INLET per inlet — TEMPERATURE_IMPOSE (T, |u|) as the shipped jet cfgs,
# TOTAL_CONDITIONS (T_total, P_total), MASS_FLOW (rho, |u|)
INLETS = {
    "TEMPERATURE_IMPOSE": ("300.0, 20.0", "800.0, 0.87"),
    "TOTAL_CONDITIONS": ("340.0, 195000.0", "900.0, 195000.0"),
    "MASS_FLOW": ("2.37, 20.0", "1.49, 0.87"),
}


SPECIES9 = ("C4H6", "H2O", "O2", "CO", "CO2", "H2", "O", "OH", "H")


def write_subset_library(wd, ns):
    """Library input files of the first `ns` species of the jet mixture (7 species = both shipped
    reactions; 4 species = reaction 1 only), written into the work dir in the reference's own formats
    (Mixture / Chemistry / list file); the per-species Thermo / Transp tables are the reference's, read in place."""
    os.makedirs(os.path.join(wd, "Mixture"))
    os.makedirs(os.path.join(wd, "Chemistry"))
    for d in ("Thermo", "Transp"):
        os.symlink(os.path.join(CASE_DIR, d), os.path.join(wd, d))
    mix = open(os.path.join(CASE_DIR, "Mixture/Test_Mixture.txt")).read().splitlines()
    rows = [ln for ln in mix if ln.split() and ln.split()[0] in SPECIES9[:ns]]
    with open(os.path.join(wd, "Mixture/Test_Mixture.txt"), "w") as f:
        f.write("//Number of species\n%d\n%s\n" % (ns, mix[2]) + "\n".join(rows) + "\n\nSTOP\n")
    chem = open(os.path.join(CASE_DIR, "Chemistry/Test_Reactions_second.txt")).read()
    if ns < 5:  # reaction 2 (CO + 0.5 O2 <=> CO2) needs CO2: reaction 1 only
        head, rest = chem.split("//Reactions", 1)
        r1 = rest.strip().split("\n\n")[0]
        chem = head.replace("2\n", "1\n", 1) + "//Reactions\n" + r1 + "\n\nSTOP\n"
    with open(os.path.join(wd, "Chemistry/Test_Reactions_second.txt"), "w") as f:
        f.write(chem)
    with open(os.path.join(wd, "test_chem_second.txt"), "w") as f:
        f.write("Mixture/Test_Mixture.txt\nChemistry/Test_Reactions_second.txt\n")
        for sp in SPECIES9[:ns]:
            f.write(f"Transp/{sp}_transp.txt\nThermo/{sp}_thermo.txt\n")


def make_workdir(case, mesh_writer, cfl, order, prec="LU_SGS", inlet="TEMPERATURE_IMPOSE", extra="",
                 time_flow="EULER_IMPLICIT", ns=9, slope_limiter="VENKATAKRISHNAN", case_dir=None, root="/tmp/rx_golden"):
    """A work dir holding a cfg of CFG_TEMPLATE, the mesh (mesh_writer) and the library files of case_dir (default:
    the reference's TURBOLENT_COMBUSTION; the tests pass the unpacked tests/golden/case_files.npz)."""
    case_dir = case_dir or CASE_DIR
    wd = os.path.join(root, case)
    shutil.rmtree(wd, ignore_errors=True)
    os.makedirs(os.path.join(wd, "out"))
    if ns == 9:
        for d in ("Mixture", "Chemistry", "Thermo", "Transp"):
            os.symlink(os.path.join(case_dir, d), os.path.join(wd, d))
        for lst in ("test_chem_second.txt", "test_chem_first.txt"):
            os.symlink(os.path.join(case_dir, lst), os.path.join(wd, lst))
    else:
        write_subset_library(wd, ns)
    mesh_name = mesh_writer(wd) if case_dir == CASE_DIR else mesh_writer(wd, case_dir)
    cfg = CFG_TEMPLATE.format(cfl=cfl, order=order, mesh=mesh_name, prec=prec, inlet_type=inlet,
                              inlet_ox=INLETS[inlet][0], inlet_fuel=INLETS[inlet][1], extra=extra, time_flow=time_flow)
    cfg = cfg.replace("SLOPE_LIMITER_FLOW= VENKATAKRISHNAN", "SLOPE_LIMITER_FLOW= " + slope_limiter)
    if ns != 9:  # the mixture's species lists
        y = lambda k: ", ".join("1.0" if q == k else "0.0" for q in range(ns))
        cfg = cfg.replace("FREESTREAM_MASS_FRAC = (0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)",
                          f"FREESTREAM_MASS_FRAC = ({y(2)})")
        cfg = cfg.replace("SPECIES_ORDER = (C4H6, H2O, O2, CO, CO2, H2, O, OH, H)",
                          "SPECIES_ORDER = (" + ", ".join(SPECIES9[:ns]) + ")")
        cfg = cfg.replace("INLET_MASS_FRAC = (Oxidizer_Inlet, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0; Fuel_Inlet, "
                          "1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)",
                          f"INLET_MASS_FRAC = (Oxidizer_Inlet, {y(2)}; Fuel_Inlet, {y(0)})")
    with open(os.path.join(wd, "case.cfg"), "w") as f:
        f.write(cfg)
    return wd


synth = _load("rx_synth", os.path.join(PKG, "synth.py"))


def fold_species(U, ns):
    """Conservative state of the first ns species (synth.fold_species, the bench's own fold)."""
    return synth.fold_species(U, ns)


def write_state(wd, U):
    with open(os.path.join(wd, "state.txt"), "w") as f:
        for g, row in enumerate(U):
            f.write(str(g) + " " + " ".join(f"{v:.17g}" for v in row) + "\n")


def run_harness(wd, bsr, extra=None):
    exe = os.path.join(HERE, "_ref", "harness")
    cmd = [exe, "case.cfg", "state.txt", "out"] + (["--bsr"] if bsr else []) + list(extra or [])
    r = subprocess.run(cmd, cwd=wd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        raise SystemExit(f"harness failed for {wd}")
    arrays = {}
    with open(os.path.join(wd, "out", "manifest.txt")) as f:
        for line in f:
            t = line.split()
            name, dt, shape = t[0], t[1], tuple(int(s) for s in t[2:])
            arrays[name] = np.fromfile(os.path.join(wd, "out", name + ".bin"), dtype="<" + dt).reshape(shape)
    return arrays


def mech_arrays(case_dir=None, list_file="test_chem_second.txt"):
    mech = _load("rx_oracle_mech", os.path.join(HERE, "mech.py"))
    m = mech.load_mechanism(case_dir or CASE_DIR, list_file)
    return {"mech_" + k: v for k, v in m.items()}


def case_mini9(nx=21, ny=11):
    pts, quads, bnd = meshgen.jet_mesh(nx, ny)
    xy, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    # nearest-point sampling of the converged field
    from scipy.spatial import cKDTree
    scale = np.array([1.0 / 0.125, 1.0 / 0.006])
    _, idx = cKDTree(xy * scale).query(pts * scale)
    U = cons[idx]

    def writer(wd):
        meshgen.write_su2(os.path.join(wd, "mesh.su2"), pts, quads, bnd)
        return "mesh.su2"

    wd = make_workdir("mini9", writer, cfl=5.0, order="1ST_ORDER")
    write_state(wd, U)
    a = run_harness(wd, bsr=True)
    wd = make_workdir("mini9_ilu", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0")
    write_state(wd, U)
    b = run_harness(wd, bsr=True)
    for k in ("ilu_factor", "ilu_rhs", "fgmres_ilu_x", "fgmres_ilu_info"):
        a[k] = b[k]
    # the SST implicit step solved with ILU0 (same system, other preconditioner)
    assert np.array_equal(a["sst_bsr_system"], b["sst_bsr_system"])
    for k in ("sst_lin_sol", "sst_new_sol", "sst_rms", "sst_post_mut", "sst_post_F1", "sst_post_F2",
              "sst_post_CDkw", "sst_post_grad"):
        a[k + "_ilu"] = b[k]
    assert np.array_equal(a["bsr_system"], b["bsr_system"])
    # keep the fixture small: the assembled system + ILU factor stay whole, per-edge Jacobians are
    # sampled (the whole-matrix assembly is checked against bsr_system)
    del a["bsr_jac_residual"]
    rng = np.random.default_rng(7)
    js = np.sort(rng.choice(len(a["edges"]), size=96, replace=False))
    a["jac_edge_sample"] = js
    for k in ("conv_jac_i", "conv_jac_j", "visc_jac_i", "visc_jac_j"):
        a[k] = a[k][js]
    ns = rng.choice(len(a["coord"]), size=64, replace=False)
    a["src_jac_sample"] = np.sort(ns)
    a["src_jac"] = a["src_jac"][a["src_jac_sample"]]
    a.update(mech_arrays())
    a["gen_points"] = pts
    a["gen_quads"] = quads
    return a


def case_rank9(split=None):
    """One MPI rank of mini9's implicit system: the reference's own CSysMatrix with domain points
    [0, P) and halo [P, N) (harness RX_RANK_SPLIT = P), its BuildILUPreconditioner / ComputeILUPreconditioner /
    ComputeLU_SGSPreconditioner on the system's blocks. The LU-SGS halo preset (halo_x.bin) is the forward-sweep
    result x* of the other rank, rows [P, N) as their own partition: the oracle's orc_lusgs_fwd_p, the restatement of
    that rank's (D+L) x* = b — what its SendReceive_Solution hands over. The golden holds the system, P, the preset and
    the reference's rank-0 outputs (rows [0, P)); tests/test_oracle_golden.py checks the oracle's partitioned
    ILU build / apply / LU-SGS (struct Parts, part_ptr = [0, P, N]) against them, tests/test_gpu_partitions.py the
    device's."""
    oracle = _load("rx_oracle_py", os.path.join(HERE, "oracle.py"))
    pts, quads, U, writer = mini9_inputs()
    wd = make_workdir("rank9", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0")
    write_state(wd, U)
    a = run_harness(wd, bsr=True)
    rp, col, A, b = a["bsr_row_ptr"], a["bsr_col"], a["bsr_system"], a["sys_rhs"]
    N = len(rp) - 1
    P = split or N // 2
    xs = oracle.lusgs_forward(rp, col, A, b.ravel(), part_ptr=np.array([0, P, N]))
    np.ascontiguousarray(xs, dtype="<f8").tofile(os.path.join(wd, "halo_x.bin"))
    env = dict(os.environ, RX_RANK_SPLIT=str(P))
    exe = os.path.join(HERE, "_ref", "harness")
    r = subprocess.run([exe, "case.cfg", "state.txt", "out", "--bsr"], cwd=wd, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        raise SystemExit("harness (RX_RANK_SPLIT) failed")
    out = {}
    with open(os.path.join(wd, "out", "manifest.txt")) as f:
        for line in f:
            t = line.split()
            out[t[0]] = np.fromfile(os.path.join(wd, "out", t[0] + ".bin"), dtype="<" + t[1]).reshape(
                tuple(int(q) for q in t[2:]))
    assert np.array_equal(out["bsr_system"], A)
    g = {k: a[k] for k in ("dims", "bsr_row_ptr", "bsr_col", "bsr_system", "sys_rhs")}
    g.update(rank_split=np.array([P]), rank_halo_x=xs, rank_ilu_factor=out["rank_ilu_factor"],
             rank_ilu_rhs=out["rank_ilu_rhs"], rank_lusgs_rhs=out["rank_lusgs_rhs"])
    return g  # the mesh and state are mini9's (the same inputs; the tests use tests/golden/mini9.npz for them)


def mini9_inputs(nx=21, ny=11):
    pts, quads, bnd = meshgen.jet_mesh(nx, ny)
    xy, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    from scipy.spatial import cKDTree
    scale = np.array([1.0 / 0.125, 1.0 / 0.006])
    _, idx = cKDTree(xy * scale).query(pts * scale)

    def writer(wd):
        meshgen.write_su2(os.path.join(wd, "mesh.su2"), pts, quads, bnd)
        return "mesh.su2"

    return pts, quads, cons[idx], writer


GEOM_KEYS = ("coord", "volume", "global_index", "nbr_ptr", "nbr", "edges", "edge_normal", "bvertex", "bvertex_normal",
             "wall_distance")


def case_bc9(inlet="TEMPERATURE_IMPOSE"):
    """next-3 / a8: the reference's Space_Integration with its boundary conditions (inlets of the given
    INLET_TYPE, outlet, isothermal walls; SST inlet / outlet / wall) on the mini9 jet, flow + SST, ILU0 cfg."""
    pts, quads, U, writer = mini9_inputs()
    wd = make_workdir("bc9_" + inlet, writer, cfl=5.0, order="1ST_ORDER", prec="ILU0", inlet=inlet)
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--bc"])
    # keep the BSR rows of the boundary points only (the interior rows are the plain assembly)
    rp = a["bsr_row_ptr"]
    rows = np.unique(a["bvertex"][:, 1])
    blk = np.concatenate([np.arange(rp[i], rp[i + 1]) for i in rows])
    a["bc_rows"] = rows
    a["bc_blk"] = blk
    for k in ("bc_pre_bsr", "bc_bsr", "sst_bc_pre_bsr", "sst_bc_bsr"):
        a[k] = a[k][blk]
    if inlet != "TEMPERATURE_IMPOSE":
        # same mesh, state and interior loops as bc9: keep only what the inlet kind changes
        return {k: a[k] for k in ("bc_res", "bc_bsr", "bc_charac", "bc_sol_old", "sst_bc_res", "sst_bc_bsr",
                                  "sst_bc_sol", "bc_marker", "bc_params")}
    a.update(mech_arrays())
    return a


def case_it9():
    """Whole reference outer iterations (CMeanFlowIteration::Iterate: flow MultiGrid_Iteration + SST
    SingleGrid_Iteration, boundary conditions included) from the mini9 state: 3 iterations, ILU0."""
    pts, quads, U, writer = mini9_inputs()
    wd = make_workdir("it9", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0")
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--iters", "3"])
    a.update(mech_arrays())
    return a


def case_gg9():
    """case_it9 with NUM_METHOD_GRAD= GREEN_GAUSS (CReactiveEulerSolver::SetPrimitive_Gradient_GG and
    CTurbSolver::SetSolution_Gradient_GG in place of the least-squares gradients): 2 outer iterations, ILU0."""
    pts, quads, U, writer = mini9_inputs()
    wd = make_workdir("gg9", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0", extra="NUM_METHOD_GRAD= GREEN_GAUSS\n%")
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--iters", "2"])
    a.update(mech_arrays())
    a["grad_method"] = np.array("GREEN_GAUSS")
    return a


def case_rst9():
    """The reference's own restart file (next-4): one reference outer iteration on the mini9 jet, then COutput's
    MergeCoordinates / MergeSolution / SetRestart (output_structure.cpp:3858-4060, the CDriver output step), as
    the harness's --restart writes it. Kept: the file's bytes, the iteration's U / (k, omega) (the doubles the file
    prints) and the point order."""
    pts, quads, U, writer = mini9_inputs()
    wd = make_workdir("rst9", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0")
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--iters", "1", "--restart"])
    with open(os.path.join(wd, "restart_flow.dat"), "rb") as f:
        text = f.read()
    return dict(restart_bytes=np.frombuffer(text, dtype=np.uint8), it1_U=a["it1_U"], it1_sst=a["it1_sst"],
                global_index=a["global_index"], dims=a["dims"])


# 3-D (config C5's extruded jet): 13 x 7 x 4 points, z planes as symmetry planes
MINI3D = (13, 7, 4)
SYM3D = "MARKER_SYM= ( sym_back, sym_front )\n"


def mini3d_inputs():
    """The extruded jet and a 3-D state: the converged 2-D field sampled at (x, y), plus a spanwise velocity
    w = 0.8 sin(pi z / depth) sin(pi x / L) m/s (zero on the symmetry planes) so that every third-component term of
    the operators is exercised; rho E gains the matching kinetic energy (T unchanged)."""
    nx, ny, nz = MINI3D
    pts, hexes, bnd = meshgen.jet_mesh3d(nx, ny, nz)
    xy, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    from scipy.spatial import cKDTree
    scale = np.array([1.0 / 0.125, 1.0 / 0.006])
    _, idx = cKDTree(xy * scale).query(pts[:, :2] * scale)
    c2 = cons[idx]  # [rho, rho u, rho v, rho E, rho Y x9, k, omega]
    depth = pts[:, 2].max()
    w = 0.8 * np.sin(np.pi * pts[:, 2] / depth) * np.sin(np.pi * pts[:, 0] / 0.125)
    rho = c2[:, 0]
    U = np.c_[c2[:, :3], rho * w, c2[:, 3] + 0.5 * rho * w * w, c2[:, 4:]]

    def writer(wd):
        meshgen.write_su2(os.path.join(wd, "mesh.su2"), pts, hexes, bnd)
        return "mesh.su2"

    return pts, hexes, U, writer


def case_mini3d():
    """mini9's dumps on the 3-D extruded jet (every operator, whole loops, BSR, LU-SGS / ILU0 / FGMRES, SST)."""
    pts, hexes, U, writer = mini3d_inputs()
    wd = make_workdir("mini3d", writer, cfl=5.0, order="1ST_ORDER", extra=SYM3D)
    write_state(wd, U)
    a = run_harness(wd, bsr=True)
    wd = make_workdir("mini3d_ilu", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0", extra=SYM3D)
    write_state(wd, U)
    b = run_harness(wd, bsr=True)
    for k in ("ilu_factor", "ilu_rhs", "fgmres_ilu_x", "fgmres_ilu_info"):
        a[k] = b[k]
    assert np.array_equal(a["sst_bsr_system"], b["sst_bsr_system"])
    for k in ("sst_lin_sol", "sst_new_sol", "sst_rms", "sst_post_mut", "sst_post_F1", "sst_post_F2",
              "sst_post_CDkw", "sst_post_grad"):
        a[k + "_ilu"] = b[k]
    assert np.array_equal(a["bsr_system"], b["bsr_system"])
    del a["bsr_jac_residual"]
    rng = np.random.default_rng(7)
    js = np.sort(rng.choice(len(a["edges"]), size=96, replace=False))
    a["jac_edge_sample"] = js
    for k in ("conv_jac_i", "conv_jac_j", "visc_jac_i", "visc_jac_j"):
        a[k] = a[k][js]
    ns = rng.choice(len(a["coord"]), size=64, replace=False)
    a["src_jac_sample"] = np.sort(ns)
    a["src_jac"] = a["src_jac"][a["src_jac_sample"]]
    a.update(mech_arrays())
    a["gen_points"] = pts
    a["gen_quads"] = hexes
    return a


def case_bc3d():
    """case_bc9 on the 3-D extruded jet (symmetry planes: no-op markers)."""
    pts, hexes, U, writer = mini3d_inputs()
    wd = make_workdir("bc3d", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0", extra=SYM3D)
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--bc"])
    rp = a["bsr_row_ptr"]
    rows = np.unique(a["bvertex"][:, 1])
    blk = np.concatenate([np.arange(rp[i], rp[i + 1]) for i in rows])
    a["bc_rows"] = rows
    a["bc_blk"] = blk
    for k in ("bc_pre_bsr", "bc_bsr", "sst_bc_pre_bsr", "sst_bc_bsr"):
        a[k] = a[k][blk]
    a.update(mech_arrays())
    return a


def case_it3d():
    """Whole reference outer iterations on the 3-D extruded jet: 2 iterations, ILU0."""
    pts, hexes, U, writer = mini3d_inputs()
    wd = make_workdir("it3d", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0", extra=SYM3D)
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--iters", "2"])
    a.update(mech_arrays())
    return a


def mix3d_inputs():
    """mini3d's extruded jet and state recipe on meshgen.mixed_mesh3d: prisms, pyramids (around added centroid points)
    and hexahedra, boundary triangles and quadrilaterals."""
    nx, ny, nz = MINI3D
    pts, elems, bnd = meshgen.mixed_mesh3d(nx, ny, nz)
    xy, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    from scipy.spatial import cKDTree
    scale = np.array([1.0 / 0.125, 1.0 / 0.006])
    _, idx = cKDTree(xy * scale).query(pts[:, :2] * scale)
    c2 = cons[idx]
    depth = pts[:, 2].max()
    w = 0.8 * np.sin(np.pi * pts[:, 2] / depth) * np.sin(np.pi * pts[:, 0] / 0.125)
    rho = c2[:, 0]
    U = np.c_[c2[:, :3], rho * w, c2[:, 3] + 0.5 * rho * w * w, c2[:, 4:]]

    def writer(wd):
        meshgen.write_su2_mixed(os.path.join(wd, "mesh.su2"), pts, elems, bnd)
        return "mesh.su2"

    return pts, elems, U, writer


def case_mix3d():
    """The SU2 reader's prism / pyramid branches (geometry_structure.cpp:8641-8794 orientation, the CPrism / CPyramid
    tables of primal_grid_structure.cpp:478-622 in the connectivity and the median dual) on a mixed-element mesh, and
    two whole reference outer iterations on it (ILU0). CFL 1: at mini3d's CFL 5 this start's FGMRES(5)+ILU0 solve
    on the mixed mesh is chaotic (reordering the inner products alone moves U by 16 %, the c2b mechanism of
    DESIGN.md §2), at CFL 1 the same perturbation moves it by 4e-15."""
    pts, elems, U, writer = mix3d_inputs()
    wd = make_workdir("mix3d", writer, cfl=1.0, order="1ST_ORDER", prec="ILU0", extra=SYM3D)
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--iters", "2"])
    a.update(mech_arrays())
    return a


def case_muscl3d():
    """a2 MUSCL branch + a13 Venkatakrishnan limiter in 3-D: the mini3d state with 2ND_ORDER_LIMITER (the
    jet9w dumps on the extruded jet: whole-loop residual, a sample of Jacobian rows, limiter, records)."""
    pts, hexes, U, writer = mini3d_inputs()
    wd = make_workdir("muscl3d", writer, cfl=0.1, order="2ND_ORDER_LIMITER", extra=SYM3D)
    write_state(wd, U)
    a = run_harness(wd, bsr=False)
    out = {k: a[k] for k in ("coord", "volume", "U", "V", "dPdU", "dTdU", "grad_prim", "limiter_out", "edges",
                             "edge_normal", "nbr_ptr", "nbr", "dims", "mach_inf", "limiter_params", "muscl_params",
                             "muscl_loop_res", "bvertex", "bvertex_normal", "wall_distance", "visc_params",
                             "src_params", "mu", "kappa", "Dij", "turb_k", "turb_omega", "mu_t",
                             "sigma_k", "grad_k", "eddy_visc_flow")}
    rng = np.random.default_rng(12345)
    N = len(a["coord"])
    rs = np.sort(rng.choice(N, size=48, replace=False))
    rp, cl, blk = a["muscl_bsr_row_ptr"], a["muscl_bsr_col"], a["muscl_bsr"]
    deg = max(int(rp[r + 1] - rp[r]) for r in rs)
    nv = blk.shape[1]
    mc = -np.ones((len(rs), deg), dtype=np.int64)
    mb = np.zeros((len(rs), deg, nv, nv))
    for q, r in enumerate(rs):
        cols = cl[rp[r]:rp[r + 1]]
        mc[q, :len(cols)] = cols
        mb[q, :len(cols)] = blk[rp[r]:rp[r + 1]]
    out["muscl_jac_rows"] = rs
    out["muscl_jac_cols"] = mc
    out["muscl_jac"] = mb
    out.update(mech_arrays())
    return out


BJ_KEYS = ("coord", "volume", "U", "V", "dPdU", "dTdU", "grad_prim", "limiter_out", "edges", "edge_normal",
           "nbr_ptr", "nbr", "dims", "mach_inf", "limiter_params", "muscl_params", "muscl_loop_res", "bvertex",
           "bvertex_normal", "wall_distance", "visc_params", "src_params", "mu", "kappa", "Dij", "turb_k",
           "turb_omega", "mu_t", "sigma_k", "grad_k", "eddy_visc_flow")


def case_bj9():
    """a13 Barth-Jespersen branch (solver_direct_reactive.cpp:1383-1440) in 2-D: the mini9 mesh and state with
    2ND_ORDER_LIMITER + SLOPE_LIMITER_FLOW= BARTH_JESPERSEN (limiter after the reference's own Preprocessing,
    and the MUSCL loop residual that reads it)."""
    pts, quads, bnd = meshgen.jet_mesh(21, 11)
    xy, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    from scipy.spatial import cKDTree
    scale = np.array([1.0 / 0.125, 1.0 / 0.006])
    _, idx = cKDTree(xy * scale).query(pts * scale)

    def writer(wd):
        meshgen.write_su2(os.path.join(wd, "mesh.su2"), pts, quads, bnd)
        return "mesh.su2"

    wd = make_workdir("bj9", writer, cfl=0.1, order="2ND_ORDER_LIMITER", slope_limiter="BARTH_JESPERSEN")
    write_state(wd, cons[idx])
    a = run_harness(wd, bsr=False)
    out = {k: a[k] for k in BJ_KEYS}
    out.update(mech_arrays())
    return out


def case_jet9w():
    def writer(wd):
        os.symlink(os.path.join(CASE_DIR, "mesh_stretched.su2"), os.path.join(wd, "mesh.su2"))
        return "mesh.su2"

    xy, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    wd = make_workdir("jet9", writer, cfl=0.1, order="2ND_ORDER_LIMITER")
    write_state(wd, cons)
    a = run_harness(wd, bsr=False)
    # window around the flame: strongest species gradients in the burning region
    coord = a["coord"]
    T = a["V"][:, 0]
    c = coord[np.argmax(T)]
    box = (np.abs(coord[:, 0] - c[0]) < 0.008) & (np.abs(coord[:, 1] - c[1]) < 0.0025)
    out = window_case(a, np.nonzero(box)[0])
    out.update(mech_arrays())
    return out


def case_jet9k():
    """The reference's whole 9 000-point jet (mesh_stretched.su2) with its converged PaSR state after the
    reference's own preprocessing: the node field the synthetic bench meshes interpolate (synth.jet_field_case),
    plus the dual-grid summary of the reference mesh. Only node records are kept (coords, U, V, k, omega, mu_t)."""
    def writer(wd):
        os.symlink(os.path.join(CASE_DIR, "mesh_stretched.su2"), os.path.join(wd, "mesh.su2"))
        return "mesh.su2"

    xy, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    wd = make_workdir("jet9k", writer, cfl=5.0, order="1ST_ORDER", prec="ILU0")
    write_state(wd, cons)
    a = run_harness(wd, bsr=False)
    out = {k: a[k] for k in ("coord", "volume", "global_index", "U", "V", "turb_k", "turb_omega", "mu_t",
                             "dims", "mach_inf", "visc_params", "src_params")}
    out["n_edge"] = np.array(len(a["edges"]))
    out.update(mech_arrays())
    return out


# keys an iteration golden keeps (the rest of the harness dump is the per-operator data the other cases hold)
ITER_KEEP = ("edges", "edge_normal", "coord", "volume", "nbr_ptr", "nbr", "bvertex", "bvertex_normal", "wall_distance",
             "bvertex_pn", "bc_marker", "bc_params", "dims", "mach_inf", "visc_params", "src_params", "dt_params",
             "p2v_params", "bsr_row_ptr", "bsr_col", "global_index")


def iteration_case(name, writer, U, ns, n_iters, cfl, prec, time_flow, extra="", order="1ST_ORDER", cfg_edit=None):
    wd = make_workdir(name, writer, cfl=cfl, order=order, prec=prec, time_flow=time_flow, ns=ns, extra=extra)
    if cfg_edit:
        path = os.path.join(wd, "case.cfg")
        text = open(path).read()
        with open(path, "w") as f:
            f.write(cfg_edit(text))
    write_state(wd, U)
    a = run_harness(wd, bsr=False, extra=["--iters", str(n_iters)])
    out = {k: a[k] for k in a if k in ITER_KEEP or k.startswith("it") or k == "limiter_params"}
    big = len(a["coord"]) > 5000  # whole-mesh cases: one iteration, no later Solution_Old needed
    out = {k: v for k, v in out.items()
           if not k.endswith("_wall") and not (big and k.endswith("_Uold") and k != "it_Uold0")}
    out.update(mech_arrays(wd) if ns != 9 else mech_arrays())
    out["time_flow"] = np.array(time_flow)
    out["lin_prec"] = np.array(prec)
    if "RK_ALPHA_COEFF" in extra:
        out["rk_alpha"] = np.array([float(x) for x in extra.split("(")[1].split(")")[0].split(",")])
    return out


def full_jet_writer(wd, case_dir=None):
    os.symlink(os.path.join(case_dir or CASE_DIR, "mesh_stretched.su2"), os.path.join(wd, "mesh.su2"))
    return "mesh.su2"


def case_itx9():
    """The reference's shipped jet setup (my_combustion_second_chem_PaSR.cfg: TIME_DISCRE_FLOW = EULER_EXPLICIT,
    CFL 0.1, implicit SST with LU_SGS) on its whole 9 000-point mesh_stretched.su2 from its converged PaSR state,
    9 species: one whole reference outer iteration (the fixture holds the whole mesh; a second iteration would
    double it)."""
    _, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    return iteration_case("itx9", full_jet_writer, cons, 9, 1, 0.1, "LU_SGS", "EULER_EXPLICIT")


def ig9_workdir(case_dir=None, root="/tmp/rx_golden"):
    """Work dir of stage 1 (my_combustion_first_chem_PaSR.cfg's keys on CFG_TEMPLATE)."""
    wd = make_workdir("ig9", full_jet_writer, cfl=0.1, order="1ST_ORDER", prec="LU_SGS", time_flow="EULER_EXPLICIT",
                      case_dir=case_dir, root=root)
    cfg = open(os.path.join(wd, "case.cfg")).read()
    cfg = cfg.replace("CONFIG_LIB_FILE = test_chem_second.txt", "CONFIG_LIB_FILE = test_chem_first.txt")
    cfg = cfg.replace("IGNITION = NO", "IGNITION = YES\nIGNITION_ITER = 8000\nFUEL_INDEX = 0\nOXIDIZER_INDEX = 2")
    with open(os.path.join(wd, "case.cfg"), "w") as f:
        f.write(cfg)
    return wd


def fp_workdir(case_dir=None, root="/tmp/rx_golden", name="fpit", cfg_edit=None):
    """Work dir of the flat plate (FP_CFG) over the plate's files (default: the reference's TURBOLENT_FLAT_PLATE);
    cfg_edit(text) -> text changes the cfg."""
    case_dir = case_dir or FP_DIR
    wd = os.path.join(root, name)
    shutil.rmtree(wd, ignore_errors=True)
    os.makedirs(os.path.join(wd, "out"))
    for d in ("Mixture", "Thermo", "Transp"):
        os.symlink(os.path.join(case_dir, d), os.path.join(wd, d))
    os.symlink(os.path.join(case_dir, "test_air.txt"), os.path.join(wd, "test_air.txt"))
    os.symlink(os.path.join(case_dir, "mesh_flatplate_turb_137x97.su2"), os.path.join(wd, "mesh.su2"))
    with open(os.path.join(wd, "case.cfg"), "w") as f:
        f.write(cfg_edit(FP_CFG) if cfg_edit else FP_CFG)
    return wd


def case_ig9():
    """Stage 1 of the reference's own procedure (my_combustion_first_chem_PaSR.cfg: the first chemistry,
    test_chem_first.txt, IGNITION = YES with IGNITION_ITER 8000, FUEL_INDEX 0, OXIDIZER_INDEX 2, EULER_EXPLICIT at
    CFL 0.1, LU_SGS SST) restarted, as that cfg is, from the converged non-reacting field (PLOT/no_chem.dat) on the
    whole 9 000-point mesh: the ignition branch of SetPrimitive_Variables (solver_direct_reactive.cpp:1013-1024)
    raises T to 1700 K at the 1 283 mixing points, in the start-up preprocessing and in the iteration. One reference
    outer iteration."""
    _, cons = read_plot(os.path.join(CASE_DIR, "PLOT/no_chem.dat"))
    wd = ig9_workdir()
    write_state(wd, cons)
    a = run_harness(wd, bsr=False, extra=["--iters", "1"])
    out = {k: a[k] for k in a if k in ITER_KEEP or k.startswith("it")}
    out = {k: v for k, v in out.items() if not k.endswith("_wall") and not (k.endswith("_Uold") and k != "it_Uold0")}
    out.update(mech_arrays(CASE_DIR, "test_chem_first.txt"))
    out["time_flow"] = np.array("EULER_EXPLICIT")
    out["lin_prec"] = np.array("LU_SGS")
    out["ignition"] = np.array([1.0, 8000.0, 1700.0, 0.0, 2.0])  # IGNITION, _ITER, _TEMPERATURE, FUEL_, OXIDIZER_INDEX
    return out


def case_itx4():
    """BASELINE configs[0] (C1): the 9 000-point jet, 4 species (reaction 1 only; library files of the mixture's
    first four species), explicit Runge-Kutta (RK_ALPHA_COEFF 0.66667 / 0.66667 / 1), SST with LU_SGS, from the
    converged state with the dropped species folded in: one reference outer iteration (three RK stages)."""
    _, cons = read_plot(os.path.join(CASE_DIR, "PLOT/flow_second_chem.dat"))
    return iteration_case("itx4", full_jet_writer, fold_species(cons, 4), 4, 1, 0.1, "LU_SGS", "RUNGE-KUTTA_EXPLICIT",
                          extra="RK_ALPHA_COEFF= ( 0.66667, 0.66667, 1.000000 )\n")


def case_it7():
    """The bench mechanism (7 species, both reactions) through the reference: the mini9 jet, implicit ILU0, two
    reference outer iterations."""
    pts, quads, U, writer = mini9_inputs()
    return iteration_case("it7", writer, fold_species(U, 7), 7, 2, 5.0, "ILU0", "EULER_IMPLICIT")


def case_it4t(limiter=False):
    """The SST's second-order upwind on a reacting state (the flat plate's composition is uniform, so there its
    density reconstruction along the gradient of X_0 — CTurbSolver::Upwind_Residual reconstructs the flow record
    entry iVar with gradient row iVar, solver_direct_turbulent.cpp:481-493 — and the flow limiter entry it reads past
    the end are invisible): the mini9 jet with the 4-species mechanism (nPrimVarGrad = 8 fits the reference's
    FlowPrimVar of nDim + 7 = 9 entries; with more species the reference writes past it), implicit ILU0 at CFL 1,
    SPATIAL_ORDER_TURB= 2ND_ORDER (it4t) or 2ND_ORDER_LIMITER with the flow at 2ND_ORDER_LIMITER (it4tl), two
    reference outer iterations."""
    pts, quads, U, writer = mini9_inputs()
    ord_t = "2ND_ORDER_LIMITER" if limiter else "2ND_ORDER"
    out = iteration_case("it4tl" if limiter else "it4t", writer, fold_species(U, 4), 4, 2, 1.0, "ILU0",
                         "EULER_IMPLICIT", extra=f"SPATIAL_ORDER_TURB= {ord_t}\n",
                         order="2ND_ORDER_LIMITER" if limiter else "1ST_ORDER")
    out["spatial_order"] = np.array(2 if limiter else 0)
    out["sst_spatial_order"] = np.array(2 if limiter else 1)
    return out


def case_itns(ns):
    """The mini9 jet with the first ns species of the jet mixture (subset library; ns 5, 6, 8: the species counts the
    device instantiates besides the shipped 3 / 9 and the bench's 4 / 7, csrc/rx_species.h), implicit ILU0 at CFL 1,
    two reference outer iterations."""
    pts, quads, U, writer = mini9_inputs()
    return iteration_case(f"it{ns}s", writer, fold_species(U, ns), ns, 2, 1.0, "ILU0", "EULER_IMPLICIT")


def case_lam4():
    """The laminar REACTIVE_NAVIER_STOKES outer iteration (KIND_TURB_MODEL= NONE: CMeanFlowIteration::Iterate runs the
    flow's MultiGrid_Iteration alone, iteration_structure.cpp:531-534; no SST solver, no eddy viscosity, the laminar
    PaSR branch): the mini9 jet with the 4-species mechanism (as it4t), implicit ILU0 at CFL 1, two reference outer
    iterations."""
    pts, quads, U, writer = mini9_inputs()
    out = iteration_case("lam4", writer, fold_species(U, 4)[:, :-2], 4, 2, 1.0, "ILU0", "EULER_IMPLICIT",
                         cfg_edit=lambda t: t.replace("KIND_TURB_MODEL= SST", "KIND_TURB_MODEL= NONE"))
    out["laminar"] = np.array(1)
    return out


def case_sup4():
    """CReactiveEulerSolver::BC_Supersonic_Inlet / BC_Supersonic_Outlet (solver_direct_reactive.cpp:2998-3206,
    :3681-3800) on the laminar lam4 setup: both inlets MARKER_SUPERSONIC_INLET (oxidizer 300 K, 130 kPa, 20 m/s; fuel
    800 K, 130 kPa, 0.87 m/s: the whole ghost state imposed; a subsonic MARKER_INLET beside them is not possible —
    BC_Inlet asserts one INLET_MASS_FRAC entry per MARKER_INLET, :3245, while the supersonic inlet reads its mass
    fractions from that same list), the outlet a MARKER_SUPERSONIC_OUTLET (ghost = the domain state); two reference
    outer iterations. Laminar because the reference's two supersonic
    BCs never hand the turbulence quantities to their viscous numerics (the MANGOTURB add-on of BC_Inlet / BC_Outlet,
    :3607-3621, is missing there), so under SST they read whatever the previous boundary call left in that object."""
    pts, quads, U, writer = mini9_inputs()

    def edit(t):
        t = t.replace("KIND_TURB_MODEL= SST", "KIND_TURB_MODEL= NONE")
        t = t.replace("MARKER_INLET= ( Oxidizer_Inlet, 300.0, 20.0, 1.0, 0.0, 0.0, Fuel_Inlet, 800.0, 0.87, 0.0, 1.0, 0.0)",
                      "MARKER_SUPERSONIC_INLET= ( Oxidizer_Inlet, 300.0, 130000.0, 20.0, 0.0, 0.0, "
                      "Fuel_Inlet, 800.0, 130000.0, 0.0, 0.87, 0.0)")
        t = t.replace("MARKER_OUTLET= ( Outlet, 101325.0)", "MARKER_SUPERSONIC_OUTLET= ( Outlet )")
        assert "MARKER_SUPERSONIC_INLET" in t and "MARKER_SUPERSONIC_OUTLET" in t
        return t

    out = iteration_case("sup4", writer, fold_species(U, 4)[:, :-2], 4, 2, 1.0, "ILU0", "EULER_IMPLICIT",
                         cfg_edit=edit)
    out["laminar"] = np.array(1)
    return out


# CSysSolve::Solve's branches (linear_solvers_structure.cpp:626-708) beside the default FGMRES: (LINEAR_SOLVER,
# LINEAR_SOLVER_PREC, LINEAR_SOLVER_RESTART_FREQUENCY) of each golden
LIN_CASES = {"lsbc": ("BCGSTAB", "ILU0", 10), "lsbj": ("BCGSTAB", "JACOBI", 10), "lsfj": ("FGMRES", "JACOBI", 10),
             "lsrs": ("RESTARTED_FGMRES", "LU_SGS", 2), "lssl": ("SMOOTHER_LUSGS", "LU_SGS", 10),
             "lssj": ("SMOOTHER_JACOBI", "LU_SGS", 10), "lssi": ("SMOOTHER_ILU0", "LU_SGS", 10)}


def lin_edit(t, solver):
    t = t.replace("LINEAR_SOLVER= FGMRES", "LINEAR_SOLVER= " + solver)
    if solver == "RESTARTED_FGMRES":  # cycles that stop early (tolerance met), so the restart loop runs several
        t = t.replace("LINEAR_SOLVER_ERROR= 1E-6", "LINEAR_SOLVER_ERROR= 0.05")
    return t


def case_lin(name):
    """The mini9 jet with the 4-species mechanism (as it4t) through one of CSysSolve::Solve's other branches
    (LIN_CASES: BCGSTAB_LinSolver, the JACOBI preconditioner, RESTARTED_FGMRES, the LU_SGS / Jacobi / ILU0 smoothers)
    for the flow and the SST solve: implicit at CFL 1, LINEAR_SOLVER_ITER 5, two reference outer iterations."""
    solver, prec, restart = LIN_CASES[name]
    pts, quads, U, writer = mini9_inputs()
    out = iteration_case(name, writer, fold_species(U, 4), 4, 2, 1.0, prec, "EULER_IMPLICIT",
                         extra=f"LINEAR_SOLVER_RESTART_FREQUENCY= {restart}\n",
                         cfg_edit=lambda t: lin_edit(t, solver))
    out["lin_solver"] = np.array(solver)
    out["lin_restart"] = np.array(restart)
    return out


FP_DIR = os.path.join(REF, "Test_Cases/TURBOLENT/TURBOLENT_FLAT_PLATE")
FP_CFG = """\
% golden-vector cfg written by oracle/make_golden.py: the reference's turbulent flat plate (air, 3 species, no
% reactions; values of Test_Cases/TURBOLENT/TURBOLENT_FLAT_PLATE/my_turbulent_flatplate_air.cfg)
CONFIG_LIB_FILE = test_air.txt
FREESTREAM_MASS_FRAC = (0.2197, 0.0302, 0.7501)
SPECIES_ORDER = (O2, CO2, N2)
PHYSICAL_PROBLEM= REACTIVE_NAVIER_STOKES
KIND_TURB_MODEL= SST
MATH_PROBLEM= DIRECT
RESTART_SOL= NO
MACH_NUMBER= 0.2
FREESTREAM_TEMPERATURE= 297.62
FREESTREAM_VELOCITY= (69.1687, 0.0, 0.0)
FREESTREAM_PRESSURE= 113303.0
REYNOLDS_LENGTH= 1.000
REYNOLDS_NUMBER= 500000
REF_DIMENSIONALIZATION= DIMENSIONAL
REF_LENGTH= 1.0
REF_AREA= 2.00
MARKER_HEATFLUX = (wall, 0.0)
MARKER_EULER= ( symmetry )
MARKER_INLET= ( inlet, 300.0, 100000.0, 1.0, 0.0, 0.0 )
INLET_MASS_FRAC = (inlet, 0.2197, 0.0302, 0.7501)
MARKER_OUTLET= ( outlet, 97250.0, farfield, 97250.0 )
NUM_METHOD_GRAD= WEIGHTED_LEAST_SQUARES
CFL_NUMBER= 9
CFL_ADAPT= NO
EXT_ITER= 1
LINEAR_SOLVER= FGMRES
LINEAR_SOLVER_PREC= LU_SGS
LINEAR_SOLVER_ERROR= 1E-6
LINEAR_SOLVER_ITER= 5
MGLEVEL= 0
CONV_NUM_METHOD_FLOW= AUSM
SPATIAL_ORDER_FLOW= 2ND_ORDER
SLOPE_LIMITER_FLOW= VENKATAKRISHNAN
TIME_DISCRE_FLOW= EULER_IMPLICIT
CONV_NUM_METHOD_TURB= SCALAR_UPWIND
SLOPE_LIMITER_TURB= VENKATAKRISHNAN
TIME_DISCRE_TURB= EULER_IMPLICIT
CONV_CRITERIA= RESIDUAL
RESIDUAL_REDUCTION= 6
RESIDUAL_MINVAL= -7
MESH_FILENAME= mesh.su2
MESH_FORMAT= SU2
OUTPUT_FORMAT= TECPLOT
CONV_FILENAME= history
WRT_SOL_FREQ= 100000
WRT_CON_FREQ= 1
"""


def case_fp3():
    """The reference's own second test case: the 137x97 turbulent flat plate (air: O2, CO2, N2, no reactions) with
    its converged state (PLOT/flow.dat), cfg SPATIAL_ORDER_FLOW = 2ND_ORDER (the unlimited MUSCL branch); a window
    of the boundary layer at the leading edge is kept, as for jet9w."""
    wd = "/tmp/rx_golden/fp3"
    shutil.rmtree(wd, ignore_errors=True)
    os.makedirs(os.path.join(wd, "out"))
    for d in ("Mixture", "Thermo", "Transp"):
        os.symlink(os.path.join(FP_DIR, d), os.path.join(wd, d))
    os.symlink(os.path.join(FP_DIR, "test_air.txt"), os.path.join(wd, "test_air.txt"))
    os.symlink(os.path.join(FP_DIR, "mesh_flatplate_turb_137x97.su2"), os.path.join(wd, "mesh.su2"))
    with open(os.path.join(wd, "case.cfg"), "w") as f:
        f.write(FP_CFG)
    xy, cons = read_plot(os.path.join(FP_DIR, "PLOT/flow.dat"), ncons=9)
    write_state(wd, cons)
    a = run_harness(wd, bsr=False)
    coord = a["coord"]
    box = (coord[:, 0] > -0.02) & (coord[:, 0] < 0.06) & (coord[:, 1] < 0.004)
    out = window_case(a, np.nonzero(box)[0])
    out.update(mech_arrays(FP_DIR, "test_air.txt"))
    return out


def case_fpit():
    """The reference's second shipped case end to end: one whole reference outer iteration of the turbulent flat plate
    (Test_Cases/TURBOLENT/TURBOLENT_FLAT_PLATE, the whole 137x97 mesh = 13 289 points, air O2 / CO2 / N2 without
    reactions, nVar 7) from its converged state (PLOT/flow.dat), with its cfg's markers: MARKER_HEATFLUX (wall, 0),
    MARKER_EULER (symmetry), a TOTAL_CONDITIONS inlet and two outlets; 2ND_ORDER (unlimited MUSCL), EULER_IMPLICIT
    with FGMRES(5) + LU_SGS at CFL 9."""
    wd = fp_workdir()
    _, cons = read_plot(os.path.join(FP_DIR, "PLOT/flow.dat"), ncons=9)
    write_state(wd, cons)
    a = run_harness(wd, bsr=False, extra=["--iters", "1"])
    out = {k: a[k] for k in a if k in ITER_KEEP or k.startswith("it")}
    out = {k: v for k, v in out.items() if not k.endswith("_wall") and not (k.endswith("_Uold") and k != "it_Uold0")}
    out.update(mech_arrays(FP_DIR, "test_air.txt"))
    out["time_flow"] = np.array("EULER_IMPLICIT")
    out["lin_prec"] = np.array("LU_SGS")
    out["spatial_order"] = np.array(1)  # 2ND_ORDER: MUSCL without limiter
    return out


def case_fpit2(limiter=False):
    """The whole flat plate (fpit) with the SST's second-order upwind: SPATIAL_ORDER_TURB= 2ND_ORDER (fpit2), or
    2ND_ORDER_LIMITER with SLOPE_LIMITER_TURB= VENKATAKRISHNAN and the flow's SPATIAL_ORDER_FLOW= 2ND_ORDER_LIMITER
    (fpit2l: CTurbSolver::Upwind_Residual's MUSCL branch, solver_direct_turbulent.cpp:464-510, on the limiters of
    CSolver::SetSolution_Limiter, solver_structure.cpp:951-1204, and of the flow's SetPrimitive_Limiter that
    CTurbSSTSolver::Preprocessing repeats, :2945-2949). One reference outer iteration from the converged state."""
    def edit(t):
        t = t.replace("SLOPE_LIMITER_TURB= VENKATAKRISHNAN",
                      "SLOPE_LIMITER_TURB= VENKATAKRISHNAN\nSPATIAL_ORDER_TURB= " +
                      ("2ND_ORDER_LIMITER" if limiter else "2ND_ORDER"))
        if limiter:
            t = t.replace("SPATIAL_ORDER_FLOW= 2ND_ORDER", "SPATIAL_ORDER_FLOW= 2ND_ORDER_LIMITER")
        return t
    wd = fp_workdir(name="fpit2l" if limiter else "fpit2", cfg_edit=edit)
    _, cons = read_plot(os.path.join(FP_DIR, "PLOT/flow.dat"), ncons=9)
    write_state(wd, cons)
    a = run_harness(wd, bsr=False, extra=["--iters", "1"])
    out = {k: a[k] for k in a if k in ITER_KEEP or k.startswith("it") or k == "limiter_params"}
    out = {k: v for k, v in out.items() if not k.endswith("_wall") and not (k.endswith("_Uold") and k != "it_Uold0")}
    out.update(mech_arrays(FP_DIR, "test_air.txt"))
    out["time_flow"] = np.array("EULER_IMPLICIT")
    out["lin_prec"] = np.array("LU_SGS")
    out["spatial_order"] = np.array(2 if limiter else 1)
    out["sst_spatial_order"] = np.array(2 if limiter else 1)
    return out


def window_case(a, keep):
    """Restrict a whole-mesh harness dump to the points `keep` (and the edges between them); interior = points
    whose whole neighbourhood is kept (where loop results are complete)."""
    coord = a["coord"]
    loc = -np.ones(len(coord), dtype=np.int64)
    loc[keep] = np.arange(len(keep))
    e = a["edges"]
    ekeep = np.nonzero((loc[e[:, 0]] >= 0) & (loc[e[:, 1]] >= 0))[0]
    nb_ptr, nb = a["nbr_ptr"], a["nbr"]
    interior = np.array([all(loc[nb[nb_ptr[i]:nb_ptr[i + 1]]] >= 0) for i in keep])
    out = {}
    node_keys = ["coord", "volume", "global_index", "U", "V", "dPdU", "dTdU", "mu", "kappa", "cp", "Dij",
                 "grad_prim", "limiter", "turb_k", "turb_omega", "mu_t", "sigma_k", "grad_k", "src_res",
                 "src_jac", "limiter_out", "grad_lsq_out", "wall_distance",
                 "eddy_visc_flow", "sst_sol", "sst_grad", "sst_F1", "sst_F2", "sst_CDkw", "strain_mag",
                 "sst_src_res", "sst_src_jac", "p2v_U", "p2v_V_before", "p2v_tke", "p2v_mut", "p2v_U_after", "p2v_V",
                 "p2v_dPdU", "p2v_dTdU", "p2v_mu", "p2v_kappa", "p2v_cp", "p2v_eddy", "p2v_Dij"]
    for k in node_keys:
        out[k] = a[k][keep]
    out["interior"] = interior
    # local neighbour CSR restricted to interior points' full lists
    lp, ln = [0], []
    for i in keep:
        nbl = loc[nb[nb_ptr[i]:nb_ptr[i + 1]]]
        ln.extend(int(x) for x in nbl if x >= 0)
        lp.append(len(ln))
    out["nbr_ptr"] = np.array(lp, dtype=np.int64)
    out["nbr"] = np.array(ln, dtype=np.int64)
    out["edges"] = loc[e[ekeep]]
    out["edge_normal"] = a["edge_normal"][ekeep]
    for k in ("conv_res", "visc_res", "sst_upw_res", "sst_upw_jac_i", "sst_upw_jac_j", "sst_visc_res",
              "sst_visc_jac_i", "sst_visc_jac_j"):
        out[k] = a[k][ekeep]
    rng = np.random.default_rng(12345)
    js = np.sort(rng.choice(len(ekeep), size=min(256, len(ekeep)), replace=False))
    out["jac_edge_sample"] = js
    for k in ("conv_jac_i", "conv_jac_j", "visc_jac_i", "visc_jac_j"):
        out[k] = a[k][ekeep][js]
    for k in ("dims", "mach_inf", "visc_params", "src_params", "limiter_params", "muscl_params", "p2v_params"):
        out[k] = a[k]
    # a2 MUSCL branch: whole-loop residual at the window points (compared at interior points, whose
    # incident edges are all in the window) and the Jacobian rows of a sample of interior points
    out["muscl_loop_res"] = a["muscl_loop_res"][keep]
    irows = np.nonzero(interior)[0]
    rs = np.sort(rng.choice(irows, size=min(48, len(irows)), replace=False))
    rp, cl, blk = a["muscl_bsr_row_ptr"], a["muscl_bsr_col"], a["muscl_bsr"]
    deg = max(int(rp[keep[r] + 1] - rp[keep[r]]) for r in rs)
    nv = blk.shape[1]
    mc = -np.ones((len(rs), deg), dtype=np.int64)
    mb = np.zeros((len(rs), deg, nv, nv))
    for q, r in enumerate(rs):
        g = keep[r]
        cols = loc[cl[rp[g]:rp[g + 1]]]
        mc[q, :len(cols)] = cols
        mb[q, :len(cols)] = blk[rp[g]:rp[g + 1]]
    out["muscl_jac_rows"] = rs
    out["muscl_jac_cols"] = mc
    out["muscl_jac"] = mb
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="mini9,jet9w")
    args = ap.parse_args()
    subprocess.run(["make", "-s", "-f", os.path.join(HERE, "ref_build.mk"), "-j8", "all", "harness"], check=True,
                   cwd=REPO)
    gold = os.path.join(REPO, "tests", "golden")
    os.makedirs(gold, exist_ok=True)
    for case in args.cases.split(","):
        a = {"mini9": case_mini9, "jet9w": case_jet9w, "bc9": case_bc9, "it9": case_it9,
             "bc9t": lambda: case_bc9("TOTAL_CONDITIONS"), "bc9m": lambda: case_bc9("MASS_FLOW"),
             "mini3d": case_mini3d, "bc3d": case_bc3d, "it3d": case_it3d, "muscl3d": case_muscl3d,
             "fp3": case_fp3, "jet9k": case_jet9k, "itx9": case_itx9, "itx4": case_itx4, "ig9": case_ig9, "rst9": case_rst9, "fpit": case_fpit, "it7": case_it7,
             "bj9": case_bj9, "gg9": case_gg9, "mix3d": case_mix3d, "fpit2": case_fpit2,
             "fpit2l": lambda: case_fpit2(limiter=True), "it4t": case_it4t,
             "it4tl": lambda: case_it4t(limiter=True), "rank9": case_rank9, "lam4": case_lam4, "sup4": case_sup4,
             **{k: (lambda k=k: case_lin(k)) for k in LIN_CASES},
             **{f"it{n}s": (lambda n=n: case_itns(n)) for n in (5, 6, 8)}}[case]()
        path = os.path.join(gold, case + ".npz")
        np.savez_compressed(path, **a)
        print(f"{case}: {len(a)} arrays -> {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
