"""C++ host path (include/rx_solver.hpp, the reference-shaped solver class over the C ABI):
tests/cpp/rx_driver.cpp drives one explicit and one implicit iteration in CIntegration order on the
golden mini jet; results are checked against the reference's golden residual / time step and the
oracle's clipped update."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from tests.parity import assert_close
from tests.rxpkg import rx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.dirname(rx.__file__)


def build_driver(out):
    cmd = ["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp",
           "rx_driver.cpp"), "-L", PKG, "-lrx", "-Wl,-rpath," + PKG, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)


def test_cpp_driver_builds(tmp_path):
    rx.lib()  # librx.so present
    exe = str(tmp_path / "rx_driver")
    build_driver(exe)
    assert os.path.exists(exe)


def write_case(d, g):
    def w(name, arr, dt):
        np.ascontiguousarray(arr, dtype=dt).tofile(os.path.join(d, name + {np.float64: ".f64", np.int64: ".i64",
                                                                             np.int32: ".i32"}[dt]))
    for k in ("edges", "nbr_ptr", "nbr"):
        w(k, g[k], np.int64)
    w("bvertex", np.asarray(g["bvertex"])[:, :2], np.int64)
    for k in ("edge_normal", "coord", "volume", "bvertex_normal", "U", "V", "dPdU", "dTdU", "mu", "kappa", "Dij",
              "grad_prim", "turb_k", "turb_omega", "mu_t", "sigma_k", "grad_k", "wall_distance", "sst_sol", "sst_F1",
              "sst_F2", "sst_CDkw"):
        w(k, g[k], np.float64)
    w("eddy_visc_flow", g.get("eddy_visc_flow", g["mu_t"]), np.float64)
    for k in ("mmass", "diff_vol", "stoich_reac", "stoich_prod", "exp_reac", "exp_prod", "A", "beta", "Ta", "A_back",
              "beta_back", "Ta_back", "tab_x", "tab_y", "tab_y2"):
        w("mech_" + k, g["mech_" + k], np.float64)
    for k in ("reversible", "has_backward"):
        w("mech_" + k, g["mech_" + k], np.int32)
    w("cfg", [g["mach_inf"][0], g["visc_params"][1], g["visc_params"][2], g["src_params"][0], g["src_params"][1],
              g["dt_params"][0]], np.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("implicit", [0, 1])
def test_cpp_driver_matches_reference(tmp_path, implicit):
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "mini9.npz")))
    d = str(tmp_path)
    write_case(d, g)
    exe = os.path.join(d, "rx_driver")
    build_driver(exe)
    r = subprocess.run([exe, d, str(implicit)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    nVar = g["U"].shape[1]
    res = np.fromfile(os.path.join(d, "out_res.f64")).reshape(-1, nVar)
    ref = g["loop_total_res"]
    assert_close(res[:, :4], ref[:, :4], what="C++ driver residual flow rows")
    assert np.max(np.abs(res[:, 4:] - ref[:, 4:])) <= 1e-10 * np.abs(ref[:, 4:]).max()
    assert_close(np.fromfile(os.path.join(d, "out_dt.f64")), g["dt"], what="C++ driver dt")
    U = np.fromfile(os.path.join(d, "out_u.f64")).reshape(-1, nVar)
    if not implicit:
        U_ref = O.update(g["U"], res, 2, 1, 1.0, g["volume"], g["dt"])
        assert_close(U, U_ref, what="C++ driver explicit update")
    else:
        assert np.all(np.isfinite(U)) and "lin_iters=5" in r.stdout
        # the SST iteration (TurbSSTSolver, ILU0) against the reference's own turbulent step
        T = np.fromfile(os.path.join(d, "out_sst_u.f64")).reshape(-1, 2)
        for v in range(2):
            assert_close(T[:, v], g["sst_new_sol_ilu"][:, v], what=f"C++ driver SST (k, omega)[{v}]")
        assert_close(np.fromfile(os.path.join(d, "out_sst_rms.f64")), g["sst_rms_ilu"], what="C++ driver SST RMS")
        assert_close(np.fromfile(os.path.join(d, "out_sst_mut.f64")), g["sst_post_mut_ilu"], what="C++ driver mu_t")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["it9", "itx9", "itx4", "lam4", "sup4"])
def test_cpp_driver_reference_iteration(tmp_path, case):
    """rx::Iterate (the reference's outer iteration with the jet's boundary conditions) from the C++ mirror, against
    the reference's own iteration: it9 (implicit, ILU0), itx9 (the shipped cfg: EULER_EXPLICIT flow, LU_SGS SST, the
    whole reference mesh), itx4 (C1: 4 species, RUNGE-KUTTA_EXPLICIT, 3 stages); lam4 (round 6): the laminar
    REACTIVE_NAVIER_STOKES iteration through rx::IterateFlow; sup4 (round 6): the same with the supersonic inlet /
    outlet markers."""
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", case + ".npz")))
    laminar = "laminar" in g
    if laminar:  # no SST records: zeros stand in for the files the RANS branch reads
        N = len(g["it_U0"])
        g.update(it_sst0=np.zeros((N, 2)), it_mut0=np.zeros(N), it_F1_0=np.zeros(N), it_F2_0=np.zeros(N),
                 it_CDkw0=np.zeros(N), it_sstgrad0=np.zeros((N, 2, 2)))
    d = str(tmp_path)

    def w(name, arr, dt):
        np.ascontiguousarray(arr, dtype=dt).tofile(os.path.join(d, name + {np.float64: ".f64", np.int64: ".i64",
                                                                             np.int32: ".i32"}[dt]))
    for k in ("edges", "nbr_ptr", "nbr", "bvertex_pn"):
        w(k, g[k], np.int64)
    w("bvertex", np.asarray(g["bvertex"])[:, :2], np.int64)
    for k in ("edge_normal", "coord", "volume", "bvertex_normal", "wall_distance", "it_U0", "it_V0", "it_sst0",
              "it_mut0", "it_F1_0", "it_F2_0", "it_CDkw0", "it_sstgrad0"):
        w(k, g[k], np.float64)
    for k in ("mmass", "diff_vol", "stoich_reac", "stoich_prod", "exp_reac", "exp_prod", "A", "beta", "Ta", "A_back",
              "beta_back", "Ta_back", "tab_x", "tab_y", "tab_y2"):
        w("mech_" + k, g["mech_" + k], np.float64)
    for k in ("reversible", "has_backward"):
        w("mech_" + k, g["mech_" + k], np.int32)
    w("cfg", [0.0] * 6, np.float64)
    bp, p2v = g["bc_params"], g["p2v_params"]
    w("cfg_it", [g["mach_inf"][0], g["visc_params"][0], g["visc_params"][1], g["visc_params"][2], g["src_params"][0],
                 g["src_params"][1], g["dt_params"][0], g["dt_params"][1], bp[19], bp[20], bp[22], p2v[1], p2v[2],
                 bp[23], bp[24]], np.float64)
    flow_imp = str(g.get("time_flow", "EULER_IMPLICIT")) == "EULER_IMPLICIT"
    w("cfg_scheme", [1.0 if flow_imp else 0.0, 0.0 if str(g.get("lin_prec", "ILU")) == "LU_SGS" else 1.0], np.float64)
    if "rk_alpha" in g:
        w("cfg_rk", g["rk_alpha"], np.float64)
    bc = rx.bc_from_reference(g["bc_marker"], g["bc_params"], g["bvertex_pn"])
    w("bc_kind", bc["kind"], np.int32)
    w("bc_data", bc["data"], np.float64)
    w("bc_scalars", [bc["inlet_kind"], bc["tke_inf"], bc["kine_inf"], bc["omega_inf"]], np.float64)
    if laminar:
        w("cfg_laminar", [1.0], np.float64)
    exe = os.path.join(d, "rx_driver")
    build_driver(exe)
    r = subprocess.run([exe, d, "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    N, nVar = g["it_U0"].shape
    U = np.fromfile(os.path.join(d, "out_u.f64")).reshape(N, nVar)
    from tests.parity import per_column_close
    per_column_close(U, g["it1_U"], floor=1e-3, what="C++ Iterate U")
    if not laminar:
        T = np.fromfile(os.path.join(d, "out_sst_u.f64")).reshape(N, 2)
        per_column_close(T, g["it1_sst"], floor=1e-3, what="C++ Iterate (k, omega)")
    assert_close(np.fromfile(os.path.join(d, "out_rms.f64")), g["it1_rms"], what="C++ Iterate RMS")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["itx9", "ig9", "fpit"])
def test_cpp_driver_from_cfg(tmp_path, case):
    """The C++ host set up entirely from a cfg by the native reader (rx_case_read: SU2 mesh + dual grid + wall
    distance, library, rx_cfg, markers, free stream) then rx::Iterate, against the reference's own iteration of the
    same cfg and files: the shipped jet cfg (itx9), stage 1 with IGNITION (ig9), the flat plate (fpit)."""
    from tests.test_gpu_case import workdir
    wd = workdir(case, tmp_path)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", case + ".npz")))
    sd = str(tmp_path / "state")
    os.makedirs(sd)
    for k in ("it_U0", "it_V0", "it_sst0", "it_mut0", "it_F1_0", "it_F2_0", "it_CDkw0", "it_sstgrad0"):
        np.ascontiguousarray(g[k], dtype=np.float64).tofile(os.path.join(sd, k + ".f64"))
    exe = str(tmp_path / "rx_driver")
    build_driver(exe)
    r = subprocess.run([exe, os.path.join(wd, "case.cfg"), "3", sd], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    N, nVar = g["it_U0"].shape
    from tests.parity import per_column_close
    per_column_close(np.fromfile(os.path.join(sd, "out_u.f64")).reshape(N, nVar), g["it1_U"], floor=1e-3,
                     what="C++ from cfg: U")
    per_column_close(np.fromfile(os.path.join(sd, "out_sst_u.f64")).reshape(N, 2), g["it1_sst"], floor=1e-3,
                     what="C++ from cfg: (k, omega)")
    assert_close(np.fromfile(os.path.join(sd, "out_rms.f64")), g["it1_rms"], what="C++ from cfg: RMS")
    assert_close(np.fromfile(os.path.join(sd, "out_sst_rms.f64")), g["it1_sst_rms"], what="C++ from cfg: SST RMS")
