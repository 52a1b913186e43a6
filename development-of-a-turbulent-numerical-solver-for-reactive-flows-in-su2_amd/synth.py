"""Synthetic workloads: a jet mesh of any size carrying realistic reacting node records.

Host-side data preparation for tests and bench.py (not the hot path). Node records (primitives,
pressure/temperature derivatives, transport properties, binary diffusion coefficients and the SST
fields) are resampled by nearest normalised position from a record set produced by the reference's
own preprocessing (tests/golden/jet9w.npz: the flame window of the reference jet with its converged
PaSR state). Every record is thermodynamically self-consistent because it is a record the
reference produced; neighbouring points of the synthetic mesh may come from different records,
which exercises the fluxes with real jumps.
"""
from __future__ import annotations

import importlib.util
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(REPO, "tests", "golden")

NODE_KEYS = ("V", "U", "dPdU", "dTdU", "mu", "kappa", "Dij", "turb_k", "turb_omega", "mu_t", "sigma_k", "grad_k",
             "eddy_visc_flow", "sst_F1", "sst_F2", "sst_CDkw")


def _meshgen():
    spec = importlib.util.spec_from_file_location("rx_meshgen", os.path.join(HERE, "meshgen.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def load_records(name="jet9w"):
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    if "eddy_visc_flow" not in g:
        g["eddy_visc_flow"] = g["mu_t"]
    return g


def species_subset(g, keep, nDim=2):
    """Restrict records + mechanism to the species indices `keep` (7 species =
    C4H6, H2O, O2, CO, CO2, H2, O; 4 species = reaction 1 only). Reactions touching a dropped species
    are removed. The dropped species carry zero mass in the jet records, so the restricted records stay
    consistent (rho, mixture properties unchanged)."""
    keep = np.asarray(keep, dtype=np.int64)
    ns0 = int(g["mech_n_species"])
    drop = np.setdiff1d(np.arange(ns0), keep)
    sr, sp = g["mech_stoich_reac"], g["mech_stoich_prod"]
    rk = np.nonzero(np.all(sr[drop] == 0, axis=0) & np.all(sp[drop] == 0, axis=0))[0]
    out = dict(g)
    fl = nDim + 2  # [rho, rho u, rho v, rho E] then species in U / dPdU / dTdU
    pv = nDim + 5  # [T, u, v, P, rho, h, a] then Y_s in V
    out["V"] = np.concatenate([g["V"][:, :pv], g["V"][:, pv + keep]], axis=1)
    for k in ("U", "dPdU", "dTdU"):
        if k in g:
            out[k] = np.concatenate([g[k][:, :fl], g[k][:, fl + keep]], axis=1)
    if "Dij" in g:
        out["Dij"] = g["Dij"][:, keep][:, :, keep]
    for k in ("mmass", "diff_vol", "form_enthalpy", "species"):
        out["mech_" + k] = g["mech_" + k][keep]
    for k in ("tab_x", "tab_y", "tab_y2"):
        out["mech_" + k] = g["mech_" + k][:, keep]
    out["mech_stoich_reac"] = sr[keep][:, rk]
    out["mech_stoich_prod"] = sp[keep][:, rk]
    out["mech_exp_reac"] = g["mech_exp_reac"][rk][:, keep]
    out["mech_exp_prod"] = g["mech_exp_prod"][rk][:, keep]
    for k in ("A", "beta", "Ta", "A_back", "beta_back", "Ta_back", "reversible", "has_backward"):
        out["mech_" + k] = g["mech_" + k][rk]
    out["mech_n_species"] = np.array(len(keep))
    out["mech_n_reactions"] = np.array(len(rk))
    return out


def lift_records_3d(g):
    """2-D node records as 3-D records of a spanwise-uniform flow: w = 0 inserted after v in V, U, dP/dU and dT/dU
    (dP/d(rho w) = -(gamma - 1) w = 0 and dT/d(rho w) = -w / (rho c_v) = 0 at w = 0), a zero third component of the
    TKE gradient; every other record (rho E included, the kinetic energy being unchanged) stays the reference's."""
    out = dict(g)
    for k in ("V", "U", "dPdU", "dTdU"):
        a = np.asarray(g[k])
        out[k] = np.concatenate([a[:, :3], np.zeros((len(a), 1)), a[:, 3:]], axis=1)
    gk = np.asarray(g["grad_k"])
    out["grad_k"] = np.concatenate([gk, np.zeros((len(gk), 1))], axis=1)
    return out


def jet_case(nx, ny, records="jet9w", seed=12345, n_species=9, n_part=1, nz=0):
    """Mesh (RCM-ordered median dual) + node records for an nx x ny jet (nz > 1: the 3-D extrusion over nz planes)
    with 9 (reference-native), 7 or 4 species."""
    mg = _meshgen()
    mesh = mg.build_jet(nx, ny, n_part=n_part, nz=nz)
    g = load_records(records)
    if n_species != int(g["mech_n_species"]):
        g = species_subset(g, np.arange(n_species))
    if nz > 1:
        g = lift_records_3d(g)
    src = g["coord"]
    lo, hi = src.min(axis=0), src.max(axis=0)
    sn = (src - lo) / np.where(hi > lo, hi - lo, 1.0)
    dst = mesh["coord"][:, :2]  # records sampled by (x, y); spanwise-uniform in 3-D
    dlo, dhi = dst.min(axis=0), dst.max(axis=0)
    dn = (dst - dlo) / np.where(dhi > dlo, dhi - dlo, 1.0)
    rng = np.random.default_rng(seed)
    dn = np.clip(dn + rng.normal(scale=0.002, size=dn.shape), 0.0, 1.0)
    from scipy.spatial import cKDTree
    _, idx = cKDTree(sn).query(dn)
    state = {k: np.ascontiguousarray(g[k][idx]) for k in NODE_KEYS if k in g}
    state["sst_sol"] = np.ascontiguousarray(np.stack([state["turb_k"], state["turb_omega"]], axis=1))
    mesh["n_dim"] = 3 if nz > 1 else 2
    mech = {k: g[k] for k in g if k.startswith("mech_")}
    return mesh, state, mech, {"mach_inf": float(g["mach_inf"][0]), "prandtl_turb": float(g["visc_params"][1]),
                               "lewis_turb": float(g["visc_params"][2]), "c_mu": float(g["src_params"][0]),
                               "pasr_lb": float(g["src_params"][1])}


JET_LENGTH, JET_HEIGHT = 0.125, 0.006  # mesh_stretched.su2's domain (meshgen.jet_points)


def fold_matrix(n_species, ns0=9):
    """[ns0][n_species] map of the 9 jet species' partial densities onto the first n_species (SPECIES_ORDER C4H6,
    H2O, O2, CO, CO2, H2, O, OH, H): the dropped radicals / H2 go to O2; for 4 species CO2 goes to H2O and CO in the
    mass ratio 0.53 : 0.47, which keeps the mixture's formation enthalpy per unit mass (CO2 -8.94 kJ/g = 0.53 x
    H2O -13.42 + 0.47 x CO -3.95), so rho, rho E and T stay close to the reference's state."""
    M = np.zeros((ns0, n_species))
    for s in range(min(ns0, n_species)):
        M[s, s] = 1.0
    for s in range(n_species, ns0):
        if s == 4:  # CO2
            M[s, 1], M[s, 3] = 0.53, 0.47
        else:
            M[s, 2] = 1.0
    return M


def fold_species(U, n_species, fl=4, ns0=9):
    """Conservative state of the first n_species species from a 9-species one (fold_matrix); columns after the
    species (k, omega) are kept."""
    U = np.asarray(U, dtype=np.float64)
    return np.concatenate([U[:, :fl], U[:, fl:fl + ns0] @ fold_matrix(n_species, ns0), U[:, fl + ns0:]], axis=1)


def field_subset(g, n_species):
    """Restrict the reference's 9-species field (and mechanism) to its first n_species species, the dropped
    partial densities folded into the kept ones (fold_species: rho unchanged, formation enthalpy kept); T is
    re-derived by Cons2PrimVar on the device."""
    ns0 = int(g["mech_n_species"])
    if n_species == ns0:
        return g
    out = species_subset(g, np.arange(n_species))
    nDim = int(np.shape(g["coord"])[1])
    out["U"] = fold_species(g["U"], n_species, fl=nDim + 2, ns0=ns0)
    return out


def field_at(xy, n_species=7, field="jet9k", y_floor=1e-6):
    """The reference's converged PaSR jet (tests/golden/jet9k.npz: its own 9 000-point mesh after its start-up
    preprocessing) linearly interpolated at the physical points xy [n][2] of the jet domain: (g, U, k, omega,
    mu_t, T) with g the (species-restricted) field dict. Species are floored at a mass fraction of 1e-10 (see
    below)."""
    g = field_subset(load_records(field), n_species)
    src = np.asarray(g["coord"]) / np.array([JET_LENGTH, JET_HEIGHT])
    dst = np.asarray(xy)[:, :2] / np.array([JET_LENGTH, JET_HEIGHT])
    vals = np.concatenate([g["U"], np.stack([g["turb_k"], g["turb_omega"], g["mu_t"], g["V"][:, 0]], axis=1)],
                          axis=1)
    from scipy.interpolate import LinearNDInterpolator
    from scipy.spatial import cKDTree
    out = LinearNDInterpolator(src, vals)(dst)
    bad = np.isnan(out[:, 0])
    if bad.any():  # outside the reference points' convex hull (curved-boundary slivers): nearest point
        _, idx = cKDTree(src).query(dst[bad])
        out[bad] = vals[idx]
    nU = g["U"].shape[1]
    U = out[:, :nU]
    # trace species. The viscous Jacobian's Ds = (1 - X_s) / sum_b X_b / D_sb (numerics_direct_reactive.cpp:1578-1588)
    # is 0/0 -> 0 (the reference's NaN guard) at a pure-species point, but once an update leaves 1e-30-level
    # partial densities there (negative ones are clamped to 1e-30, reacting_model_library.cpp:65-79) it is
    # rounding / 1e-30 ~ 1e280 and the ILU(0) factor overflows (the Ds discontinuity). The
    # reference's oxidiser stream is pure O2, so every species is floored at a mass fraction y_floor and the
    # partial densities rescaled to the interpolated density. 1e-6 rather than just above the 1e-30 clamp: with
    # 1e-10 trace species the Ds cancellation (1 - X_s carries 1e-16 / 1e-10 relative rounding) and the PaSR
    # rates' C^(nu-1) derivatives make the FGMRES(5) update amplify last-bit residual differences ~1e6-fold
    # (tools/size_diag.py: device vs oracle U 3e-7 column-relative at C3 with 1e-10, 1e-12 with 1e-6).
    rho = U[:, 0]
    rs = U[:, 4:]
    np.maximum(rs, y_floor * rho[:, None], out=rs)
    rs *= (rho / rs.sum(axis=1))[:, None]
    return g, U, out[:, nU], out[:, nU + 1], out[:, nU + 2], out[:, nU + 3]


def jet_field_case(nx, ny, n_species=7, n_part=1, nz=0, field="jet9k", y_floor=1e-6):
    """Mesh (RCM-ordered median dual, partitioned) + a smooth, physically consistent initial state for an nx x ny
    (x nz) jet: the reference's converged PaSR field on its own 9 000-point mesh (tests/golden/jet9k.npz, after the
    reference's preprocessing) linearly interpolated onto the synthetic mesh, which covers the same physical domain
    (SURVEY.md §8(d) 'bilinearly interpolate flow_second_chem.dat onto the finer mesh'; field_at). Interpolated
    quantities are the conservatives U, (k, omega), mu_t and T (the secant's starting temperature); a convex
    combination of valid conservative states is a valid conservative state. The other node records (V, dP/dU,
    dT/dU, mu, kappa, D_ij, SST fields) are produced on the device by the reference's preprocessing sequence
    (device_preprocess). 3-D: spanwise-uniform (rho w = 0)."""
    mg = _meshgen()
    mesh = mg.build_jet(nx, ny, n_part=n_part, nz=nz)
    g, U, k, om, mut, T = field_at(mesh["coord"], n_species, field, y_floor)
    nDim = 3 if nz > 1 else 2
    if nDim == 3:
        U = np.concatenate([U[:, :3], np.zeros((len(U), 1)), U[:, 3:]], axis=1)
    ns = n_species
    V = np.zeros((len(U), ns + nDim + 5))
    V[:, 0] = T
    state = dict(U=np.ascontiguousarray(U), V=V, turb_k=np.ascontiguousarray(k), turb_omega=np.ascontiguousarray(om),
                 mu_t=np.ascontiguousarray(mut), eddy_visc_flow=np.ascontiguousarray(mut))
    state["sst_sol"] = np.ascontiguousarray(np.stack([k, om], axis=1))
    mesh["n_dim"] = nDim
    mech = {q: g[q] for q in g if q.startswith("mech_")}
    return mesh, state, mech, {"mach_inf": float(g["mach_inf"][0]), "prandtl_turb": float(g["visc_params"][1]),
                               "lewis_turb": float(g["visc_params"][2]), "c_mu": float(g["src_params"][0]),
                               "pasr_lb": float(g["src_params"][1])}


def device_preprocess(flow, turb, mesh, state):
    """The reference's start-up preprocessing on the device (the sequence its driver runs before the first
    iteration, as oracle/ref_harness reproduces it: flow Preprocessing, turbulence Postprocessing, flow
    Preprocessing, turbulence Preprocessing + Postprocessing), from U, the starting T, (k, omega) and mu_t. Returns
    the completed node records (host copies, NODE_KEYS + sst_sol) for the CPU baseline and the parity tests."""
    flow.upload("U", state["U"])
    flow.upload("V", state["V"])
    flow.upload("TKE", state["turb_k"])
    flow.upload("OMEGA", state["turb_omega"])
    flow.upload("MUT", state["mu_t"])
    flow.upload("EDDY", state["eddy_visc_flow"])
    turb.set_state(state["sst_sol"], mesh["wall_distance"])

    def flow_pre():
        flow.SetPrimitive_Variables(0)
        flow.SetPrimitive_Gradient()
        flow.SetStrainMag()

    flow_pre()
    turb.Preprocessing()
    turb.Postprocessing()
    flow_pre()
    turb.Preprocessing()
    turb.Postprocessing()
    flow.sync()
    N, nDim = flow.N, flow.nDim
    out = {}
    for key, fld in (("V", "V"), ("U", "U"), ("dPdU", "DPDU"), ("dTdU", "DTDU"), ("mu", "MU"), ("kappa", "KAPPA"),
                     ("Dij", "DIJ"), ("turb_k", "TKE"), ("turb_omega", "OMEGA"), ("mu_t", "MUT"),
                     ("sigma_k", "SIGMAK"), ("grad_k", "GRADK"), ("eddy_visc_flow", "EDDY"), ("grad_prim", "GRAD")):
        out[key] = flow.download(fld).reshape(N, -1)
    for key in ("mu", "kappa", "turb_k", "turb_omega", "mu_t", "sigma_k", "eddy_visc_flow"):
        out[key] = out[key].ravel()
    ns = flow.mech.ns
    out["Dij"] = out["Dij"].reshape(N, ns, ns)
    out["grad_prim"] = out["grad_prim"].reshape(N, -1, nDim)
    for key, fld in (("sst_F1", "F1"), ("sst_F2", "F2"), ("sst_CDkw", "CDKW")):
        out[key] = turb.download(fld)
    out["sst_sol"] = turb.download("U").reshape(N, 2)
    return out


# MARKER_* of the reference's jet cfg (Test_Cases/TURBOLENT/TURBOLENT_COMBUSTION/*.cfg, oracle/make_golden.py):
# INLET_TYPE = TEMPERATURE_IMPOSE, MARKER_INLET = (Oxidizer_Inlet, 300 K, 20 m/s, (1, 0, 0); Fuel_Inlet, 800 K,
# 0.87 m/s, (0, 1, 0)), INLET_MASS_FRAC pure O2 / pure C4H6, MARKER_OUTLET = (Outlet, 101325 Pa),
# MARKER_ISOTHERMAL = (upper_wall 300 K, lower_wall_pre 300 K, lower_wall_post 600 K).
JET_MARKERS = {  # in meshgen.MARKERS order: (kind, a, b, flow direction, inlet species)
    "Oxidizer_Inlet": ("inlet", 300.0, 20.0, (1.0, 0.0, 0.0), "O2"),
    "Outlet": ("outlet", 101325.0, 0.0, (0.0, 0.0, 0.0), None),
    "upper_wall": ("isothermal", 300.0, 0.0, (0.0, 0.0, 0.0), None),
    "Fuel_Inlet": ("inlet", 800.0, 0.87, (0.0, 1.0, 0.0), "C4H6"),
    "lower_wall_pre": ("isothermal", 300.0, 0.0, (0.0, 0.0, 0.0), None),
    "lower_wall_post": ("isothermal", 600.0, 0.0, (0.0, 0.0, 0.0), None),
}
SPECIES_ORDER = ("C4H6", "H2O", "O2", "CO", "CO2", "H2", "O", "OH", "H")  # the golden cfg's SPECIES_ORDER


def jet_bc(mesh, n_species):
    """rx_bc_desc inputs of the jet's markers for a meshgen mesh (bvertex markers in meshgen.MARKERS order), with
    the free-stream turbulence values the reference derives from the same cfg (golden bc9 bc_params)."""
    mg = _meshgen()
    g = dict(np.load(os.path.join(GOLDEN, "bc9.npz")))
    bp = g["bc_params"]
    kinds = {"inlet": 1, "outlet": 2, "isothermal": 3, "symmetry": 0}  # MARKER_SYM: no action (BC_Sym_Plane)
    rows, kk = [], []
    names = mg.MARKERS3 if np.shape(mesh["coord"])[1] == 3 else mg.MARKERS
    for name in names:
        kind, a, b, d, sp = JET_MARKERS.get(name, ("symmetry", 0.0, 0.0, (0.0, 0.0, 0.0), None))
        y = np.zeros(n_species)
        if sp is not None:
            y[SPECIES_ORDER.index(sp)] = 1.0
        rows.append(np.r_[0.0, a, b, d, y])
        kk.append(kinds[kind])
    return dict(kind=np.array(kk, dtype=np.int32), data=np.array(rows), normal_neighbor=mesh["bvertex_pn"],
                inlet_kind=2, tke_inf=float(bp[1]), kine_inf=float(bp[2]), omega_inf=float(bp[3]))
