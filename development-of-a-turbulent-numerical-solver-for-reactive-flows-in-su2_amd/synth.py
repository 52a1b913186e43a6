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
             "eddy_visc_flow")


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


def jet_case(nx, ny, records="jet9w", seed=12345):
    """Mesh (RCM-ordered median dual) + node records for an nx x ny jet."""
    mg = _meshgen()
    mesh = mg.build_jet(nx, ny)
    g = load_records(records)
    src = g["coord"]
    lo, hi = src.min(axis=0), src.max(axis=0)
    sn = (src - lo) / np.where(hi > lo, hi - lo, 1.0)
    dst = mesh["coord"]
    dlo, dhi = dst.min(axis=0), dst.max(axis=0)
    dn = (dst - dlo) / np.where(dhi > dlo, dhi - dlo, 1.0)
    rng = np.random.default_rng(seed)
    dn = np.clip(dn + rng.normal(scale=0.002, size=dn.shape), 0.0, 1.0)
    from scipy.spatial import cKDTree
    _, idx = cKDTree(sn).query(dn)
    state = {k: np.ascontiguousarray(g[k][idx]) for k in NODE_KEYS if k in g}
    mesh["n_dim"] = 2
    mech = {k: g[k] for k in g if k.startswith("mech_")}
    return mesh, state, mech, {"mach_inf": float(g["mach_inf"][0]), "prandtl_turb": float(g["visc_params"][1]),
                               "lewis_turb": float(g["visc_params"][2]), "c_mu": float(g["src_params"][0]),
                               "pasr_lb": float(g["src_params"][1])}
