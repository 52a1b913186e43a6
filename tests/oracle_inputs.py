"""Inputs of the CPU oracle's whole outer iteration (O.outer_iteration) for a synthetic jet run on the device:
the device cfg / rx_bc_desc restated in the oracle's terms. Test infrastructure (tests + bench.py's cpu_baseline
leg)."""
import os

import numpy as np

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def outer_iteration_inputs(mesh, st, cfg, bc):
    """(state, bc, cfg) dicts for O.outer_iteration from a synth.jet_case mesh / state, the rx cfg and the
    synth.jet_bc descriptor. Marker kinds are mapped to the reference's KindBC values (golden bc9 bc_params);
    symmetry markers (rx kind 0) become a value no reference BC uses (no action)."""
    nDim = int(np.shape(mesh["coord"])[1])
    bp = np.asarray(dict(np.load(os.path.join(GOLD, "bc9.npz")))["bc_params"])
    md = np.array(bc["data"], dtype=np.float64)
    # the supersonic kinds (round 6): the reference's SUPERSONIC_INLET / SUPERSONIC_OUTLET enum values (golden sup4's
    # bc_params[28:30])
    sup = np.asarray(dict(np.load(os.path.join(GOLD, "sup4.npz")))["bc_params"])[28:30]
    md[:, 0] = [{1: bp[11], 2: bp[12], 3: bp[13], 4: bp[14], 5: O.EULER_WALL, 6: sup[0], 7: sup[1]}.get(int(k), -1.0)
                for k in bc["kind"]]
    prm = O.bc_prm(bp, cfg.mach_inf, cfg.prandtl_turb, cfg.lewis_turb)
    prm[22:24] = sup
    bco = dict(marker=md, prm=prm)
    c = dict(cfl=cfg.cfl, max_delta_time=cfg.max_delta_time, prandtl_lam=cfg.prandtl_lam,
             prandtl_turb=cfg.prandtl_turb, lewis_turb=cfg.lewis_turb, mach_inf=cfg.mach_inf, c_mu=cfg.c_mu,
             pasr_lb=cfg.pasr_lb, lin_tol=cfg.lin_tol, lin_iter=cfg.lin_iter, relaxation=cfg.relaxation,
             p2v=[cfg.t_min, cfg.t_max, cfg.T_ref, cfg.E_ref, cfg.R_ref, cfg.p_ref, cfg.visc_ref, cfg.cond_ref,
                  cfg.vel_ref, cfg.len_ref, 0.0, float(cfg.clip_temp), float(cfg.ignition), float(cfg.ignition_iter),
                  cfg.ignition_temp, float(cfg.fuel_index), float(cfg.oxidizer_index)])
    T = np.ascontiguousarray(st["sst_sol"])
    state = dict(U=st["U"], V=st["V"], Uold=st["U"], T=T,
                 TG=O.sol_grad_ls(nDim, mesh["coord"], T, mesh["nbr_ptr"], mesh["nbr"]),
                 F1=st["sst_F1"], F2=st["sst_F2"], CDkw=st["sst_CDkw"], mut=st["mu_t"])
    mesh_o = dict(mesh, bvertex=np.c_[np.asarray(mesh["bvertex"])[:, :2], np.zeros(len(mesh["bvertex"]))])
    return mesh_o, state, bco, c
