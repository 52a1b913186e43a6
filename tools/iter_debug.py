"""Debug: whole reference iterations on the device vs the oracle / reference goldens (it9), per iteration."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from tests.rxpkg import rx  # noqa: E402
from tests.test_gpu_bc import golden, solvers  # noqa: E402
from tests.test_oracle_bc import iteration_cfg  # noqa: E402

g = golden("it9")
N = len(g["it_U0"])
s, t = solvers(g, 1)
s.upload("V", g["it_V0"])
s.upload("U", g["it_U0"])
T0 = g["it_sst0"]
for f, v in (("TKE", T0[:, 0]), ("OMEGA", T0[:, 1]), ("MUT", g["it_mut0"]), ("SIGMAK", np.full(N, 0.85)),
             ("GRADK", np.ascontiguousarray(g["it_sstgrad0"][:, 0, :]))):
    s.upload(f, v)
t.set_state(T0, g["wall_distance"], g["it_F1_0"], g["it_F2_0"], g["it_CDkw0"])
cfg, bc, st = iteration_cfg(g)
m = O.Mechanism(g)


def cr(a, b):
    return float((np.abs(a - b).max(0) / np.maximum(np.abs(b).max(0), 1e-300)).max())


rp, col = g["bsr_row_ptr"], g["bsr_col"]
bnodes = set(np.unique(g["bvertex"][:, 1]).tolist())
row_of = np.repeat(np.arange(N), np.diff(rp))
for k in range(3):
    if k < 2:
        rms, rms_t, its = rx.Iterate(s, t, ext_iter=k)
    else:  # phase by phase
        s.SetPrimitive_Variables(k)
        s.SetPrimitive_Gradient_LS()
        s.SetStrainMag()
        s.SetTime_Step()
        s.sync()
        pre_dev = {f: s.download(f) for f in ("V", "DPDU", "DTDU", "MU", "KAPPA", "DIJ", "GRAD", "TKE", "MUT", "SIGMAK",
                                              "GRADK", "EDDY", "U")}
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.Viscous_Residual()
        s.Source_Residual()
        s.spmv("RHS", "SOL")  # forces the assembly (ensure_assembled) before the BCs
        s.sync()
        J_cv = s.download("JAC").reshape(-1, 13, 13)
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.spmv("RHS", "SOL")
        s.sync()
        J_c = s.download("JAC").reshape(-1, 13, 13)
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.Viscous_Residual()
        s.Source_Residual()
        s.spmv("RHS", "SOL")
        s.sync()
        J_loops = s.download("JAC").reshape(-1, 13, 13)
        R_loops = s.download("RES").reshape(N, -1)
        s.BC()
        s.sync()
        J_bc = s.download("JAC").reshape(-1, 13, 13)
        rms, it = s.ImplicitEuler_Iteration()
        s.SetPrimitive_Variables(k)
        s.SetPrimitive_Gradient_LS()
        s.SetStrainMag()
        t.Preprocessing(); t.Upwind_Residual(); t.Viscous_Residual(); t.Source_Residual(); t.BC()
        rms_t, it_t = t.ImplicitEuler_Iteration()
        t.Postprocessing()
        its = (it, it_t)
    s.sync()
    st_prev = st
    st = O.outer_iteration(m, 2, g, st, bc, cfg, k, (g["bsr_row_ptr"], g["bsr_col"]))
    U, V, T = s.download("U").reshape(N, -1), s.download("V").reshape(N, -1), t.download("U").reshape(N, 2)
    p = f"it{k + 1}_"
    print(f"iter {k + 1}: lin {its} oracle lin ({st['lin_iters']}, {st['sst_lin_iters']})")
    print(f"   dev-ref U {cr(U, g[p + 'U']):.3e} V {cr(V, g[p + 'V']):.3e} T {cr(T, g[p + 'sst']):.3e}"
          f" | dev-orc U {cr(U, st['U']):.3e} T {cr(T, st['T']):.3e} | orc-ref U {cr(st['U'], g[p + 'U']):.3e}")
    print(f"   rms dev {rms[:4]} ref {g[p + 'rms'][:4]}  sst {rms_t} ref {g[p + 'sst_rms']}")
    if k == 2:
        for nm, dv, oc in (("JAC loops", J_loops, st["jac_loops"]), ("JAC after BC", J_bc, None)):
            oc = st["jac_loops"] if oc is not None else None
        d = np.abs(J_loops - st["jac_loops"]).reshape(len(J_loops), -1).max(1)
        bad = np.nonzero(d > 1e-8 * np.abs(st["jac_loops"]).max())[0]
        print("   JAC loops bad blocks", len(bad), "rows", sorted(set(row_of[bad].tolist()))[:20],
              "boundary rows among them", len(set(row_of[bad].tolist()) & bnodes))
        o = st["pre"]
        for f, key in (("V", "V"), ("DPDU", "dPdU"), ("DTDU", "dTdU"), ("MU", "mu"), ("KAPPA", "kappa"), ("DIJ", "Dij"),
                       ("EDDY", "eddy"), ("U", "U")):
            dv, oc = pre_dev[f], o[key].ravel()
            dd = np.abs(dv - oc)
            print(f"   pre {f} dev-orc {dd.max() / max(np.abs(oc).max(), 1e-300):.3e} at {int(np.argmax(dd))}")
        dd = np.abs(pre_dev["GRAD"] - st["pre_grad"].ravel())
        print(f"   pre GRAD dev-orc {dd.max() / np.abs(st['pre_grad']).max():.3e}")
        for b in bad[:7]:
            e = np.abs(J_loops[b] - st["jac_loops"][b])
            print("   bad block", b, "row", row_of[b], "col", col[b], "entries", np.argwhere(e > 1e-8 * np.abs(st["jac_loops"]).max())[:6].tolist())
        # oracle pieces on the oracle's own iteration-3 state
        T_prev = st_prev["T"]
        gk = np.ascontiguousarray(st_prev["TG"][:, 0, :])
        rc, Jci, Jcj = O.ausm_edges(2, 9, g["edges"], g["edge_normal"], o["V"], o["dPdU"], cfg["mach_inf"], True)
        rv, Jvi, Jvj = O.visc_edges(m, 2, g["edges"], g["edge_normal"], g["coord"], o["V"], st["pre_grad"], o["mu"],
                                    o["kappa"], o["Dij"], o["dTdU"], T_prev[:, 0].copy(), st_prev["mut"],
                                    np.full(N, 0.85), gk, True, True, [1, 1, 1, cfg["prandtl_turb"], cfg["lewis_turb"]])
        Ac = O.assemble(rp, col, g["edges"], rc, Jci, Jcj, None, None, None, None, None, g["volume"],
                        np.full(N, np.inf), 13)[1]
        Acv = O.assemble(rp, col, g["edges"], rc, Jci, Jcj, rv, Jvi, Jvj, None, None, g["volume"], np.full(N, np.inf),
                         13)[1]
        sc = np.abs(Acv).max()
        for nm, dv, oc in (("conv", J_c, Ac), ("conv+visc", J_cv, Acv)):
            dd = np.abs(dv - oc).reshape(len(oc), -1).max(1)
            bb = np.nonzero(dd > 1e-8 * sc)[0]
            print(f"   {nm}: bad blocks {bb.tolist()[:8]}")
            for b in bb[:2]:
                print("     dev row3", dv[b][3], "\n     orc row3", oc[b][3])
        for b in (733, 785):
            print(f"   block {b}: dev loops row3 {J_loops[b][3][3:]}\n              orc loops row3 {st['jac_loops'][b][3][3:]}"
                  f"\n              dev cv    row3 {J_cv[b][3][3:]}\n              orc cv    row3 {Acv[b][3][3:]}"
                  f"\n              dev c     row3 {J_c[b][3][3:]}\n              orc c     row3 {Ac[b][3][3:]}")
        e = int(np.nonzero((g["edges"][:, 0] == 154) & (g["edges"][:, 1] == 165))[0][0])
        print("   edge", e, "orc visc Ji row3", Jvi[e][3], "\n   orc visc Jj row3", Jvj[e][3])
        print("   RES loops dev-orc", np.abs(R_loops - st["res_loops"]).max() / np.abs(st["res_loops"]).max())
    for name, dev, orc in (("DT", s.download("DT"), st["dt"]), ("MUT", t.download("MUT"), st["mut"]),
                           ("F1", t.download("F1"), st["F1"]), ("JAC", s.download("JAC"), st["sys"].ravel()),
                           ("RHS", s.download("RHS"), st["rhs"].ravel()), ("SOL", s.download("SOL"), st["sol"].ravel()),
                           ("SST JAC", t.download("JAC"), st["sst_sys"].ravel()),
                           ("SST RHS", t.download("RHS"), st["sst_rhs"].ravel()),
                           ("SST SOL", t.download("SOL"), st["sst_sol"].ravel())):
        if dev is not None:
            d = np.abs(dev - orc)
            print(f"   {name} dev-orc {d.max() / np.abs(orc).max():.3e} at {int(np.argmax(d))}")
s.close()
