"""Debug: one reference outer iteration (it3d / it9 from the reference's state) on the device, phase by phase,
against the oracle in the device's inner-product order."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_bc import golden, load_iteration_state, solvers  # noqa: E402
from tests.test_oracle_bc import iteration_cfg  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "it3d"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # start from the reference's state after K iterations
g = golden(case)
nDim = int(g["dims"][0])
N = len(g["it_U0"])
s, t = solvers(g, 1)
load_iteration_state(g, s, t, K)
cfg, bc, st = iteration_cfg(g)
if K:
    p = f"it{K}_"
    st = dict(U=g[p + "U"], V=g[p + "V"], Uold=g[p + "Uold"], T=g[p + "sst"], TG=g[p + "sstgrad"], F1=g[p + "F1"],
              F2=g[p + "F2"], CDkw=g[p + "CDkw"], mut=g[p + "mut"])
m = O.Mechanism(g)
with O.dot_order("device"):
    o = O.outer_iteration(m, nDim, g, st, bc, cfg, K, (g["bsr_row_ptr"], g["bsr_col"]))


def cr(a, b, floor=1e-300):
    a, b = np.asarray(a).reshape(len(b), -1), np.asarray(b).reshape(len(b), -1)
    return np.abs(a - b).max(0) / np.maximum(np.abs(b).max(0), floor)


s.SetPrimitive_Variables(K)
s.SetPrimitive_Gradient_LS()
s.SetStrainMag()
s.SetTime_Step()
s.sync()
for f, key in (("V", "V"), ("DPDU", "dPdU"), ("DTDU", "dTdU"), ("MU", "mu"), ("KAPPA", "kappa"), ("DIJ", "Dij"),
               ("EDDY", "eddy"), ("U", "U")):
    print(f"pre {f:6s} max col rel {cr(s.download(f), o['pre'][key]).max():.3e}")
print(f"pre GRAD   max col rel {cr(s.download('GRAD'), o['pre_grad']).max():.3e}")
print(f"dt         max rel {cr(s.download('DT'), o['dt']).max():.3e}")
s.Preprocessing_zero()
s.Upwind_Residual()
s.Viscous_Residual()
s.Source_Residual()
s.BC()
s.sync()
R = s.download("RES").reshape(N, -1)
print("RES after BC per col", np.array2string(cr(R, -o["rhs"].reshape(N, -1)), precision=2))
rms, it = s.ImplicitEuler_Iteration()
s.sync()
nv = R.shape[1]
A = s.download("JAC").reshape(-1, nv, nv)
As = np.asarray(o["sys"]).reshape(-1, nv, nv)
sc = np.abs(As).max(axis=(1, 2), keepdims=True)
e = (np.abs(A - As) / sc).reshape(len(A), -1).max(1)
print(f"system blocks max block-rel err {e.max():.3e}; worst blocks {np.argsort(e)[-5:][::-1].tolist()}")
wb = int(np.argmax(e))
ee = np.abs(A[wb] - As[wb]) / sc[wb, 0, 0]
print("   worst entries", np.argwhere(ee > 0.1 * ee.max()).tolist()[:8], ee.max())
print("RHS per col", np.array2string(cr(s.download("RHS"), o["rhs"]), precision=2))
print("SOL per col", np.array2string(cr(s.download("SOL"), o["sol"]), precision=2), "lin", it, o["lin_iters"])
print("U per col", np.array2string(cr(s.download("U"), o["U"], 1e-3), precision=2))
U1 = s.download("U").reshape(N, -1)
s.SetPrimitive_Variables(K)
s.SetPrimitive_Gradient_LS()
s.SetStrainMag()
s.sync()
U2 = s.download("U").reshape(N, -1)
V2 = s.download("V").reshape(N, -1)
print("after 2nd preprocessing: U per col", np.array2string(cr(U2, o["U"], 1e-3), precision=2))
print("   V per col", np.array2string(cr(V2, o["V"], 1e-3), precision=2))
ch = np.nonzero(np.any(U1 != U2, axis=1))[0]
print("   nodes whose U changed in the 2nd preprocessing:", ch.tolist()[:20])
d = np.abs(U2[:, 2] - o["U"][:, 2])
i = int(np.argmax(d))
print("   worst var-2 node", i, U1[i, 2], U2[i, 2], o["U"][i, 2], "ref", g[f"it{K + 1}_U"][i, 2])
print("dev vs ref U per col", np.array2string(cr(U2, g[f"it{K + 1}_U"], 1.0), precision=2))
print("orc vs ref U per col", np.array2string(cr(o["U"], g[f"it{K + 1}_U"], 1.0), precision=2))
