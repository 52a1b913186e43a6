"""Locate device-vs-oracle differences of one outer iteration at a full size (GPU only): primitives after the
first SetPrimitive_Variables, the assembled flow system (JAC incl. BCs and Vol/dt) and rhs, the FGMRES solution
and U, worst points first.

usage: python tools/size_diag.py [c2|c3|c5]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from tests.oracle_inputs import outer_iteration_inputs  # noqa: E402
from tests.rxpkg import rx, synth  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "c3"
nx, ny, nz = {"c2": (500, 200, 0), "c3": (2000, 500, 0), "c5": (1000, 50, 20)}[case]
ns = 7
y_floor = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-10
mesh, st0, mech, kw = synth.jet_field_case(nx, ny, n_species=ns, n_part=256, nz=nz, y_floor=y_floor)
cfg = rx.default_cfg(implicit=1, lin_prec=1, **kw)
bc = synth.jet_bc(mesh, ns)
s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), cfg)
s.set_bc(bc)
t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
st = synth.device_preprocess(s, t, mesh, st0)
N = len(st["V"])
nDim = 3 if nz else 2
mesh_o, state, bco, c = outer_iteration_inputs(mesh, st, cfg, bc)
s.upload("GRADK", np.ascontiguousarray(state["TG"][:, 0, :]))
s.upload("SIGMAK", np.full(N, 0.85))
nv = s.nVar
runs = []
for rep in range(2):  # determinism: the same iteration twice from the same records
    synth.device_preprocess(s, t, mesh, st0)
    s.upload("GRADK", np.ascontiguousarray(state["TG"][:, 0, :]))
    s.upload("SIGMAK", np.full(N, 0.85))
    rms, rms_t, its = rx.Iterate(s, t, ext_iter=0)
    s.sync()
    runs.append({k: s.download(k) for k in ("U", "JAC", "RHS", "SOL", "DT")})
dev = runs[0]
for k in dev:
    print(f"repeat {k}: bitwise {np.array_equal(runs[0][k], runs[1][k])} max abs diff "
          f"{np.nanmax(np.abs(runs[0][k] - runs[1][k])):.3e}")
pat = O.bsr_pattern(N, mesh["edges"])
with O.dot_order("device"):
    o = O.outer_iteration(O.Mechanism(mech), nDim, mesh_o, state, bco, c, 0, pat, part_ptr=mesh["part_ptr"], keep=True)
rp, col = pat


def worst(name, a, b, per_row, k=5):
    a = np.asarray(a).reshape(per_row.shape[0] if per_row is not None else len(b), -1)
    b = np.asarray(b).reshape(a.shape)
    scale = np.maximum(np.abs(b).max(axis=0), 1e-300)
    rel = np.abs(a - b) / scale
    r = rel.max(axis=1)
    idx = np.argsort(r)[-k:][::-1]
    print(f"{name}: max col-rel {r.max():.3e}; per column {np.array2string(rel.max(axis=0), precision=1)}; worst rows "
          f"{idx.tolist()} {np.array2string(r[idx], precision=2)}")
    return idx


print(f"{case}: lin iters device {its} oracle {(o['lin_iters'], o['sst_lin_iters'])}; rms rel "
      f"{np.max(np.abs(rms - o['rms']) / np.abs(o['rms'])):.3e}")
worst("dt", dev["DT"], o["dt"], np.zeros((N, 1)))
ir = worst("rhs", dev["RHS"], o["rhs"], np.zeros((N, nv)))
Rd, Ro = dev["RHS"].reshape(N, nv), o["rhs"].reshape(N, nv)
for r in ir[:3]:
    v = int(np.argmax(np.abs(Rd[r] - Ro[r]) / np.maximum(np.abs(Ro).max(axis=0), 1e-300)))
    print(f"  rhs row {r} var {v}: device {Rd[r, v]:.17e} oracle {Ro[r, v]:.17e} (col max {np.abs(Ro[:, v]).max():.3e}) "
          f"coord {mesh['coord'][r]} boundary {r in set(np.asarray(mesh['bvertex'])[:, 1].tolist())}")
    print(f"    V {np.array2string(st['V'][r], precision=5)}")
J = dev["JAC"].reshape(-1, nv * nv)
Jo = o["sys"].reshape(-1, nv * nv)
blk_scale = np.maximum(np.abs(Jo).max(axis=1), 1e-300)
brel = (np.abs(J - Jo).max(axis=1) / blk_scale)
bi = np.argsort(brel)[-8:][::-1]
rows = np.searchsorted(rp, bi, side="right") - 1
print(f"JAC: max block-rel {brel.max():.3e}; worst blocks (row, col, rel): "
      f"{[(int(r), int(col[b]), float(brel[b])) for r, b in zip(rows, bi)]}")
for r in rows[:3]:
    print(f"  row {r}: coord {mesh['coord'][r]} V {np.array2string(st['V'][r], precision=4)}")
worst("SOL", dev["SOL"], o["sol"], np.zeros((N, nv)))
ix = worst("U", dev["U"], o["U"], np.zeros((N, nv)))
for r in ix[:3]:
    print(f"  point {r}: coord {mesh['coord'][r]} partition {int(np.searchsorted(mesh['part_ptr'], r, side='right') - 1)}")
