"""Debug: phase timing of the ILU(0) factorisation kernel (partition 0) on the GPU.

python tools/ilu_trace.py [nx ny parts [nz]]  — prints median shader-clock cycles per row phase:
  0-1 row/staging loads, 1-2 lower-block products and updates, 2-3 inverse of D_i, 3-4 write-back.
With the grouped kernel (k_ilu_build_grp, the default on the jet meshes) the phases are
  0-1 loads + lower-block products + diagonal updates, 1-2 factor of D_i, 2-3 solve + stores,
and the level durations of partition 0.
"""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.rxpkg import rx, synth  # noqa: E402

nx, ny, P = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (500, 200, 256)))
nz = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # 3-D extrusion (C5: 1000 50 256 20)
mesh, st, mech, kw = synth.jet_case(nx, ny, n_species=7, n_part=P, nz=nz)
s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), rx.default_cfg(implicit=1, lin_prec=1, **kw))
s.set_state(st)
s.SetPrimitive_Gradient_LS()
s.SetTime_Step()
s.Preprocessing_zero()
s.Upwind_Residual()
s.Viscous_Residual()
s.Source_Residual()
s.ImplicitEuler_Iteration()
G, R, LV = 64, 64, 512
n = 1 + G * R * 8 + LV
buf = np.zeros(n, dtype=np.int64)
rc = rx.lib().rx_debug_ilu_trace(s.h, buf.ctypes.data_as(C.c_void_p), C.c_int64(n))
assert rc == 0, rc
if buf[1 + G * R * 8] > 0:  # grouped kernel: per-level stamps present
    t = buf[1:1 + G * R * 8].reshape(G, R, 8)
    rows = t[(t[:, :, 0] > 0) & (t[:, :, 3] > 0)]
    lv = buf[1 + G * R * 8:]
    lv = lv[lv > 0]
    t0 = rows[:, 0].min()
    print("rows traced", len(rows), "kernel span (cycles)", buf[0] - t0, "levels traced", len(lv))
    two = rows[(rows[:, 6] > 0) & (rows[:, 7] > 0)]
    print("rows with two lower blocks:", len(two))
    seq = [(0, 4, "first loads"), (4, 5, "W0"), (5, 6, "X0 + 2nd loads"), (6, 7, "W1"), (7, 1, "X1 + D store"),
           (1, 2, "factor"), (2, 3, "solve + store")]
    for a_, b_, name in seq:
        d = two[:, b_] - two[:, a_]
        print(f"{name:16s} median {np.median(d):8.0f}  mean {d.mean():8.0f}  max {d.max():8.0f}")
    print("row total median", np.median(rows[:, 3] - rows[:, 0]), "max", (rows[:, 3] - rows[:, 0]).max())
    dl = np.diff(np.concatenate([[t0], lv]))
    print("level duration median", np.median(dl), "mean", dl.mean(), "max", dl.max())
    print("first levels:", dl[:12].tolist())
else:
    t = buf[1:1 + 16 * 5 * 64].reshape(16, 64, 5)
    rows = t[(t[:, :, 0] > 0) & (t[:, :, 4] > 0)]
    t0 = rows[:, 0].min()
    d = np.diff(rows, axis=1)
    print("rows traced", len(rows), "kernel span (cycles)", buf[0] - t0)
    for k, name in enumerate(["loads", "products", "inverse", "writeback"]):
        print(f"{name:10s} median {np.median(d[:, k]):8.0f}  mean {d[:, k].mean():8.0f}  max {d[:, k].max():8.0f}")
    print("row total median", np.median(rows[:, 4] - rows[:, 0]))
