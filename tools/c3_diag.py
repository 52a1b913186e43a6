"""Diagnose the bench state at a workload / partition count: run outer iterations, print the RMS, the
linear-solver counts and the first failure (status, index, that point's record). GPU only.

usage: python tools/c3_diag.py [--workload c3] [--parts 1024] [--steps 8]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from tests.rxpkg import rx, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
ap.add_argument("--parts", type=int, default=256)
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--cfl", type=float, default=0.0)
a = ap.parse_args()
wl = bench.WORKLOADS[a.workload]
t0 = time.time()
mesh, st, mech, kw = bench.build_workload(wl["nx"], wl["ny"], wl["ns"], a.parts, wl.get("nz", 0))
if a.cfl:
    kw["cfl"] = a.cfl
print(f"setup {time.time() - t0:.1f}s N={len(st['V'])} parts={a.parts} lds_apply={'RX_NO_LDS_APPLY' not in os.environ}",
      flush=True)
cfg = rx.default_cfg(implicit=1, rans=1, lin_prec=1, lin_iter=5, **kw)
s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), cfg, device=0)
s.set_bc(synth.jet_bc(mesh, wl["ns"]))
t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
st = synth.device_preprocess(s, t, mesh, st)
for k in range(a.steps):
    try:
        rms, trms, its = rx.Iterate(s, t, ext_iter=k)
        s.sync()
    except rx.RxError as e:
        print(f"step {k}: FAILED {e}", flush=True)
        msg = str(e)
        if "index" in msg:
            idx = int(msg.rsplit("index", 1)[1].strip(" )"))
            if 0 <= idx < len(st["V"]):
                print("  coord", mesh["coord"][idx], "V", np.array2string(st["V"][idx], precision=4))
                pp = np.asarray(mesh.get("part_ptr", [0, len(st["V"])]))
                print("  partition", int(np.searchsorted(pp, idx, side="right") - 1))
        J = s.download("JAC")
        nv = s.nVar
        bad = ~np.isfinite(J.reshape(-1, nv * nv)).all(axis=1)
        print(f"  JAC non-finite blocks: {int(bad.sum())}; max |JAC| {np.nanmax(np.abs(J[np.isfinite(J)])):.3e}")
        big = np.abs(J.reshape(-1, nv * nv)).max(axis=1)
        rp, col = s.bsr_pattern()
        kk = np.argsort(big)[-5:]
        rows = np.searchsorted(rp, kk, side="right") - 1
        for kb, r in zip(kk, rows):
            print(f"  big block row {r} col {col[kb]} |max| {big[kb]:.3e} coord {mesh['coord'][r]} "
                  f"Y {np.array2string(st['V'][r][-wl['ns']:], precision=3)}")
        L = s.download("ILU")
        print(f"  ILU non-finite entries: {int((~np.isfinite(L)).sum())}")
        break
    print(f"step {k}: log10 rms flow {np.array2string(np.log10(np.maximum(rms, 1e-300)), precision=2)} "
          f"sst {np.array2string(np.log10(np.maximum(trms, 1e-300)), precision=2)} lin {its}", flush=True)
s.close()
