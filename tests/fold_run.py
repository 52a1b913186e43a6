"""Two outer iterations (rx.Iterate) of a partitioned synthetic jet with its boundary conditions, the flow and SST
solutions and the RMS written to an .npz (helper of tests/test_gpu_fold.py, run as a subprocess so that RX_NO_FOLD,
read once per process by rx_set_system_fold, can differ between runs).

usage: python tests/fold_run.py NZ OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.rxpkg import rx, synth  # noqa: E402


def main():
    nz, out = int(sys.argv[1]), sys.argv[2]
    mesh, st, mech, kw = synth.jet_case(24, 10, n_species=7, n_part=4, nz=nz)
    cfg = rx.default_cfg(implicit=1, lin_prec=1, **kw)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), cfg)
    s.set_bc(synth.jet_bc(mesh, 7))
    t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
    s.set_state(st)
    t.set_state(st["sst_sol"], mesh["wall_distance"], st["sst_F1"], st["sst_F2"], st["sst_CDkw"])
    rms = []
    for k in range(2):
        r, rt, its = rx.Iterate(s, t, ext_iter=k)
        rms.append(np.r_[r, rt, its])
    s.sync()
    np.savez(out, U=s.download("U"), T=t.download("U"), rms=np.array(rms))
    t.close()
    s.close()


if __name__ == "__main__":
    main()
