#!/usr/bin/env python3
"""Per-rank floor of the C4 strong-scaling run (VERDICT r04 #2c), on one GPU: one rank's shard of the decomposition
`bench.py --gpus 8 --scaling strong` builds (the 2000 x 500 C3 jet, 7 species, 256 partitions per rank = 2048 in all;
meshgen.shard: 125 000 owned points + one halo layer) with its boundary conditions, timed as bench.py times a step
(rx.Iterate: the reference's whole outer iteration), but with no communicator attached: every halo exchange and
all-reduce returns at once (rx_la_exchange_on / rx_la_allreduce: not distributed), so what is left is the rank's
compute. Halo rows keep their start-up values. Prints one JSON line (ms per step, Mcells*iters/s of the owned points,
the phase split) for DESIGN §6's budget: floor + exchanges x their latency.

usage: python tools/c4_rank_floor.py [--rank 3] [--world 8] [--parts 256] [--steps 10] [--warmup 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--parts", type=int, default=256, help="partitions per rank")
    ap.add_argument("--nx", type=int, default=2000)
    ap.add_argument("--ny", type=int, default=500)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch

    import bench
    from tests.rxpkg import meshgen, rx, synth
    ns = 7
    mesh, st, mech_arrays, kw = bench.build_workload(a.nx, a.ny, ns, a.parts * a.world)
    sh = meshgen.shard(mesh, a.world, a.rank)
    st_l = {k: np.asarray(v)[sh["l2g"]] for k, v in st.items()}
    cfg = rx.default_cfg(implicit=1, rans=1, lin_prec=1, lin_iter=5, **kw)
    s = rx.ReactiveNSSolver(sh, rx.Mechanism(mech_arrays), cfg)
    s.set_bc(synth.jet_bc(sh, ns))
    t = rx.TurbSSTSolver(sh, s, rx.sst_cfg())
    st_l = synth.device_preprocess(s, t, sh, st_l)
    bench.set_states(s, t, sh, st_l)
    its = []
    ext = [0]

    def step():
        rms, trms, it = rx.Iterate(s, t, ext_iter=ext[0])
        ext[0] += 1
        its.append(it)

    for _ in range(a.warmup):
        step()
    s.sync()
    torch.cuda.synchronize()
    s.profile(True)
    t.profile(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    s.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    prof = {k: s.profile_read(k) for k in rx.K}
    tprof = {k: t.profile_read(k) for k in rx.K}
    phases = {k: round((prof[k][0] + tprof[k][0]) / a.steps, 4) for k in rx.K if prof[k][1] + tprof[k][1] > 0}
    s.profile(False)
    t.profile(False)
    # the SOLVE phase's kernels per launch (as bench.py: one more step with the solve launched eagerly, flow context)
    os.environ["RX_NO_GRAPH"] = "1"
    s.profile(True)
    step()
    s.sync()
    in_solve = {k: round(s.profile_read(k)[0] / max(1, s.profile_read(k)[1]) * 1e3, 1) for k in ("SPMV", "ILU_APPLY")}
    s.profile(False)
    os.environ.pop("RX_NO_GRAPH")
    nd = int(sh["n_domain"])
    out = dict(what="C4 rank floor (no communicator: exchanges and all-reduces skipped)", rank=a.rank,
               world=a.world, parts_per_rank=a.parts, owned_points=nd, halo_points=len(sh["l2g"]) - nd,
               neighbours=[int(x) for x in sh["neigh"]], send_points=int(len(sh["send_idx"])),
               ms_per_step=round(el / a.steps * 1e3, 3), mcells_iters_per_s_owned=round(nd * a.steps / el / 1e6, 3),
               lin_iters=[list(map(int, x)) for x in its[-a.steps:]][:3], phase_ms_per_step=phases,
               in_solve_us_per_launch=in_solve)
    s.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
