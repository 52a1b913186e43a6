"""The sharded path bench.py --gpus N runs (bench.py:setup_sharded), on the device: meshgen.shard + set_bc + the
start-up preprocessing (synth.device_preprocess) + whole reference outer iterations (rx.Iterate: flow
Preprocessing, time step, loops + jet boundary conditions, update, Preprocessing(Output), SST iteration with its
boundary conditions) on 2 and 3 ranks, in 2-D and 3-D, against one context on the same global mesh and partitions.
Reference: CMeanFlowIteration::Iterate (iteration_structure.cpp:486-560) run on MPI ranks, each rank's
CGeometry holding its domain points plus one halo layer (geometry_structure.cpp:11465-11530), halos refreshed by
Set_MPI_Solution / Set_MPI_Primitive_Gradient (solver_direct_reactive.cpp:1530-1990), every inner product and RMS
all-reduced (vector_structure.cpp:397-419).

The ranks share the test box's one GPU, so they use the host-staged transport over gloo (RCCL refuses two ranks on
one device); the RCCL transport itself is checked bitwise against one context at world size 1
(test_gpu_shard.py::test_rccl_world1_matches_single_context) and runs the same exchange plan.

Bars:
- EULER_EXPLICIT flow (the shipped cfgs' scheme; LU_SGS SST solve): U, (k, omega) and both RMS vectors within 1e-10
  of one context; the ranks' local edge order (reference: a rank numbers its own edges) changes only summation
  order. Two chained iterations.
- EULER_IMPLICIT (FGMRES(5)+ILU0, the bench step): identical linear-iteration counts, RMS within 1e-10, dU and
  (k, omega) within 5e-8 normwise per column (the FGMRES amplification of the edge-order rounding,
  test_gpu_shard.py; measured values are printed).
- Every rank: halo rows of U and (k, omega) equal their owners' rows after the iteration (Set_MPI_Solution)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from tests.parity import assert_close, per_column_close, rel_err
from tests.rxpkg import meshgen, rx, synth

pytestmark = pytest.mark.gpu

NS = 7
GEOM = {"2d": (48, 20, 0, 12), "3d": (20, 8, 4, 12)}  # nx, ny, nz, global partitions (block-Jacobi ILU)


def _setup(geom, implicit, world=1, rank=0, transport=None):
    nx, ny, nz, parts = GEOM[geom]
    mesh, st0, mech, kw = synth.jet_field_case(nx, ny, n_species=NS, n_part=parts, nz=nz)
    kw = dict(kw, cfl=5.0 if implicit else 0.5)
    cfg = rx.default_cfg(implicit=implicit, rans=1, lin_prec=1, lin_iter=5, **kw)
    if world > 1:
        m = meshgen.shard(mesh, world, rank)
        st = {k: np.asarray(v)[m["l2g"]] for k, v in st0.items()}
    else:
        m, st = mesh, st0
    s = rx.ReactiveNSSolver(m, rx.Mechanism(mech), cfg)
    if transport is not None:
        s.comm_init_host(world, rank, transport)
    s.set_bc(synth.jet_bc(m, NS))
    t = rx.TurbSSTSolver(m, s, rx.sst_cfg(lin_prec=1 if implicit else 0))
    synth.device_preprocess(s, t, m, st)
    return s, t, m


def _iterate(s, t, n_iter):
    out = []
    for k in range(n_iter):
        rms, rms_t, its = rx.Iterate(s, t, ext_iter=k)
        out.append((np.r_[rms, rms_t], its))
    s.sync()
    U = s.download("U").reshape(s.N, -1)
    T = t.download("U").reshape(s.N, 2)
    return out, U, T


def _worker(rank, world, port, q, geom, implicit, n_iter):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, t, m = _setup(geom, implicit, world, rank, rx.TorchHostTransport())
        U0 = s.download("U").reshape(s.N, -1)
        hist, U, T = _iterate(s, t, n_iter)
        s.close()
        q.put((rank, dict(l2g=m["l2g"], nd=int(m["n_domain"]), U0=U0, U=U, T=T, hist=hist)))
    except Exception as e:  # reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run_ranks(world, geom, implicit, n_iter):
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, geom, implicit, n_iter)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=600) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=120)
    for r in range(world):
        assert isinstance(res[r], dict), res[r]
    return res


@pytest.mark.parametrize("world,geom,implicit", [(2, "2d", 0), (3, "2d", 0), (2, "3d", 0),
                                                  (2, "2d", 1), (3, "2d", 1), (2, "3d", 1)])
def test_sharded_iterate_matches_single_context(world, geom, implicit):
    n_iter = 1 if implicit else 2
    s, t, _ = _setup(geom, implicit)
    U_init = s.download("U").reshape(s.N, -1)
    hist0, U0, T0 = _iterate(s, t, n_iter)
    s.close()
    res = _run_ranks(world, geom, implicit, n_iter)
    U_sh, T_sh = np.zeros_like(U0), np.zeros_like(T0)
    owned = np.zeros(len(U0), dtype=np.int64)
    for r in range(world):
        d = res[r]
        l2g, nd = d["l2g"], d["nd"]
        assert np.array_equal(d["U0"][:nd], U_init[l2g[:nd]]), "start state"
        U_sh[l2g[:nd]] = d["U"][:nd]
        T_sh[l2g[:nd]] = d["T"][:nd]
        owned[l2g[:nd]] += 1
        for k, (rms, its) in enumerate(d["hist"]):
            # all-reduced: the same numbers on every rank
            assert np.array_equal(rms, res[0]["hist"][k][0]), f"rank {r} iteration {k}: RMS differs across ranks"
            assert its == hist0[k][1], f"rank {r} iteration {k}: linear iterations {its} vs {hist0[k][1]}"
    assert np.all(owned == 1), "every global point owned by exactly one rank"
    for r in range(world):
        d = res[r]
        l2g, nd = d["l2g"], d["nd"]
        assert np.array_equal(d["U"][nd:], U_sh[l2g[nd:]]), f"rank {r}: halo rows of U = owners' rows"
        assert np.array_equal(d["T"][nd:], T_sh[l2g[nd:]]), f"rank {r}: halo rows of (k, omega) = owners' rows"
    tag = f"{geom} x{world} {'implicit' if implicit else 'explicit'}"
    for k in range(n_iter):
        assert_close(res[0]["hist"][k][0], hist0[k][0], rtol=1e-10, what=f"{tag}: RMS iteration {k}")
    bar = 5e-8 if implicit else 1e-10
    eU = per_column_close(U_sh - U_init, U0 - U_init, rtol=bar, floor=1e-14, what=f"{tag}: dU vs one context")
    eT = per_column_close(T_sh, T0, rtol=bar, floor=1e-14, what=f"{tag}: (k, omega) vs one context")
    print(f"{tag}: dU {eU:.2e}, (k, omega) {eT:.2e}, RMS {rel_err(res[0]['hist'][-1][0], hist0[-1][0]):.2e}")
