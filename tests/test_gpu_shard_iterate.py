"""The sharded path bench.py --gpus N runs (bench.py:setup_sharded), on the device: meshgen.shard + set_bc + the
start-up preprocessing (synth.device_preprocess) + whole reference outer iterations (rx.Iterate: flow
Preprocessing, time step, loops + jet boundary conditions, update, Preprocessing(Output), SST iteration with its
boundary conditions) on 2 and 3 ranks, in 2-D and 3-D (tests/shard_run.py). Reference: CMeanFlowIteration::Iterate
(iteration_structure.cpp:486-560) on MPI ranks (geometry_structure.cpp:11465-11530), Set_MPI_Solution /
Set_MPI_Primitive_Gradient (solver_direct_reactive.cpp:1530-1990), dotProd's MPI_Allreduce
(vector_structure.cpp:397-419).

A shard keeps the global edge order and orientation, and its BSR rows the global column order (meshgen.shard,
rx_mesh_desc.global_id), so an owned point's residual, Jacobian rows, gradient, time step and SpMV rows are the
undivided mesh's, operation for operation; the ranks differ from one context only in the inner products (each rank's
partial over its own rows, then the rank-ordered sum of the all-reduce). Bars:
- start-up preprocessing: every owned record bitwise equal to one context's;
- EULER_EXPLICIT flow (the shipped cfgs' scheme; LU_SGS SST solve), two chained iterations: U, (k, omega) and both RMS
  vectors within 1e-10 of one context;
- EULER_IMPLICIT (FGMRES(5)+ILU0, the bench step), one iteration from the reference's iteration-start state: against
  the CPU oracle's O.outer_iteration on the same global mesh and partitions with the inner products in the ranks'
  order (O.dot_order("device", ranks=rank_ptr)) at 1e-10 — U per column, every species elementwise, (k, omega), both
  RMS vectors, identical linear-iteration counts (this replaces round 3's 5e-8 bar against one context);
- every rank: halo rows of U and (k, omega) equal their owners' rows after the iteration (Set_MPI_Solution)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.oracle_inputs import outer_iteration_inputs
from tests.parity import assert_close, per_column_close, rel_err, species_close
from tests.rxpkg import rx, synth
from tests.shard_run import NS, STATE_KEYS, gather, run_ranks, write_shards

pytestmark = pytest.mark.gpu

GEOM = {"2d": (48, 20, 0, 12), "3d": (20, 8, 4, 12)}  # nx, ny, nz, global partitions (block-Jacobi ILU)


def single_context(mesh, st0, mech, kw, implicit, cfl):
    cfg = rx.default_cfg(implicit=implicit, rans=1, lin_prec=1, lin_iter=5, **dict(kw, cfl=cfl))
    bc = synth.jet_bc(mesh, NS)
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), cfg)
    s.set_bc(bc)
    t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg(lin_prec=1 if implicit else 0))
    st = synth.device_preprocess(s, t, mesh, st0)
    return s, t, st, cfg, bc


def check_preprocessing(pre, st, tag):
    for k in STATE_KEYS:
        a, b = np.asarray(pre[k]).reshape(len(pre[k]), -1), np.asarray(st[k]).reshape(len(st[k]), -1)
        assert np.array_equal(a, b), f"{tag}: start-up record {k} differs from one context ({rel_err(a, b):.2e})"


def check_vs_oracle(mesh, mech, st, cfg, bc, rank_ptr, U, T, hist, nd, tag):
    """One implicit outer iteration of the oracle on the global mesh, the inner products in the ranks' order."""
    N = len(st["V"])
    mesh_o, state, bco, c = outer_iteration_inputs(mesh, st, cfg, bc)
    pat = O.bsr_pattern(N, mesh["edges"])
    with O.dot_order("device", ranks=rank_ptr):
        o = O.outer_iteration(O.Mechanism(mech), nd, mesh_o, state, bco, c, 0, pat, part_ptr=mesh["part_ptr"],
                              keep=False)
    rms, its = hist[0]
    assert tuple(its) == (o["lin_iters"], o["sst_lin_iters"]), f"{tag}: linear iterations {its}"
    cols = [v for v in range(U.shape[1]) if not 1 <= v <= nd]
    eU = per_column_close(U[:, cols], o["U"][:, cols], rtol=1e-10, floor=1.0, what=f"{tag}: U vs oracle")
    eS = species_close(U, o["U"], nd, rtol=1e-10, what=f"{tag}: species (elementwise) vs oracle")
    mom = np.abs(o["U"][:, 1:nd + 1]).max()
    eM = assert_close(U[:, 1:nd + 1], o["U"][:, 1:nd + 1], rtol=1e-10, floor=1.0, scale=mom,
                      what=f"{tag}: momentum vs oracle (momentum magnitude scale)")
    eT = per_column_close(T, o["T"], rtol=1e-10, floor=1.0, what=f"{tag}: (k, omega) vs oracle")
    nv = U.shape[1]
    assert_close(rms[:nv], o["rms"], rtol=1e-10, what=f"{tag}: RMS flow")
    assert_close(rms[nv:], o["sst_rms"], rtol=1e-10, what=f"{tag}: RMS SST")
    print(f"{tag}: vs oracle (rank-ordered inner products): U {eU:.2e}, species {eS:.2e}, momentum {eM:.2e}, "
          f"(k, omega) {eT:.2e}; bitwise U {np.array_equal(U, o['U'])}, (k, omega) {np.array_equal(T, o['T'])}")


@pytest.mark.parametrize("world,geom", [(2, "2d"), (3, "2d"), (2, "3d")])
def test_sharded_explicit_matches_single_context(world, geom, tmp_path):
    nx, ny, nz, parts = GEOM[geom]
    mesh, st0, mech, kw = synth.jet_field_case(nx, ny, n_species=NS, n_part=parts, nz=nz)
    s, t, st, cfg, bc = single_context(mesh, st0, mech, kw, 0, 0.5)
    U_init = s.download("U").reshape(s.N, -1)
    hist0 = []
    for k in range(2):
        rms, rms_t, its = rx.Iterate(s, t, ext_iter=k)
        hist0.append((np.r_[rms, rms_t], its))
    s.sync()
    U0, T0 = s.download("U").reshape(s.N, -1), t.download("U").reshape(s.N, 2)
    s.close()
    write_shards(tmp_path, mesh, st0, mech, kw, world)
    res = run_ranks(tmp_path, world, 0, 2, 0.5)
    U, T, pre = gather(res, len(U0), U0.shape[1])
    tag = f"{geom} x{world} explicit"
    check_preprocessing(pre, st, tag)
    for r, d in res.items():
        for k, (rms, its) in enumerate(d["hist"]):
            assert np.array_equal(rms, res[0]["hist"][k][0]), f"rank {r} iteration {k}: RMS differs across ranks"
            assert its == hist0[k][1], f"rank {r} iteration {k}: linear iterations {its} vs {hist0[k][1]}"
    for k in range(2):
        assert_close(res[0]["hist"][k][0], hist0[k][0], rtol=1e-10, what=f"{tag}: RMS iteration {k}")
    eU = per_column_close(U - U_init, U0 - U_init, rtol=1e-10, floor=1e-14, what=f"{tag}: dU vs one context")
    eT = per_column_close(T, T0, rtol=1e-10, floor=1e-14, what=f"{tag}: (k, omega) vs one context")
    print(f"{tag}: dU {eU:.2e}, (k, omega) {eT:.2e}, bitwise U {np.array_equal(U, U0)}")


@pytest.mark.parametrize("world,geom", [(2, "2d"), (3, "2d"), (2, "3d")])
def test_sharded_implicit_matches_oracle_on_the_ranks(world, geom, tmp_path):
    nx, ny, nz, parts = GEOM[geom]
    mesh, st0, mech, kw = synth.jet_field_case(nx, ny, n_species=NS, n_part=parts, nz=nz)
    s, t, st, cfg, bc = single_context(mesh, st0, mech, kw, 1, rx.BENCH_CFL)
    s.close()
    _, state, _, _ = outer_iteration_inputs(mesh, st, cfg, bc)
    shards = write_shards(tmp_path, mesh, st0, mech, kw, world, tg=state["TG"])
    res = run_ranks(tmp_path, world, 1, 1, rx.BENCH_CFL)
    N, nv = len(st["V"]), st["U"].shape[1]
    U, T, pre = gather(res, N, nv)
    tag = f"{geom} x{world} implicit"
    check_preprocessing(pre, st, tag)
    for r, d in res.items():
        assert np.array_equal(d["hist"][0][0], res[0]["hist"][0][0]), f"rank {r}: RMS differs across ranks"
    check_vs_oracle(mesh, mech, st, cfg, bc, shards[0]["rank_ptr"], U, T, res[0]["hist"], 3 if nz else 2, tag)
