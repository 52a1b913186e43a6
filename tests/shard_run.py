"""Run the sharded device path (meshgen.shard, one process per rank, the host-staged transport over gloo on the test
box's one GPU) the way bench.py --gpus N runs it, for the multi-rank parity tests (test_gpu_shard_iterate.py,
test_gpu_c4.py). Reference: CMeanFlowIteration::Iterate (iteration_structure.cpp:486-560) on MPI ranks, each rank's
CGeometry holding its domain points plus one halo layer (geometry_structure.cpp:11465-11530), halos refreshed by
Set_MPI_Solution / Set_MPI_Primitive_Gradient (solver_direct_reactive.cpp:1530-1990), every inner product and RMS
all-reduced (vector_structure.cpp:397-419).

The parent builds the global mesh and state once, writes every rank's shard to an .npz file and spawns the ranks;
each rank completes its records with the start-up preprocessing (synth.device_preprocess), optionally takes the
oracle's iteration-start (grad k, sigma_k), runs rx.Iterate and returns its owned rows. RCCL refuses two ranks on one
device, so the ranks use rx.TorchHostTransport; the RCCL transport runs the same plan and the same rank-ordered
all-reduce (rx_comm.hip)."""
import json
import multiprocessing as mp
import os
import socket

import numpy as np

NS = 7
STATE_KEYS = ("V", "U", "dPdU", "dTdU", "mu", "kappa", "Dij", "turb_k", "turb_omega", "mu_t", "sigma_k", "grad_k",
              "eddy_visc_flow", "grad_prim", "sst_F1", "sst_F2", "sst_CDkw", "sst_sol")


def write_shards(tmpdir, mesh, st0, mech, kw, world, tg=None):
    """Every rank's shard + its rows of the raw initial state (+ of the oracle's turbulent gradient tg) in
    tmpdir/rank{r}.npz; returns the shards (l2g, n_domain, rank_ptr)."""
    from tests.rxpkg import meshgen
    out = []
    for r in range(world):
        sh = meshgen.shard(mesh, world, r)
        arr = {"m_" + k: np.asarray(v) for k, v in sh.items()}
        arr.update({"s_" + k: np.asarray(v)[sh["l2g"]] for k, v in st0.items()})
        arr.update({k: np.asarray(v) for k, v in mech.items()})
        if tg is not None:
            arr["tg"] = np.ascontiguousarray(np.asarray(tg)[sh["l2g"]])
        arr["kw"] = np.array(json.dumps(kw))
        np.savez(os.path.join(tmpdir, f"rank{r}.npz"), **arr)
        out.append(dict(l2g=sh["l2g"], n_domain=int(sh["n_domain"]), rank_ptr=sh["rank_ptr"],
                        n_point=len(sh["coord"]), n_edge=len(sh["edges"]), n_part=len(sh["part_ptr"]) - 1))
    return out


def _worker(rank, world, port, q, tmpdir, implicit, n_iter, cfl, rk):
    import torch.distributed as dist

    from tests.rxpkg import rx, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = dict(np.load(os.path.join(tmpdir, f"rank{rank}.npz")))
        m = {k[2:]: (v if v.ndim else v.item()) for k, v in z.items() if k.startswith("m_")}
        st = {k[2:]: v for k, v in z.items() if k.startswith("s_")}
        mech = {k: v for k, v in z.items() if k.startswith("mech_")}
        kw = json.loads(str(z["kw"]))
        kw = dict(kw, cfl=cfl)
        cfg = rx.default_cfg(implicit=implicit, rans=1, lin_prec=1, lin_iter=5, **kw)
        s = rx.ReactiveNSSolver(m, rx.Mechanism(mech), cfg)
        s.comm_init_host(world, rank, rx.TorchHostTransport())
        s.set_bc(synth.jet_bc(m, NS))
        t = rx.TurbSSTSolver(m, s, rx.sst_cfg(lin_prec=1 if implicit else 0))
        pre = synth.device_preprocess(s, t, m, st)
        nd = int(m["n_domain"])
        if "tg" in z:  # the reference's iteration-start state (test_gpu_size.py): grad k of the SST solution, sigma_k
            s.upload("GRADK", np.ascontiguousarray(z["tg"][:, 0, :]))
            s.upload("SIGMAK", np.full(s.N, 0.85))
        U0 = s.download("U").reshape(s.N, -1)
        hist = []
        for k in range(n_iter):
            rms, rms_t, its = rx.Iterate(s, t, ext_iter=k, rk_alpha=rk)
            hist.append((np.r_[rms, rms_t], its))
        s.sync()
        U = s.download("U").reshape(s.N, -1)
        T = t.download("U").reshape(s.N, 2)
        s.close()
        q.put((rank, dict(l2g=m["l2g"], nd=nd, U0=U0[:nd], U=U, T=T, hist=hist,
                          pre={k: np.asarray(pre[k])[:nd] for k in STATE_KEYS})))
    except Exception as e:  # reported to the parent
        import traceback
        q.put((rank, repr(e) + "\n" + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def run_ranks(tmpdir, world, implicit, n_iter, cfl, rk=None, timeout=900):
    """Spawn `world` ranks on the shards of write_shards; returns {rank: result dict}."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, str(tmpdir), implicit, n_iter, cfl, rk))
          for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=timeout) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert isinstance(res[r], dict), f"rank {r}: {res[r]}"
    return res


def gather(res, N, nvar):
    """Owned rows of every rank in global order: U, T, and the preprocessed records; checks each point is owned
    once and every rank's halo rows of U / (k, omega) equal their owners' (Set_MPI_Solution)."""
    U = np.zeros((N, nvar))
    T = np.zeros((N, 2))
    pre = {}
    owned = np.zeros(N, dtype=np.int64)
    for r, d in res.items():
        l2g, nd = d["l2g"], d["nd"]
        U[l2g[:nd]] = d["U"][:nd]
        T[l2g[:nd]] = d["T"][:nd]
        owned[l2g[:nd]] += 1
        for k, v in d["pre"].items():
            if k not in pre:
                pre[k] = np.zeros((N,) + v.shape[1:])
            pre[k][l2g[:nd]] = v
    assert np.all(owned == 1), "every global point owned by exactly one rank"
    for r, d in res.items():
        l2g, nd = d["l2g"], d["nd"]
        assert np.array_equal(d["U"][nd:], U[l2g[nd:]]), f"rank {r}: halo rows of U = owners' rows"
        assert np.array_equal(d["T"][nd:], T[l2g[nd:]]), f"rank {r}: halo rows of (k, omega) = owners' rows"
    return U, T, pre
