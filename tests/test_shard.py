"""Sharding of the dual grid across ranks (meshgen.shard): one halo layer, exchange plan, and the
residual of every owned point equal to the unsharded one (CPU oracle). The N>1 exchange itself is
exercised with torch.distributed (gloo, world_size 2) on CPU."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.rxpkg import meshgen, synth


def sharded_case(R, nx=60, ny=24, n_part=8, ns=7):
    mesh, st, mech, kw = synth.jet_case(nx, ny, n_species=ns, n_part=n_part)
    return mesh, st, mech, kw, [meshgen.shard(mesh, R, r) for r in range(R)]


@pytest.mark.parametrize("R", [2, 3])
def test_exchange_plan_is_symmetric(R):
    mesh, st, mech, kw, sh = sharded_case(R)
    assert sum(s["n_domain"] for s in sh) == len(mesh["coord"])
    for r, s in enumerate(sh):
        halo_g = s["l2g"][s["n_domain"]:]
        for k, q in enumerate(s["neigh"]):
            recv = halo_g[s["recv_ptr"][k]:s["recv_ptr"][k + 1]]
            o = sh[q]
            kq = list(o["neigh"]).index(r)
            sent = o["l2g"][o["send_idx"][o["send_ptr"][kq]:o["send_ptr"][kq + 1]]]
            assert np.array_equal(recv, sent)


def local_residual(om, s, st_l, kw):
    """Explicit residual of the local mesh with the oracle, gathered in local edge order."""
    nDim, ns = 2, om.ns
    N = len(s["coord"])
    G = O.grad_lsq(om, nDim, np.arange(N), s["coord"], st_l["V"], s["nbr_ptr"], s["nbr"])
    rc, _, _ = O.ausm_edges(nDim, ns, s["edges"], s["edge_normal"], st_l["V"], st_l["dPdU"], kw["mach_inf"], False)
    return G, rc


@pytest.mark.parametrize("R", [2, 3])
def test_owned_residual_matches_global(R):
    mesh, st, mech, kw, sh = sharded_case(R)
    om = O.Mechanism(mech)
    N = len(mesh["coord"])
    nDim, ns = 2, om.ns
    G = O.grad_lsq(om, nDim, np.arange(N), mesh["coord"], st["V"], mesh["nbr_ptr"], mesh["nbr"])
    rc, _, _ = O.ausm_edges(nDim, ns, mesh["edges"], mesh["edge_normal"], st["V"], st["dPdU"], kw["mach_inf"], False)
    R_glob = np.zeros((N, rc.shape[1]))
    np.add.at(R_glob, mesh["edges"][:, 0], rc)
    np.add.at(R_glob, mesh["edges"][:, 1], -rc)
    for s in sh:
        st_l = {k: v[s["l2g"]] for k, v in st.items()}
        Gl, rcl = local_residual(om, s, st_l, kw)
        nd = s["n_domain"]
        # LSQ neighbour order is kept for owned points: bitwise
        assert np.array_equal(Gl[:nd], G[s["l2g"][:nd]])
        R_loc = np.zeros((len(s["coord"]), rc.shape[1]))
        np.add.at(R_loc, s["edges"][:, 0], rcl)
        np.add.at(R_loc, s["edges"][:, 1], -rcl)
        ref = R_glob[s["l2g"][:nd]]
        # local edges keep the global order and orientation: every owned point adds the same fluxes in the same
        # order, bitwise
        assert np.array_equal(R_loc[:nd], ref)
        assert np.array_equal(s["l2g"][s["edges"]], mesh["edges"][np.isin(mesh["edges"], s["l2g"][:nd]).any(axis=1)])


def _exchange_worker(rank, world, port, R_nx, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mesh = meshgen.build_jet(*R_nx, n_part=8)
        s = meshgen.shard(mesh, world, rank)
        nd, n = s["n_domain"], len(s["l2g"])
        # field = global id * 10 + component, halo filled with -1 until exchanged
        f = np.full((n, 3), -1.0)
        f[:nd] = s["l2g"][:nd, None] * 10.0 + np.arange(3)
        reqs, bufs = [], []
        for k, q_ in enumerate(s["neigh"]):
            sb = torch.from_numpy(f[s["send_idx"][s["send_ptr"][k]:s["send_ptr"][k + 1]]].copy())
            rb = torch.empty((s["recv_ptr"][k + 1] - s["recv_ptr"][k], 3), dtype=torch.float64)
            reqs.append(dist.isend(sb, int(q_)))
            reqs.append(dist.irecv(rb, int(q_)))
            bufs.append((k, rb))
        for r_ in reqs:
            r_.wait()
        for k, rb in bufs:
            f[nd + s["recv_ptr"][k]:nd + s["recv_ptr"][k + 1]] = rb.numpy()
        ok = np.array_equal(f, s["l2g"][:, None] * 10.0 + np.arange(3))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_halo_exchange_gloo_world2():
    import multiprocessing as mp
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_exchange_worker, args=(r, 2, port, (60, 24), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _allreduce_worker(rank, world, port, q):
    import ctypes as C

    import torch.distributed as dist

    from tests.rxpkg import rx
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = rx.TorchHostTransport()
        # rank sums whose total depends on the addition order: ((1e16 + 1) + -1e16) + 1 = 1 in rank order,
        # 2 in exact arithmetic, 0 or 1 in other orders
        vals = {0: [1e16, 3.0], 1: [1.0, 0.5], 2: [-1e16, 0.25], 3: [1.0, 0.125]}[rank]
        a = np.array(vals)
        out = np.zeros(2)
        rc = t._cb[1](None, a.ctypes.data_as(C.POINTER(C.c_double)), out.ctypes.data_as(C.POINTER(C.c_double)), 2)
        q.put((rank, (rc, out.tolist())))
    finally:
        dist.destroy_process_group()


def test_host_transport_allreduce_is_rank_ordered():
    """rx_host_comm's all-reduce contract (include/rx.h): the rank-ordered sum ((in_0 + in_1) + in_2) + ..., the same
    doubles on every rank, as the RCCL path's all-gather + k_sum_ranks; the oracle's rank-split inner products
    (O.dot_order("device", ranks=...)) restate it."""
    import multiprocessing as mp
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_allreduce_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    want = [((1e16 + 1.0) + -1e16) + 1.0, ((3.0 + 0.5) + 0.25) + 0.125]
    for r in range(4):
        assert res[r] == (0, want), res[r]


def test_oracle_rank_split_dot():
    """O.dot_order("device", ranks=rank_ptr): each rank's rows in the device's reduction order, then the rank-ordered
    sum; a single rank is the plain device order."""
    rng = np.random.default_rng(3)
    nb, rp = 3, np.array([0, 700, 1500, 2300], dtype=np.int64)
    a, c = rng.normal(size=rp[-1] * nb), rng.normal(size=rp[-1] * nb)
    L = O.lib()
    with O.dot_order("device"):
        dev = [L.orc_dot(C_i64(q1 - q0), O._p(a[q0:q1]), O._p(c[q0:q1])) for q0, q1 in zip(rp[:-1] * nb, rp[1:] * nb)]
        whole = L.orc_dot(C_i64(len(a)), O._p(a), O._p(c))
    with O.dot_order("device", ranks=rp):
        split = L.orc_dot(C_i64(len(a)), O._p(a), O._p(c))
    with O.dot_order("device", ranks=np.array([0, rp[-1]])):
        one = L.orc_dot(C_i64(len(a)), O._p(a), O._p(c))
    assert split == (dev[0] + dev[1]) + dev[2] and one == whole


def C_i64(v):
    import ctypes as C
    return C.c_int64(int(v))
