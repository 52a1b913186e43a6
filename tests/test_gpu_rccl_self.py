"""The RCCL halo path with real traffic on the test box's one GPU (VERDICT r04 #2a). At world size 1 an ordinary
mesh has no neighbour, so rx_la_exchange_on returns before ncclSend / ncclRecv (rx_comm.hip); every multi-rank test
uses the host transport. Here a world-1 communicator gets an exchange plan that names rank 0 as its own neighbour:
rank 0's shard of a 2-rank split of a partitioned jet (meshgen.shard) whose halo strip is fed from the owned points
next to the cut (each halo point receives its nearest owned point: a zero-gradient strip), so the reference's
SendReceive_Solution / Set_MPI_Solution / Set_MPI_Primitive_Gradient pattern (matrix_structure.cpp:794-880,
solver_direct_reactive.cpp:1530-1636, 1877-1990) moves data on every exchange. Two outer iterations (flow implicit
FGMRES(5)+ILU0 step, then the SST step) run

  (a) over RCCL: grouped ncclSend / ncclRecv to self, the gradient exchange forked onto comm_stream, the Krylov z
      exchange forked around the interior SpMV rows inside the captured FGMRES hipGraph (the second iteration replays
      it), the inner products through ncclAllGather + k_sum_ranks;
  (b) over the synchronous host transport (the same plan through pinned host buffers, eager solve);

and must agree bitwise: gradients, RMS vectors, linear-iteration counts, U, the primitives after the update and
(k, omega) including the halo rows, which must hold the values of the owned points they are fed from. With RCCL the
post-update Set_MPI_Solution runs on comm_stream while SetPrimitive_Variables computes the owned points (round 5).
Requires an MI355X."""
import numpy as np
import pytest

from tests.rxpkg import meshgen, rx
from tests.test_gpu_shard import NS, _case, _set

pytestmark = pytest.mark.gpu


def self_halo_shard():
    from scipy.spatial import cKDTree
    mesh, st, mech_arrays, cfg = _case(implicit=1)
    sh = meshgen.shard(mesh, 2, 0)
    nd, n = int(sh["n_domain"]), len(sh["l2g"])
    _, near = cKDTree(sh["coord"][:nd]).query(sh["coord"][nd:])
    near = np.asarray(near, dtype=np.int64)
    sh.update(neigh=np.array([0], dtype=np.int32), send_ptr=np.array([0, n - nd], dtype=np.int64),
              send_idx=near, recv_ptr=np.array([0, n - nd], dtype=np.int64))
    st_l = {k: np.array(np.asarray(v)[sh["l2g"]]) for k, v in st.items()}
    for v in st_l.values():  # the halo rows start as the values they will receive
        v[nd:] = v[near]
    return sh, st_l, mech_arrays, cfg, nd, near


class SelfTransport:
    """rx_host_comm for a world of one rank whose only neighbour is itself: sendrecv copies each neighbour's send
    segment into its receive segment; the all-reduce of one rank is the identity."""

    def __init__(self):
        self.calls = 0

        def sendrecv(user, n_neigh, neigh, send_ptr, send, recv_ptr, recv, stride):
            for k in range(n_neigh):
                assert neigh[k] == 0
                s0, s1 = send_ptr[k] * stride, send_ptr[k + 1] * stride
                r0, r1 = recv_ptr[k] * stride, recv_ptr[k + 1] * stride
                src = np.ctypeslib.as_array(send, shape=(s1,))[s0:s1]
                np.ctypeslib.as_array(recv, shape=(r1,))[r0:r1] = src
            self.calls += 1
            return 0

        def allreduce(user, inp, out, count):
            np.ctypeslib.as_array(out, shape=(count,))[:] = np.ctypeslib.as_array(inp, shape=(count,))
            return 0

        self._cb = (rx.SENDRECV_FN(sendrecv), rx.ALLREDUCE_FN(allreduce))
        self.desc = rx.HostComm(None, self._cb[0], self._cb[1])


def _step(s, t):
    """One outer iteration in rx.Iterate's order: the flow implicit step, the flow SetPrimitive_Variables on the updated
    solution (with RCCL its owned points run while the post-update Set_MPI_Solution is in flight on comm_stream, then
    the halo points), then the SST step."""
    s.SetPrimitive_Gradient_LS()
    grad = s.download("GRAD")
    s.SetStrainMag()
    s.SetTime_Step()
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    rms, it = s.ImplicitEuler_Iteration()
    s.SetPrimitive_Variables(1)
    V = s.download("V")
    t.Preprocessing()
    t.Upwind_Residual()
    t.Viscous_Residual()
    t.Source_Residual()
    trms, tit = t.ImplicitEuler_Iteration()
    t.Postprocessing()
    return grad, V, np.r_[rms, trms], (it, tit)


def run(transport):
    sh, st_l, mech_arrays, cfg, nd, near = self_halo_shard()
    s = rx.ReactiveNSSolver(sh, rx.Mechanism(mech_arrays), cfg)
    tr = None
    if transport == "rccl":
        s.comm_init(1, 0, rx.comm_unique_id())
    else:
        tr = SelfTransport()
        s.comm_init_host(1, 0, tr)
    t = rx.TurbSSTSolver(sh, s, rx.sst_cfg())
    _set(s, t, sh, st_l)
    out = []
    for _ in range(2):  # RCCL: the second iteration replays the captured solve graphs
        g, V, rms, it = _step(s, t)
        out.append(dict(grad=g, V=V, rms=rms, it=it, U=s.download("U"), T=t.download("U")))
    s.close()
    if tr is not None:
        assert tr.calls > 0
    return out, nd, near, sh


def test_rccl_self_halo_matches_host_transport():
    a, nd, near, sh = run("rccl")
    b, _, _, _ = run("host")
    nvar = NS + 4
    for k in range(2):
        assert a[k]["it"] == b[k]["it"], k
        assert np.array_equal(a[k]["grad"], b[k]["grad"]), f"iteration {k}: gradients"
        assert np.array_equal(a[k]["rms"], b[k]["rms"]), f"iteration {k}: RMS"
        assert np.array_equal(a[k]["U"], b[k]["U"]), f"iteration {k}: U"
        assert np.array_equal(a[k]["V"], b[k]["V"]), f"iteration {k}: primitives after the update"
        assert np.array_equal(a[k]["T"], b[k]["T"]), f"iteration {k}: (k, omega)"
        U = a[k]["U"].reshape(-1, nvar)
        T = a[k]["T"].reshape(-1, 2)
        # Set_MPI_Solution after the update: every halo row holds the value of the owned point that feeds it
        assert np.array_equal(U[nd:], U[near]) and np.array_equal(T[nd:], T[near])
        V = a[k]["V"].reshape(len(sh["l2g"]), -1)
        assert np.array_equal(V[nd:], V[near])  # the halo points' primitives from the exchanged solution
        assert np.all(np.isfinite(U)) and a[k]["it"][0] >= 1
    G = a[1]["grad"].reshape(len(sh["l2g"]), -1)
    assert np.array_equal(G[nd:], G[near])  # Set_MPI_Primitive_Gradient
    assert not np.array_equal(a[0]["U"], a[1]["U"])  # the second iteration moved the state
    print(f"self-halo RCCL: {len(near)} halo points of {len(sh['l2g'])}, lin iters {[x['it'] for x in a]}")
