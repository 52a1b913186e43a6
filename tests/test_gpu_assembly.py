"""The implicit system's assembly paths: the 2-D node-centric assembly that also evaluates the AUSM
flux and Jacobians (k_asm_visc's fused pass, the default) against the per-edge convective kernel path
(k_ausm_edge + k_asm_visc's non-fused pass, RX_ASM_CONV=0), bitwise, for 1st order and both MUSCL branches; the
3-D fused default (round 5) against the edge kernel path, 1st order and MUSCL; and a re-assembly of the same residual after
an intermediate download (Upwind, Viscous, RES download, then Source) against the straight sequence and the
reference's golden system. Round 6: the edge-side-team assembly (k_asm_es, the default) against the node-serial
k_asm_visc (RX_ASMV_ES=0), fused and per-edge convective, 2-D and 3-D, every spatial order. Requires an MI355X."""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.parity import assert_close
from tests.test_gpu_parity import golden, make_solver

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def run_variant(tmp_path, case, order, env_val, es=None):
    env = dict(os.environ)
    env.pop("RX_ASM_CONV", None)
    env.pop("RX_ASMV_ES", None)
    if env_val is not None:
        env["RX_ASM_CONV"] = env_val
    if es is not None:
        env["RX_ASMV_ES"] = es
    out = str(tmp_path / f"{case}_{order}_{env_val}_{es}.npz")
    subprocess.run([sys.executable, os.path.join(HERE, "asm_variant_run.py"), case, str(order), out], env=env,
                   check=True, timeout=300)
    return dict(np.load(out))


@pytest.mark.parametrize("case,order", [("mini9", 0), ("mini9", 1), ("mini9", 2), ("jet9w", 2)])
def test_fused_ausm_assembly_is_bitwise_the_edge_kernel_path(tmp_path, case, order):
    fused = run_variant(tmp_path, case, order, None)  # 2-D default: the fused pass
    edge = run_variant(tmp_path, case, order, "0")    # k_ausm_edge's per-edge blocks
    assert np.array_equal(fused["res"], edge["res"])
    assert np.array_equal(fused["jac"], edge["jac"])


@pytest.mark.parametrize("order", [0, 2])
def test_fused_ausm_assembly_3d_is_bitwise(tmp_path, order):
    fused = run_variant(tmp_path, "mini3d", order, None)  # 3-D default since round 5: the fused pass
    edge = run_variant(tmp_path, "mini3d", order, "0")
    assert np.array_equal(fused["res"], edge["res"])
    assert np.array_equal(fused["jac"], edge["jac"])


@pytest.mark.parametrize("case,order", [("mini9", 0), ("mini9", 1), ("mini9", 2), ("jet9w", 2), ("mini3d", 0),
                                        ("mini3d", 2)])
@pytest.mark.parametrize("conv", [None, "0"])
def test_edge_side_teams_are_bitwise_the_node_serial_assembly(tmp_path, case, order, conv):
    """k_asm_es (each team one adjacency entry, the node's contributions added in phase B in k_asm_visc's order)
    against k_asm_visc: residual and every BSR block bitwise, with the fused AUSM pass and with k_ausm_edge's blocks."""
    es = run_variant(tmp_path, case, order, conv)
    serial = run_variant(tmp_path, case, order, conv, es="0")
    assert np.array_equal(es["res"], serial["res"])
    assert np.array_equal(es["jac"], serial["jac"])


@pytest.mark.parametrize("case", ["mini9", "mini3d"])
def test_reassembly_after_download(case):
    """a RES download between the viscous and the source loop assembles the system once; the
    source loop then invalidates it, and the second assembly must rebuild it from this residual's convective terms
    (fused pass again, or the per-edge blocks) — bitwise the straight sequence, and the reference's system."""
    g = golden(case)
    nVar = int(g["dims"][1])
    nDim = int(g["dims"][0])
    F = nDim + 2

    def system(download_between):
        s, _ = make_solver(g, implicit=True)
        s.upload("DT", g["dt"])
        s.Preprocessing_zero()
        s.Upwind_Residual()
        s.Viscous_Residual()
        if download_between:
            s.sync()
            s.download("RES")
        s.Source_Residual()
        s.sync()
        R, A = s.download("RES").reshape(-1, nVar), s.download("JAC").reshape(-1, nVar, nVar)
        rp, col = s.bsr_pattern()
        s.close()
        return R, A, rp, col

    R1, A1, rp, col = system(False)
    R2, A2, _, _ = system(True)
    assert np.array_equal(R1, R2)
    assert np.array_equal(A1, A2)
    ref = g["loop_total_res"]
    assert_close(R2[:, :F], ref[:, :F], what="re-assembled residual flow rows")
    assert np.max(np.abs(R2[:, F:] - ref[:, F:])) <= 1e-10 * np.abs(ref[:, F:]).max()
    Aref = g["bsr_system"].copy()
    diag = np.array([rp[i] + np.nonzero(col[rp[i]:rp[i + 1]] == i)[0][0] for i in range(len(rp) - 1)])
    Aref[diag] -= np.einsum("i,ab->iab", g["volume"] / g["dt"], np.eye(nVar))
    scale = np.abs(Aref).max(axis=(1, 2), keepdims=True)
    assert (np.abs(A2 - Aref) / np.where(scale == 0, 1, scale)).max() <= 1e-10
