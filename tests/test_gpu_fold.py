"""rx_set_system_fold (round 5): rx.Iterate lets the node-centric assembly add ImplicitEuler_Iteration's V / dt to
the diagonal of the rows no boundary condition changes afterwards (k_asm_visc, SysFold), and the system build then
leaves those rows' diagonals alone (k_build_system_elem). Two outer iterations of a partitioned synthetic jet with its
inlet / outlet / wall markers, 2-D and 3-D: the flow and SST solutions, the RMS and the linear-solver counts bitwise
those of the unfolded build (RX_NO_FOLD=1). Requires an MI355X."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def run(tmp_path, nz, no_fold, es=None):
    env = dict(os.environ)
    env.pop("RX_NO_FOLD", None)
    env.pop("RX_ASMV_ES", None)
    if no_fold:
        env["RX_NO_FOLD"] = "1"
    if es is not None:
        env["RX_ASMV_ES"] = es
    out = str(tmp_path / f"fold_{nz}_{int(no_fold)}_{es}.npz")
    subprocess.run([sys.executable, os.path.join(HERE, "fold_run.py"), str(nz), out], env=env, check=True,
                   timeout=300)
    return dict(np.load(out))


@pytest.mark.parametrize("nz", [0, 4])
def test_folded_system_is_bitwise_the_unfolded_build(tmp_path, nz):
    folded, plain = run(tmp_path, nz, False), run(tmp_path, nz, True)
    for key in ("U", "T", "rms"):
        assert np.array_equal(folded[key], plain[key]), key


@pytest.mark.parametrize("nz", [0, 4])
def test_folded_edge_side_assembly_is_bitwise_the_node_serial_one(tmp_path, nz):
    """Round 6: the folded k_asm_es (default) against the folded k_asm_visc (RX_ASMV_ES=0), whole outer iterations."""
    es, serial = run(tmp_path, nz, False), run(tmp_path, nz, False, es="0")
    for key in ("U", "T", "rms"):
        assert np.array_equal(es[key], serial[key]), key
