"""A case run from its files (next-4 end to end, on the device): the cfg read by rx.case_from_cfg, the mesh by the
native SU2 reader + dual-grid preprocessing (rx_mesh_read_su2), the mechanism by the native library readers
(rx_mech_read), then one whole reference outer iteration (rx.Iterate) from the reference's own state, against the
reference's own iteration of the same cfg. The input files are the reference's shipped ones
(tests/golden/case_files.npz) with cfgs written from oracle/make_golden.py's templates:

  itx9  the shipped jet cfg (my_combustion_second_chem_PaSR.cfg's keys: EULER_EXPLICIT, CFL 0.1, LU_SGS SST)
  ig9   stage 1 of the reference's procedure (first chemistry, IGNITION = YES) from its non-reacting start
  fpit  the turbulent flat plate (heat-flux and Euler walls, TOTAL_CONDITIONS inlet, 2ND_ORDER, implicit LU_SGS)

Bar: U, V, (k, omega), mu_t, both RMS vectors at 1e-10 (test_gpu_bc.check_iteration). Requires an MI355X."""
import os

import numpy as np
import pytest

from tests.casefiles import unpack
from tests.rxpkg import rx
from tests.test_gpu_bc import check_iteration, golden, load_iteration_state

pytestmark = pytest.mark.gpu


def workdir(case, tmp_path):
    from oracle import make_golden as MG
    if case == "fpit":
        return MG.fp_workdir(case_dir=unpack(tmp_path / "files", "plate"), root=str(tmp_path))
    files = unpack(tmp_path / "files", "jet")
    if case == "ig9":
        return MG.ig9_workdir(case_dir=files, root=str(tmp_path))
    return MG.make_workdir(case, MG.full_jet_writer, cfl=0.1, order="1ST_ORDER", prec="LU_SGS",
                           time_flow="EULER_EXPLICIT", case_dir=files, root=str(tmp_path))


@pytest.mark.parametrize("case", ["itx9", "ig9", "fpit"])
def test_case_from_files_runs_the_reference_iteration(case, tmp_path):
    c = rx.case_from_cfg(os.path.join(workdir(case, tmp_path), "case.cfg"))
    mesh = c["mesh"].mesh()
    s = rx.ReactiveNSSolver(mesh, rx.Mechanism(c["mech"]), rx.default_cfg(**c["flow_cfg"]))
    s.set_bc(c["bc"])
    t = rx.TurbSSTSolver(mesh, s, rx.default_cfg(**c["sst_cfg"]))
    g = golden(case)
    load_iteration_state(g, s, t, 0)
    rms, rms_t, _ = rx.Iterate(s, t, ext_iter=0, rk_alpha=c["rk_alpha"])
    s.sync()
    check_iteration(g, s, t, 1, rms, rms_t, 1e-10)
    s.close()
    c["mesh"].close()
