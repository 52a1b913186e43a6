"""FGMRES on a non-finite system: the matrix-free initial residual (k_fg_residual0, the default: LinSysSol is zeroed
before the solve, solver_direct_reactive.cpp:2373, so A x = +0 for a finite A) against the A x product path
(RX_FG_X_PRODUCT=1, read once per process, hence one child process per path). A NaN in one point's dP/dU puts NaN
in the convective Jacobian blocks of its edges while the residual stays finite. The reference's A * 0 then makes w0
NaN at the first residual; the matrix-free path meets the NaN one Krylov step later, in the preconditioned vector.
Both must report the same outcome: rx_implicit_euler returns RX_ERR_DIVERGED (the breakdown test of ModGramSchmidt,
linear_solvers_structure.cpp:97-100, on a NaN norm) and no finite update is claimed."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, ".")
from tests.rxpkg import rx, synth
mesh, st, mech, kw = synth.jet_case(24, 10, n_species=7, n_part=4)
s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), rx.default_cfg(implicit=1, lin_prec=int(sys.argv[1]), **kw))
s.set_state(st)
s.SetPrimitive_Gradient_LS()
s.SetTime_Step()
# dP/dU enters only the convective Jacobian (the AUSM residual and the time step read V): A gets NaN blocks, b stays
# finite
dpdu = s.download("DPDU")
dpdu[17 * s.nVar + 2] = np.nan
s.upload("DPDU", dpdu)
s.Preprocessing_zero()
s.Upwind_Residual()
s.Viscous_Residual()
s.Source_Residual()
out = {"rhs_finite": bool(np.isfinite(s.download("RES")).all())}
out["status"] = 0
try:
    rms, it = s.ImplicitEuler_Iteration()
    out["iters"] = it
    out["finite"] = bool(np.isfinite(s.download("U")).all())
except rx.RxError as e:
    out["status"] = e.status
s.close()
print("RESULT " + json.dumps(out))
"""


def run_child(product, prec):
    env = dict(os.environ)
    env.pop("RX_FG_X_PRODUCT", None)
    if product:
        env["RX_FG_X_PRODUCT"] = "1"
    p = subprocess.run([sys.executable, "-c", CHILD, str(prec)], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


@pytest.mark.parametrize("prec", [1, 0])  # ILU0, LU_SGS
def test_nan_jacobian_same_status_on_both_residual_paths(prec):
    import tests.rxpkg as rxpkg
    a = run_child(False, prec)
    b = run_child(True, prec)
    assert a == b, (a, b)
    assert a["rhs_finite"], a
    assert a["status"] == rxpkg.rx.RX_ERR_DIVERGED, a
