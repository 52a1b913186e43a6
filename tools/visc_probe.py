"""Time the viscous edge sweep (k_visc_edge, phase VISC) and the Jacobian kernel (VISC_JAC) alone on the C3 state,
for the build variant named by RX_LIB (tools/build_variant.sh). Prints one line: tag, ms per call of each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tests.rxpkg import rx, synth  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "base"
nx, ny = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (2000, 500)
mesh, st, mech, kw = bench.build_workload(nx, ny, 7, 256)
s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), rx.default_cfg(implicit=1, rans=1, lin_prec=1, lin_iter=5, **kw))
t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
st = synth.device_preprocess(s, t, mesh, st)
bench.set_states(s, t, mesh, st)
for _ in range(2):
    s.Preprocessing_zero()
    s.Viscous_Residual()
s.sync()
s.profile(True)
for _ in range(10):
    s.Preprocessing_zero()
    s.Viscous_Residual()
s.sync()
out = {k: s.profile_read(k) for k in ("VISC", "VISC_JAC")}
print(tag, " ".join(f"{k} {ms / max(n, 1):.3f} ms/call (n={n})" for k, (ms, n) in out.items()), flush=True)
s.close()
