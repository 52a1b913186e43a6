"""Time the ILU(0) factorisation (phase ILU_BUILD: k_ilu_build_grp on the jet meshes) alone on the C3 system, for the
build variant named by RX_LIB (tools/build_variant_fast.sh, e.g. the RX_GRP_PROBE knobs of csrc/rx_sweeps.hip).
Prints one line: tag, ms per call (HIP events on the launch stream)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tests.rxpkg import rx, synth  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "base"
nx, ny, nz = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (2000, 500, 0)
mesh, st, mech, kw = bench.build_workload(nx, ny, 7, 256, nz)
s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), rx.default_cfg(implicit=1, rans=1, lin_prec=1, lin_iter=5, **kw))
t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
st = synth.device_preprocess(s, t, mesh, st)
bench.set_states(s, t, mesh, st)


def once():
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    s.sync()
    s.download("RES")  # assembles the system (rx_launch_assemble)


once()
for _ in range(2):
    s.ilu0_build()
s.profile(True)
for _ in range(10):
    s.ilu0_build()
s.sync()
ms, n = s.profile_read("ILU_BUILD")
print(tag, f"ILU_BUILD {ms / max(n, 1):.3f} ms/call (n={n})", flush=True)
s.close()
