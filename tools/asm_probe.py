"""Time the node-centric assembly (phase ASSEMBLE: k_asm_es or k_asm_visc, with the fused AUSM pass) alone on the C3
state, for the build variant named by RX_LIB (tools/build_variant.sh, e.g. the RX_ASMES_PROBE knobs of
csrc/rx_kernels.hip). Prints one line: tag, ms per call (HIP events on the launch stream)."""
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


for _ in range(2):
    once()
s.profile(True)
for _ in range(10):
    once()
s.sync()
out = {k: s.profile_read(k) for k in ("ASSEMBLE", "VISC")}
print(tag, " ".join(f"{k} {ms / max(n, 1):.3f} ms/call (n={n})" for k, (ms, n) in out.items()), flush=True)
s.close()
