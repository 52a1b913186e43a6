"""Probe (librx_probe.so, built by: bash tools/build_variant.sh probe -DRX_PROBE): where a level of the wide ILU(0)
forward sweep spends its time at C3. Builds the bench's C3 system (one implicit iteration, so JAC / ILU / RHS are the
bench's), then times forward-sweep variants that drop the x dependence (1), the level barrier (2) or the factor
loads (4), against the production forward (8) and backward (9) sweeps. Prints ms per launch."""
import ctypes as C
import os
import sys

sys.path.insert(0, ".")
os.environ.setdefault("RX_LIB", os.path.abspath(
    "development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd/librx_probe.so"))
from tests.rxpkg import rx, synth  # noqa: E402

mesh, st0, mech, kw = synth.jet_field_case(2000, 500, n_species=7, n_part=256)
s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech), rx.default_cfg(implicit=1, lin_prec=1, **kw))
s.set_bc(synth.jet_bc(mesh, 7))
t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
synth.device_preprocess(s, t, mesh, st0)
rx.Iterate(s, t, ext_iter=0)
s.sync()
names = {0: "fwd as production (probe kernel)", 1: "no x dependence", 2: "no level barrier", 3: "no x dep + no barrier",
         4: "no factor loads", 5: "no factor loads + no x dep", 6: "no factor loads + no barrier", 7: "x from b, no F, no barrier",
         8: "production k_ilu_fwd_wide", 9: "production k_ilu_bwd_wide", 10: "fwd, compact lower blocks",
         11: "bwd, compact upper blocks + inv(D)"}
import numpy as np  # noqa: E402


def run(mode, reps):
    ms = C.c_double()
    rc = rx.lib().rx_debug_sweep_probe(s.h, C.c_int(mode), C.c_int(reps), C.byref(ms))
    assert rc == 0, rc
    return ms.value


# the compact layouts against the production sweeps, bitwise (forward: x from b; backward: from the same x)
run(8, 1)
xf = s.download("SOL").copy()
run(10, 1)
print("fwd compact bitwise:", np.array_equal(s.download("SOL"), xf), flush=True)
run(9, 1)
xb = s.download("SOL").copy()
s.upload("SOL", xf)
run(11, 1)
print("bwd compact bitwise:", np.array_equal(s.download("SOL"), xb), flush=True)
modes = [int(m) for m in sys.argv[1:]] or [8, 9, 10, 11, 8, 9, 10, 11, 0, 1, 2, 3, 4, 5, 6, 7]
for mode in modes:
    print(f"mode {mode}: {run(mode, 20) * 1e3:8.1f} us  {names[mode]}", flush=True)
