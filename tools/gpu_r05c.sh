#!/bin/bash
# Round-5 cycle c: the reworked solver-step test (the device's own system through the oracle), then same-box A/B of
# the fused assembly's off-diagonal handling: librx.so (single write, RX_ASMV_PARK=0) vs librx_park.so (round 4's
# parked 0 -+ Jc, RX_ASMV_PARK=1), C3 twice each and C5 once each.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05c
timeout -k 10 300 python -u -m pytest "tests/test_gpu_linsolve.py::test_implicit_step_with_solver_vs_oracle" -v --timeout 170 --timeout-method thread > gpurun_out/fix_tests_$T.log 2>&1; rc=$?; echo "fix tests rc=$rc"; grep -E "PASSED|FAILED|^E " gpurun_out/fix_tests_$T.log | tail -8
[ $rc -gt 1 ] && exit $rc
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {k: p[k] for k in sorted(p) if p[k] > 0.3})"; }
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && show gpurun_out/bench_${T}_$1.log "$1"; }
run5() { timeout -k 10 400 env $2 python bench.py --workload c5 --no-cpu-baseline --steps 8 > gpurun_out/bench_${T}_$1.log 2>&1 && show gpurun_out/bench_${T}_$1.log "$1"; }
run new RX_LIB=$PKG/librx.so && run park RX_LIB=$PKG/librx_park.so && run newb RX_LIB=$PKG/librx.so && \
run parkb RX_LIB=$PKG/librx_park.so && run5 c5new RX_LIB=$PKG/librx.so && run5 c5park RX_LIB=$PKG/librx_park.so || exit 2
