#!/bin/bash
# Round-6 cycle b: where k_asm_es's time goes (RX_ASMES_PROBE build variants, tools/asm_probe.py, timing only), and the
# cost of rx_div's range guard (librx_noguard.so: RX_FDIV_GUARD=0) in a same-box bench A/B.
mkdir -p gpurun_out
T=r06b
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_fdiv.py "tests/test_gpu_linsolve.py::test_restarted_fgmres_stops_when_a_cycle_starts_converged" -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -n 1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
for v in base p1 p2 p3 p4 p5 base2; do
  lib=$PKG/librx.so; [ "${v#p}" != "$v" ] && lib=$PKG/librx_$v.so
  timeout -k 10 300 env RX_LIB=$lib python tools/asm_probe.py $v >> gpurun_out/asm_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/asm_probe_$T.log
done
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run guard RX_LIB=$PKG/librx.so && run noguard RX_LIB=$PKG/librx_noguard.so && run guardb RX_LIB=$PKG/librx.so && \
run noguardb RX_LIB=$PKG/librx_noguard.so || exit 2
