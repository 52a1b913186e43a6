#!/bin/bash
# Round-5 cycle f: shared-divisor divisions in the viscous / AUSM kernels (rx_fdiv.h) and the two-group LDS-ring ILU
# apply with predicated row loads: the division check, the whole GPU suite, then same-box bench A/B against the
# round's previous build (librx_r5d.so), the build without rx_fdiv (librx_nofdiv.so) and the one-group plan.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05f
timeout -k 10 120 python -u -m pytest tests/test_gpu_fdiv.py -v --timeout 100 --timeout-method thread > gpurun_out/fdiv_$T.log 2>&1; rc=$?; echo "fdiv rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/fdiv_$T.log | head -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -2 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run old RX_LIB=$PKG/librx_r5d.so && run new RX_LIB=$PKG/librx.so && run nofdiv RX_LIB=$PKG/librx_nofdiv.so && \
run g1 "RX_LIB=$PKG/librx.so RX_ILU_RING_G=1" && run oldb RX_LIB=$PKG/librx_r5d.so && run newb RX_LIB=$PKG/librx.so || exit 2
run5() { timeout -k 10 400 env $2 python bench.py --workload c5 --no-cpu-baseline --steps 8 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run5 c5old RX_LIB=$PKG/librx_r5d.so && run5 c5new RX_LIB=$PKG/librx.so || exit 3
