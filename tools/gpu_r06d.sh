#!/bin/bash
# Round-6 cycle d: k_asm_es with the node records staged through LDS and the summary loads in flight during the AUSM
# pass (RX_ASMES_STAGE=1, default) against staging the summary first (librx_st0.so): assembly parity tests, then
# tools/asm_probe.py and a same-box bench A/B.
mkdir -p gpurun_out
T=r06d
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_assembly.py tests/test_gpu_fold.py tests/test_gpu_muscl.py -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -n 1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
for v in st1:librx st0:librx_st0 st1b:librx st0b:librx_st0; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/asm_probe.py ${v%%:*} >> gpurun_out/asm_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/asm_probe_$T.log
done
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run st1 RX_LIB=$PKG/librx.so && run st0 RX_LIB=$PKG/librx_st0.so && run c5st1 RX_LIB=$PKG/librx.so "--workload c5" || exit 2
