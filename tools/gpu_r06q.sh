#!/bin/bash
# Round-6 cycle q: the grouped ILU build's inverse solved from DPP row broadcasts (RX_GRP_SOLVE_DPP=1, in-tree) against
# the LDS-slot solve (librx_lds): the factor / apply parity tests, the build timed alone (tools/ilu_probe.py), then
# bench lines alternating.
mkdir -p gpurun_out
T=r06q
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_c4.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || exit $rc
for v in base:librx lds:librx_lds base2:librx lds2:librx_lds; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/ilu_probe.py ${v%%:*} >> gpurun_out/ilu_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ilu_probe_$T.log
done
for r in 1 2; do
  for v in base:librx lds:librx_lds; do
    RX_LIB=$PKG/${v#*:}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_${v%%:*}_$r.log 2>&1 || exit 2
  done
done
python3 tools/ab_table.py base1=gpurun_out/bench_${T}_base_1.log lds1=gpurun_out/bench_${T}_lds_1.log base2=gpurun_out/bench_${T}_base_2.log lds2=gpurun_out/bench_${T}_lds_2.log
