#!/bin/bash
# Round-6 cycle t: the staged SpMV with the next step's x gather issued during this step (RX_SPMV_XPRE=1, in-tree)
# against the gather issued in its own step (librx_xp0): the Krylov and triangular parity tests, then bench lines.
mkdir -p gpurun_out
T=r06t
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_c4.py tests/test_gpu_linsolve.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base:librx xp0:librx_xp0; do
    RX_LIB=$PKG/${v#*:}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_${v%%:*}_$r.log 2>&1 || exit 2
  done
done
python3 tools/ab_table.py base1=gpurun_out/bench_${T}_base_1.log xp0_1=gpurun_out/bench_${T}_xp0_1.log base2=gpurun_out/bench_${T}_base_2.log xp0_2=gpurun_out/bench_${T}_xp0_2.log
for f in gpurun_out/bench_${T}_*.log; do python3 -c "
import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); k=d['roofline_kernels']; print('$f', 'apply', k['ILU_APPLY']['avg_launch_us'], 'spmv', k['SPMV']['avg_launch_us'])"; done
timeout -k 10 300 env RX_RING_FIRST=1 python tools/c4_rank_floor.py > gpurun_out/c4floor_$T.log 2>&1 && tail -c 250 gpurun_out/c4floor_$T.log
