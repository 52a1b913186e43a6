#!/bin/bash
# Round-6 cycle u: the FGMRES in-place walks (MGS projections, normalisation) loading round r + 1 before storing round r
# (RX_FG_PIPE=1, in-tree) against the plain walks (librx_fp0): the Krylov / outer-iteration parity tests, then bench lines.
mkdir -p gpurun_out
T=r06u
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_linsolve.py tests/test_gpu_bc.py tests/test_gpu_c4.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base:librx fp0:librx_fp0; do
    RX_LIB=$PKG/${v#*:}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_${v%%:*}_$r.log 2>&1 || exit 2
  done
done
python3 tools/ab_table.py base1=gpurun_out/bench_${T}_base_1.log fp0_1=gpurun_out/bench_${T}_fp0_1.log base2=gpurun_out/bench_${T}_base_2.log fp0_2=gpurun_out/bench_${T}_fp0_2.log
for f in gpurun_out/bench_${T}_*.log; do python3 -c "
import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); k=d['roofline_kernels']; print('$f', 'apply', k['ILU_APPLY']['avg_launch_us'], 'spmv', k['SPMV']['avg_launch_us'], 'solve', d['phase_ms_per_step']['SOLVE'], 'sst_solve', d['phase_ms_per_step']['SST_SOLVE'])"; done
timeout -k 10 300 env RX_RING_FIRST=1 python tools/c4_rank_floor.py > gpurun_out/c4floor_$T.log 2>&1 && tail -c 250 gpurun_out/c4floor_$T.log
