#!/bin/bash
# Round-6 cycle aa: the grouped ILU build prefetching each row's second lower block with its first (RX_GRP_PF2=1,
# in-tree) against loading it after the first block's product (librx_pf0): factor / apply / outer-iteration parity
# tests, the build timed alone (tools/ilu_probe.py), bench lines alternating, the C4 floor of each, C5.
mkdir -p gpurun_out
T=r06aa
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_c4.py tests/test_gpu_bc.py tests/test_gpu_linsolve.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || exit $rc
for v in base:librx pf0:librx_pf0 base2:librx pf0b:librx_pf0; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/ilu_probe.py ${v%%:*} >> gpurun_out/ilu_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ilu_probe_$T.log
done
for r in 1 2; do
  for v in base:librx pf0:librx_pf0; do
    RX_LIB=$PKG/${v#*:}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_${v%%:*}_$r.log 2>&1 || exit 2
  done
done
python3 tools/ab_table.py base1=gpurun_out/bench_${T}_base_1.log pf0_1=gpurun_out/bench_${T}_pf0_1.log base2=gpurun_out/bench_${T}_base_2.log pf0_2=gpurun_out/bench_${T}_pf0_2.log
timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_$T.log 2>&1 && tail -c 400 gpurun_out/c4floor_$T.log
timeout -k 10 300 env RX_LIB=$PKG/librx_pf0.so python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_pf0.log 2>&1 && tail -c 400 gpurun_out/c4floor_${T}_pf0.log
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 6 > gpurun_out/bench_${T}_c5.log 2>&1 && python3 tools/ab_table.py c5=gpurun_out/bench_${T}_c5.log
