#!/bin/bash
# Round-6 cycle p: the SST loops reading the node's own record once (k_sst_upwind first order, k_sst_visc): the SST
# and outer-iteration parity tests, then bench lines alternating the new library and HEAD's SST kernels (librx_sst0).
mkdir -p gpurun_out
T=r06p
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_sst.py tests/test_gpu_bc.py tests/test_gpu_fold.py tests/test_gpu_size.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base:librx sst0:librx_sst0; do
    RX_LIB=$PKG/${v#*:}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_${v%%:*}_$r.log 2>&1 || exit 2
  done
done
python3 tools/ab_table.py base1=gpurun_out/bench_${T}_base_1.log sst0_1=gpurun_out/bench_${T}_sst0_1.log base2=gpurun_out/bench_${T}_base_2.log sst0_2=gpurun_out/bench_${T}_sst0_2.log
for f in gpurun_out/bench_${T}_*.log; do python3 -c "
import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$f', p['SST_UPW'], p['SST_VISC'])"; done
