#!/bin/bash
# Round-6 cycle x: the node-gather loops (SST upwind / viscous, LSQ gradient) with their workgroups in XCD order
# (RX_SST_XCD=1 / RX_GRAD_XCD=1, in-tree) against the hardware order (librx_xc0): parity tests, bench lines alternating,
# then a FETCH_SIZE pass of each.
mkdir -p gpurun_out
T=r06x
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_sst.py tests/test_gpu_bc.py tests/test_gpu_parity.py tests/test_gpu_shard_iterate.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base:librx xc0:librx_xc0; do
    RX_LIB=$PKG/${v#*:}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_${v%%:*}_$r.log 2>&1 || exit 2
  done
done
python3 tools/ab_table.py base1=gpurun_out/bench_${T}_base_1.log xc0_1=gpurun_out/bench_${T}_xc0_1.log base2=gpurun_out/bench_${T}_base_2.log xc0_2=gpurun_out/bench_${T}_xc0_2.log
for f in gpurun_out/bench_${T}_*.log; do python3 -c "
import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$f', 'SST_UPW', p['SST_UPW'], 'SST_VISC', p['SST_VISC'], 'GRAD', p['GRAD'], 'SST_GRAD', p['SST_GRAD'])"; done
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_${T}_base -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fetch_${T}_base.log 2>&1 && echo "pmc base ok" &&
RX_LIB=$PKG/librx_xc0.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_${T}_xc0 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fetch_${T}_xc0.log 2>&1 && echo "pmc xc0 ok"
