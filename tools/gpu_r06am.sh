#!/bin/bash
# Round-6 cycle am: C5 same-box A/B, the final build against the r06y-era build (librx_old.so, commit 13d604a), to
# separate the box from the code in C5's SOLVE (15.21 ms in r06y, 16.17 in r06al).
mkdir -p gpurun_out
T=r06am
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
for v in new old new2 old2; do
  L=$PWD/$PKG/librx.so; case $v in old*) L=$PWD/$PKG/librx_old.so;; esac
  RX_LIB=$L timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 8 > gpurun_out/bench_${T}_$v.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; r=d['roofline_kernels']; print('c5 $v', d['ms_per_step'], 'SOLVE', p['SOLVE'], 'SST_SOLVE', p['SST_SOLVE'], 'PRIM', p['PRIMITIVE'], 'ring', r['ILU_APPLY']['avg_launch_us'], 'spmv', r['SPMV']['avg_launch_us'])"
done
