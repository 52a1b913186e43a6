#!/bin/bash
# Round-6 cycle aj: the FGMRES solve in two captured parts with the host's stop check between them (the SST solve
# stops after 2 of its 5 iterations; the empty launches after it are skipped): parity tests, then same-box A/B
# against the previous commit's build (librx_old.so), C4 rank floor and C3 bench.
mkdir -p gpurun_out
T=${T:-r06aj}
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sst.py \
  tests/test_gpu_c4.py tests/test_gpu_partitions.py tests/test_gpu_fold.py tests/test_gpu_linsolve.py \
  tests/test_gpu_p2v.py tests/test_gpu_bc.py > gpurun_out/tests_${T}.log 2>&1 || { tail -30 gpurun_out/tests_${T}.log; exit 1; }
tail -2 gpurun_out/tests_${T}.log
for v in new old new2 old2; do
  L=$PWD/$PKG/librx.so; case $v in old*) L=$PWD/$PKG/librx_old.so;; esac
  RX_LIB=$L timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_$v.log 2>&1 || exit 3
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('c4 $v', d['ms_per_step'], 'SOLVE', round(p['SOLVE'],4), 'SST_SOLVE', round(p['SST_SOLVE'],4), 'PRIM', round(p['PRIMITIVE'],4), d['lin_iters'])"
done
for v in new old new2 old2; do
  L=$PWD/$PKG/librx.so; case $v in old*) L=$PWD/$PKG/librx_old.so;; esac
  RX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$v.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$v', d['ms_per_step'], 'SOLVE', p['SOLVE'], 'SST_SOLVE', p['SST_SOLVE'], 'PRIM', p['PRIMITIVE'])"
done
