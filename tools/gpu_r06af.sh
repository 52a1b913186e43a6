#!/bin/bash
# Round-6 cycle af: the spline interval searched once per temperature (DevMech::xshared) and the secant's carried
# h(Told): parity tests, then same-box A/B against the previous build (librx_old.so) at C3 and the C4 rank floor.
mkdir -p gpurun_out
T=${T:-r06af}
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_p2v.py \
  tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_gpu_sst.py tests/test_gpu_bc.py > gpurun_out/tests_${T}.log 2>&1 || { tail -30 gpurun_out/tests_${T}.log; exit 1; }
tail -2 gpurun_out/tests_${T}.log
for v in new old new2 old2; do
  L=""; case $v in old*) L=$PWD/$PKG/librx_old.so;; esac
  RX_LIB=${L:-$PWD/$PKG/librx.so} timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$v.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$v', d['ms_per_step'], 'PRIM', p['PRIMITIVE'], 'VISC', p['VISC'], 'SOURCE', p['SOURCE'], 'ASM', p['ASSEMBLE'])"
done
for v in new old; do
  L=""; case $v in old*) L=$PWD/$PKG/librx_old.so;; esac
  RX_LIB=${L:-$PWD/$PKG/librx.so} timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_$v.log 2>&1 || exit 3
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('c4 $v', d['ms_per_step'], 'PRIM', round(p['PRIMITIVE'],4), 'VISC', round(p['VISC'],4), 'SOURCE', round(p['SOURCE'],4))"
done
