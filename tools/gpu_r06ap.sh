#!/bin/bash
# Round-6 cycle ap: the 2x2 (SST) ILU sweeps' pass loop unrolled by the slot ring's length with 4 passes of blocks in
# flight (librx_u8.so: RX_SST_UNROLL=1, RX_SST_D2=4; the rings rotate by renaming, 26 instead of 77 register moves
# per pass): SST parity tests on the variant, then C3 bench and C4 rank floor against the default build.
mkdir -p gpurun_out
T=r06ap
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
U=$PWD/$PKG/librx_u8.so; N=$PWD/$PKG/librx.so
RX_LIB=$U timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sst.py \
  tests/test_gpu_c4.py tests/test_gpu_linsolve.py > gpurun_out/tests_${T}.log 2>&1 || { tail -30 gpurun_out/tests_${T}.log; exit 1; }
tail -1 gpurun_out/tests_${T}.log
for v in base u8 base2 u8b; do
  L=$N; case $v in u8*) L=$U;; esac
  RX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$v.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$v', d['ms_per_step'], 'SST_SOLVE', p['SST_SOLVE'], 'SST_SYSTEM', p['SST_SYSTEM'])"
done
for v in base u8 base2 u8b; do
  L=$N; case $v in u8*) L=$U;; esac
  RX_LIB=$L timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_$v.log 2>&1 || exit 3
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('c4 $v', d['ms_per_step'], 'SST_SOLVE', round(p['SST_SOLVE'],4), d['lin_iters'])"
done
