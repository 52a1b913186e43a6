#!/bin/bash
# Round-6 cycle ai: timing probe — the FGMRES second-projection launches (k_fg_reo, no-ops unless the
# re-orthogonalisation test fires) left out (librx_noreo.so, RX_FG_NOREO_PROBE), C4 rank floor and C3 bench.
mkdir -p gpurun_out
T=r06ai
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
for v in base noreo base2 noreo2; do
  L=$PWD/$PKG/librx.so; case $v in noreo*) L=$PWD/$PKG/librx_noreo.so;; esac
  RX_LIB=$L timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_$v.log 2>&1 || exit 3
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('c4 $v', d['ms_per_step'], 'SOLVE', round(p['SOLVE'],4), 'SST_SOLVE', round(p['SST_SOLVE'],4), d['lin_iters'])"
done
for v in base noreo; do
  L=$PWD/$PKG/librx.so; case $v in noreo*) L=$PWD/$PKG/librx_noreo.so;; esac
  RX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$v.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$v', d['ms_per_step'], 'SOLVE', p['SOLVE'], 'SST_SOLVE', p['SST_SOLVE'])"
done
