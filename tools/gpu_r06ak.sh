#!/bin/bash
# Round-6 cycle ak: the split FGMRES solve with the host waits polled (rx_la_host_wait) and the RMS / state
# read-backs under one wait: parity tests, then C4 rank floor and C3 bench: new (spin on, tail graph), spin off,
# tail eager, the previous commit's build (librx_old.so).
mkdir -p gpurun_out
T=${T:-r06ak}
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sst.py \
  tests/test_gpu_c4.py tests/test_gpu_fold.py tests/test_gpu_linsolve.py tests/test_gpu_shard_iterate.py \
  tests/test_gpu_rccl_self.py > gpurun_out/tests_${T}.log 2>&1 || { tail -30 gpurun_out/tests_${T}.log; exit 1; }
tail -2 gpurun_out/tests_${T}.log
run() {  # tag, env..., tool
  local v=$1; shift
  env "$@" timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_$v.log 2>&1 || exit 3
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('c4 $v', d['ms_per_step'], 'SOLVE', round(p['SOLVE'],4), 'SST_SOLVE', round(p['SST_SOLVE'],4), d['lin_iters'])"
}
N=$PWD/$PKG/librx.so; O=$PWD/$PKG/librx_old.so
run new RX_LIB=$N; run nospin RX_LIB=$N RX_SYNC_SPIN=0; run eager RX_LIB=$N RX_FG_TAIL_EAGER=1; run old RX_LIB=$O
run new2 RX_LIB=$N; run nospin2 RX_LIB=$N RX_SYNC_SPIN=0; run eager2 RX_LIB=$N RX_FG_TAIL_EAGER=1; run old2 RX_LIB=$O
for v in new old new2 old2; do
  L=$N; case $v in old*) L=$O;; esac
  RX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$v.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$v', d['ms_per_step'], 'SOLVE', p['SOLVE'], 'SST_SOLVE', p['SST_SOLVE'], 'PRIM', p['PRIMITIVE'])"
done
