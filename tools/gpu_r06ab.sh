#!/bin/bash
# Round-6 cycle ab: the grouped ILU build with two lane groups per row (PAIR). Parity tests with the default choice and
# with PAIR forced on (RX_GRP_PAIR=1) / off, then the C4 rank floor and the C3 build timed alone with PAIR on / off.
mkdir -p gpurun_out
T=r06ac
timeout -k 10 500 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_c4.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_${T}_def.log 2>&1; rc=$?
echo "tests default rc=$rc"; tail -n 2 gpurun_out/gpu_tests_${T}_def.log; [ $rc -eq 0 ] || exit $rc
RX_GRP_PAIR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_c4.py tests/test_gpu_bc.py tests/test_gpu_size.py -k "not whole_mesh" -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_${T}_on.log 2>&1; rc=$?
echo "tests PAIR on rc=$rc"; tail -n 2 gpurun_out/gpu_tests_${T}_on.log; [ $rc -eq 0 ] || exit $rc
for v in on:1 off:0 on2:1 off2:0; do
  RX_GRP_PAIR=${v#*:} timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_${v%%:*}.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_${v%%:*}.log') if x.startswith('{')][-1]); print('c4 ${v%%:*}', d['ms_per_step'], 'ILU_BUILD', round(d['phase_ms_per_step']['ILU_BUILD'],3), 'SOLVE', round(d['phase_ms_per_step']['SOLVE'],3))"
done
for v in on:1 off:0; do
  RX_GRP_PAIR=${v#*:} timeout -k 10 300 python tools/ilu_probe.py c3_${v%%:*} >> gpurun_out/ilu_probe_$T.log 2>&1 || exit 3
  tail -n 1 gpurun_out/ilu_probe_$T.log
done
