#!/bin/bash
# Round-6 cycle h: the C4 per-rank floor (tools/c4_rank_floor.py) with the LDS-resident ILU apply (default at 490-row
# partitions) against the ring sweeps (RX_RING_FIRST=1) with 2, 4 and 8 wavefront groups; then the partition parity
# tests with the ring first and 8 groups.
mkdir -p gpurun_out
T=r06h
for v in lds: g2:"RX_RING_FIRST=1 RX_ILU_RING_G=2" g4:"RX_RING_FIRST=1 RX_ILU_RING_G=4" g8:"RX_RING_FIRST=1 RX_ILU_RING_G=8"; do
  timeout -k 10 300 env ${v#*:} python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_${v%%:*}.log 2>&1 || exit 1
  python3 -c "
import json,sys; l=[x for x in open('gpurun_out/c4floor_${T}_${v%%:*}.log') if x.startswith('{')][-1]; d=json.loads(l)
p=d['phase_ms_per_step']; print('${v%%:*}', d['ms_per_step'], {k: round(v,3) for k,v in p.items() if v > 0.1})"
done
timeout -k 10 600 env RX_RING_FIRST=1 RX_ILU_RING_G=8 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_c4.py -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -n 1 gpurun_out/gpu_tests_$T.log
