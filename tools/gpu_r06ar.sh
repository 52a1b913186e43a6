#!/bin/bash
# Round-6 cycle ar: the C4 rank floor of the final code three times on one box (box-to-box spread of the floor:
# 4.47 ms in the closing cycle r06aq against 4.24 in r06ap's A/B).
mkdir -p gpurun_out
T=r06ar
for v in 1 2 3; do
  timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_$v.log 2>&1 || exit 3
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('c4 $v', d['ms_per_step'], 'phase sum', round(sum(p.values()),3), 'SOLVE', round(p['SOLVE'],4), 'SST_SOLVE', round(p['SST_SOLVE'],4))"
done
