#!/bin/bash
# Round-6 cycle ae: the ring sweeps' wavefront groups (RX_ILU_RING_G 1 / 2 / 4) re-measured after the late x stores,
# C3 bench lines and the C4 rank floor.
mkdir -p gpurun_out
T=r06ae
for g in 2 1 4 2b; do
  RX_ILU_RING_G=${g%b} timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_g$g.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_g$g.log') if x.startswith('{')][-1]); k=d['roofline_kernels']['ILU_APPLY']; print('g$g', d['ms_per_step'], k['kernel'], k['avg_launch_us'], 'SOLVE', d['phase_ms_per_step']['SOLVE'])"
done
for g in 2 1 4; do
  RX_ILU_RING_G=$g timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_g$g.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4floor_${T}_g$g.log') if x.startswith('{')][-1]); print('c4 g$g', d['ms_per_step'], 'SOLVE', round(d['phase_ms_per_step']['SOLVE'],3), d['in_solve_us_per_launch'])"
done
