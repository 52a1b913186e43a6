#!/bin/bash
# Round-6 cycle i: the whole GPU suite on the round's kernels (edge-side assembly, ring sweeps first), then the C4
# per-rank floor with 2 and 4 ring groups (in-solve kernel times included).
mkdir -p gpurun_out
T=r06i
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -n 1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
for v in g2: g4:"RX_ILU_RING_G=4"; do
  timeout -k 10 300 env ${v#*:} python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}_${v%%:*}.log 2>&1 || exit 1
  python3 -c "
import json,sys; l=[x for x in open('gpurun_out/c4floor_${T}_${v%%:*}.log') if x.startswith('{')][-1]; d=json.loads(l)
p=d['phase_ms_per_step']; print('${v%%:*}', d['ms_per_step'], d['in_solve_us_per_launch'], {k: round(v,3) for k,v in p.items() if v > 0.05})"
done
