#!/bin/bash
# A/B bench on one box: the default path, then the same with the environment in $B (e.g. RX_NO_FUSED_ASM=1).
mkdir -p gpurun_out
T=${TAG:-ab}
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {k: p[k] for k in sorted(p) if p[k] > 0.4})"; }
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_${T}_a.log 2>&1 && show gpurun_out/bench_${T}_a.log A &&
timeout -k 10 300 env $B python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_${T}_b.log 2>&1 && show gpurun_out/bench_${T}_b.log "B($B)" &&
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_${T}_c.log 2>&1 && show gpurun_out/bench_${T}_c.log A2
