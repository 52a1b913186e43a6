#!/bin/bash
# Quick GPU check through gpurun: the -m gpu suite and one bench line (no CPU baseline, no profiles).
mkdir -p gpurun_out
T=${TAG:-quick}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$T.log 2>&1 && echo "bench ok" && python3 -c "
import json,sys
l=[x for x in open('gpurun_out/bench_$T.log') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step']); print({k: v for k, v in d.get('phase_ms_per_step', {}).items()})"
