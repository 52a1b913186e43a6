#!/bin/bash
# Round-4 check of the sharded path: shard / C4 / ILU-state tests, then one bench line.
mkdir -p gpurun_out
T=${TAG:-r04a}
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard_iterate.py tests/test_gpu_c4.py tests/test_gpu_shard.py \
  "tests/test_gpu_parity.py::test_ilu_field_needs_a_factor" -v -s -x --timeout 900 --timeout-method thread \
  > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$T.log; exit 1; }
grep -E "PASS|FAIL|vs oracle|explicit|passed|failed" gpurun_out/gpu_tests_$T.log | tail -40
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$T.log 2>&1 && python3 -c "
import json
l=[x for x in open('gpurun_out/bench_$T.log') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step']); print(d['roofline']); print(d['roofline_longest_launch']['kernel'])
print({k: v for k, v in d.get('phase_ms_per_step', {}).items()})"
