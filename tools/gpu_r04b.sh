#!/bin/bash
# Round-4 cycle: the -m gpu suite without the 8M-point C5 test, then one bench line with the phase split.
mkdir -p gpurun_out
T=${TAG:-r04b}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -x --timeout 900 --timeout-method thread \
  --deselect tests/test_gpu_size.py::test_c5_whole_mesh > gpurun_out/gpu_tests_$T.log 2>&1 \
  || { grep -E "PASS|FAIL|Error|error" gpurun_out/gpu_tests_$T.log | tail -30; tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests_$T.log | tail -3
grep -E "vs oracle|explicit x|dU " gpurun_out/gpu_tests_$T.log | tail -20
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$T.log 2>&1 && python3 -c "
import json
l=[x for x in open('gpurun_out/bench_$T.log') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step']); print(d['roofline']); print(d['roofline_longest_launch']['kernel'])
print({k: v for k, v in d.get('phase_ms_per_step', {}).items()})"
