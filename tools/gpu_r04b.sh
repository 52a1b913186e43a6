#!/bin/bash
# Round-4 cycle: the -m gpu suite without the 8M-point C5 test, then one bench line with the phase split.
# gpurun_out/gpu_dirty stays behind unless every GPU step ended by itself (pytest exit 0 or 1: pass / assertion
# failures); later scripts of the same call (tools/gpu_r04d.sh) refuse to start while it exists.
mkdir -p gpurun_out
touch gpurun_out/gpu_dirty
T=${TAG:-r04b}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=8 --timeout 900 --timeout-method thread \
  --deselect tests/test_gpu_size.py::test_c5_whole_mesh > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_$T.log | tail -3
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests_$T.log | grep -v PASSED | tail -30
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; tail -40 gpurun_out/gpu_tests_$T.log; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$T.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/bench_$T.log; exit 2; }
python3 -c "
import json
l=[x for x in open('gpurun_out/bench_$T.log') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step']); print(d['roofline']); print(d['roofline_longest_launch']['kernel'])
print({k: v for k, v in d.get('phase_ms_per_step', {}).items()})"
rm -f gpurun_out/gpu_dirty
exit $rc
