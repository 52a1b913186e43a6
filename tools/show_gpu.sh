#!/bin/bash
# Summarise the files one tools/gpu_check.sh run merged back into gpurun_out/.
cd "$(dirname "$0")/.."
grep -E "passed|failed|Error" gpurun_out/gpu_tests.log | tail -5
grep -v amdgpu.ids gpurun_out/trace.log 2>/dev/null
python -c "
import json;d=json.loads(open('gpurun_out/bench.log').read().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['phase_ms_per_step'])"
python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv x | sed -n 5,${1:-16}p
