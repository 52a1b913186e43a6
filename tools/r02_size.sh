#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_size.py tests/test_gpu_bc.py -k "size or graph" -v -x --timeout 400 --timeout-method thread > gpurun_out/gpu_size.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/gpu_size.log | head -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_solve.log 2>&1; echo "bench rc=$?"; python -c "
import json;d=json.loads(open('gpurun_out/bench_solve.log').read().strip().splitlines()[-1]);print(d['value']); [print(k, v) for k,v in d['roofline_kernels'].items()]"
