#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bc.py tests/test_cpp_driver.py tests/test_gpu_size.py -v -x --timeout 400 --timeout-method thread > gpurun_out/gpu_iter.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/gpu_iter.log | head -60
