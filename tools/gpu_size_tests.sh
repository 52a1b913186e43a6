#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_size.py -v -x --timeout 400 --timeout-method thread > gpurun_out/gpu_size.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/gpu_size.log | head -30
