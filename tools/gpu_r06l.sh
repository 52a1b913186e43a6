#!/bin/bash
# Round-6 cycle l: the laminar outer iteration against golden lam4.
mkdir -p gpurun_out
T=r06l
timeout -k 10 300 python -u -m pytest tests/test_gpu_bc.py -k laminar -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -n 30 gpurun_out/gpu_tests_$T.log | grep -E "Error|error|assert|passed|failed|max" | head -20
