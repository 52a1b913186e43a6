#!/bin/bash
# Round-6 cycle z: the full-size (configs[1]) laminar / supersonic outer iteration against the oracle.
mkdir -p gpurun_out
T=r06z
timeout -k 10 600 python -u -m pytest tests/test_gpu_size.py -k laminar -x -v -s --timeout 500 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|species elementwise|Error|assert" gpurun_out/gpu_tests_$T.log | tail -n 12
exit $rc
