#!/bin/bash
# Round-6 cycle m: supersonic inlet / outlet (golden sup4), laminar, the C++ driver, then the whole GPU suite.
mkdir -p gpurun_out
T=r06m
timeout -k 10 400 python -u -m pytest tests/test_gpu_bc.py tests/test_cpp_driver.py -k "laminar or supersonic or cpp_driver_reference" -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_${T}a.log 2>&1; rc=$?
echo "targeted rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/gpu_tests_${T}a.log | tail -n 20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_${T}b.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -n 15 gpurun_out/gpu_tests_${T}b.log
exit $rc
