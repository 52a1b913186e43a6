#!/bin/bash
# The whole 8M-point C5 mesh on one MI355X (tests/test_gpu_size.py::test_c5_whole_mesh), through gpurun from the repo
# root; progress lines go to gpurun_out/c5_full.log as the test runs.
mkdir -p gpurun_out
RX_FULL_C5=1 timeout -k 10 1000 python -u -m pytest tests/test_gpu_size.py -m gpu -k c5_whole -x -v -s --timeout 980 \
  --timeout-method thread > gpurun_out/c5_full.log 2>&1; rc=$?; tail -25 gpurun_out/c5_full.log; exit $rc
