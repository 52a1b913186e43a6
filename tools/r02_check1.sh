#!/bin/bash
# Round-2 re-entry check: GPU parity tests, then the C3 bench state at several partition counts.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/gpu_tests.log
for p in 256 1024 2048; do
  timeout -k 10 240 python -u tools/c3_diag.py --parts $p --steps 8 > gpurun_out/diag_c3_$p.log 2>&1; rc=$?; echo "diag c3 $p rc=$rc"; cat gpurun_out/diag_c3_$p.log | grep -v amdgpu
  case $rc in 0|1) ;; *) exit $rc;; esac
done
RX_NO_LDS_APPLY=1 timeout -k 10 240 python -u tools/c3_diag.py --parts 1024 --steps 8 > gpurun_out/diag_c3_1024_nolds.log 2>&1; echo "nolds rc=$?"; grep -v amdgpu gpurun_out/diag_c3_1024_nolds.log
