#!/bin/bash
# Round-6 cycle k: the device's partition semantics against the reference's own rank (golden rank9), the linear-solver
# and partition tests, then the C3 bench line (RMS partials staged through LDS).
mkdir -p gpurun_out
T=r06k
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_linsolve.py -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -n 1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}.log 2>&1 && python tools/ab_table.py c3=gpurun_out/bench_${T}.log
