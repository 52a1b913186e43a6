#!/bin/bash
# Confirmation cycle without the profiler passes: the whole -m gpu suite, smoke, the c3 and c5 bench lines.
mkdir -p gpurun_out
T=${TAG:-r04c}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/gpu_tests_$T.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_$T.log 2>&1 && echo "bench ok" || exit 1
timeout -k 10 400 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${T}_c5.log 2>&1 && echo "c5 ok"
