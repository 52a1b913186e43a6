#!/bin/bash
# Round-5 cycle a: the new assembly / self-halo RCCL / linear-solver tests, the whole GPU suite (bench CFL 1, C4 at 2048
# partitions), the bench line, the C4 per-rank floor. Each GPU step has its own limit; a failing step ends the script.
mkdir -p gpurun_out
T=r05a
timeout -k 10 600 python -u -m pytest tests/test_gpu_assembly.py tests/test_gpu_rccl_self.py tests/test_gpu_linsolve.py -v --timeout 300 --timeout-method thread > gpurun_out/new_tests_$T.log 2>&1; rc=$?; tail -15 gpurun_out/new_tests_$T.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread --ignore=tests/test_gpu_linsolve.py > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests_$T.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.log 2>&1 && echo "bench ok" && tail -c 1500 gpurun_out/bench_$T.log || exit 1
timeout -k 10 600 python tools/c4_rank_floor.py > gpurun_out/c4floor_$T.log 2>&1 && tail -c 1500 gpurun_out/c4floor_$T.log
