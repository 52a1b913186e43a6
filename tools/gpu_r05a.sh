#!/bin/bash
# Round-5 cycle a: the linear-solver tests, the whole GPU suite (bench CFL 1, C4 at 2048 partitions, species 5 / 6 / 8,
# the ls* solver goldens), the bench line, the C4 per-rank floor, then the self-halo RCCL test (it hung once: last, with
# RCCL's own log and a short limit). Each GPU step has its own limit; a timeout / crash ends the script. pytest runs
# with -v into files under gpurun_out/ (a line per test start and end).
mkdir -p gpurun_out
T=r05a
ok() { [ $1 -le 1 ]; }  # pytest: 0 pass, 1 failures; anything else (timeout 124 / 137, crash) ends the script
timeout -k 10 420 python -u -m pytest tests/test_gpu_linsolve.py -v --timeout 170 --timeout-method thread > gpurun_out/linsolve_$T.log 2>&1; rc=$?; echo "linsolve rc=$rc"; tail -4 gpurun_out/linsolve_$T.log
ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread --ignore=tests/test_gpu_linsolve.py --ignore=tests/test_gpu_rccl_self.py --ignore=tests/test_gpu_assembly.py > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/gpu_tests_$T.log | head -20; tail -2 gpurun_out/gpu_tests_$T.log
ok $rc || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$T.log 2>&1 && echo "bench ok" && tail -c 1200 gpurun_out/bench_$T.log || exit 1
timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_$T.log 2>&1 && tail -c 800 gpurun_out/c4floor_$T.log || exit 1
NCCL_DEBUG=INFO timeout -k 10 170 python -u -m pytest tests/test_gpu_rccl_self.py -v -s --timeout 150 --timeout-method thread > gpurun_out/rccl_self_$T.log 2>&1; rc=$?; echo "rccl_self rc=$rc"; tail -5 gpurun_out/rccl_self_$T.log
exit 0
