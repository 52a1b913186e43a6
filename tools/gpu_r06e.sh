#!/bin/bash
# Round-6 cycle e: k_asm_es with per-entry side records ({edge | side, n0, n1, block}: one 16-B load instead of the
# adjacency -> edge -> node chain), the workgroup plan carrying its first adjacency entry, and phase B's loads issued
# before the barrier: parity tests, tools/asm_probe.py, bench C3 and C5.
mkdir -p gpurun_out
T=r06e
timeout -k 10 600 python -u -m pytest tests/test_gpu_assembly.py tests/test_gpu_fold.py tests/test_gpu_muscl.py tests/test_gpu_parity.py -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -n 1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
for v in a b; do timeout -k 10 300 python tools/asm_probe.py $v >> gpurun_out/asm_probe_$T.log 2>&1 || exit 1; tail -n 1 gpurun_out/asm_probe_$T.log; done
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run c3 "" && run c5 "" "--workload c5" || exit 2
