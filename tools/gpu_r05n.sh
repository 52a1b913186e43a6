#!/bin/bash
# Round-5 cycle n: the grouped ILU build issuing a row's next lower block A_ij before W (librx.so) against after W
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05n
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_linsolve.py -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ilu_trace.py 2000 500 256 > gpurun_out/ilu_trace_$T.log 2>&1; echo "trace rc=$?"; tail -12 gpurun_out/ilu_trace_$T.log
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC')})"; }
run new RX_LIB=$PKG/librx.so && run latebl RX_LIB=$PKG/librx_latebl.so && run newb RX_LIB=$PKG/librx.so && \
run lateblb RX_LIB=$PKG/librx_latebl.so && run c5new RX_LIB=$PKG/librx.so "--workload c5" && run c5latebl RX_LIB=$PKG/librx_latebl.so "--workload c5" || exit 2
