#!/bin/bash
# Round-5 cycle h: the grouped ILU build's divisions through rx_fdiv (the ILU / linear-solver parity tests), and the
# ring apply's pair-interleaved load probe (librx_probe2.so: the same factor bytes, each load instruction reading a
# contiguous 16-byte pair per lane) against librx.so, ILU_APPLY phase times.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05h
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_linsolve.py tests/test_gpu_size.py -x -v \
  --timeout 170 --timeout-method thread > gpurun_out/ilu_tests_$T.log 2>&1; rc=$?; echo "ilu tests rc=$rc"; grep -cE "PASSED" gpurun_out/ilu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/ilu_tests_$T.log | head -5
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: (v['kernel'], v['avg_launch_us']) for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD')})"; }
run new RX_LIB=$PKG/librx.so && run probe2 RX_LIB=$PKG/librx_probe2.so && run newb RX_LIB=$PKG/librx.so || exit 2
