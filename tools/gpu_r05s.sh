#!/bin/bash
# Round-5 cycle s: the FGMRES SpMV with its blocks staged through LDS (k_fg_spmv_stage, librx.so) against one element
# per lane reading its block rows from global memory (k_fg_spmv_full, librx_spmv0.so); both with k_asm_visc writing
# each off-diagonal block once (RX_ASMV_PARK=0, cycle r); librx_stage2.so = RX_SPMV_STAGE=2 (column indices read once,
# each step's blocks loaded during the previous step). The whole GPU suite first, then same-box bench A/B at C3, C5.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05s
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run stage RX_LIB=$PKG/librx.so && run full RX_LIB=$PKG/librx_spmv0.so && run stageb RX_LIB=$PKG/librx.so && \
run fullb RX_LIB=$PKG/librx_spmv0.so && \
run stage2 RX_LIB=$PKG/librx_stage2.so && run stage2b RX_LIB=$PKG/librx_stage2.so && \
run c5stage RX_LIB=$PKG/librx.so "--workload c5" && run c5full RX_LIB=$PKG/librx_spmv0.so "--workload c5" && \
run c5stage2 RX_LIB=$PKG/librx_stage2.so "--workload c5" || exit 2
