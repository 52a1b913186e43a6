#!/bin/bash
# Round-5 cycle w: the grouped ILU build without the stores of the eliminated diagonal blocks (no sweep reads them; a
# download of the ILU field remakes them, k_ilu_diag_materialize; librx.so) against storing them (librx_dstore.so):
# the whole GPU suite (the ILU factor downloads against the oracle), then same-box bench A/B at C3 and C5.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05w
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run nodiag RX_LIB=$PKG/librx.so && run store RX_LIB=$PKG/librx_dstore.so && run nodiagb RX_LIB=$PKG/librx.so && \
run storeb RX_LIB=$PKG/librx_dstore.so && \
run c5nodiag RX_LIB=$PKG/librx.so "--workload c5" && run c5store RX_LIB=$PKG/librx_dstore.so "--workload c5" || exit 2
