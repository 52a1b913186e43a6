#!/bin/bash
# Round-5 cycle q: k_asm_visc with nVar-lane teams (5 nodes per wavefront; librx.so) against 16-lane teams
# (librx_w16.so), and the 3-D shape of the LDS-ring sweeps (RX_RING_3D) and the fused AUSM assembly (RX_ASM_CONV=1)
# at C5: the whole GPU suite, then same-box bench A/B at C3 and C5.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05q
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run narrow RX_LIB=$PKG/librx.so && run w16 RX_LIB=$PKG/librx_w16.so && run narrowb RX_LIB=$PKG/librx.so && \
run w16b RX_LIB=$PKG/librx_w16.so && \
run c5 RX_LIB=$PKG/librx.so "--workload c5" && run c5w16 RX_LIB=$PKG/librx_w16.so "--workload c5" && \
run c5ring2 "RX_LIB=$PKG/librx.so RX_RING_3D=0" "--workload c5" && run c5fused "RX_LIB=$PKG/librx.so RX_ASM_CONV=1" "--workload c5" && \
run c5b RX_LIB=$PKG/librx.so "--workload c5" || exit 2
