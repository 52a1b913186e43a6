#!/bin/bash
# Round-5 cycle g: shared-divisor divisions in SetPrimitive_Variables too (the whole GPU suite), same-box bench A/B
# (librx_r5d.so = the round's cycle-d build, librx_nofdiv.so = this build without rx_fdiv), and the ring apply's
# timing probe (librx_probe1.so: no factor-block loads) for the ILU_APPLY phase time.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05g
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: (v['kernel'], v['avg_launch_us']) for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ASSEMBLE', 'VISC')})"; }
run new RX_LIB=$PKG/librx.so && run nofdiv RX_LIB=$PKG/librx_nofdiv.so && run old RX_LIB=$PKG/librx_r5d.so && \
run probe1 RX_LIB=$PKG/librx_probe1.so && run newb RX_LIB=$PKG/librx.so || exit 2
