#!/bin/bash
# Round-5 cycle r: k_asm_visc writing each off-diagonal block once (RX_ASMV_PARK=0: the own-side AUSM column made
# again in the viscous pass; librx_park0.so) against parking it (librx.so), now that the column evaluates only its
# own side's entries: same-box bench A/B at C3 and C5.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05r
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run park RX_LIB=$PKG/librx.so && run once RX_LIB=$PKG/librx_park0.so && run parkb RX_LIB=$PKG/librx.so && \
run onceb RX_LIB=$PKG/librx_park0.so && \
run c5park RX_LIB=$PKG/librx.so "--workload c5" && run c5once RX_LIB=$PKG/librx_park0.so "--workload c5" || exit 2
