#!/bin/bash
# Round-5 cycle u: occupancy targets. k_asm_visc<., 2> at 2 waves per SIMD (198 VGPRs, no spill; librx_aw2.so) and
# k_set_primitive at 2 (176 VGPRs, no VGPR spill; librx_pw2.so) against 3 (librx.so): same-box bench A/B, C3 and C5.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05u
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run base RX_LIB=$PKG/librx.so && run aw2 RX_LIB=$PKG/librx_aw2.so && run pw2 RX_LIB=$PKG/librx_pw2.so && \
run baseb RX_LIB=$PKG/librx.so && run aw2b RX_LIB=$PKG/librx_aw2.so && run pw2b RX_LIB=$PKG/librx_pw2.so && \
run c5 RX_LIB=$PKG/librx.so "--workload c5" && run c5pw2 RX_LIB=$PKG/librx_pw2.so "--workload c5" || exit 2
