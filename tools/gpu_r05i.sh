#!/bin/bash
# Round-5 cycle i: same-box bench A/B of non-temporal factor / matrix block loads (librx_nt.so, RX_NT_LOADS=1)
# against librx.so; ILU_APPLY / SPMV phase times.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05i
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: (v['kernel'], v['avg_launch_us']) for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD')})"; }
run new RX_LIB=$PKG/librx.so && run nt RX_LIB=$PKG/librx_nt.so && run newb RX_LIB=$PKG/librx.so && run ntb RX_LIB=$PKG/librx_nt.so || exit 2
