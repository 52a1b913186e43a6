#!/bin/bash
# Round-5 cycle t: the SST 2x2 ILU apply with its blocks 4 / 6 passes ahead instead of 3 (librx_d4.so, librx_d6.so),
# and the staged SpMV with XCD-grouped workgroups (librx_sx.so), against librx.so: the SST and linear-solver parity
# tests on each variant, then same-box bench A/B at C3.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05t
for v in d6 sx; do
  RX_LIB=$PKG/librx_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sst.py tests/test_gpu_linsolve.py tests/test_gpu_rccl_self.py -x -q --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_${T}_$v.log 2>&1; rc=$?; echo "tests $v rc=$rc"; tail -1 gpurun_out/gpu_tests_${T}_$v.log; [ $rc -ne 0 ] && exit $rc
done
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run base RX_LIB=$PKG/librx.so && run d4 RX_LIB=$PKG/librx_d4.so && run d6 RX_LIB=$PKG/librx_d6.so && run sx RX_LIB=$PKG/librx_sx.so && \
run baseb RX_LIB=$PKG/librx.so && run d4b RX_LIB=$PKG/librx_d4.so && run d6b RX_LIB=$PKG/librx_d6.so && run sxb RX_LIB=$PKG/librx_sx.so || exit 2
