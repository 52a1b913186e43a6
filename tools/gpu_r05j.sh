#!/bin/bash
# Round-5 cycle j: the pair-interleaved ILU(0) factor (grouped build -> LDS-ring sweeps; rx_download of the factor
# de-interleaves it): the ILU / linear-solver parity tests, then same-box bench A/B: librx.so vs RX_ILU_ROWMAJOR=1,
# and the k_asm_visc next-edge index prefetch (librx_pf.so, built before the interleave, so row-major).
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05j
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_linsolve.py tests/test_gpu_size.py -x -v \
  --timeout 170 --timeout-method thread > gpurun_out/ilu_tests_$T.log 2>&1; rc=$?; echo "ilu tests rc=$rc"; grep -cE "PASSED" gpurun_out/ilu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/ilu_tests_$T.log | head -5
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: (v['kernel'], v['avg_launch_us']) for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE')})"; }
run il RX_LIB=$PKG/librx.so && run rowmajor "RX_LIB=$PKG/librx.so RX_ILU_ROWMAJOR=1" && run pf RX_LIB=$PKG/librx_pf.so && \
run ilb RX_LIB=$PKG/librx.so && run rowmajorb "RX_LIB=$PKG/librx.so RX_ILU_ROWMAJOR=1" && run pfb RX_LIB=$PKG/librx_pf.so || exit 2
