#!/bin/bash
# Round-5 cycle p: the 3-D shape of the LDS-ring sweeps (768 threads, three factor blocks of a row in registers):
# the ILU / linear-solver parity tests, then same-box C5 A/B against RX_RING_3D=0 (the 2-D shape), and C3.
mkdir -p gpurun_out
T=r05p
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_linsolve.py -x -v --timeout 170 \
  --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run c5ring3 RX_RING_3D=1 "--workload c5" && run c5ring2 RX_RING_3D=0 "--workload c5" && run c5ring3b RX_RING_3D=1 "--workload c5" && \
run c5ring2b RX_RING_3D=0 "--workload c5" && run c3 RX_RING_3D=1 || exit 2
