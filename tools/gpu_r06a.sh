#!/bin/bash
# Round-6 cycle a: the edge-side-team assembly (k_asm_es, default) against the node-serial k_asm_visc (RX_ASMV_ES=0):
# the assembly / fold parity tests, then a same-box bench A/B at C3 and C5.
mkdir -p gpurun_out
T=r06a
timeout -k 10 600 python -u -m pytest tests/test_gpu_assembly.py tests/test_gpu_fold.py -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run es RX_ASMV_ES=1 && run serial RX_ASMV_ES=0 && run esb RX_ASMV_ES=1 && run serialb RX_ASMV_ES=0 && \
run c5es RX_ASMV_ES=1 "--workload c5" && run c5serial RX_ASMV_ES=0 "--workload c5" || exit 2
