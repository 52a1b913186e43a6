#!/bin/bash
# Round-5 cycle v: the implicit system's V/dt folded into the node-centric assembly under rx.Iterate
# (rx_set_system_fold): the whole GPU suite (tests/test_gpu_fold.py: bitwise the unfolded build), then same-box bench
# A/B against RX_NO_FOLD=1 at C3 and C5.
mkdir -p gpurun_out
T=r05v
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -1 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 $3 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log && python3 -c "
import json; l=[x for x in open('gpurun_out/bench_${T}_$1.log') if x.startswith('{')][-1]; k=json.loads(l)['roofline_kernels']
print('   ', {p: v['avg_launch_us'] for p, v in k.items() if p in ('ILU_APPLY', 'SPMV', 'ILU_BUILD', 'ASSEMBLE', 'VISC', 'CONV')})"; }
run fold RX_NO_FOLD= && run plain RX_NO_FOLD=1 && run foldb RX_NO_FOLD= && run plainb RX_NO_FOLD=1 && \
run c5fold RX_NO_FOLD= "--workload c5" && run c5plain RX_NO_FOLD=1 "--workload c5" || exit 2
