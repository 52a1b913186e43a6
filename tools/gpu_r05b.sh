#!/bin/bash
# Round-5 cycle b: the LDS-ring ILU(0) apply + the single-write fused assembly + the SST second-order upwind (in-tree
# librx.so) through the parity tests that exercise them, then same-box bench A/B: librx_r4.so (round-4 kernels) /
# librx_rc.so (single-write assembly) / librx.so (both + SST 2nd order) / librx.so with RX_ILU_NO_RING=1.
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05b
timeout -k 10 900 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_assembly.py \
  tests/test_gpu_parity.py tests/test_gpu_bc.py "tests/test_gpu_size.py::test_full_size_iteration_vs_oracle[c3]" \
  "tests/test_gpu_size.py::test_full_size_iteration_vs_oracle[c5]" -x -q --timeout 600 --timeout-method thread > gpurun_out/ring_tests_$T.log 2>&1
rc=$?; tail -4 gpurun_out/ring_tests_$T.log; [ $rc -gt 1 ] && exit $rc
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']; r=d['roofline_kernels']
print('$2', d['value'], d['ms_per_step'], 'lin', d['config']['lin_iters_mean'], {k: p[k] for k in sorted(p) if p[k] > 0.3}, {k: (r[k]['avg_launch_us'], r[k]['frac']) for k in ('ASSEMBLE','ILU_APPLY','SPMV') if k in r})"; }
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && show gpurun_out/bench_${T}_$1.log "$1"; }
run r4 RX_LIB=$PKG/librx_r4.so && run rc RX_LIB=$PKG/librx_rc.so && run new RX_LIB=$PKG/librx.so && \
run noring "RX_LIB=$PKG/librx.so RX_ILU_NO_RING=1" && run r4b RX_LIB=$PKG/librx_r4.so && run newb RX_LIB=$PKG/librx.so || exit 2
run5() { timeout -k 10 400 env $2 python bench.py --workload c5 --no-cpu-baseline --steps 8 > gpurun_out/bench_${T}_$1.log 2>&1 && show gpurun_out/bench_${T}_$1.log "$1"; }
run5 c5r4 RX_LIB=$PKG/librx_r4.so && run5 c5new RX_LIB=$PKG/librx.so && run5 c5fused "RX_LIB=$PKG/librx.so RX_ASM_CONV=1" || exit 3
