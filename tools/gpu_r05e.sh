#!/bin/bash
# Round-5 cycle e: the LDS-ring ILU apply with its wavefronts in two groups taking turns by level (loads issued two
# levels ahead) and unconditional loads, and the post-update exchange overlapped with SetPrimitive_Variables: the ILU /
# linear-solver parity tests and the RCCL self-halo test, then same-box bench A/B against the round's previous build
# (librx_r5d.so), the one-group plan (RX_ILU_RING_G=1) and the SpMV chunk variant (librx_spmv2.so).
mkdir -p gpurun_out
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=r05e
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitions.py tests/test_gpu_linsolve.py tests/test_gpu_size.py -x -v \
  --timeout 170 --timeout-method thread > gpurun_out/ilu_tests_$T.log 2>&1; rc=$?; echo "ilu tests rc=$rc"; grep -cE "PASSED" gpurun_out/ilu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/ilu_tests_$T.log | head -5
[ $rc -ne 0 ] && exit $rc
NCCL_DEBUG=WARN timeout -k 10 170 python -u -m pytest tests/test_gpu_rccl_self.py -v -s --timeout 150 --timeout-method thread > gpurun_out/rccl_self_$T.log 2>&1; rc=$?; echo "rccl_self rc=$rc"; grep -E "PASSED|FAILED|self-halo" gpurun_out/rccl_self_$T.log | tail -3
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run old RX_LIB=$PKG/librx_r5d.so && run g2 RX_LIB=$PKG/librx.so && run g1 "RX_LIB=$PKG/librx.so RX_ILU_RING_G=1" && \
run oldb RX_LIB=$PKG/librx_r5d.so && run g2b RX_LIB=$PKG/librx.so && run g1b "RX_LIB=$PKG/librx.so RX_ILU_RING_G=1" && \
run spmv2 RX_LIB=$PKG/librx_spmv2.so || exit 2
run5() { timeout -k 10 400 env $2 python bench.py --workload c5 --no-cpu-baseline --steps 8 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run5 c5old RX_LIB=$PKG/librx_r5d.so && run5 c5g2 RX_LIB=$PKG/librx.so || exit 3
