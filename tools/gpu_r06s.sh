#!/bin/bash
# Round-6 cycle s: k_asm_es with the off-diagonal column stored after phase B's loads and an LDS-only phase barrier
# (RX_ASMES_LATE_STORE=1, in-tree) against the stores inside the viscous column + __syncthreads (librx_als0): the
# assembly parity tests, the kernel timed alone, then bench lines alternating.
mkdir -p gpurun_out
T=r06s
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_assembly.py tests/test_gpu_fold.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || exit $rc
for v in base:librx als0:librx_als0 base2:librx als0b:librx_als0; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/asm_probe.py ${v%%:*} >> gpurun_out/asm_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/asm_probe_$T.log
done
for r in 1 2; do
  for v in base:librx als0:librx_als0; do
    RX_LIB=$PKG/${v#*:}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_${v%%:*}_$r.log 2>&1 || exit 2
  done
done
python3 tools/ab_table.py base1=gpurun_out/bench_${T}_base_1.log als0_1=gpurun_out/bench_${T}_als0_1.log base2=gpurun_out/bench_${T}_base_2.log als0_2=gpurun_out/bench_${T}_als0_2.log
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 6 > gpurun_out/bench_${T}_c5.log 2>&1 && python3 tools/ab_table.py c5=gpurun_out/bench_${T}_c5.log
