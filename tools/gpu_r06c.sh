#!/bin/bash
# Round-6 cycle c: k_asm_es occupancy / layout variants timed alone (tools/asm_probe.py): 3- and 2-wave workgroups at
# 4 waves per SIMD, edge-major summary records (RX_SUMM_TILE=1, VISC changes too); then the default's bench line.
mkdir -p gpurun_out
T=r06c
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
for v in base:librx w2:librx_w2 tile1:librx_tile1 base2:librx w2b:librx_w2 tile1b:librx_tile1; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/asm_probe.py ${v%%:*} >> gpurun_out/asm_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/asm_probe_$T.log
done
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 8 > gpurun_out/bench_${T}.log 2>&1 && python tools/ab_table.py base=gpurun_out/bench_${T}.log
