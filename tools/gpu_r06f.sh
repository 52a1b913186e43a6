#!/bin/bash
# Round-6 cycle f: where k_asm_es's time goes after cycle e (RX_ASMES_PROBE variants, tools/asm_probe.py, timing only).
mkdir -p gpurun_out
T=r06f
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
for v in base:librx p1:librx_p1 p2:librx_p2 p3:librx_p3 p5:librx_p5; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/asm_probe.py ${v%%:*} >> gpurun_out/asm_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/asm_probe_$T.log
done
