#!/bin/bash
# Round-6 cycle g: k_asm_es without its off-diagonal stores (p6), without the source loads of phase B (p7), and with
# edge-major summary records (tile1: RX_SUMM_TILE=1, k_visc_edge's stores change too); timing only.
mkdir -p gpurun_out
T=r06g
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
for v in base:librx p6:librx_p6 p7:librx_p7 tile1:librx_tile1 base2:librx tile1b:librx_tile1; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/asm_probe.py ${v%%:*} >> gpurun_out/asm_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/asm_probe_$T.log
done
