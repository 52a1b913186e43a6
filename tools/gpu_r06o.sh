#!/bin/bash
# Round-6 cycle o: where the grouped ILU build's row time goes — inv(A_jj) loads redirected to one block (gp1), the
# later lower blocks' A loads too (gp3), the A loads alone (gp2), against the default, timed alone (tools/ilu_probe.py).
mkdir -p gpurun_out
T=r06o
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
for v in base:librx gp1:librx_gp1 gp2:librx_gp2 gp3:librx_gp3 base2:librx gp1b:librx_gp1; do
  timeout -k 10 300 env RX_LIB=$PKG/${v#*:}.so python tools/ilu_probe.py ${v%%:*} >> gpurun_out/ilu_probe_$T.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ilu_probe_$T.log
done
