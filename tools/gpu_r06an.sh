#!/bin/bash
# Round-6 cycle an: occupancy variants after the primitive rework — k_set_primitive at 4 waves per SIMD (128 VGPRs,
# 164 B/lane of spills; librx_prim4.so) and k_source at 2 (no spills; librx_src2.so) against the default build, C3.
mkdir -p gpurun_out
T=r06an
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
for v in base prim4 src2 base2 prim4b src2b; do
  L=$PWD/$PKG/librx.so; case $v in prim4*) L=$PWD/$PKG/librx_prim4.so;; src2*) L=$PWD/$PKG/librx_src2.so;; esac
  RX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$v.log 2>&1 || exit 2
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/bench_${T}_$v.log') if x.startswith('{')][-1]); p=d['phase_ms_per_step']; print('$v', d['ms_per_step'], 'PRIM', p['PRIMITIVE'], 'SOURCE', p['SOURCE'])"
done
