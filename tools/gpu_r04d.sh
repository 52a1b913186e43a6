#!/bin/bash
# Viscous edge sweep probes: time k_visc_edge / k_visc_jac alone at C3 for the base build and the section-skip
# variants (RX_VISC_PROBE 1: no BiCGSTAB, 2: no QR, 3: neither), then any extra variants named in $VARIANTS.
mkdir -p gpurun_out
[ -f gpurun_out/gpu_dirty ] && { echo "previous GPU step did not end cleanly: skipping"; exit 3; }
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
: > gpurun_out/visc_probe.txt
timeout -k 10 200 python tools/visc_probe.py base >> gpurun_out/visc_probe.txt 2>&1 || { tail -20 gpurun_out/visc_probe.txt; exit 1; }
for v in vp1 vp2 vp3 $VARIANTS; do
  RX_LIB=$PWD/$PKG/librx_$v.so timeout -k 10 200 python tools/visc_probe.py $v >> gpurun_out/visc_probe.txt 2>&1 || { tail -20 gpurun_out/visc_probe.txt; exit 1; }
done
grep ms/call gpurun_out/visc_probe.txt
