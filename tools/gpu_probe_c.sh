#!/bin/bash
# Compact-layout sweep probe (librx_probe.so: bash tools/build_variant.sh probe -DRX_PROBE) + the ILU build phase trace
# at C3, each with its own time limit.
mkdir -p gpurun_out
T=${TAG:-pc}
timeout -k 10 400 python -u tools/sweep_probe.py ${MODES:-} > gpurun_out/sweep_probe_$T.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/sweep_probe_$T.log | tail -20; [ $rc = 0 ] || exit $rc
if [ "${TRACE:-1}" = "1" ]; then
  timeout -k 10 300 python -u tools/ilu_trace.py 2000 500 256 > gpurun_out/ilu_trace_$T.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ilu_trace_$T.log | tail -16; exit $rc
fi
