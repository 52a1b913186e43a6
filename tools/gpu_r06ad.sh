#!/bin/bash
# Round-6 cycle ad: the whole GPU suite and smoke() on the final code (two-groups-per-row ILU build by default on the
# small meshes).
mkdir -p gpurun_out
T=r06ad
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 && echo "smoke ok"
