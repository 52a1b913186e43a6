# Staged ILU(0) sweeps: probe timings + bitwise check vs the wide sweeps, parity tests that run them, bench A/B.
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep_probe.py > gpurun_out/stage_probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stage_probe.log | tail -17; [ $rc = 0 ] || exit $rc
rm -f development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd/librx_probe.so
RX_STAGE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "partitions or size" --timeout 300 --timeout-method thread > gpurun_out/stage_tests.log 2>&1; rc=$?; tail -2 gpurun_out/stage_tests.log; [ $rc = 0 ] || exit $rc
TAG=stage B="RX_STAGE=1" bash tools/gpu_ab.sh
