mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep_probe.py > gpurun_out/sweep_probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/sweep_probe.log | tail -12; [ $rc = 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "partitions or size or shard or parity" --timeout 300 --timeout-method thread > gpurun_out/fgs_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fgs_tests.log; [ $rc = 0 ] || exit $rc
TAG=fgs B="RX_FG_FUSED_SPMV=1" bash tools/gpu_ab.sh
