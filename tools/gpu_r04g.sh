#!/bin/bash
# cycle g: A/B of the sweeps' column prefetch (pf) and the shared spline interval (sp), then a wave-state PMC pass
set -o pipefail
TAG=abg VARIANTS="sp pf" TESTS="tests/test_gpu_parity.py tests/test_gpu_bc.py tests/test_gpu_partitions.py tests/test_gpu_sst.py tests/test_gpu_shard_iterate.py tests/test_gpu_fgmres_nan.py" bash tools/gpu_ab.sh || exit $?
[ -f gpurun_out/gpu_dirty ] && exit 3
RX_LIB=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd/librx_pf.so TAG=g bash tools/gpu_pmc_stall.sh
