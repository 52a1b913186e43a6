#!/bin/bash
# Parity tests of the working tree's librx.so, then an A/B bench: A = working tree, B = librx_head.so (the last
# commit, built in-tree by: git worktree + make + cp), A2 = working tree again. TESTS: pytest -k filter.
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
mkdir -p gpurun_out
T=${TAG:-head}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "${TESTS:-parity or bc or size or muscl or partitions}" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
TAG=$T B="RX_LIB=$PWD/$PKG/librx_head.so" bash tools/gpu_ab.sh
