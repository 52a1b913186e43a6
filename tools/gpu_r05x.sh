#!/bin/bash
# Round-5 cycle x: the C4 per-rank floor (one rank's shard of the 8-GPU strong-scaling run, no communicator) with the
# round's closing kernels, twice.
mkdir -p gpurun_out
T=r05x
timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_$T.log 2>&1 && tail -c 900 gpurun_out/c4floor_$T.log && \
timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_${T}b.log 2>&1 && tail -c 900 gpurun_out/c4floor_${T}b.log || exit 1
