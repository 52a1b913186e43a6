#!/bin/bash
# Round-4 closing cycle: the whole -m gpu suite (C5 whole mesh included), smoke, the default bench line (with the
# reference CPU baseline), rocprof kernel trace + PMC traffic (tools/gpu_cycle.sh), then a 3-D C5 bench line.
TAG=${TAG:-r04f} bash tools/gpu_cycle.sh || exit $?
timeout -k 10 400 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${TAG:-r04f}_c5.log 2>&1 && \
  tail -c 400 gpurun_out/bench_${TAG:-r04f}_c5.log
