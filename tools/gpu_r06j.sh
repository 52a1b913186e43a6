#!/bin/bash
# Round-6 cycle j: rocprofv3 kernel statistics of one C4 rank (tools/c4_rank_floor.py) — where the per-rank floor goes.
mkdir -p gpurun_out
T=r06j
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4_$T -o run --output-format csv -- python3 $R/tools/c4_rank_floor.py --steps 5 --warmup 2 > $R/gpurun_out/c4prof_$T.log 2>&1 && echo "rocprof ok" || exit 1
cd $R && f=$(find gpurun_out/prof_c4_$T -name "*kernel_stats.csv" | head -n 1) && python3 tools/prof_summary.py $f "C4 rank 3 of 8, c4_rank_floor.py (5 steps + warm-up)" > gpurun_out/c4_kernel_stats_$T.md && head -45 gpurun_out/c4_kernel_stats_$T.md
