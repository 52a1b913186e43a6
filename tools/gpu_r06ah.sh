#!/bin/bash
# Round-6 cycle ah: kernel trace of the C4 rank floor (which launches make SST_SOLVE / SOLVE at the rank shape).
mkdir -p gpurun_out
T=r06ah
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_c4 -o run --output-format csv -- python3 $R/tools/c4_rank_floor.py > $R/gpurun_out/prof_${T}_c4.log 2>&1 && echo "prof c4 ok" && tail -c 600 $R/gpurun_out/prof_${T}_c4.log
