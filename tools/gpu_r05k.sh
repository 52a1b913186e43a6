#!/bin/bash
# Round-5 cycle k: the grouped ILU build's phase trace at C3 (tools/ilu_trace.py), the C5 bench line of the current
# build, and its C3 rocprofv3 kernel trace.
mkdir -p gpurun_out
T=r05k
timeout -k 10 300 python tools/ilu_trace.py 2000 500 256 > gpurun_out/ilu_trace_$T.log 2>&1; echo "trace rc=$?"; tail -14 gpurun_out/ilu_trace_$T.log
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline --steps 8 > gpurun_out/bench_${T}_c5.log 2>&1 && python tools/ab_table.py c5=gpurun_out/bench_${T}_c5.log || exit 2
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$T.log 2>&1 && echo "prof ok"
