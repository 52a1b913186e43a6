#!/bin/bash
# configs[2] (1M-cell jet, 7 species PaSR + SST): bench line + kernel-trace profile. Run through gpurun.
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 && echo "bench c3 ok" &&
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o run --output-format csv -- python3 $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c3.log 2>&1 && echo "prof c3 ok"
