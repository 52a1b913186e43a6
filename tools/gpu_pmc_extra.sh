#!/bin/bash
# Extra PMC passes on the default bench (through gpurun, from the repo root): FP64 VALU instruction counts
# (viscous FP64 fraction) and WRITE_SIZE. One counter group per pass, each with its own limit.
mkdir -p gpurun_out
T=${TAG:-x}
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES -d $R/gpurun_out/pmc_fp64_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fp64_$T.log 2>&1 && echo "pmc fp64 ok" &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_write_$T.log 2>&1 && echo "pmc write ok" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fetch_$T.log 2>&1 && echo "pmc fetch ok"
