#!/bin/bash
# Wave-state PMC pass on the default bench (through gpurun): where each kernel's wave cycles go (SQ_WAIT_ANY =
# parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stalls, SQ_ACTIVE_INST_ANY = issuing; quad-cycles).
mkdir -p gpurun_out
T=${TAG:-s}
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_stall_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_stall_$T.log 2>&1 && echo "pmc stall ok"
