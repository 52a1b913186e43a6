#!/bin/bash
# Round-6 measurement cycle of the in-tree librx.so: (unless SKIP_TESTS=1) the whole GPU suite and smoke(), the
# default bench line (C3, the all-core reference CPU baseline), a rocprofv3 kernel-trace summary, the PMC passes
# (FETCH_SIZE / WRITE_SIZE traffic, FP64 VALU counts, wave states) on C3, C5's bench line and kernel trace, then the
# C4 per-rank floor. One rocprofv3 counter group per run, each with its own limit; a failing step ends the script.
# Usage: tools/gpu_r06_final.sh TAG
mkdir -p gpurun_out
T=${1:-r06f}
# the box's clocks and memory state (for the box-to-box spread of the bandwidth-bound kernels), read-only
{ date; rocm-smi --showclocks --showperflevel --showmeminfo vram --showpower 2>&1; } > gpurun_out/box_clocks_$T.txt 2>&1 || true
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; grep -cE "PASSED" gpurun_out/gpu_tests_$T.log; grep -E "FAILED|Error" gpurun_out/gpu_tests_$T.log | head -5; tail -n 1 gpurun_out/gpu_tests_$T.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_$T.log 2>&1 && echo "bench ok" && tail -c 400 gpurun_out/bench_$T.log || exit 1
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$T.log 2>&1 && echo "prof ok" &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fetch_$T.log 2>&1 && echo "pmc fetch ok" &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_write_$T.log 2>&1 && echo "pmc write ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES -d $R/gpurun_out/pmc_fp64_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fp64_$T.log 2>&1 && echo "pmc fp64 ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_stall_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_stall_$T.log 2>&1 && echo "pmc stall ok" || exit 2
cd $R
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_${T}_c5.log 2>&1 && echo "bench c5 ok" && tail -c 300 gpurun_out/bench_${T}_c5.log || exit 3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_c5 -o run --output-format csv -- python3 $R/bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_${T}_c5.log 2>&1 && echo "prof c5 ok" || exit 4
cd $R
timeout -k 10 300 python tools/c4_rank_floor.py > gpurun_out/c4floor_$T.log 2>&1 && echo "c4 floor ok" && tail -c 300 gpurun_out/c4floor_$T.log || exit 5
{ date; rocm-smi --showclocks --showperflevel --showpower 2>&1; } >> gpurun_out/box_clocks_$T.txt 2>&1 || true
