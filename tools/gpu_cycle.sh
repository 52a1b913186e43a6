#!/bin/bash
# One full GPU verification cycle (through gpurun, from the repo root): parity tests, smoke, the default bench
# line (c3, with the all-core CPU baseline), a rocprofv3 kernel-trace summary and the PMC traffic passes.
# Each GPU step has its own time limit; a failing step ends the script.
mkdir -p gpurun_out
T=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_$T.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$T.log 2>&1 && echo "bench ok" && tail -c 600 gpurun_out/bench_$T.log || exit 1
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/prof_$T.log 2>&1 && echo "prof ok" || exit 1
if [ "${PMC:-1}" = "1" ]; then
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/pmc_fetch_$T.log 2>&1 && echo "pmc fetch ok" &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$T -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/pmc_write_$T.log 2>&1 && echo "pmc write ok"
fi
