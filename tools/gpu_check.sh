#!/bin/bash
# One GPU verification cycle (run through gpurun from the repo root): GPU parity tests, the ILU
# phase trace, a bench line and a rocprofv3 kernel-trace summary. Every GPU step has its own time
# limit; a failing step ends the script (set -e semantics via &&).
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -rA --tb=short > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python tools/ilu_trace.py > gpurun_out/trace.log 2>&1 && echo "trace ok" &&
timeout -k 10 400 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1 && echo "bench ok" &&
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1 && echo "prof ok"
if [ "${DIST2:-0}" = "1" ]; then
  R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=/root/repo
  cd $R && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench2.log 2>&1 && echo "bench2 ok"
fi
if [ "${PMC:-0}" = "1" ]; then
  R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=/root/repo
  cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1 && echo "pmc fetch ok" &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1 && echo "pmc write ok"
fi
