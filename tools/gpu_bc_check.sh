mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 40 --warmup 2 --no-cpu-baseline > gpurun_out/stab.log 2>&1; echo "stab rc=$?"; tail -c 400 gpurun_out/stab.log
R=$PWD && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1 && echo "prof ok"
