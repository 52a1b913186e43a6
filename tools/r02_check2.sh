#!/bin/bash
# Interpolated-field bench state: stability at several partition counts and workloads, then the default bench.
mkdir -p gpurun_out
for a in "--parts 256" "--parts 1024" "--parts 2048" "--workload c2 --parts 256" "--workload c5 --parts 256"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 240 python -u tools/c3_diag.py $a --steps 10 > gpurun_out/diag2_$n.log 2>&1; rc=$?; echo "diag $a rc=$rc"; grep -v amdgpu gpurun_out/diag2_$n.log | cut -c1-200
  case $rc in 0|1) ;; *) exit $rc;; esac
done
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; echo "bench rc=$?"; tail -c 1500 gpurun_out/bench_c3.log
