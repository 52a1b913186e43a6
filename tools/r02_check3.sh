#!/bin/bash
mkdir -p gpurun_out
for a in "--parts 2048" "--workload c5 --parts 256" "--parts 256"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 240 python -u tools/c3_diag.py $a --steps 12 > gpurun_out/diag3_$n.log 2>&1; rc=$?; echo "diag $a rc=$rc"; grep -v amdgpu gpurun_out/diag3_$n.log | cut -c1-250
  case $rc in 0|1) ;; *) exit $rc;; esac
done
