#!/bin/bash
mkdir -p gpurun_out
for a in "--parts 2048" "--workload c5 --parts 256" "--parts 1024" "--workload c2 --parts 512"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 240 python -u tools/c3_diag.py $a --steps 15 > gpurun_out/diag4_$n.log 2>&1; rc=$?; echo "diag $a rc=$rc"; grep -v amdgpu gpurun_out/diag4_$n.log | cut -c1-250 | tail -8
  case $rc in 0|1) ;; *) exit $rc;; esac
done
