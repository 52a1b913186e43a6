#!/bin/bash
# C3 partition-count sweep (the reference's MPI-rank count of the ILU(0) preconditioner), bench lines only.
mkdir -p gpurun_out
for p in ${PARTS:-256 512 1024 2048}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --parts $p ${BENCH_ARGS:-} > gpurun_out/parts_${TAG:-c3}_$p.log 2>&1; rc=$?; echo "parts $p rc=$rc"
  python -c "
import json,sys;d=json.loads(open('gpurun_out/parts_${TAG:-c3}_$p.log').read().strip().splitlines()[-1]);ph=d['phase_ms_per_step'];print(d['value'], d['ms_per_step'], d['config']['lin_iters_mean'], {k:ph[k] for k in ('SOLVE','ILU_BUILD','SST_SOLVE','SST_SYSTEM')})" || tail -3 gpurun_out/parts_${TAG:-c3}_$p.log
  case $rc in 0|1) ;; *) exit $rc;; esac
done
