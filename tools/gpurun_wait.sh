#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool reports no free box / slot (status=transient: nothing ran,
# nothing charged). Any call that ran (pass or fail) ends the loop. Usage: tools/gpurun_wait.sh OUT TIMEOUT CMD
OUT=$1; TO=$2; shift 2
for i in $(seq 1 400); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$OUT" 2>&1
  rc=$?
  if grep -q "status=transient" "$OUT"; then sleep 90; continue; fi
  exit $rc
done
exit 3
