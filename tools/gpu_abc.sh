#!/bin/bash
# A/B/C bench on one box: the default path, then each environment in $B1, $B2 (e.g. RX_ILU_ROWWAVE=1,
# RX_LIB=$PWD/<pkg>/librx_x.so), each a separate bench process; optional parity tests first ($TESTS).
mkdir -p gpurun_out
T=${TAG:-abc}
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {k: p[k] for k in sorted(p) if p[k] > 0.4})"; }
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 1; }
  tail -1 gpurun_out/tests_$T.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_${T}_a.log 2>&1 && show gpurun_out/bench_${T}_a.log A || exit 1
for V in "$B1" "$B2" "$B3"; do
  [ -z "$V" ] && continue
  timeout -k 10 300 env $V python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_${T}_v.log 2>&1 && show gpurun_out/bench_${T}_v.log "($V)" || exit 1
done
