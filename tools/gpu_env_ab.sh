#!/bin/bash
# Same-library A/B of an environment switch: bench lines alternating default / $ENVB (twice), after the given tests
# run with the default. usage: ENVB="RX_NO_ASM_VISC=1" TESTS="tests/..." TAG=x bash tools/gpu_env_ab.sh
mkdir -p gpurun_out
touch gpurun_out/gpu_dirty
T=${TAG:-eab}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -q -x --timeout 600 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
  rc=$?; echo "tests: $(tail -1 gpurun_out/${T}_tests.log)"; [ $rc -gt 1 ] && exit $rc
fi
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {k: p[k] for k in sorted(p) if p[k] > 0.2}, d['roofline']['kernel'], d['roofline']['frac'])"; }
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${T}_bench_$1.log 2>&1 && show gpurun_out/${T}_bench_$1.log "$1"; }
for r in 1 2; do run a$r "${ENVA:-RX_NOTHING=1}" || exit 2; run b$r "$ENVB" || exit 2; done
rm -f gpurun_out/gpu_dirty
