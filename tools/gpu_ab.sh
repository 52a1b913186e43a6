#!/bin/bash
# Same-box A/B of in-tree build variants: parity tests of each variant (TESTS), the viscous probe, then bench lines
# alternating base / variants twice. usage: VARIANTS="vn2 ..." TESTS="tests/test_gpu_parity.py ..." bash tools/gpu_ab.sh
mkdir -p gpurun_out
touch gpurun_out/gpu_dirty
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
T=${TAG:-ab}
BASE=${BASE:-base}  # "base" = the in-tree librx.so; or the name of a variant built the same way as the others
for v in $VARIANTS; do
  if [ -n "$TESTS" ]; then
    RX_LIB=$PKG/librx_$v.so timeout -k 10 600 python -u -m pytest $TESTS -q -x --timeout 300 --timeout-method thread \
      > gpurun_out/${T}_tests_$v.log 2>&1
    rc=$?; echo "$v tests: $(tail -1 gpurun_out/${T}_tests_$v.log)"; [ $rc -gt 1 ] && exit $rc
  fi
done
: > gpurun_out/${T}_visc_probe.txt
for v in $BASE $VARIANTS; do
  lib=$PKG/librx_$v.so; [ $v = base ] && lib=$PKG/librx.so
  RX_LIB=$lib timeout -k 10 200 python tools/visc_probe.py $v >> gpurun_out/${T}_visc_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_visc_probe.txt; exit 1; }
done
grep ms/call gpurun_out/${T}_visc_probe.txt
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {k: p[k] for k in sorted(p) if p[k] > 0.2})"; }
run() { lib=$PKG/librx_$1.so; [ $1 = base ] && lib=$PKG/librx.so
  RX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${T}_bench_$1_$2.log 2>&1 && show gpurun_out/${T}_bench_$1_$2.log "$1#$2"; }
for r in 1 2; do for v in $BASE $VARIANTS; do run $v $r || exit 2; done; done
rm -f gpurun_out/gpu_dirty
