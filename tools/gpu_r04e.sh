#!/bin/bash
# Round-4 cycle e: the viscous rewrite (librx_vnew.so: short live ranges, Dm streamed through LDS, interleaved LDS
# scratch, unrolled pivoted QR) — its parity tests, the viscous probe against the current librx.so, then the
# step-level A/B of the other build knobs against it.
mkdir -p gpurun_out
touch gpurun_out/gpu_dirty
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
RX_LIB=$PKG/librx_vnew.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bc.py tests/test_gpu_sst.py \
  tests/test_gpu_muscl.py tests/test_gpu_case.py -q -x --timeout 300 --timeout-method thread > gpurun_out/vnew_tests.log 2>&1
rc=$?; tail -3 gpurun_out/vnew_tests.log; [ $rc -gt 1 ] && exit $rc
: > gpurun_out/visc_probe_e.txt
for v in base vnew vnewrl; do
  lib=$PKG/librx_$v.so; [ $v = base ] && lib=$PKG/librx.so
  RX_LIB=$lib timeout -k 10 200 python tools/visc_probe.py $v >> gpurun_out/visc_probe_e.txt 2>&1 || { tail -20 gpurun_out/visc_probe_e.txt; exit 1; }
done
grep ms/call gpurun_out/visc_probe_e.txt
T=r04e
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']; r=d['roofline_kernels']
print('$2', d['value'], d['ms_per_step'], {k: p[k] for k in sorted(p) if p[k] > 0.3}, 'CONV', r['CONV']['frac'], r['CONV']['avg_launch_us'], 'SPMV', r.get('SPMV',{}).get('avg_launch_us'), 'ILU_APPLY', r.get('ILU_APPLY',{}).get('avg_launch_us'))"; }
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && show gpurun_out/bench_${T}_$1.log "$1($2)"; }
run vnew RX_LIB=$PKG/librx_vnew.so && run touch RX_LIB=$PKG/librx_touch.so && run ausm0 RX_LIB=$PKG/librx_ausm0.so && \
run ausm1 RX_LIB=$PKG/librx_ausm1.so && run split "RX_LIB=$PKG/librx_vnew.so RX_ILU_SPLIT=1" && \
run old2 "RX_LIB=$PKG/librx_vnew.so RX_ILU2_OLD=1 RX_ILU2_APPLY_OLD=1" && run vnew2 RX_LIB=$PKG/librx_vnew.so || exit 2
rm -f gpurun_out/gpu_dirty
