#!/bin/bash
# Round-4 A/B on one box: HEAD, the AUSM store variants, the split ILU sweeps, the previous 2x2 kernels.
mkdir -p gpurun_out
T=${TAG:-r04c}
PKG=$PWD/development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
show() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l); p=d['phase_ms_per_step']; r=d['roofline_kernels']
print('$2', d['value'], d['ms_per_step'], {k: p[k] for k in sorted(p) if p[k] > 0.3}, 'CONV', r['CONV']['frac'], r['CONV']['avg_launch_us'], 'SPMV', r.get('SPMV',{}).get('avg_launch_us'), 'ILU_APPLY', r.get('ILU_APPLY',{}).get('avg_launch_us'))"; }
run() { timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_${T}_$1.log 2>&1 && show gpurun_out/bench_${T}_$1.log "$1($2)"; }
run a RX_NOTHING=1 && run touch RX_LIB=$PKG/librx_touch.so && run ausm0 RX_LIB=$PKG/librx_ausm0.so && run ausm1 RX_LIB=$PKG/librx_ausm1.so && \
run split RX_ILU_SPLIT=1 && run old2 "RX_ILU2_OLD=1 RX_ILU2_APPLY_OLD=1" && run a2 RX_NOTHING=1
