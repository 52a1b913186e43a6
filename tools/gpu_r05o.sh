#!/bin/bash
# Round-5 cycle o: C5 with the AUSM fluxes fused into the node-centric assembly (RX_ASM_CONV=1) against the edge kernel,
# now that the fused pass evaluates only its own side's entries.
mkdir -p gpurun_out
T=r05o
run() { timeout -k 10 400 env $2 python bench.py --no-cpu-baseline --steps 8 --workload c5 > gpurun_out/bench_${T}_$1.log 2>&1 && python tools/ab_table.py $1=gpurun_out/bench_${T}_$1.log; }
run edge RX_ASM_CONV= && run fused RX_ASM_CONV=1 && run edgeb RX_ASM_CONV= && run fusedb RX_ASM_CONV=1 || exit 2
