mkdir -p gpurun_out
for p in 256 512 1024; do timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --parts $p > gpurun_out/parts_c2_$p.log 2>&1; echo "c2 parts $p rc=$?"; done
for p in 256 1024 2048; do timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --parts $p > gpurun_out/parts_c3_$p.log 2>&1; echo "c3 parts $p rc=$?"; done
