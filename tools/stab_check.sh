mkdir -p gpurun_out
for c in 5 1; do
timeout -k 10 200 python bench.py --steps 40 --warmup 2 --no-cpu-baseline --cfl $c > gpurun_out/stab_$c.log 2>&1; echo "cfl $c rc=$?"; tail -c 300 gpurun_out/stab_$c.log; echo
done
