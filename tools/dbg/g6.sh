mkdir -p gpurun_out/g6
for c in 0 512 256 128 64; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --chunk $c > gpurun_out/g6/bench_c$c.log 2>&1 || exit 1
done
echo "rc=$?"
