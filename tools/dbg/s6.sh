mkdir -p gpurun_out/s6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s6/full_gpu.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for c in botsort bytetrack ocsort boosttrack strongsort; do
  timeout -k 10 200 python -u bench.py --dropin --config $c --steps 300 --warmup 30 > gpurun_out/s6/$c.json 2> gpurun_out/s6/$c.err || exit 1
done
echo done
