mkdir -p gpurun_out/s5
for c in botsort bytetrack ocsort boosttrack strongsort; do
  timeout -k 10 200 python -u bench.py --dropin --config $c --steps 200 --warmup 30 > gpurun_out/s5/$c.json 2> gpurun_out/s5/$c.err || exit 1
done
echo done
