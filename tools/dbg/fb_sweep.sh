mkdir -p gpurun_out
for gg in 1 2 4; do
  BX_SS_NN_G=$gg timeout -k 10 200 python -u bench.py --config strongsort_c4 --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/fbc4_g$gg.log 2>&1 || exit 1
done
