mkdir -p gpurun_out
for gg in 4 2 1; do
  BX_SS_NN_G=$gg timeout -k 10 200 python -u bench.py --config strongsort --no-cpu-baseline > gpurun_out/fb_g$gg.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fb_bot.log 2>&1
timeout -k 10 200 python -u bench.py --config boosttrack --no-cpu-baseline > gpurun_out/fb_boost.log 2>&1
