mkdir -p gpurun_out
for nd in 2 4; do
  BX_SS_NN_NDT=$nd timeout -k 10 200 python -u bench.py --config strongsort --no-cpu-baseline > gpurun_out/fb_nd$nd.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --config strongsort_c4 --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/fb_c4.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "strongsort or ss_ or nn" > gpurun_out/ss_gpu.log 2>&1
