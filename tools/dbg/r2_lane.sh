mkdir -p gpurun_out/r2lane
for v in 16 8 4 3 0; do
  BX_LAP_LANE_ROWS=$v timeout -k 10 300 python -u bench.py --config botsort_crowded --no-cpu-baseline --steps 30 > gpurun_out/r2lane/crowd_$v.log 2>&1 || exit 1
done
for v in 16 3; do
  BX_LAP_LANE_ROWS=$v timeout -k 10 300 python -u bench.py --config botsort --no-cpu-baseline --steps 30 > gpurun_out/r2lane/grid_$v.log 2>&1 || exit 1
  BX_LAP_LANE_ROWS=$v timeout -k 10 300 python -u bench.py --config bytetrack --no-cpu-baseline --steps 30 > gpurun_out/r2lane/byte_$v.log 2>&1 || exit 1
done
BX_LAP_LANE_ROWS=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "botsort or bytetrack or lap or batched or c3 or fixture" > gpurun_out/r2lane/t3.log 2>&1
BX_LAP_LANE_ROWS=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "botsort or bytetrack or lap or batched or c3 or fixture" > gpurun_out/r2lane/t0.log 2>&1
echo "rc=$?"
