mkdir -p gpurun_out/g9
for m in 0 1 2; do BX_FORK1=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/g9/f$m.log 2>&1 || exit 1; done
BX_FORK1=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "botsort or batched or c3 or float64 or pending" > gpurun_out/g9/t.log 2>&1
echo "rc=$?"
