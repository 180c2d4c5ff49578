mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "warp or c4" > gpurun_out/g3_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g3_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config strongsort_c4 --steps 20 --warmup 10 > gpurun_out/g3_c4.log 2>&1
echo "rc=$?"
