mkdir -p gpurun_out/s3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "kf_ or per_class or lapjv" > gpurun_out/s3/t.log 2>&1
echo "rc=$?"
