mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "perclass or per_class or fusefirst or noreid" > gpurun_out/s2/t.log 2>&1
echo "rc=$?"
