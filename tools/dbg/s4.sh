mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "strongsort or occ or runner" > gpurun_out/s4/t.log 2>&1
echo "rc=$?"
