mkdir -p gpurun_out/g10
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "state_set" > gpurun_out/g10/t.log 2>&1
echo "rc=$?"
