mkdir -p gpurun_out/s18
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -s -k "strongsort or ss_ or lsap or occ" > gpurun_out/s18/t.log 2>&1
echo done
