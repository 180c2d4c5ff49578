mkdir -p gpurun_out/g7
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/g7/p16.log 2>&1 && \
BX_LIB_PATH=boxmot_amd/lib/libbxassoc_p8.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/g7/p8.log 2>&1 && \
BX_LIB_PATH=boxmot_amd/lib/libbxassoc_p8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "botsort or c3 or float64 or smoke or batched" > gpurun_out/g7/p8_tests.log 2>&1
echo "rc=$?"
