mkdir -p gpurun_out/r2ss
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "strongsort or ss_ or lsap or occ or c4 or lapjv or ocsort or boost" > gpurun_out/r2ss/t.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config strongsort_c4 --no-cpu-baseline > gpurun_out/r2ss/b_c4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config strongsort --no-cpu-baseline > gpurun_out/r2ss/b_ss.log 2>&1
echo "rc=$?"
