mkdir -p gpurun_out/g5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g5/gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/g5/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config botsort_crowded > gpurun_out/g5/bench_crowded.log 2>&1
echo "rc=$?"
