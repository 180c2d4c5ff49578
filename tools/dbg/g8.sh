mkdir -p gpurun_out/g8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g8/gpu.log 2>&1 && \
bash tools/trace_only.sh g8 botsort 1024
echo "rc=$?"
