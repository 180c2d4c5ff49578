mkdir -p gpurun_out/r2full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2full/gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2full/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r2full/b_default.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config strongsort_c4 > gpurun_out/r2full/b_c4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config botsort_crowded > gpurun_out/r2full/b_crowd.log 2>&1
echo "rc=$?"
