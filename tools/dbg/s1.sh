mkdir -p gpurun_out/s1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s1/full_gpu.log 2>&1 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.log 2>&1 && timeout -k 10 400 python -u bench.py > gpurun_out/s1/bench.log 2>&1
echo "rc=$?"
