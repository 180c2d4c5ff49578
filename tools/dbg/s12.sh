mkdir -p gpurun_out/s12
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "strongsort or ss_ or lsap or occ" > gpurun_out/s12/t.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/ss_phases.py --no-build --config strongsort_c4 > gpurun_out/s12/ph.log 2>&1 || { echo "phases rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --config strongsort_c4 --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/s12/c4.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config strongsort --no-cpu-baseline > gpurun_out/s12/ss.log 2>&1
echo done
