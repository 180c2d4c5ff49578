export TMPDIR=/tmp
mkdir -p gpurun_out/s34
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "strongsort or ss_ or lsap or occ" > gpurun_out/s34/t.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s34/v0 -o run -- python3 bench.py --config strongsort_c4 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/s34/v0.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config strongsort --no-cpu-baseline > gpurun_out/s34/ss.log 2>&1
echo done
