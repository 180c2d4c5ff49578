set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_bench_workload.py -k "strongsort or ss_ or nn_ or lsap" > gpurun_out/r6_nn_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_nn_tests.log; exit 1; }
tail -1 gpurun_out/r6_nn_tests.log
bash tools/r6_nn_ab.sh "$@"
