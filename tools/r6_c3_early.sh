# C3 early-features: parity tests, then interleaved bench A/B (normal vs early) and a trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_workload.py -k "c3_bench or crowded" > gpurun_out/r6_c3e_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_c3e_tests.log; exit 1; }
tail -1 gpurun_out/r6_c3e_tests.log
for r in 1 2; do
  for f in "" "--early-features"; do
    timeout -k 10 150 python bench.py --config botsort --no-cpu-baseline $f > gpurun_out/r6_c3e.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r6_c3e.json')); print('early' if d['config'].get('early_features') else 'normal', d['value'], d['ms_per_step'])"
  done
done
export TMPDIR=/tmp
OUT=gpurun_out/tlc3_early; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --config botsort --steps 20 --warmup 10 --no-cpu-baseline --early-features > $OUT/bench.log 2>&1 || exit 1
python3 tools/timeline.py $OUT det_feature_kernel 10 | tail -10
