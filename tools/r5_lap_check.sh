# LAP checks on the GPU box: LAP / tie / ByteTrack / BoT-SORT parity, the tie-path timing, C3 and
# crowded C3 bench lines
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_bench_workload.py -k "linear_assignment or lapjv or botsort or bytetrack or dup or crowd" > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 300 python tools/tie_timing.py > gpurun_out/${tag}_ties.jsonl 2> gpurun_out/${tag}_ties.err && cat gpurun_out/${tag}_ties.jsonl
for c in botsort_crowded botsort; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/${tag}_$c.json 2> gpurun_out/${tag}_$c.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_$c.json').read()); print('$c', d['value'], d['ms_per_step'], d['roofline'].get('stage_ms_probe'))"
done
