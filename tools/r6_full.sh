# Full GPU suite + the headline and StrongSort bench lines (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r6}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
for c in "botsort" "strongsort_c4" "strongsort"; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/${tag}_bench_$c.json 2> gpurun_out/${tag}_bench.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_bench_$c.json').read()); print('$c', d['value'], d['ms_per_step'], d['roofline'].get('stage_ms_after_timed'))"
done
