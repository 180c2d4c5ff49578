# StrongSort checks on the GPU box: parity subset, C4 phase split (timing build), C4 / 256-seq bench
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r6}
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_bench_workload.py -k "strongsort or ss_ or nn_ or lsap" > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
grep -E "outcomes|LSAPs|lsap_fast" gpurun_out/${tag}_tests.log
timeout -k 10 240 python tools/ss_phases.py --no-build --frames 30 > gpurun_out/${tag}_phases.txt 2>&1 && grep -E "stage1|stage2|updates|lsap|slow|R x CC|KiB|those|ncont" gpurun_out/${tag}_phases.txt
for c in "strongsort_c4" "strongsort_c4 --start-frame 150" "strongsort"; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_bench.json').read()); print('$c', d['value'], d['ms_per_step'], d['roofline'].get('stage_ms_after_timed'))"
done
