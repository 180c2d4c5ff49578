# Round-end check at HEAD: the GPU suite, smoke(), and the StrongSort lines (fp64 roofline vs spec)
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/final/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
for c in strongsort_c4 strongsort; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/final/$c.json 2> gpurun_out/final/$c.err || exit 1
done
timeout -k 10 300 python bench.py --config strongsort_c4 --start-frame 150 --no-cpu-baseline > gpurun_out/final/strongsort_c4_steady.json 2> gpurun_out/final/steady.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final/botsort.json 2> gpurun_out/final/botsort.err || exit 1
for f in gpurun_out/final/*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['peak'], (d.get('cpu_baseline') or {}).get('value'))" $f; done
