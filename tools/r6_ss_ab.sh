# StrongSort A/B on the GPU box: solve + certify vs scipy's order, C4 and 256-seq; phases
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r6ab}
for c in "strongsort_c4" "strongsort_c4 --lsap-exact" "strongsort" "strongsort --lsap-exact"; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_bench.json').read()); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r.get('stage_ms_after_timed'), r['units_last_frame'].get('lsap_all_frames'))"
done
timeout -k 10 240 python tools/ss_phases.py --no-build --frames 30 > gpurun_out/${tag}_phases.txt 2>&1 && head -16 gpurun_out/${tag}_phases.txt && grep -E "lsap|fast" gpurun_out/${tag}_phases.txt
