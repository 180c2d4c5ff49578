#!/bin/bash
# Every bench config once (GPU box, repo root) into gpurun_out/bench_all/<config>.json; the
# default C3 line and C5 with their CPU baselines.
set -euo pipefail
mkdir -p gpurun_out/bench_all
timeout -k 10 300 python bench.py > gpurun_out/bench_all/botsort.json 2> gpurun_out/bench_all/botsort.err
timeout -k 10 300 python bench.py --config boosttrack_mot8 > gpurun_out/bench_all/boosttrack_mot8.json 2> gpurun_out/bench_all/boosttrack_mot8.err
for c in botsort_crowded bytetrack ocsort boosttrack strongsort strongsort_c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_all/$c.json 2> gpurun_out/bench_all/$c.err
done
timeout -k 10 300 python bench.py --config strongsort_c4 --start-frame 150 --no-cpu-baseline > gpurun_out/bench_all/strongsort_c4_steady.json 2> gpurun_out/bench_all/strongsort_c4_steady.err
# the C3 line with every frame's outputs delivered to pinned host memory (bench.py --with-d2h)
timeout -k 10 300 python bench.py --with-d2h --no-cpu-baseline > gpurun_out/bench_all/botsort_with_d2h.json 2> gpurun_out/bench_all/botsort_with_d2h.err
# the multi-GPU entry point on the one-GPU box: two ranks over gloo sharing the card (rehearsal)
BX_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config boosttrack_mot8 --no-cpu-baseline > gpurun_out/bench_all/boosttrack_mot8_gpus2_gloo.json 2> gpurun_out/bench_all/boosttrack_mot8_gpus2_gloo.err
