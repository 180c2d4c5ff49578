#!/bin/bash
# dev sweep (GPU box, repo root): default (C3) bench per variant lib, interleaved twice
set -euo pipefail
CFG=${CFG:-botsort}
for rep in 1 2; do for v in "$@"; do
  BX_LIB_PATH=boxmot_amd/lib/libbxassoc_$v.so timeout -k 10 150 python bench.py --config $CFG \
    --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/${CFG}_${v}_$rep.json 2> gpurun_out/${CFG}_${v}_$rep.err
done; done
