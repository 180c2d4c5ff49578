#!/bin/bash
# dev sweep (GPU box, repo root): strongsort_c4 bench per variant lib, then a kernel-trace timeline
# of the first variant.  Usage: c4_variants.sh CONFIG VARIANT...
set -euo pipefail
CFG=$1; shift
for v in "$@"; do
  BX_LIB_PATH=boxmot_amd/lib/libbxassoc_$v.so timeout -k 10 150 python bench.py --config $CFG \
    --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${CFG}_$v.json 2> gpurun_out/${CFG}_$v.err
done
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
BX_LIB_PATH=boxmot_amd/lib/libbxassoc_$1.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/tl/$1 -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/tl/$1.log 2>&1
python3 tools/timeline.py gpurun_out/tl/$1 ${FIRST:-ss_prep_kernel} 10 > gpurun_out/tl/${CFG}_$1.txt
rm -rf gpurun_out/tl/$1
