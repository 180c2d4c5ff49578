#!/bin/bash
# quick per-kernel timing of the bench workload: rocprofv3 kernel trace + stats only
#   $1 = tag, $2 = config, $3 = seqs
set -euo pipefail
TAG=${1:-dev}; CFG=${2:-botsort}; SEQS=${3:-1024}
OUT=gpurun_out/trace_${TAG}_${CFG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 bench.py --config $CFG --seqs $SEQS --steps 50 --warmup 10 --no-cpu-baseline > "$OUT/bench.log" 2>&1
