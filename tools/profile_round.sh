#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root).
#   $1 = tag (e.g. r01), $2 = config (botsort|bytetrack), $3 = seqs
# kernel trace + stats in one pass; HBM counters in their own passes (FETCH_SIZE and WRITE_SIZE
# cannot share a pass on gfx950, MI355X_MICROARCH.md §rocprofv3 PMC slots).
set -euo pipefail
TAG=${1:-r01}; CFG=${2:-botsort}; SEQS=${3:-1024}
OUT=gpurun_out/prof_${TAG}_${CFG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="--config $CFG --seqs $SEQS --steps 30 --warmup 10 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/bench_traced.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/bench_write.log" 2>&1
find "$OUT" -name "*.csv" | head -50
