#!/bin/bash
# Round evidence for one config (GPU box, repo root): rocprofv3 kernel trace + stats of the bench
# command, then the PMC passes, summarised ON the box into gpurun_out/summary_<tag>/ (the raw
# traces stay on the box: gpurun copies back at most 64 MiB).
#   $1 = tag (e.g. r01), $2 = config (bench.py --config), $3 = sequences (default 1024)
set -euo pipefail
TAG=${1:-r01}; CFG=${2:-botsort}; SEQS=${3:-1024}
bash tools/trace_only.sh "$TAG" "$CFG" "$SEQS"
bash tools/pmc_passes.sh "$TAG" "$CFG" "$SEQS"
python3 tools/summarize_profile.py "$TAG" "$CFG" "gpurun_out/summary_${TAG}"
cp "gpurun_out/trace_${TAG}_${CFG}/run_kernel_stats.csv" "gpurun_out/summary_${TAG}/${TAG}_${CFG}_kernel_stats.csv"
cp "gpurun_out/trace_${TAG}_${CFG}/bench.log" "gpurun_out/summary_${TAG}/${TAG}_${CFG}_bench_traced.log"
rm -rf "gpurun_out/trace_${TAG}_${CFG}" "gpurun_out/pmc_${TAG}_${CFG}"
