#!/bin/bash
# Per-kernel PMC counters of the bench workload (run on the GPU box from the repo root), one
# counter group per pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE need their own passes;
# no trace domains are combined with --pmc).
#   $1 = tag, $2 = config, $3 = seqs
set -euo pipefail
TAG=${1:-dev}; CFG=${2:-botsort}; SEQS=${3:-1024}
OUT=gpurun_out/pmc_${TAG}_${CFG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--config $CFG --seqs $SEQS --steps 50 --warmup 10 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT/sq" -o run -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/misc" -o run -- python3 bench.py $ARGS > "$OUT/misc.log" 2>&1
