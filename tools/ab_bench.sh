#!/bin/bash
# A/B of library variants on one bench config (GPU box, repo root), interleaved rounds:
#   $1 = config, $2 = rounds, $3.. = variant names ("base" = libbxassoc.so, else libbxassoc_<name>.so)
set -euo pipefail
CFG=$1; R=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    lib=boxmot_amd/lib/libbxassoc.so
    [ "$v" != base ] && lib=boxmot_amd/lib/libbxassoc_$v.so
    BX_LIB_PATH=$lib timeout -k 10 150 python bench.py --config "$CFG" --no-cpu-baseline \
      > "gpurun_out/ab/${CFG}_${v}_$r.json" 2>/dev/null
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: round(v, 4) for k, v in d['roofline']['stage_ms_probe'].items()})" \
      "gpurun_out/ab/${CFG}_${v}_$r.json" "$v" "$r"
  done
done
