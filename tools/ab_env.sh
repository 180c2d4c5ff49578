#!/bin/bash
# A/B of environment settings on one bench config (GPU box, repo root), interleaved rounds:
#   $1 = config, $2 = rounds, $3.. = "name:VAR=val,VAR2=val" (lib=<variant> selects libbxassoc_<variant>.so)
set -uo pipefail
CFG=$1; R=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 "$R"); do
  for spec in "$@"; do
    name=${spec%%:*}; kv=${spec#*:}
    envs=(); lib=boxmot_amd/lib/libbxassoc.so
    IFS=',' read -ra parts <<< "$kv"
    for p in "${parts[@]}"; do
      [ -z "$p" ] && continue
      if [ "${p%%=*}" = lib ]; then lib=boxmot_amd/lib/libbxassoc_${p#*=}.so; else envs+=("$p"); fi
    done
    env "${envs[@]}" BX_LIB_PATH=$lib timeout -k 10 150 python bench.py --config "$CFG" --no-cpu-baseline \
      > "gpurun_out/ab/${CFG}_${name}_$r.json" 2>/dev/null || { echo "$name $r FAILED"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: round(v, 4) for k, v in d['roofline']['stage_ms_probe'].items()})" \
      "gpurun_out/ab/${CFG}_${name}_$r.json" "$name" "$r"
  done
done
