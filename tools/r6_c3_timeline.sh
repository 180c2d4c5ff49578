# rocprofv3 kernel trace of the C3 headline for library variants, then the per-frame timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cfg=${CFG:-botsort}
for v in "$@"; do
  lib=boxmot_amd/lib/libbxassoc.so
  [ "$v" != base ] && lib=boxmot_amd/lib/libbxassoc_$v.so
  OUT=gpurun_out/tlc3_$v
  mkdir -p $OUT
  BX_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --config $cfg --steps 20 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
  echo "== $v"; tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; python3 tools/timeline.py $OUT det_feature_kernel 10 | tail -12
done
