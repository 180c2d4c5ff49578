# rocprofv3 kernel trace of C4 for library variants, then the per-frame timeline of each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  lib=boxmot_amd/lib/libbxassoc.so
  [ "$v" != base ] && lib=boxmot_amd/lib/libbxassoc_$v.so
  OUT=gpurun_out/tl_$v
  mkdir -p $OUT
  BX_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --config ${SSCFG:-strongsort_c4} --steps 20 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
  echo "== $v"; python3 tools/timeline.py $OUT ss_prep_kernel 10 | tail -16
done
