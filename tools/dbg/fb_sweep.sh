mkdir -p gpurun_out
for v in lq16 lq8 lq4; do
  BX_LIB_PATH=boxmot_amd/lib/libbxassoc_$v.so timeout -k 10 200 python -u bench.py --config strongsort --no-cpu-baseline > gpurun_out/fb_$v.log 2>&1 || exit 1
  BX_LIB_PATH=boxmot_amd/lib/libbxassoc_$v.so timeout -k 10 200 python -u bench.py --config strongsort_c4 --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/fbc4_$v.log 2>&1 || exit 1
done
