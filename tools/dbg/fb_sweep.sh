mkdir -p gpurun_out
for v in k1np4 k1np8 k1p16 k1np16; do
  BX_LIB_PATH=boxmot_amd/lib/libbxassoc_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fb_$v.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fb_base.log 2>&1
