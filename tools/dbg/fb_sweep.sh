mkdir -p gpurun_out
for fb in 4 8 32; do
  BX_LIB_PATH=boxmot_amd/lib/libbxassoc_fb$fb.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fb$fb.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fb16.log 2>&1
