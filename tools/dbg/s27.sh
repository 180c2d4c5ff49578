export TMPDIR=/tmp
mkdir -p gpurun_out/s27
for v in v0 v1; do
  BX_LIB_PATH=$PWD/boxmot_amd/lib/libbxassoc_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s27/$v -o run -- python3 bench.py --config strongsort_c4 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/s27/$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
done
echo done
