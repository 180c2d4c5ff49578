export TMPDIR=/tmp
mkdir -p gpurun_out/s28
run() { timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s28/$1 -o run -- python3 bench.py --config strongsort_c4 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/s28/$1.log 2>&1; }
run v0 &&
BX_SS_NN_NDT=2 run v1 &&
BX_SS_NN_G=2 run v2 &&
BX_SS_NN_G=2 BX_SS_NN_NDT=2 run v3
echo done
