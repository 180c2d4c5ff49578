mkdir -p gpurun_out/r2ph
timeout -k 10 300 python -u tools/ss_phases.py --no-build --config strongsort_c4 --frames 20 > gpurun_out/r2ph/c4.log 2>&1
echo "rc=$?"
