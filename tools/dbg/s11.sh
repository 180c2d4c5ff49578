mkdir -p gpurun_out/s11
timeout -k 10 300 python -u tools/ss_phases.py --no-build --config strongsort_c4 > gpurun_out/s11/ph.log 2>&1 || { echo "phases rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --config strongsort_c4 --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/s11/c4.log 2>&1
echo done
