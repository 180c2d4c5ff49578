mkdir -p gpurun_out/s14
timeout -k 10 300 python -u tools/ss_phases.py --no-build --config strongsort_c4 > gpurun_out/s14/ph.log 2>&1 || { echo "phases rc=$?"; exit 1; }
echo done
