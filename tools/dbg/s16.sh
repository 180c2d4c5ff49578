mkdir -p gpurun_out/s16
for v in t16f t16 t8f; do
timeout -k 10 300 python -u tools/ss_phases.py --no-build --lib $PWD/boxmot_amd/lib/libbxassoc_$v.so --config strongsort_c4 > gpurun_out/s16/$v.log 2>&1 || { echo "phases rc=$?"; exit 1; }
done
echo done
