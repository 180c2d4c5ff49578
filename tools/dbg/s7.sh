mkdir -p gpurun_out/s7
bash tools/trace_only.sh s7 botsort 1024 && python3 tools/timeline.py gpurun_out/trace_s7_botsort det_feature_kernel 10 > gpurun_out/s7/timeline.txt 2>&1
cp gpurun_out/trace_s7_botsort/run_kernel_stats.csv gpurun_out/s7/ ; cp gpurun_out/trace_s7_botsort/bench.log gpurun_out/s7/
rm -rf gpurun_out/trace_s7_botsort
echo done
