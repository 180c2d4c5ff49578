mkdir -p gpurun_out/s8
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "botsort or bytetrack or batched or pending or kalman or per_class or c3" > gpurun_out/s8/t.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s8/b.log 2>&1
bash tools/trace_only.sh s8 botsort 1024 && python3 tools/timeline.py gpurun_out/trace_s8_botsort det_feature_kernel 10 > gpurun_out/s8/timeline.txt 2>&1
rm -rf gpurun_out/trace_s8_botsort
echo done
