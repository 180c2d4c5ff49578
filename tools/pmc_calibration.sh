mkdir -p gpurun_out/g4 && export TMPDIR=/tmp && \
timeout -k 10 120 ./tools/probes/fetch_calib > gpurun_out/g4/calib_plain.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/g4/calf -o run -- ./tools/probes/fetch_calib > gpurun_out/g4/calf.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/g4/calw -o run -- ./tools/probes/fetch_calib > gpurun_out/g4/calw.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/g4/bench_botsort.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config botsort_crowded > gpurun_out/g4/bench_crowded.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config strongsort_c4 --steps 20 --warmup 5 > gpurun_out/g4/bench_c4.log 2>&1 && \
(timeout -k 10 60 rocprofv3 -L > gpurun_out/g4/counters.txt 2>&1 || true) && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/g4/mfma_ss -o run -- python3 bench.py --config strongsort --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/g4/mfma_ss.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/g4/grbm_ss -o run -- python3 bench.py --config strongsort --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/g4/grbm_ss.log 2>&1
echo "rc=$?"
