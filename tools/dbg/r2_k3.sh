mkdir -p gpurun_out/r2k3
timeout -k 10 300 python -u tools/phase_profile.py --no-build --config botsort_crowded --seqs 1024 > gpurun_out/r2k3/crowd.log 2>&1 && \
timeout -k 10 300 python -u tools/phase_profile.py --no-build --config botsort --seqs 1024 > gpurun_out/r2k3/grid.log 2>&1
echo "rc=$?"
