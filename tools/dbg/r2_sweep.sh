# round-2 bench sweep (one line per config) + r02 rocprof/PMC profile of the headline config
mkdir -p gpurun_out/r2sweep
for c in botsort bytetrack botsort_crowded ocsort boosttrack strongsort strongsort_c4; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/r2sweep/$c.log 2>&1 || { echo "fail $c"; exit 1; }
done
bash tools/profile_round.sh r02 botsort 1024 > gpurun_out/prof_r02_bot.log 2>&1
echo "rc=$?"
