set -e
bash tools/profile_round.sh r01 botsort 1024
bash tools/profile_round.sh r01 strongsort 256
bash tools/profile_round.sh r01 strongsort_c4 1
