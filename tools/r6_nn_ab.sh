# C4 timelines of NN variants (kernel durations from the trace) and their step times
set -o pipefail
for v in "$@"; do bash tools/r6_ss_timeline.sh $v | grep -E "==|ss_nn_kernel|span"; done
bash tools/ab_bench.sh strongsort_c4 1 "$@"
