# StrongSort parity subset, C4 timeline and the NN kernel's HBM bytes (FETCH / WRITE passes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_bench_workload.py -k "strongsort or ss_ or nn_ or lsap" > gpurun_out/r6_nn_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_nn_tests.log; exit 1; }
tail -1 gpurun_out/r6_nn_tests.log
bash tools/r6_ss_timeline.sh base | tail -13
export TMPDIR=/tmp
ARGS="--config strongsort_c4 --steps 20 --warmup 10 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/nnf -o run -- python3 bench.py $ARGS > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/nnw -o run -- python3 bench.py $ARGS > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for tag, d in (("FETCH_SIZE", "gpurun_out/nnf"), ("WRITE_SIZE", "gpurun_out/nnw")):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "ss_nn_kernel" in r["Kernel_Name"]:
                acc[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    vals = [sum(v) for v in acc.values()]
    vals = vals[-20:]
    print(tag, "KiB per launch (last 20 mean):", sum(vals) / max(len(vals), 1))
PY
