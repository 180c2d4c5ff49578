# MFMA-busy / clock / wait counters of the C4 gallery distance (one pass, SQ + GRBM only)
set -o pipefail
export TMPDIR=/tmp
ARGS="--config strongsort_c4 --steps 20 --warmup 10 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/nnpmc -o run -- python3 bench.py $ARGS > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
dur = {}
for f in glob.glob("gpurun_out/nnpmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ss_nn_kernel" in r["Kernel_Name"]:
            acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(acc, key=int)[-20:]
keys = sorted({k for i in ids for k in acc[i]})
for k in keys:
    print(k, sum(acc[i][k] for i in ids) / len(ids))
PY
