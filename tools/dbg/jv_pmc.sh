# instruction counters of the JV diagnostic (crowd, skip on, LDS state)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python $R/tools/dbg/jv_dump.py $R/gpurun_out/jvm || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/jvpmc -o p1 --output-format csv -- $R/tools/dbg/jv_clock $R/gpurun_out/jvm/crowd.bin 0.8 0 1 0 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM -d $R/gpurun_out/jvpmc -o p2 --output-format csv -- $R/tools/dbg/jv_clock $R/gpurun_out/jvm/crowd.bin 0.8 0 1 0 || exit 1
rm -rf $R/gpurun_out/jvm
find $R/gpurun_out/jvpmc -name "*counter_collection.csv" | while read f; do echo "== $f"; cat "$f"; done
