python tools/dbg/jv_dump.py gpurun_out/jvm || exit 1
for c in 8 4 2; do for m in crowd crowd2 eq512; do timeout -k 5 60 tools/dbg/jv_clock_ch$c gpurun_out/jvm/$m.bin 0.8 0 1 0 | tail -1 | sed "s/^/ch$c /" || exit 1; done; done
rm -rf gpurun_out/jvm
