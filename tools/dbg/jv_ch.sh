python tools/dbg/jv_dump.py gpurun_out/jvm || exit 1
for b in jv_clock jv_clock_ch1; do for m in crowd crowd2; do timeout -k 5 60 tools/dbg/$b gpurun_out/jvm/$m.bin 0.8 0 1 0 | tail -1 | sed "s/^/$b /" || exit 1; done; done
rm -rf gpurun_out/jvm
