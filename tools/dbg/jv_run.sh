python tools/dbg/jv_dump.py gpurun_out/jvm || exit 1
for m in ${JVM:-crowd crowd2 eq512}; do for sk in ${JVS:-0 1}; do for e in ${JVE:-0}; do
  timeout -k 5 60 tools/dbg/jv_clock gpurun_out/jvm/$m.bin 0.8 0 $sk $e || exit 1
done; done; done
rm -rf gpurun_out/jvm
