#!/bin/bash
# Tie path: JV phase clocks (skip off/on), the LAP parity tests, op-level and engine timings.
set -o pipefail
mkdir -p gpurun_out
JVS=1 bash tools/dbg/jv_run.sh > gpurun_out/r6_jv_clock.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "linear_assignment or lapjv or dup or tied or legacy" \
  > gpurun_out/r6_tie_tests.log 2>&1 || { tail -30 gpurun_out/r6_tie_tests.log; exit 1; }
tail -2 gpurun_out/r6_tie_tests.log
timeout -k 10 120 python -u tools/tie_probe.py > gpurun_out/r6_tie_probe.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/tie_timing.py > gpurun_out/r6_tie_timing.jsonl 2>&1 || exit 1
cat gpurun_out/r6_jv_clock.txt gpurun_out/r6_tie_probe.txt gpurun_out/r6_tie_timing.jsonl
