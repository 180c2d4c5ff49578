timeout -k 10 240 python tools/ss_phases.py --no-build --frames 30 > gpurun_out/r6d_phases.txt 2>&1; grep -E "lsap|fast|slow" gpurun_out/r6d_phases.txt
