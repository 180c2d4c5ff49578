#!/usr/bin/env python
"""Diagnostic: host enqueue time of bench.py's steps vs the GPU time they take (is the frame
loop launch-bound?).  Usage: enqueue_rate.py [config] [steps]"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from boxmot_amd.workloads import BenchFrames, bench_engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "botsort"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
S = 1024
dev = torch.device("cuda:0")
src = BenchFrames(cfg, S, dev)
eng, _ = bench_engine(cfg, S)
frames = [src.frame(t) for t in range(1, 2 * K + 12)]
max_n = max(int(f[1][-1].item()) for f in frames)
out = torch.empty((max_n, 8), dtype=torch.float64, device=dev)
cnt = torch.empty(S, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream()
for k in range(10):
    d, off, e = frames[k]
    eng.step(d, off, e, None, out, cnt, stream=st.cuda_stream)
torch.cuda.synchronize()
res = {}
for rep in range(2):
    t0 = time.perf_counter()
    marks = []
    for k in range(10 + rep * K, 10 + (rep + 1) * K):
        d, off, e = frames[k]
        eng.step(d, off, e, None, out, cnt, stream=st.cuda_stream)
        marks.append(time.perf_counter() - t0)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    res[f"rep{rep}"] = {"enqueue_us_per_step": round(t_enq / K * 1e6, 1),
                        "gpu_us_per_step": round(t_all / K * 1e6, 1),
                        "enqueue_marks_us": [round(m * 1e6) for m in marks[:8]]}
print(json.dumps(res))
