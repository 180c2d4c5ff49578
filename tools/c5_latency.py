#!/usr/bin/env python
"""C5 at one sequence per launch (configs[4]'s one-sequence-per-GPU shape): for each of the eight
boosttrack_mot8 sequences (the LPT shard a rank of an 8-GPU job gets), the per-frame latency of
one BoostEngine step on its own (host-synchronised every frame) and the back-to-back rate without
the per-frame sync, over the bench's timed frames (14-63).  Prints one JSON line per sequence."""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from boxmot_amd.workloads import BenchFrames, bench_engine  # noqa: E402

dev = torch.device("cuda:0")
first, last = 14, 63
for k in range(8):
    src = BenchFrames("boosttrack_mot8", 1, dev, rank=k, world=8)
    frames = [src.frame(t) for t in range(1, last + 1)]
    max_n = max(int(f[1][-1].item()) for f in frames)
    out = torch.empty((max(max_n, 1), 8), dtype=torch.float64, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    res = {"sequence": [int(g) for g in src.mine]}
    for mode in ("sync", "stream"):
        eng, _ = bench_engine("boosttrack_mot8", 1)
        st = torch.cuda.current_stream()
        for t in range(first - 1):
            d, off, e = frames[t]
            eng.step(d, off, e, None, out, cnt, stream=st.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(first - 1, last):
            d, off, e = frames[t]
            eng.step(d, off, e, None, out, cnt, stream=st.cuda_stream)
            if mode == "sync":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        res[f"ms_per_frame_{mode}"] = round((time.perf_counter() - t0) / (last - first + 1) * 1e3, 4)
        eng.close()
    res["dets_mean"] = round(float(sum(int(f[1][-1]) for f in frames[first - 1:]) /
                                   (last - first + 1)), 1)
    print(json.dumps(res), flush=True)
