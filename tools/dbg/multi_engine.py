#!/usr/bin/env python
"""Experiment: the C3 workload (botsort, 1024 sequences) split over G engines of 1024/G sequences,
each stepped on its own stream (so the G frame pipelines interleave on the GPU).  Prints
ms/step for G = 1 and the requested G.  Usage: multi_engine.py [G ...]"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from boxmot_amd.workloads import BenchFrames, bench_engine  # noqa: E402


def run(G, S=1024, warm=10, steps=50):
    dev = torch.device("cuda", 0)
    src = BenchFrames("botsort", S, dev)
    frames = [src.frame(t) for t in range(1, warm + steps + 1)]
    per = S // G
    engs = [bench_engine("botsort", per)[0] for _ in range(G)]
    streams = [torch.cuda.Stream() for _ in range(G)]
    max_n = max(int(f[1][-1].item()) for f in frames)
    out = torch.empty((max_n, 8), dtype=torch.float64, device=dev)
    cnt = torch.empty(S, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def step(k):
        d, off, e = frames[k]
        for g in range(G):
            c0, c1 = g * per, (g + 1) * per
            engs[g].step(d, off[c0:c1 + 1], e, None, out, cnt[c0:c1], seq0=0, nseq=per,
                         stream=streams[g].cuda_stream)

    for k in range(warm):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        step(k)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    for e in engs:
        assert e.status() == 0
    print(f"G={G}: {ms:.4f} ms/step  {S / ms * 1e3:.0f} frames/s", flush=True)


if __name__ == "__main__":
    for g in [1] + [int(x) for x in sys.argv[1:]]:
        run(g)
