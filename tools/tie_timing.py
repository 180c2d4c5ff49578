#!/usr/bin/env python
"""Cost of the LAP tie path: a tied optimum is re-solved by lapx's own
JV on the (R+C)^2 cost_limit extension, on one wave with its state in HBM.

1. BoT-SORT at C3 sizes (256 objects, ~128 detections, 512-d) on the crowded layout, with and
   without duplicated detections (every 3rd emitted twice: a detector without NMS; every such
   frame's first association ties): ms per step and the number of re-solved LAPs.
2. bx_linear_assignment_ex on fully tied problems (all costs equal, below the threshold) up to the
   documented size limit (8192): the re-solve's time.
Prints one JSON line per measurement."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def c3_dups(S, frames, dup_every):
    import torch

    from boxmot_amd.engine import Engine, EngineParams
    from boxmot_amd.synth import SyntheticScene
    from boxmot_amd.workloads import CONFIGS

    _, n_obj, F, params = CONFIGS["botsort"]
    scenes = [SyntheticScene(n_obj=n_obj, seed=3000 + s, emb_dim=F, layout="crowded",
                             dup_every=dup_every) for s in range(S)]
    eng = Engine("botsort", n_seq=S, track_cap=512, det_cap=384, emb_dim=F,
                 params=EngineParams(**params))
    inputs = []
    for t in range(1, frames + 1):
        fr = [sc.frame(t) for sc in scenes]
        off = np.zeros(S + 1, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in fr])
        inputs.append((torch.from_numpy(np.concatenate([f[0] for f in fr]).astype(np.float32)).cuda(),
                       torch.from_numpy(off).cuda(),
                       torch.from_numpy(np.concatenate([f[1] for f in fr])).cuda()))
    out = torch.empty((max(int(i[1][-1]) for i in inputs), 8), dtype=torch.float64, device="cuda")
    cnt = torch.empty(S, dtype=torch.int32, device="cuda")
    warm = frames // 3
    for k in range(warm):
        eng.step(*inputs[k], None, out, cnt)
    torch.cuda.synchronize()
    t0, ties0 = time.perf_counter(), eng.lap_ties()
    for k in range(warm, frames):
        eng.step(*inputs[k], None, out, cnt)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / (frames - warm) * 1e3
    assert eng.status() == 0
    return {"what": "botsort crowded C3 sizes", "seqs": S, "dup_every": dup_every,
            "ms_per_step": round(ms, 4), "lap_ties_timed": eng.lap_ties() - ties0,
            "timed_frames": frames - warm}


def lap_tied(n, reps=3):
    import torch

    from boxmot_amd import _native as N

    L = N.load()
    c = torch.full((n, n), 0.5, dtype=torch.float64, device="cuda")
    x = torch.empty(n, dtype=torch.int32, device="cuda")
    y = torch.empty(n, dtype=torch.int32, device="cuda")
    t = torch.zeros(1, dtype=torch.int32, device="cuda")
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        N.check(L.bx_linear_assignment_ex(c.data_ptr(), n, n, 0.8, x.data_ptr(), y.data_ptr(),
                                          t.data_ptr(), None))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return {"what": "bx_linear_assignment_ex all-equal costs", "n": n, "tied": int(t.item()),
            "ms": round(best * 1e3, 3)}


def main():
    for dup in (0, 3):
        print(json.dumps(c3_dups(128, 30, dup)), flush=True)
    for n in (64, 128, 256, 512):
        print(json.dumps(lap_tied(n)), flush=True)


if __name__ == "__main__":
    main()
