#!/usr/bin/env python
"""Where the LAP tie path's time goes: the op-level lapx JV alone (bx_lapjv with
cost_limit: the (R+C)^2 extension) against bx_linear_assignment_ex (sparse SSP + certificate,
then the same JV on a tie), on all-equal costs and on a crowded IoU matrix with every third
detection duplicated.  One JSON line per measurement."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def crowd(seed=1, nt=256, nd=128):
    rng = np.random.default_rng(seed)

    def boxes(k):
        xy = rng.uniform(0, 1000, (k, 2))
        return np.hstack([xy, xy + rng.uniform(30, 80, (k, 2))])

    T = boxes(nt)
    D = T[rng.choice(nt, nd, replace=False)] + rng.normal(0, 5, (nd, 4))
    D = np.vstack([np.repeat(D[i:i + 1], 2 if i % 3 == 0 else 1, 0) for i in range(nd)])
    x1 = np.maximum(T[:, None, 0], D[None, :, 0]); y1 = np.maximum(T[:, None, 1], D[None, :, 1])
    x2 = np.minimum(T[:, None, 2], D[None, :, 2]); y2 = np.minimum(T[:, None, 3], D[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    ar = lambda z: (z[:, 2] - z[:, 0]) * (z[:, 3] - z[:, 1])
    return 1.0 - inter / (ar(T)[:, None] + ar(D)[None, :] - inter)


def timed(fn, reps=3):
    import torch
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return round(best * 1e3, 3)


def main():
    import torch

    from boxmot_amd import _native as N
    L = N.load()
    cases = [("equal", np.full((n, n), 0.5)) for n in (128, 256, 512)] + [("crowd", crowd())]
    for name, c in cases:
        nr, nc = c.shape
        ct = torch.from_numpy(c).cuda()
        x = torch.empty(nr + nc, dtype=torch.int32, device="cuda")
        y = torch.empty(nr + nc, dtype=torch.int32, device="cuda")
        t = torch.zeros(1, dtype=torch.int32, device="cuda")
        ms_jv = timed(lambda: N.check(L.bx_lapjv(ct.data_ptr(), nr, nc, 1, 0.8, x.data_ptr(),
                                                 y.data_ptr(), None)))
        xj = x[:nr].cpu().numpy().copy()
        ms_ex = timed(lambda: N.check(L.bx_linear_assignment_ex(
            ct.data_ptr(), nr, nc, 0.8, x.data_ptr(), y.data_ptr(), t.data_ptr(), None)))
        print(json.dumps({"case": name, "nr": nr, "nc": nc, "lapjv_ms": ms_jv,
                          "linear_assignment_ex_ms": ms_ex, "tied": int(t.item()),
                          "jv_rows_matched": int((xj >= 0).sum())}), flush=True)


if __name__ == "__main__":
    main()
