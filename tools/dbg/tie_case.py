"""Debug: the (150, 300) rep-2 tie case — lapx via bx_lapjv (LDS state) on the extension, square
on the explicit extension, and bx_linear_assignment_ex (global-state fallback) vs the oracle."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import pyoracle as po  # noqa: E402
from tests.test_gpu_parity import gpu_lapjv, gpu_linear_assignment, tie_heavy_costs  # noqa: E402

shape = (150, 300)
rng = np.random.default_rng(sum(shape) * 7919 + shape[0])
for rep in range(3):
    c, thr = tie_heavy_costs(rng, shape, rep)
nr, nc = shape
ox, oy = po.lapjv(c, extend_cost=True, cost_limit=thr)
gx, gy = gpu_lapjv(torch, c, extend_cost=True, cost_limit=thr)
print("bx_lapjv limit mode == oracle:", np.array_equal(gx, ox), np.array_equal(gy, oy))
n = nr + nc
E = np.full((n, n), thr / 2.0)
E[nr:, nc:] = 0
E[:nr, :nc] = c
ex, ey = po.lapjv(E)
sx, sy = gpu_lapjv(torch, E)
print("bx_lapjv square == oracle:", np.array_equal(sx, ex), np.array_equal(sy, ey))
print("oracle limit vs square:", np.array_equal(np.where(ex[:nr] >= nc, -1, ex[:nr]), ox))
om, oua, oub = po.linear_assignment(c, thr)
t = []
gm, gua, gub = gpu_linear_assignment(torch, c, thr, t)
print("linear_assignment == oracle:", np.array_equal(gm, om), np.array_equal(gua, oua),
      np.array_equal(gub, oub), "tied", t)
d = np.flatnonzero(gx != ox)
print("x diffs", d[:10], gx[d[:10]], ox[d[:10]])
