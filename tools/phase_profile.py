#!/usr/bin/env python
"""Diagnostic: per-phase cycle shares of the association kernel (K3) from s_memtime stamps.

Builds boxmot_amd/lib/libbxassoc_timing.so with -DBX_PHASE_TIMING (a separate diagnostic build;
the stamps' barriers forbid overlaps the real kernel has, so read SHARES, not totals), runs the
bench workload and prints the mean / max cycles per phase over all sequences of the last frame.
"""
import argparse
import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
LIB = ROOT / "boxmot_amd" / "lib" / "libbxassoc_timing.so"
PHASES = ["dets split", "lists", "-", "assoc1 CSR+costs", "assoc1 LAP", "assoc1 records",
          "assoc2 CSR", "assoc2 LAP+records", "assoc3 CSR", "assoc3 LAP", "assoc3 rec+new",
          "expiry+lists+writeback"]


def build():
    from boxmot_amd import _native as N

    cmd = ["/opt/rocm/bin/hipcc", *N.HIPCC_FLAGS, "-DBX_PHASE_TIMING", "-o", str(LIB),
           *[str(N.CSRC / s) for s in N.SOURCES]]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="botsort")
    ap.add_argument("--seqs", type=int, default=256)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--no-build", action="store_true")
    a = ap.parse_args()
    if not a.no_build:
        build()
    os.environ["BX_LIB_PATH"] = str(LIB)
    import torch

    from bench import CONFIGS
    from boxmot_amd import _native as N
    from boxmot_amd.engine import Engine, EngineParams
    from boxmot_amd.synth import TorchSceneBatch

    kind, n_obj, F, params = CONFIGS[a.config]
    eng = Engine(kind, n_seq=a.seqs, track_cap=512, det_cap=256, emb_dim=F,
                 params=EngineParams(**params))
    layout = "crowded" if a.config.endswith("_crowded") else "grid"
    gen = TorchSceneBatch(a.seqs, n_obj, emb_dim=F, seed=7, device="cuda", layout=layout)
    L = N.load()
    L.bx_debug_stamps_host.argtypes = [C.c_void_p, C.c_void_p]
    out = torch.empty((a.seqs * n_obj, 8), dtype=torch.float64, device="cuda")
    cnt = torch.empty(a.seqs, dtype=torch.int32, device="cuda")
    for t in range(1, a.frames + 1):
        d, off, e = gen.frame(t)
        eng.step(d, off, e, None, out, cnt)
    torch.cuda.synchronize()
    st = np.zeros((a.seqs, 64), np.uint64)
    L.bx_debug_stamps_host(eng._h, st.ctypes.data)
    st = st.astype(np.int64)
    d = np.diff(st[:, :13], axis=1)
    tot = st[:, 12] - st[:, 0]
    print(f"{a.config}: {a.seqs} seqs, frame {a.frames}: total cycles mean {tot.mean():.0f} "
          f"max {tot.max():.0f}")
    sub = [("row boxes", 3, 20), ("pass1 count", 20, 21), ("scan", 21, 22), ("pass2 emit", 22, 23),
           ("pass3 costs", 23, 4)]
    for name, a0, a1 in sub:
        dd = st[:, a1] - st[:, a0]
        if (st[:, a1] > 0).all():
            print(f"    assoc1 {name:12s} mean {dd.mean():10.0f}  max {dd.max():10.0f}")
    ne = st[:, 24]
    if ne.any():
        print(f"    assoc1 edges mean {ne.mean():.1f} max {ne.max()}  rows {st[:, 25].mean():.1f}")
    if st[:, 28].any():
        print(f"    assoc1 LAP: dijkstra roots mean {st[:, 26].mean():.1f} max {st[:, 26].max()}, "
              f"steps mean {st[:, 27].mean():.1f} max {st[:, 27].max()}, rows {st[:, 28].mean():.1f}")
        pre = st[:, 29] - st[:, 4]
        print(f"    assoc1 LAP init+fast path mean {pre.mean():.0f}, dijkstra mean "
              f"{(st[:, 5] - st[:, 29]).mean():.0f}")
        print(f"    assoc1 LAP components mean {st[:, 30].mean():.1f}, max rows/component "
              f"mean {st[:, 31].mean():.1f} max {st[:, 31].max()}, label iters mean "
              f"{st[:, 32].mean():.1f} max {st[:, 32].max()}")
        print(f"    assoc1 LAP labels {(st[:, 34] - st[:, 29]).mean():.0f}, lane solves "
              f"{(st[:, 35] - st[:, 34]).mean():.0f}, rest {(st[:, 33] - st[:, 35]).mean():.0f}, "
              f"after {(st[:, 5] - st[:, 33]).mean():.0f}")
    for k, name in enumerate(PHASES):
        print(f"  {name:18s} mean {d[:, k].mean():10.0f}  max {d[:, k].max():10.0f}  "
              f"share {d[:, k].mean() / tot.mean() * 100:5.1f}%")


if __name__ == "__main__":
    main()
