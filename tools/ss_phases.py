#!/usr/bin/env python
"""Diagnostic: per-phase cycle shares of the StrongSort frame kernel from s_memtime stamps.

Builds boxmot_amd/lib/libbxassoc_timing.so with -DBX_PHASE_TIMING (separate diagnostic build),
runs a bench StrongSort workload (``--config strongsort`` or ``strongsort_c4``) and prints mean
cycles per frame per phase (s_memtime counts shader clocks, ~2.4 GHz: 2400 cycles ~ 1 us) plus the
assignment counters.
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
PHASES = ["setup", "crowd", "camera+quality+sort+predict", "lists", "stage1 cascade",
          "stage2 cascade", "stage3 iou", "updates+misses", "recovery", "births", "deaths",
          "partial_fit", "masks+outputs"]
COUNTERS = ["cost build cyc", "lsap cyc", "lsap calls", "sum rows (tracks)", "sum cols (dets)",
            "dijkstra steps", "matches", "solver rows R", "solver cols CC", "slow rows",
            "slow-row cyc", "lsap loop cyc", "pre: detection quality cyc",
            "pre: detection sort cyc", "(unused)", "(unused)", "sum R x CC", "calls R*CC*8 > 64 KiB",
            "rows in those calls", "lsap cyc in those calls", "fast: contested rows",
            "fast: certificate row expansions", "fast: certificate candidates",
            "fast: (A) minima + claims cyc", "fast: (C) contested searches cyc",
            "fast: (D) certificate cyc", "fast: (D) rows rescanned",
            "sparse (A): list check cyc", "sparse (A): tables cyc", "sparse (A): minima cyc",
            "sparse (A): claims cyc"]


def build():
    from boxmot_amd import _native as N

    cmd = ["/opt/rocm/bin/hipcc", *N.HIPCC_FLAGS, "-DBX_PHASE_TIMING", "-o", str(LIB),
           *[str(N.CSRC / s) for s in N.SOURCES]]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="strongsort_c4")
    ap.add_argument("--seqs", type=int, default=None)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--no-build", action="store_true")
    ap.add_argument("--lib", default=None, help="a timing build of tools/build_variant.py")
    a = ap.parse_args()
    if not a.no_build:
        build()
    os.environ["BX_LIB_PATH"] = a.lib or str(LIB)
    import torch

    from bench import CONFIGS, DEFAULT_SEQS, OCS_CONF_LO
    from boxmot_amd import _native as N
    from boxmot_amd.engine import SsEngine, SsParams
    from boxmot_amd.synth import TorchSceneBatch

    kind, n_obj, F, params = CONFIGS[a.config]
    S = a.seqs or DEFAULT_SEQS.get(a.config, 1)
    eng = SsEngine(n_seq=S, track_cap=min(1024, max(96, 2 * n_obj)),
                   det_cap=min(1024, max(64, n_obj)), emb_dim=F, vec_cap=64,
                   params=SsParams(**params))
    gen = TorchSceneBatch(S, n_obj, emb_dim=F, seed=1000, device="cuda", conf_lo=OCS_CONF_LO)
    L = N.load()
    L.bx_ss_debug_host.argtypes = [C.c_void_p, C.c_void_p]
    out = torch.empty((S * n_obj, 10), dtype=torch.float64, device="cuda")
    cnt = torch.empty(S, dtype=torch.int32, device="cuda")
    for t in range(1, a.frames + 1):
        d, off, e = gen.frame(t)
        eng.step(d.double(), off, e.double(), None, out, cnt)
        torch.cuda.synchronize()
    dbg = np.zeros((S, 48), np.uint64)
    N.check(L.bx_ss_debug_host(eng._h, dbg.ctypes.data), "debug")
    per = dbg.astype(np.float64) / a.frames
    tot = per[:, :len(PHASES)].sum(1)
    print(f"{a.config}: {S} seqs x {a.frames} frames: cycles/frame mean {tot.mean():.0f} "
          f"max {tot.max():.0f} (~2400 cycles = 1 us)")
    for k, name in enumerate(PHASES):
        col = per[:, k]
        print(f"  {name:28s} mean {col.mean():11.0f} max {col.max():11.0f} "
              f"share {100 * col.mean() / max(tot.mean(), 1):5.1f}%")
    cs = per[:, 16:16 + len(COUNTERS)].mean(0)
    for k, name in enumerate(COUNTERS):
        print(f"  {name:20s} per frame {cs[k]:.1f}")


if __name__ == "__main__":
    main()
