#!/usr/bin/env python
"""Diagnostic: per-phase cycle shares of the OCSort frame kernel from s_memtime stamps.

Builds boxmot_amd/lib/libbxassoc_timing.so with -DBX_PHASE_TIMING (separate diagnostic build),
runs the bench's OCSort workload and prints per-frame mean cycles per phase (over sequences and
frames) plus the assignment counters.
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
PHASES = ["load+splits", "predict", "costs1", "fastpath/LAP1", "validate+updates1", "BYTE",
          "OCR costs", "OCR LAP+updates", "none updates+births", "outputs+deaths"]
COUNTERS = ["LAP1 calls", "LAP1 n", "BYTE LAPs", "OCR LAPs", "OCR n", "tracks", "high dets",
            "frames", "JV free rows", "JV scans", "JV relax steps", "JV sequential scans"]


def build():
    from boxmot_amd import _native as N

    cmd = ["/opt/rocm/bin/hipcc", *N.HIPCC_FLAGS, "-DBX_PHASE_TIMING", "-o", str(LIB),
           *[str(N.CSRC / s) for s in N.SOURCES]]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ocsort")
    ap.add_argument("--seqs", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--no-build", action="store_true")
    a = ap.parse_args()
    if not a.no_build:
        build()
    os.environ["BX_LIB_PATH"] = str(LIB)
    import torch

    from bench import CONFIGS, OCS_CONF_LO
    from boxmot_amd import _native as N
    from boxmot_amd.engine import OcsortEngine, OcsortParams
    from boxmot_amd.synth import TorchSceneBatch

    kind, n_obj, F, params = CONFIGS[a.config]
    eng = OcsortEngine(n_seq=a.seqs, track_cap=max(64, 2 * n_obj), det_cap=max(64, n_obj),
                       params=OcsortParams(**params))
    gen = TorchSceneBatch(a.seqs, n_obj, seed=7, device="cuda", conf_lo=OCS_CONF_LO)
    L = N.load()
    L.bx_ocsort_debug_host.argtypes = [C.c_void_p, C.c_void_p]
    out = torch.empty((a.seqs * n_obj, 8), dtype=torch.float64, device="cuda")
    cnt = torch.empty(a.seqs, dtype=torch.int32, device="cuda")
    frames = [gen.frame(t) for t in range(1, a.frames + 1)]
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for d, off, _ in frames:
        eng.step(d, off, out, cnt)
    ev1.record()
    torch.cuda.synchronize()
    print(f"kernel time per frame (all sequences, timing build): "
          f"{ev0.elapsed_time(ev1) / a.frames:.3f} ms")
    dbg = np.zeros((a.seqs, 40), np.uint64)
    N.check(L.bx_ocsort_debug_host(eng._h, dbg.ctypes.data), "debug")
    per = dbg.astype(np.float64) / a.frames
    tot = per[:, :len(PHASES)].sum(1)
    print(f"{a.config}: {a.seqs} seqs x {a.frames} frames: cycles/frame mean {tot.mean():.0f} "
          f"max {tot.max():.0f}")
    for k, name in enumerate(PHASES):
        col = per[:, k]
        print(f"  {name:22s} mean {col.mean():10.0f} max {col.max():10.0f} "
              f"share {100 * col.mean() / tot.mean():5.1f}%")
    cs = dbg[:, 16:16 + 8].astype(np.float64).sum(0)
    js = dbg[:, 24:28].astype(np.float64).sum(0)
    vals = list(cs) + list(js)
    for name, v in zip(COUNTERS, vals):
        print(f"  {name:16s} total {v:12.0f}  per seq-frame {v / (a.seqs * a.frames):8.2f}")


if __name__ == "__main__":
    main()
