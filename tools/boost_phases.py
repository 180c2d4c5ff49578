#!/usr/bin/env python
"""Diagnostic: per-phase cycle shares of the BoostTrack frame kernel from s_memtime stamps.

Builds boxmot_amd/lib/libbxassoc_timing.so with -DBX_PHASE_TIMING (separate diagnostic build),
runs the bench's BoostTrack workload and prints per-frame mean cycles per phase (over sequences
and frames) plus the assignment counters.
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
PHASES = ["load", "warp+predict", "DLO", "DUO", "keep+colsum", "cost", "fastpath/LAP",
          "validate", "updates", "births", "outputs+deaths"]
COUNTERS = ["LAP calls", "LAP n", "kept dets", "tracks", "frames", "LAP calls n > 64", "LAP tied (lapjv ran)", "-",
            "JV free rows", "JV scans", "JV relax steps", "JV sequential scans",
            "JV64 setup (ccrrt+ARR) cyc", "JV64 find cyc", "JV64 scan cyc", "JV64 writeout cyc",
            "JV64 find events", "JV64 scan events", "JV64 path steps", "JV64 ARR iterations",
            "JV64 row init cyc", "JV64 v update cyc", "JV64 path cyc", "JV64 loop top cyc"]


def build():
    from boxmot_amd import _native as N

    cmd = ["/opt/rocm/bin/hipcc", *N.HIPCC_FLAGS, "-DBX_PHASE_TIMING", "-o", str(LIB),
           *[str(N.CSRC / s) for s in N.SOURCES]]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--no-build", action="store_true")
    ap.add_argument("--c5", action="store_true", help="the boosttrack_mot8 sequences (MOT dets)")
    ap.add_argument("--lib", default=None, help="a timing build of tools/build_variant.py")
    a = ap.parse_args()
    if not a.no_build:
        build()
    os.environ["BX_LIB_PATH"] = a.lib or str(LIB)
    import torch

    from bench import CONFIGS, OCS_CONF_LO
    from boxmot_amd import _native as N
    from boxmot_amd.engine import BoostEngine, BoostParams
    from boxmot_amd.synth import TorchSceneBatch

    kind, n_obj, F, params = CONFIGS["boosttrack_mot8" if a.c5 else "boosttrack"]
    if a.c5:  # bench.py's C5 frames: MOT17-02/04 public detections + 6 synthetic sequences
        from bench import MOT_DETS
        from boxmot_amd.synth import c5_sequences

        seqs = c5_sequences(MOT_DETS, F)
        a.seqs = len(seqs)
        a.frames = min(a.frames, min(nf for _, _, nf in seqs))

        def c5_frame(t):
            fr = [sc.frame(t) for _, sc, _ in seqs]
            off = np.zeros(a.seqs + 1, np.int32)
            off[1:] = np.cumsum([f[0].shape[0] for f in fr])
            d = np.concatenate([f[0] for f in fr], 0).astype(np.float32)
            e = np.concatenate([f[1] for f in fr], 0).astype(np.float64)
            return (torch.from_numpy(d).cuda(), torch.from_numpy(off).cuda(),
                    torch.from_numpy(e).cuda())

        frames = [c5_frame(t) for t in range(1, a.frames + 1)]
        dmax = max(int((f[1][1:] - f[1][:-1]).max().item()) for f in frames)
        eng = BoostEngine(n_seq=a.seqs, track_cap=256, det_cap=max(64, dmax), emb_dim=F,
                          params=BoostParams(**params))
        n_obj = dmax
    else:
        eng = BoostEngine(n_seq=a.seqs, track_cap=128, det_cap=max(64, n_obj), emb_dim=F,
                          params=BoostParams(**params))
        gen = TorchSceneBatch(a.seqs, n_obj, emb_dim=F, seed=7, device="cuda",
                              conf_lo=OCS_CONF_LO)
        frames = [(d, o, e.double()) for d, o, e in (gen.frame(t) for t in range(1, a.frames + 1))]
    L = N.load()
    L.bx_boost_debug_host.argtypes = [C.c_void_p, C.c_void_p]
    out = torch.empty((a.seqs * n_obj, 8), dtype=torch.float64, device="cuda")
    cnt = torch.empty(a.seqs, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for d, off, e in frames:
        eng.step(d, off, e, None, out, cnt)
    torch.cuda.synchronize()
    dbg = np.zeros((a.seqs, 40), np.uint64)
    N.check(L.bx_boost_debug_host(eng._h, dbg.ctypes.data), "debug")
    per = dbg.astype(np.float64) / a.frames
    tot = per[:, :len(PHASES)].sum(1)
    print(f"boosttrack: {a.seqs} seqs x {a.frames} frames: cycles/frame mean {tot.mean():.0f} "
          f"max {tot.max():.0f}")
    for k, name in enumerate(PHASES):
        col = per[:, k]
        print(f"  {name:16s} mean {col.mean():10.0f} max {col.max():10.0f} "
              f"share {100 * col.mean() / tot.mean():5.1f}%")
    lap = PHASES.index("fastpath/LAP")
    for q in range(a.seqs):
        calls = max(dbg[q, 16], 1)
        print(f"  seq {q}: cycles/frame {tot[q]:9.0f}  LAP {per[q, lap]:9.0f}  LAP calls {dbg[q, 16]:5d} "
              f"mean n {dbg[q, 17] / calls:6.1f}  n > 64: {dbg[q, 21]:4d}  JV64 scans+relax {dbg[q, 25] + dbg[q, 26]:7d}")
    cs = dbg[:, 16:16 + len(COUNTERS)].astype(np.float64).sum(0)
    for k, name in enumerate(COUNTERS):
        if name != "-":
            print(f"  {name:20s} total {cs[k]:.0f}")


if __name__ == "__main__":
    main()
