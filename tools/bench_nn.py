#!/usr/bin/env python
"""Kernel benchmark: StrongSort's NN gallery cosine distance (bx_nn_cosine_distance) at the C4
geometry (BASELINE.json configs[3]: 1024 targets x 512 detections x 2048-d, gallery of S samples
per target, budget 150).  Inputs resident in HBM, the gallery kept normalised
(BX_NN_SAMPLES_NORMALIZED, as an engine would store it) or raw; HIP events on the launch
stream.  Prints one JSON line per S with the achieved fp64 TFLOP/s of the contraction."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets", type=int, default=1024)
    ap.add_argument("--dets", type=int, default=512)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--samples", type=int, nargs="+", default=[1, 10, 50, 150])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--raw", action="store_true", help="normalise the gallery inside the op")
    ap.add_argument("--peak", type=float, default=78.6, help="fp64 matrix peak, TFLOP/s")
    a = ap.parse_args()
    import torch

    from boxmot_amd import _native as N

    L = N.load()
    dev = torch.device("cuda", 0)
    T, D, F = a.targets, a.dets, a.dim
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    feats = torch.randn(D, F, generator=g, device=dev, dtype=torch.float64)
    out = torch.empty(T, D, device=dev, dtype=torch.float64)
    st = torch.cuda.current_stream()
    for S in a.samples:
        G = T * S
        gal = torch.randn(G, F, generator=g, device=dev, dtype=torch.float64)
        if not a.raw:
            gal /= gal.norm(dim=1, keepdim=True) + 1e-8
        off = torch.arange(0, G + 1, S, device=dev, dtype=torch.int32)
        flags = 0 if a.raw else 1

        def run():
            N.check(L.bx_nn_cosine_distance(gal.data_ptr(), G, off.data_ptr(), T, feats.data_ptr(),
                                            D, F, flags, out.data_ptr(), st.cuda_stream), "nn")
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        flop = 2.0 * G * D * F
        tf = flop / (ms * 1e-3) / 1e12
        print(json.dumps({"op": "bx_nn_cosine_distance", "targets": T, "samples_per_target": S,
                          "dets": D, "dim": F, "gallery_normalised": not a.raw,
                          "ms": round(ms, 4), "gflop": round(flop / 1e9, 2),
                          "tflops_fp64": round(tf, 2), "mfma_frac": round(tf / a.peak, 3)}),
              flush=True)
        del gal


if __name__ == "__main__":
    main()
