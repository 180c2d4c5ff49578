#!/usr/bin/env python
"""Diagnostic: StrongSort batched scenes (test_strongsort_batched_vs_oracle's default variant) on
the library BX_LIB_PATH names; prints the first frame whose rows differ from the oracle and the
engine status then (a -DSS_TAB_VERIFY build latches 9001/9002 when the first-step table disagrees
with a re-derivation)."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    import torch

    from boxmot_amd.engine import SsEngine, SsParams
    from boxmot_amd.synth import SyntheticScene
    from oracle import pyoracle as po

    args = dict(min_conf=0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50, n_init=2,
                nn_budget=150, mc_lambda=0.995, ema_alpha=0.9, conf_thresh_high=0.7,
                conf_thresh_low=0.3, id_preservation_weight=0.1, crowd_detection=True,
                born_confirmed=True)
    kw = dict(emb_dim=48, emb_dtype=np.float64, conf_lo=0.15)
    scenes = [SyntheticScene(n_obj=16 + 8 * s, seed=800 + s, layout="crowded" if s % 2 else "grid",
                             **kw) for s in range(4)]
    S = len(scenes)
    eng = SsEngine(n_seq=S, track_cap=256, det_cap=256, emb_dim=48, vec_cap=32,
                   params=SsParams(**args))
    orcs = [po.OracleTracker("strongsort", **args) for _ in range(S)]
    for t in range(1, 51):
        fr = [sc.frame(t) for sc in scenes]
        off = np.zeros(S + 1, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in fr])
        out = torch.empty((int(off[-1]) + 1, 10), dtype=torch.float64, device="cuda")
        cnt = torch.empty(S, dtype=torch.int32, device="cuda")
        eng.step(torch.from_numpy(np.concatenate([f[0] for f in fr])).cuda(),
                 torch.from_numpy(off).cuda(),
                 torch.from_numpy(np.concatenate([f[1] for f in fr])).cuda(), None, out, cnt)
        torch.cuda.synchronize()
        o, c = out.cpu().numpy(), cnt.cpu().numpy()
        bad = []
        for s in range(S):
            ref = orcs[s].update(fr[s][0], fr[s][1])
            got = o[off[s]: off[s] + c[s]]
            if got.shape != ref.shape or not np.array_equal(got, ref):
                bad.append(s)
        st = eng.status()
        print(f"frame {t}: status {st} mismatched seqs {bad}", flush=True)
        if bad or st:
            break


if __name__ == "__main__":
    main()
