"""Debug: per-frame track-state diff GPU engine vs oracle on a StrongSort fixture."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import pyoracle as po  # noqa: E402
from tests.golden_util import fixture_frames, fixture_tracker_args  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "churn24_s2"
fx = np.load(ROOT / "tests" / "golden" / f"trk_strongsort_{name}.npz")
kind, args = fixture_tracker_args(fx)
args = dict(args, born_confirmed=True)
from boxmot_amd.engine import SsEngine, SsParams  # noqa: E402

keys = SsParams.__dataclass_fields__.keys()
orc = po.OracleTracker("strongsort", **args)
eng = None
for f, d, e in fixture_frames(fx):
    if eng is None:
        eng = SsEngine(n_seq=1, track_cap=256, det_cap=256, emb_dim=e.shape[1], vec_cap=64,
                       params=SsParams(**{k: v for k, v in args.items() if k in keys}))
    o = eng.update_host(0, d, e)
    oo = orc.update(d, e)
    g = eng.tracks(0)
    n = po.lib().bxo_ss_tracks(orc.h, 0, None, None, None, None)
    ids = np.zeros(n, np.int32); st = np.zeros(n, np.int32); mean = np.zeros((n, 8))
    po.lib().bxo_ss_tracks(orc.h, n, ids.ctypes.data, st.ctypes.data, mean.ctypes.data, None)
    same = (len(g["id"]) == n and np.array_equal(g["id"], ids) and np.array_equal(g["state"], st)
            and np.array_equal(g["mean"], mean))
    print(f"frame {f}: out {o.shape[0]} vs {oo.shape[0]} eq={np.array_equal(o, oo)} tracks "
          f"{len(g['id'])} vs {n} same={same}")
    if not same:
        print(" gpu ids", g["id"].tolist(), "st", g["state"].tolist())
        print(" orc ids", ids.tolist(), "st", st.tolist())
        if len(g["id"]) == n:
            dm = np.abs(g["mean"] - mean).max(1)
            print(" mean diff per track", dm.tolist())
        break
