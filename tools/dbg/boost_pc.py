"""Debug: BoostTrack per-class active-track views vs output rows."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from boxmot_amd import BoostTrack, create_tracker  # noqa: E402

BoostTrack._id_count = 0
tr = create_tracker("boosttrack", None, None, "cuda", False, True)
det = np.array([[100, 100, 300, 250, 0.95, 0], [400, 300, 550, 450, 0.90, 65]])
e = np.random.default_rng(2).random((2, 512))
out = tr.update(det, np.zeros((640, 640, 3), np.uint8), e)
print("out", out[:, [4, 6]].tolist())
print("out_ids", tr._out_ids)
print("trackers", [int(t["id"]) for t in tr.trackers])
snap = tr.engine.tracks(0)
print("snap", snap["id"])
