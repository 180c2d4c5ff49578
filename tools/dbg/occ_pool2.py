import os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
os.environ["GITHUB_ACTIONS"] = "true"
from boxmot_amd import StrongSort
from boxmot_amd.synth import SyntheticScene
img = np.zeros((1080, 1920, 3), np.uint8)
for pd, lay in ((0.8, "grid"), (1.0, "grid"), (0.9, "crowded")):
    sc = SyntheticScene(n_obj=24, seed=3, layout=lay, emb_dim=64, emb_dtype=np.float64,
                        conf_lo=0.3, p_det=pd)
    tr = StrongSort(handle_occlusions=False, vec_cap=64)
    try:
        for t in range(1, 601):
            d, e, _ = sc.frame(t)
            tr.update(d, img, e)
        print(pd, lay, "ok 600")
    except Exception as ex:
        print(pd, lay, "fail at", t, ex)
