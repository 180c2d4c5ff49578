import os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
os.environ["GITHUB_ACTIONS"] = "true"
from boxmot_amd import StrongSort
from boxmot_amd.synth import SyntheticScene
skw = dict(n_obj=24, seed=42, layout="corner", emb_dim=32, emb_dtype=np.float64, conf_lo=0.3,
           p_det=0.8, corner=((30, .9), (55, .9), (95, .9), (160, .9)))
img = np.zeros((1080, 1920, 3), np.uint8)
for occ in (False, True):
    for vc in (32, 64):
        sc = SyntheticScene(**skw)
        tr = StrongSort(handle_occlusions=occ, vec_cap=vc)
        try:
            for t in range(1, 81):
                d, e, _ = sc.frame(t)
                tr.update(d, img, e)
            print(occ, vc, "ok")
        except Exception as ex:
            print(occ, vc, "fail at", t, ex)
