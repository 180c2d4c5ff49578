"""Drop-in engines grow instead of failing (VERDICT r2 Missing 3 / What's weak 8).

The reference's track and detection lists are unbounded (bytetrack.py:272-346,
sort/tracker.py:118-181, sort/track.py:98-105); the engines have fixed slot arenas.  Each drop-in
checks before a frame that its slots in use plus the frame's detections fit and otherwise moves
the tracker state into an engine with twice the capacity (bx_*_copy_state).  These tests start
from tiny capacities so the growth happens many times mid-sequence, and require every frame to
stay bitwise equal to the oracle."""
import os

import numpy as np
import pytest

from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a HIP device")
    from boxmot_amd import _native

    _native.load()
    return torch


CASES = [
    ("bytetrack", dict(min_conf=0.1, track_thresh=0.6, match_thresh=0.9, track_buffer=30),
     dict(n_obj=70, seed=61, layout="crowded", conf_lo=0.05)),
    ("botsort", dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8),
     dict(n_obj=60, seed=62, layout="crowded", emb_dim=32, conf_lo=0.05)),
    ("ocsort", dict(det_thresh=0.6, max_age=30, min_hits=3, inertia=0.1),
     dict(n_obj=60, seed=63, layout="crowded", conf_lo=0.3)),
    ("boosttrack", dict(max_age=60, min_hits=3, det_thresh=0.6, with_reid=True),
     dict(n_obj=50, seed=64, layout="crowded", emb_dim=32, emb_dtype=np.float64, conf_lo=0.3)),
]


def make(kind, args, caps, per_class=False):
    from boxmot_amd import BoostTrack, BotSort, ByteTrack, OcSort

    a = dict(args, per_class=per_class, **caps)
    if kind == "bytetrack":
        ByteTrack.clear_count()
        return ByteTrack(**a)
    if kind == "ocsort":
        return OcSort(**a)
    if kind == "boosttrack":
        BoostTrack._id_count = 0
        return BoostTrack(reid_weights=None, device="cuda", half=False, **a)
    return BotSort(reid_weights=None, device="cuda", half=False, **a)


@pytest.mark.parametrize("per_class", [False, True], ids=["single", "per_class"])
@pytest.mark.parametrize("kind,args,skw", CASES, ids=[c[0] for c in CASES])
def test_dropin_grows_bitwise(native, kind, args, skw, per_class):
    from boxmot_amd.synth import SyntheticScene

    if per_class:
        skw = dict(skw, classes=(0, 2, 5))
    tr = make(kind, args, dict(track_cap=8, det_cap=4), per_class)
    orc = po.OracleTracker(kind, **dict(args, per_class=per_class))
    sc = SyntheticScene(**skw)
    img = np.zeros((1080, 1920, 3), np.uint8)
    for t in range(1, 41):
        d, e, _ = sc.frame(t)
        o = tr.update(d, img, e) if e is not None else tr.update(d, img)
        oo = orc.update(d, e)
        np.testing.assert_array_equal(np.asarray(o, np.float64).reshape(-1, 8), oo,
                                      err_msg=f"{kind} frame {t}")
    assert tr.engine.track_cap > 8 and tr.engine.det_cap > 4  # it did grow


def test_strongsort_tentative_accumulation_grows(native):
    """StrongSort outside CI: tracks are born Tentative and, in this fork, never leave the list
    (SURVEY App. A D8), so they accumulate past the default 512 slots (876 after 300 frames of
    this 6-object scene); the drop-in grows and stays bitwise equal to the oracle
    (born_confirmed=False) for 300 frames.  (The StrongSort engine's ceiling is 1024 slots: its
    LSAP state is sized for them; past it the drop-in raises.)"""
    from boxmot_amd import StrongSort
    from boxmot_amd.synth import SyntheticScene

    old = {k: os.environ.pop(k, None) for k in ("GITHUB_ACTIONS", "GITHUB_JOB")}
    try:
        args = dict(min_conf=0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50, n_init=2,
                    nn_budget=100)
        tr = StrongSort(reid_weights=None, device="cuda", half=False, handle_occlusions=False,
                        **args)
        orc = po.OracleTracker("strongsort", born_confirmed=False, **args)
        sc = SyntheticScene(n_obj=6, seed=65, emb_dim=32, emb_dtype=np.float64, conf_lo=0.2)
        img = np.zeros((1080, 1920, 3), np.uint8)
        for t in range(1, 301):
            d, e, _ = sc.frame(t)
            o = np.asarray(tr.update(d, img, e), np.float64).reshape(-1, 10)
            oo = orc.update(d, e).reshape(-1, 10)
            np.testing.assert_array_equal(o, oo, err_msg=f"frame {t}")
        assert tr.engine.track_cap > 512, tr.engine.track_cap
    finally:
        for k, v in old.items():
            if v is not None:
                os.environ[k] = v
