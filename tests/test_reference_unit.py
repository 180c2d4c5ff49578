"""The reference's tracker unit tests (tests/unit/test_trackers.py:27-281) re-expressed for every
tracker on the MI355X engine, through the drop-ins and ``create_tracker`` like the reference.

Where the reference's own test cannot pass on the fork, the test states the
fork's behaviour as the oracle restates it instead of the test's expectation, and says so:
* StrongSort crashes on frame 1 (D5) and never confirms a track outside CI (D8): it runs here with
  the minimal patch P6 and ``GITHUB_ACTIONS=true`` (born Confirmed, as the reference's CI runs it),
  and its rows have 10 columns (strongsort.py ``_format_outputs``: + quality, occlusion);
* BoostTrack's per-class mode shares its tracker list across classes (D10), so two overlapping
  detections of different classes get one id, exactly as the reference;
* OCSort's "same id twice" fails on the fork (D3, UnboundLocalError); with P3 it passes.
Every output is also compared bitwise with the oracle on the same inputs.
"""
from pathlib import Path

import numpy as np
import pytest
import yaml

from oracle import pyoracle as po

pytestmark = pytest.mark.gpu

ALL_TRACKERS = ["botsort", "ocsort", "bytetrack", "strongsort", "boosttrack"]
PER_CLASS_TRACKERS = ["botsort", "ocsort", "bytetrack", "boosttrack"]
APPEARANCE = ["botsort", "strongsort", "boosttrack"]
WEIGHTS = Path("weights")  # never read: ReID inference is outside the association path


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a HIP device")
    from boxmot_amd import _native

    _native.load()
    return torch


@pytest.fixture(autouse=True)
def _ci_env(monkeypatch):
    # the reference's CI environment (sort/track.py:98-105): StrongSort tracks born Confirmed
    monkeypatch.setenv("GITHUB_ACTIONS", "true")
    monkeypatch.delenv("GITHUB_JOB", raising=False)


def yaml_args(name):
    from boxmot_amd import get_tracker_config

    return {k: v["default"] for k, v in yaml.safe_load(open(get_tracker_config(name))).items()}


def make(name, per_class=False):
    """create_tracker exactly as the reference's tests call it, plus the oracle with the same
    YAML defaults.  Class-global id counters are reset so the two start together."""
    from boxmot_amd import BoostTrack, ByteTrack, create_tracker, get_tracker_config

    ByteTrack.clear_count()
    BoostTrack._id_count = 0
    tr = create_tracker(tracker_type=name, tracker_config=get_tracker_config(name),
                        reid_weights=WEIGHTS / "mobilenetv2_x1_4_dukemtmcreid.pt", device="cpu",
                        half=False, per_class=per_class)
    args = yaml_args(name)
    if name == "strongsort":
        args.update(handle_occlusions=True, born_confirmed=True)
    else:
        args["per_class"] = per_class
    if name == "ocsort":  # the drop-in latches the image size for centroid-style asso_funcs
        args.update(frame_w=640, frame_h=640)
    return tr, po.OracleTracker(name, **args)


def step(name, tr, orc, det, img, embs):
    uses_embs = name in APPEARANCE
    out = tr.update(det, img, embs) if uses_embs else tr.update(det, img)
    ref = orc.update(det if det is not None and len(det) else np.empty((0, 6)),
                     embs if uses_embs else None)
    w = 10 if name == "strongsort" else 8
    got = np.asarray(out, np.float64).reshape(-1, w) if np.asarray(out).size else np.empty((0, w))
    np.testing.assert_array_equal(got, np.asarray(ref, np.float64).reshape(-1, w), err_msg=name)
    return out


def test_motion_n_appearance_trackers_instantiation(torch_cuda):
    """test_trackers.py:27-34 (DeepOcSort is not on the engine)."""
    from boxmot_amd import BoostTrack, BotSort, StrongSort

    for T in (StrongSort, BotSort, BoostTrack):
        T(reid_weights=WEIGHTS / "osnet_x0_25_msmt17.pt", device="cpu", half=True)


def test_motion_only_trackers_instantiation(torch_cuda):
    """test_trackers.py:37-39."""
    from boxmot_amd import ByteTrack, OcSort

    OcSort()
    ByteTrack()


@pytest.mark.parametrize("name", ALL_TRACKERS)
def test_tracker_output_size(torch_cuda, name):
    """test_trackers.py:42-58: two detections in, two rows out."""
    tr, orc = make(name)
    rgb = np.random.randint(255, size=(640, 640, 3), dtype=np.uint8)
    det = np.array([[144, 212, 400, 480, 0.82, 0], [425, 281, 576, 472, 0.72, 65]])
    embs = np.random.default_rng(0).random((2, 512))
    out = step(name, tr, orc, det, rgb, embs)
    assert out.shape == (2, 10 if name == "strongsort" else 8)


def test_dynamic_max_obs_based_on_max_age(torch_cuda):
    """test_trackers.py:61-64 (and BoostTrack's BaseTracker defaults)."""
    from boxmot_amd import BoostTrack, OcSort

    assert OcSort(max_age=400).max_obs == 405
    assert OcSort(max_age=30).max_obs == 50
    # BoostTrack passes only per_class to BaseTracker (boosttrack.py:182): its max_obs stays the
    # default 50 whatever max_age is
    assert BoostTrack(max_age=400).max_obs == 50


@pytest.mark.parametrize("qxy,qs", [(0.05, 0.0005), (0.01, 0.0001)])
def test_Q_matrix_scaling(torch_cuda, qxy, qs):
    """test_trackers.py:90-118 for OcSort: the process noise the engine's predict adds is
    Q[4,4] = Q[5,5] = Q_xy_scaling and Q[6,6] = Q_s_scaling — read back as
    P_pred - F P F^T over one predict of a fresh track (ocsort.py:73-96; F constant velocity)."""
    from boxmot_amd import OcSort

    tr = OcSort(Q_xy_scaling=qxy, Q_s_scaling=qs)
    img = np.zeros((640, 640, 3), np.uint8)
    tr.update(np.array([[0, 0, 100, 100, 0.9, 1]], np.float64), img)
    P0 = tr.active_tracks[0]["P"].copy()
    tr.update(np.empty((0, 6)), img)  # predict only: the unmatched update leaves P alone
    P1 = tr.active_tracks[0]["P"]
    F = np.eye(7)
    F[0, 4] = F[1, 5] = F[2, 6] = 1.0
    Q = P1 - F @ P0 @ F.T
    np.testing.assert_allclose([Q[4, 4], Q[5, 5], Q[6, 6]], [qxy, qxy, qs], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(np.diag(Q)[:4], [1.0, 1.0, 1.0, 1.0], rtol=1e-9)


@pytest.mark.parametrize("name", PER_CLASS_TRACKERS)
def test_per_class_tracker_output_size(torch_cuda, name):
    """test_trackers.py:121-143: per_class, second frame, two rows."""
    tr, orc = make(name, per_class=True)
    rgb = np.random.randint(255, size=(640, 640, 3), dtype=np.uint8)
    det = np.array([[100, 100, 300, 250, 0.95, 0], [400, 300, 550, 450, 0.90, 65]])
    embs = np.random.default_rng(1).random((2, 512))
    step(name, tr, orc, det, rgb, embs)
    out = step(name, tr, orc, det, rgb, embs)
    assert out.shape == (2, 8)


@pytest.mark.parametrize("name", PER_CLASS_TRACKERS)
def test_per_class_tracker_active_tracks(torch_cuda, name):
    """test_trackers.py:146-165: after one per_class update classes 0 and 65 hold a track, and no
    other class does."""
    tr, orc = make(name, per_class=True)
    rgb = np.random.randint(255, size=(640, 640, 3), dtype=np.uint8)
    det = np.array([[100, 100, 300, 250, 0.95, 0], [400, 300, 550, 450, 0.90, 65]])
    embs = np.random.default_rng(2).random((2, 512))
    assert not any(tr.per_class_active_tracks.values())
    out = step(name, tr, orc, det, rgb, embs)
    pcat = tr.per_class_active_tracks
    assert pcat[0], f"No active tracks for class 0 (rows {out[:, [4, 6]].tolist()})"
    assert pcat[65], "No active tracks for class 65"
    assert all(not v for c, v in pcat.items() if c not in (0, 65))
    ids = lambda v: sorted(int(t["id"] if isinstance(t, dict) else t.id) for t in v)  # noqa: E731
    if name != "ocsort":  # OCSort rows carry id + 1 (ocsort.py:430)
        assert ids(pcat[0] + pcat[65]) == sorted(int(i) for i in out[:, 4])
    else:
        assert ids(pcat[0] + pcat[65]) == sorted(int(i) - 1 for i in out[:, 4])
    assert not make(name)[0].per_class_active_tracks  # None without per_class


@pytest.mark.parametrize("name", ALL_TRACKERS)
@pytest.mark.parametrize("dets", [None, np.array([])], ids=["none", "empty"])
def test_tracker_with_no_detections(torch_cuda, name, dets):
    """test_trackers.py:168-185."""
    tr, orc = make(name)
    rgb = np.random.randint(255, size=(640, 640, 3), dtype=np.uint8)
    embs = np.random.random(size=(0, 512))
    out = tr.update(dets, rgb, embs)
    assert out.size == 0, "Output should be empty when no detections are provided"
    assert orc.update(np.empty((0, 6)), embs if name in APPEARANCE else None).size == 0


@pytest.mark.parametrize("name", PER_CLASS_TRACKERS)
def test_per_class_isolation(torch_cuda, name):
    """test_trackers.py:188-208: two overlapping boxes of different classes get two ids — except
    BoostTrack, whose per-class calls share one tracker list in the reference (D10): the class-2
    box updates the track the class-1 box started, so one id, as the oracle restates."""
    tr, orc = make(name, per_class=True)
    det = np.array([[100, 100, 150, 150, 0.9, 1], [102, 102, 152, 152, 0.9, 2]])
    rgb = np.zeros((640, 640, 3), dtype=np.uint8)
    embs = np.random.default_rng(3).random((2, 512))
    out = step(name, tr, orc, det, rgb, embs)
    ids = set(out[:, 4].tolist())
    assert len(ids) == (1 if name == "boosttrack" else 2)


@pytest.mark.parametrize("name", APPEARANCE)
def test_emb_trackers_requires_embeddings(torch_cuda, name):
    """test_trackers.py:211-226: detections and embeddings must pair up."""
    tr, _ = make(name)
    det = np.array([[10, 10, 20, 20, 0.7, 0]])
    rgb = np.zeros((640, 640, 3), dtype=np.uint8)
    with pytest.raises(AssertionError):
        tr.update(det, rgb, np.random.rand(2, 512))


@pytest.mark.parametrize("name", ALL_TRACKERS)
def test_invalid_det_array_shape(torch_cuda, name):
    """test_trackers.py:229-242."""
    tr, _ = make(name)
    img = np.zeros((640, 640, 3), dtype=np.uint8)
    with pytest.raises(AssertionError):
        tr.update(np.random.rand(2, 5), img, np.random.rand(2, 512))


@pytest.mark.parametrize("name", ALL_TRACKERS)
def test_track_id_stable_over_frames(torch_cuda, name):
    """test_trackers.py:251-281: the same detection twice keeps its id (column 4)."""
    tr, orc = make(name)
    det = np.array([[50, 50, 100, 100, 0.95, 3]])
    rgb = np.zeros((640, 640, 3), dtype=np.uint8)
    embs = np.random.default_rng(4).random((1, 512))
    out1 = step(name, tr, orc, det, rgb, embs)
    out2 = step(name, tr, orc, det, rgb, embs)
    w = 10 if name == "strongsort" else 8
    assert out1.shape == out2.shape == (1, w), "Unexpected output shape"
    assert out1[0, 4] == out2[0, 4], "Track ID should remain the same across frames"
