"""Host-side logic that needs no GPU: registry, configs, synthetic generator, oracle baseline."""
import numpy as np
import pytest
import yaml

from boxmot_amd import get_tracker_config
from boxmot_amd.synth import SyntheticScene
from boxmot_amd.tracker_zoo import create_tracker


def test_yaml_defaults_match_reference():
    # reference configs/trackers/{bytetrack,botsort}.yaml `default`s
    bt = {k: v["default"] for k, v in yaml.safe_load(open(get_tracker_config("bytetrack"))).items()}
    assert bt == {"min_conf": 0.1, "track_thresh": 0.6, "track_buffer": 30, "match_thresh": 0.9,
                  "frame_rate": 30}
    bs = {k: v["default"] for k, v in yaml.safe_load(open(get_tracker_config("botsort"))).items()}
    assert bs == {"track_high_thresh": 0.6, "track_low_thresh": 0.1, "new_track_thresh": 0.7,
                  "track_buffer": 30, "match_thresh": 0.8, "proximity_thresh": 0.5,
                  "appearance_thresh": 0.25, "cmc_method": "ecc"}


def test_unknown_tracker_raises_keyerror(capsys):
    with pytest.raises(KeyError):
        create_tracker("not_a_tracker", evolve_param_dict={})
    assert "No such tracker" in capsys.readouterr().out


def test_ocsort_yaml_defaults_reach_the_engine(monkeypatch):
    """create_tracker('ocsort') passes the YAML defaults to the OcSort constructor; without a GPU
    building the engine fails loudly (no CPU fallback)."""
    import boxmot_amd._native as N
    from boxmot_amd.trackers import ocsort as mod

    seen = {}

    class Probe:
        def __init__(self, **kw):
            seen.update(kw)
            raise N.NativeUnavailable("no device")

    monkeypatch.setattr(mod, "OcsortEngine", Probe)
    with pytest.raises(N.NativeUnavailable):
        create_tracker("ocsort")
    p = seen["params"]
    assert (p.det_thresh, p.max_age, p.min_hits, p.delta_t, p.inertia, p.use_byte) == \
        (0.6, 30, 3, 3, 0.1, False)
    assert (p.min_conf, p.Q_xy_scaling, p.Q_s_scaling, p.asso_threshold) == (0.1, 0.01, 1e-4, 0.3)


@pytest.mark.parametrize("name", ["deepocsort", "hybridsort"])
def test_not_yet_on_engine(name):
    with pytest.raises(NotImplementedError):
        create_tracker(name, evolve_param_dict={})


def test_boosttrack_yaml_defaults_match_reference_constructor_names():
    """configs/trackers/boosttrack.yaml keys are BoostTrack.__init__ parameters (plugin path)."""
    import inspect

    import yaml

    from boxmot_amd import BoostTrack, get_tracker_config

    cfg = yaml.safe_load(open(get_tracker_config("boosttrack")))
    params = inspect.signature(BoostTrack.__init__).parameters
    assert set(cfg) <= set(params)
    d = {k: v["default"] for k, v in cfg.items()}
    assert d["use_rich_s"] and d["use_sb"] and d["use_vt"] and d["with_reid"]  # BoostTrack++
    assert (d["max_age"], d["min_hits"], d["det_thresh"]) == (60, 3, 0.6)


def test_synthetic_scene_is_deterministic_per_frame():
    a = SyntheticScene(n_obj=50, seed=3, emb_dim=16)
    b = SyntheticScene(n_obj=50, seed=3, emb_dim=16)
    for t in (1, 7, 40):
        da, ea, ia = a.frame(t)
        db, eb, ib = b.frame(t)
        np.testing.assert_array_equal(da, db)
        np.testing.assert_array_equal(ea, eb)
        np.testing.assert_array_equal(ia, ib)
    d, e, _ = a.frame(5)
    assert d.shape[1] == 6 and e.dtype == np.float32
    np.testing.assert_allclose(np.linalg.norm(e, axis=1), 1.0, rtol=1e-6)


def test_oracle_multi_sequence_is_independent():
    from oracle import pyoracle as po

    sc = SyntheticScene(n_obj=30, seed=9)
    t1, t2 = po.OracleTracker("bytetrack", track_thresh=0.6), po.OracleTracker("bytetrack", track_thresh=0.6)
    for t in range(1, 20):
        d, _, _ = sc.frame(t)
        np.testing.assert_array_equal(t1.update(d), t2.update(d))


def test_with_index_empty_inputs():
    """The detection-index column appended before a CMC call, on empty frames in every shape
    the trackers can pass (a 1-D np.array([]) included)."""
    from boxmot_amd.trackers.basetracker import _with_index

    assert _with_index(np.array([])).shape == (0, 7)
    assert _with_index(np.zeros((0, 6))).shape == (0, 7)
    d = _with_index(np.ones((3, 6)))
    assert d.shape == (3, 7) and list(d[:, 6]) == [0, 1, 2]
