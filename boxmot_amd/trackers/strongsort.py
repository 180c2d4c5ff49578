"""StrongSort (the fork's "enhanced" tracker) on the MI355X engine — drop-in for
boxmot.trackers.strongsort.strongsort.StrongSort (reference trackers/strongsort/strongsort.py:17-345).

Same constructor, same ``update(dets, img, embs)`` contract and output rows ([M, 10]: x1, y1, x2,
y2, id, conf, cls, det_ind, track quality, occlusion level).  Per frame the engine runs the
detection-feature kernel, the NN-gallery cosine distance on the fp64 matrix cores, the recovery
similarities and one wave per sequence for everything else (include/bxstrongsort.h).

Differences from the reference, by design or because the fork cannot run otherwise
(SURVEY.md Appendix A):
* the fork crashes on frame 1 (D5); the engine applies the minimal patch P6;
* ``handle_occlusions`` (default True, as the reference): the OcclusionAwareTracker post-process
  (utils/occlusion_handler.py:312-439) runs on the host over the engine's track state
  (``boxmot_amd.occlusion``) and raises TypeError where the reference crashes on mutual
  occlusion (D7); with False the occlusion column is 0;
* tracks are born Confirmed when ``GITHUB_ACTIONS=true`` (and GITHUB_JOB is not the MOT
  benchmark), Tentative otherwise — read from the environment like the reference (D8);
* ReID features are inputs (``embs`` required, used as float64).  CMC: ``self.cmc.apply(img,
  dets)`` supplies the 2x3 warp, identity by default.
"""
from __future__ import annotations

import os

import numpy as np

from ..engine import SsEngine, SsParams
from ..occlusion import OcclusionHandler
from .basetracker import BaseTracker, CapacityGuard
from .boosttrack import IdentityCMC


def _born_confirmed() -> bool:
    # sort/track.py:98-105
    return (os.getenv("GITHUB_ACTIONS") == "true"
            and os.getenv("GITHUB_JOB") != "mot-metrics-benchmark")


class StrongSort:
    def __init__(self, reid_weights=None, device=None, half: bool = False, per_class: bool = False,
                 min_conf: float = 0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50,
                 n_init=2, nn_budget=150, mc_lambda=0.995, ema_alpha=0.9, conf_thresh_high=0.7,
                 conf_thresh_low=0.3, id_preservation_weight=0.1, adaptive_matching=True,
                 appearance_weight=0.6, motion_weight=0.4, occlusion_threshold=0.3,
                 handle_occlusions=True, crowd_detection=True, track_cap: int = 512,
                 det_cap: int = 256, vec_cap: int = 64):
        if per_class:
            # create_tracker pops per_class for StrongSort (tracker_zoo.py:84-85); constructed
            # directly with per_class=True the reference fails in its first update (StrongSort
            # never runs BaseTracker.__init__, so the decorator's nr_classes does not exist)
            raise NotImplementedError("StrongSort has no per-class mode (the reference's "
                                      "create_tracker drops per_class for it)")
        self.per_class = per_class
        self.min_conf = min_conf
        self.conf_thresh_high = conf_thresh_high
        self.conf_thresh_low = conf_thresh_low
        self.id_preservation_weight = id_preservation_weight
        self.adaptive_matching = adaptive_matching
        self.appearance_weight = appearance_weight
        self.motion_weight = motion_weight
        self.handle_occlusions = handle_occlusions
        self.crowd_detection = crowd_detection
        self.occlusion_threshold = occlusion_threshold
        self.frame_count = 0
        self.cmc = IdentityCMC()
        self._params = SsParams(
            min_conf=min_conf, max_cos_dist=max_cos_dist, max_iou_dist=max_iou_dist,
            max_age=max_age, n_init=n_init, nn_budget=nn_budget, mc_lambda=mc_lambda,
            ema_alpha=ema_alpha, conf_thresh_high=conf_thresh_high,
            conf_thresh_low=conf_thresh_low, id_preservation_weight=id_preservation_weight,
            crowd_detection=crowd_detection, born_confirmed=_born_confirmed())
        self._cap = CapacityGuard()
        self._caps = (track_cap, det_cap, vec_cap)
        self.engine = None
        self._pending = 0
        self.occlusion_tracker = None  # OcclusionHandler, created with the engine
        self.occlusion_stats = {}

    @BaseTracker.per_class_decorator
    def update(self, dets: np.ndarray, img: np.ndarray, embs: np.ndarray = None) -> np.ndarray:
        assert isinstance(dets, np.ndarray), (
            f"Unsupported 'dets' input format '{type(dets)}', valid format is np.ndarray")
        assert isinstance(img, np.ndarray), (
            f"Unsupported 'img' input format '{type(img)}', valid format is np.ndarray")
        assert len(dets.shape) == 2, "Unsupported 'dets' dimensions, valid number of dimensions is two"
        assert dets.shape[1] == 6, "Unsupported 'dets' 2nd dimension lenght, valid lenghts is 6"
        if embs is not None:
            assert dets.shape[0] == embs.shape[0], "Missmatch between detections and embeddings sizes"
        if embs is None and np.any(dets[:, 4] >= self.min_conf):
            raise ValueError("StrongSort on the engine needs precomputed embeddings")
        self.frame_count += 1
        if self.engine is None:
            if embs is None:  # nothing to associate yet; the engine is sized by the first embs
                self._pending += 1
                return np.array([])
            tc, dc, vc = self._caps
            self.engine = SsEngine(n_seq=1, track_cap=tc, det_cap=dc,
                                   emb_dim=int(np.asarray(embs).shape[1]), vec_cap=vc,
                                   params=self._params)
            for _ in range(self._pending):  # replay the empty frames (predict + bookkeeping)
                self.engine.update_host(0, np.empty((0, 6)), np.empty((0, self.engine.emb_dim)))
            if self.handle_occlusions:
                self.occlusion_tracker = OcclusionHandler(self.engine, 0, self.occlusion_threshold)
        eng = self._cap.fit(self.engine, {0: dets.shape[0]}, dets.shape[0])
        if eng is not self.engine:  # grown: the occlusion handler reads the new engine
            self.engine = eng
            if self.occlusion_tracker is not None:
                self.occlusion_tracker.engine = eng
        warp = None
        if self.cmc is not None:
            warp = np.asarray(self.cmc.apply(img, dets[:, :4]), np.float64)
            warp = warp[:2] if warp.shape == (3, 3) else warp
        e = embs if embs is not None else np.empty((dets.shape[0], self.engine.emb_dim))
        out = self.engine.update_host(0, dets, e, warp)
        if self.occlusion_tracker is not None:  # strongsort.py:150-154, 195-201
            out = self.occlusion_tracker(self.frame_count, out)
            if np.any(dets[:, 4] >= self.min_conf):  # not refreshed by the no-detection branch
                self.occlusion_stats = self.occlusion_tracker.statistics()
        return out if out.shape[0] else np.array([])

    def reset(self):
        if self.engine is not None:
            self.engine.reset()
        self.frame_count = 0
        self._cap = CapacityGuard()

    @property
    def tracks(self):
        if self.engine is None:
            return []
        snap = self.engine.tracks(0)
        return [dict(id=int(i), state=int(s), mean=m, covariance=c)
                for i, s, m, c in zip(snap["id"], snap["state"], snap["mean"], snap["covariance"])]
