"""BoostTrack / BoostTrack++ on the MI355X engine — drop-in for
boxmot.trackers.boosttrack.boosttrack.BoostTrack (reference trackers/boosttrack/boosttrack.py:123-341).

Same constructor, same ``update(dets, img, embs)`` contract and output rows.  Per frame the engine
runs the ReID contraction ``dets_embs @ trk_embs.T`` on the fp64 matrix cores, then one wave per
sequence for CMC warp + Kalman predict, the DLO/DUO confidence boosts, the IoU / Mahalanobis /
shape / ReID cost, the one-to-one fast path or lapx JV, validation, Kalman updates, births and
deaths, then the embedding EMA (include/bxboost.h).

Differences from the reference, by design:
* ReID features are inputs: ``with_reid`` needs ``embs`` (the reference would run its ReID model
  on ``img``; the model zoo is out of the engine's scope).  Embeddings are used as float64 (the
  dtype ``boxmot eval`` loads them in); float32 inputs are widened.
* Camera motion: ``self.cmc.apply(img, dets)`` supplies the 2x3 warp like the reference, but the
  default ``cmc`` is the identity (OpenCV ECC estimation from images is out of scope); assign an
  object with ``apply(img, dets) -> (2, 3)`` to feed real warps.
"""
from __future__ import annotations

import numpy as np

from ..engine import BoostEngine, BoostParams
from .basetracker import BaseTracker, CapacityGuard, _with_index, class_warps


def _boost_warp(w) -> np.ndarray:
    """camera_update's transform (boosttrack.py:243-246): a 2x3 or 3x3 affine, as 2x3."""
    w = np.asarray(w, np.float64)
    if w.shape == (3, 3):
        w = w[:2]
    if w.shape != (2, 3):
        raise ValueError(f"Expected 2x3 or 3x3 matrix, got {w.shape}")
    return w


class IdentityCMC:
    """2x3 identity warp (what a static camera's ECC estimate is)."""

    def apply(self, img, dets=None):
        return np.eye(2, 3)


class BoostTrack(BaseTracker):
    # KalmanBoxTracker.count is class-global and never reset by BoostTrack (boosttrack.py:50,
    # 53-56): every instance continues the same id sequence.
    _id_count = 0

    def __init__(self, reid_weights=None, device=None, half: bool = False, max_age: int = 60,
                 min_hits: int = 3, det_thresh: float = 0.6, iou_threshold: float = 0.3,
                 use_ecc: bool = True, min_box_area: int = 10,
                 aspect_ratio_thresh: float = 1.6, cmc_method: str = "ecc",
                 lambda_iou: float = 0.5, lambda_mhd: float = 0.25, lambda_shape: float = 0.25,
                 use_dlo_boost: bool = True, use_duo_boost: bool = True,
                 dlo_boost_coef: float = 0.65, s_sim_corr: bool = False,
                 use_rich_s: bool = False, use_sb: bool = False, use_vt: bool = False,
                 with_reid: bool = False, per_class: bool = False, track_cap: int = 256,
                 det_cap: int = 256):
        super().__init__(per_class=per_class)
        self._out_ids = {}  # class call -> ids of the trackers it output (its active_tracks)
        self.frame_count = 0
        self.max_age = max_age
        self.min_hits = min_hits
        self.det_thresh = det_thresh
        self.iou_threshold = iou_threshold
        self.use_ecc = use_ecc
        self.min_box_area = min_box_area
        self.aspect_ratio_thresh = aspect_ratio_thresh
        self.cmc_method = cmc_method
        self.lambda_iou = lambda_iou
        self.lambda_mhd = lambda_mhd
        self.lambda_shape = lambda_shape
        self.use_dlo_boost = use_dlo_boost
        self.use_duo_boost = use_duo_boost
        self.dlo_boost_coef = dlo_boost_coef
        self.s_sim_corr = s_sim_corr
        self.use_rich_s = use_rich_s
        self.use_sb = use_sb
        self.use_vt = use_vt
        self.with_reid = with_reid
        self.cmc = IdentityCMC() if use_ecc else None
        self._params = BoostParams(
            max_age=max_age, min_hits=min_hits, det_thresh=det_thresh,
            iou_threshold=iou_threshold, use_ecc=use_ecc, min_box_area=min_box_area,
            aspect_ratio_thresh=aspect_ratio_thresh, lambda_iou=lambda_iou,
            lambda_mhd=lambda_mhd, lambda_shape=lambda_shape, use_dlo_boost=use_dlo_boost,
            use_duo_boost=use_duo_boost, dlo_boost_coef=dlo_boost_coef, s_sim_corr=s_sim_corr,
            use_rich_s=use_rich_s, use_sb=use_sb, use_vt=use_vt, with_reid=with_reid)
        self._cap = CapacityGuard()
        self._caps = (track_cap, det_cap)
        self.engine = None if with_reid else self._make_engine(0)
        self._engine_ids = 0

    def _make_engine(self, emb_dim):
        return BoostEngine(n_seq=1, track_cap=self._caps[0], det_cap=self._caps[1],
                           emb_dim=emb_dim, params=self._params)

    @BaseTracker.setup_decorator
    @BaseTracker.per_class_decorator
    def update(self, dets: np.ndarray, img: np.ndarray, embs: np.ndarray = None) -> np.ndarray:
        self.check_inputs(dets, img, embs)
        if self.with_reid and embs is None and len(dets):
            raise ValueError("BoostTrack with_reid on the engine needs precomputed embeddings")
        if self.engine is None:  # with_reid: the embedding dimension arrives with the first frame
            if embs is None or not len(dets):
                # nothing can be associated before the first embeddings; the reference's
                # frame counter still advances and its CMC still sees the frame (a stateful CMC
                # keeps it as the previous image), with no tracker to warp
                if self.cmc is not None:
                    if self.per_class:
                        class_warps(self.cmc, img, dets, self.nr_classes, _boost_warp)
                    else:
                        self.cmc.apply(img, _with_index(dets))
                self.frame_count += 1
                self._pending_frames = getattr(self, "_pending_frames", 0) + 1
                return np.empty((0, 8))
            self.engine = self._make_engine(int(np.asarray(embs).shape[1]))
            for _ in range(getattr(self, "_pending_frames", 0)):
                self.engine.update_host(0, np.empty((0, 6), np.float32),
                                        np.empty((0, self.engine.emb_dim)))
        n = int(np.asarray(dets).reshape(-1, 6).shape[0])
        self.engine = self._cap.fit(self.engine, {0: n}, n)
        if self._engine_ids != BoostTrack._id_count:
            self.engine.set_id_count(0, BoostTrack._id_count)
        self.frame_count += 1
        warp = None
        if self.per_class:  # every class call sees every track (D10; basetracker.py:155-201)
            # cmc.apply runs once per class call (boosttrack.py:243-246), each warp applied to
            # every tracker
            warps = None if self.cmc is None else class_warps(self.cmc, img, dets,
                                                              self.nr_classes, _boost_warp)
            out = self.engine.update_classes_host(0, dets, embs if self.with_reid else None,
                                                  warps, n_classes=self.nr_classes)
        else:
            if self.cmc is not None:
                warp = _boost_warp(self.cmc.apply(img, _with_index(dets)))
            out = self.engine.update_host(0, dets, embs if self.with_reid else None, warp)
        self._engine_ids = BoostTrack._id_count = self.engine.counters(0)["id_count"]
        # active_tracks = the trackers a call output (boosttrack.py:320-329); an output row's
        # class is its call's class (only trackers updated or born in the call are output)
        if self.per_class:
            self._out_ids = {c: out[out[:, 6] == c, 4].astype(np.int64) for c in
                             np.unique(out[:, 6]).astype(np.int64)}
        else:
            self._out_ids = {0: out[:, 4].astype(np.int64)}
        return out if out.shape[0] else np.empty((0, 8))

    def _output_trackers(self, c):
        ids = self._out_ids.get(c)
        if ids is None or not len(ids):
            return []
        # the reference keeps the tracker objects a class call output even when a later class
        # call of the same frame drops them (D10: every call predicts every tracker, so a tracker
        # unmatched for max_age calls dies mid-frame); those come back with no live state
        by_id = {int(t["id"]): t for t in self.trackers}
        return [by_id.get(int(i), {"id": np.int32(i), "x": None, "P": None}) for i in ids]

    @property
    def active_tracks(self):
        """The trackers the last update output (per_class: the last class call's)."""
        return self._output_trackers(self.nr_classes - 1 if self.per_class else 0)

    def _class_active_lists(self):
        return [self._output_trackers(c) for c in range(self.nr_classes)]

    @property
    def trackers(self):
        """Track list snapshot (list order): ids, Kalman state x [8], P [8, 8] (+ emb)."""
        if self.engine is None:
            return []
        snap = self.engine.tracks(0)
        keys = [k for k in ("id", "x", "P", "emb") if k in snap]
        return [dict(zip(keys, vals)) for vals in zip(*(snap[k] for k in keys))]
