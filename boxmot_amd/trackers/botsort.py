"""BoT-SORT on the MI355X engine — drop-in for boxmot.trackers.botsort.botsort.BotSort
(reference trackers/botsort/botsort.py:27-411).

Same constructor signature (``reid_weights``, ``device``, ``half`` are accepted for
compatibility), same ``update(dets, img, embs)`` contract.  Out of scope and therefore required
as inputs: the ReID embeddings (``embs``; the reference would run its ReID backend when they are
missing) and the camera-motion warp — ``self.cmc.apply(img, dets)`` must return a 2x3 affine
(identity by default; the reference's OpenCV ECC/ORB/SIFT/SOF estimators are image processing
outside the association path).
"""
from __future__ import annotations

import numpy as np

from ..engine import Engine, EngineParams
from .basetracker import BaseTracker, CapacityGuard, _with_index, class_warps


class IdentityCMC:
    def apply(self, img, dets=None):
        return np.eye(2, 3)


def _xywh_box(mean):
    r = mean[:4]
    return np.array([r[0] - r[2] / 2, r[1] - r[3] / 2, r[0] + r[2] / 2, r[1] + r[3] / 2])


class BotSort(BaseTracker):
    def __init__(self, reid_weights=None, device=None, half: bool = False,
                 per_class: bool = False, track_high_thresh: float = 0.5,
                 track_low_thresh: float = 0.1, new_track_thresh: float = 0.6,
                 track_buffer: int = 30, match_thresh: float = 0.8,
                 proximity_thresh: float = 0.5, appearance_thresh: float = 0.25,
                 cmc_method: str = "ecc", frame_rate=30, fuse_first_associate: bool = False,
                 with_reid: bool = True, track_cap: int = 1024, det_cap: int = 384):
        super().__init__(per_class=bool(per_class))
        self.track_high_thresh = track_high_thresh
        self.track_low_thresh = track_low_thresh
        self.new_track_thresh = new_track_thresh
        self.match_thresh = match_thresh
        self.buffer_size = int(frame_rate / 30.0 * track_buffer)
        self.max_time_lost = self.buffer_size
        self.proximity_thresh = proximity_thresh
        self.appearance_thresh = appearance_thresh
        self.with_reid = with_reid
        self.fuse_first_associate = fuse_first_associate
        self.cmc_method = cmc_method
        self.cmc = IdentityCMC()
        self._params = EngineParams(
            track_high_thresh=track_high_thresh, track_low_thresh=track_low_thresh,
            new_track_thresh=new_track_thresh, track_buffer=track_buffer,
            match_thresh=match_thresh, proximity_thresh=proximity_thresh,
            appearance_thresh=appearance_thresh, frame_rate=frame_rate,
            fuse_first_associate=fuse_first_associate, with_reid=with_reid)
        self._caps = (track_cap, det_cap)
        self._cap = CapacityGuard()
        self.engine = None if with_reid else self._make_engine(0, False)

    def _make_engine(self, emb_dim: int, emb_f64: bool) -> Engine:
        return Engine("botsort", n_seq=1, track_cap=self._caps[0], det_cap=self._caps[1],
                      emb_dim=emb_dim, emb_f64=emb_f64, params=self._params)

    @BaseTracker.setup_decorator
    @BaseTracker.per_class_decorator
    def update(self, dets: np.ndarray, img: np.ndarray, embs: np.ndarray = None) -> np.ndarray:
        self.check_inputs(dets, img, embs)
        if self.with_reid and dets.shape[0] and embs is None:
            raise ValueError("BotSort(with_reid=True) on the MI355X engine needs `embs`: ReID "
                             "inference is outside the association path")
        if self.engine is None:
            if embs is None or embs.ndim != 2 or embs.shape[0] == 0:
                # nothing to learn the embedding width from yet; an empty frame is still a frame
                self.engine = self._make_engine(
                    embs.shape[1] if embs is not None and embs.ndim == 2 and embs.shape[1] else 512,
                    embs is not None and embs.dtype == np.float64)
            else:
                self.engine = self._make_engine(embs.shape[1], embs.dtype == np.float64)
        self.frame_count += 1
        n = int(np.asarray(dets).reshape(-1, 6).shape[0])
        self.engine = self._cap.fit(self.engine, {0: n}, n)
        if self.per_class:  # one update per class id, lost list shared (basetracker.py:155-201)
            # the reference's cmc.apply runs once per class call (botsort.py:218) on the class's
            # detections: a stateful CMC (ECC keeps the previous frame) gives class 0 the frame's
            # warp and the identity to the later calls
            warps = class_warps(self.cmc, img, dets, self.nr_classes)
            return self.engine.update_classes_host(0, dets, embs if self.with_reid else None,
                                                   warps, n_classes=self.nr_classes)
        warp = np.asarray(self.cmc.apply(img, _with_index(dets)), np.float64).reshape(2, 3)
        warp = None if np.array_equal(warp, np.eye(2, 3)) else warp
        out = self.engine.update_host(0, dets, embs if self.with_reid else None, warp)
        return out if out.shape[0] else np.asarray([])

    @property
    def active_tracks(self):
        return [] if self.engine is None else self._track_views(self.engine, _xywh_box)[0]

    def _class_active_lists(self):
        return self._class_track_views(self.engine, _xywh_box)

    @property
    def lost_stracks(self):
        return [] if self.engine is None else self._track_views(self.engine, _xywh_box)[1]
