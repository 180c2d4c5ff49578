"""OCSort on the MI355X engine — drop-in for boxmot.trackers.ocsort.ocsort.OcSort
(reference trackers/ocsort/ocsort.py:195-439).  Same constructor, same ``update`` contract and
output rows; the whole frame (XYSR Kalman predict/update with ORU, asso_func (iou, hmiou, giou,
diou, ciou or centroid) + direction-consistency costs, the legacy-lapx JV rounds, OCR/BYTE recovery, births and deaths) is one kernel launch.

The fork's OCSort does not run as shipped; this follows it with the minimal patches P1-P5
(SURVEY.md Appendix A), exactly as oracle/bxo_ocsort.c and the golden fixtures do.
"""
from __future__ import annotations

import numpy as np

from ..engine import OcsortEngine, OcsortParams
from ..iou import KINDS
from .basetracker import BaseTracker, CapacityGuard


class OcSort(BaseTracker):
    # KalmanBoxTracker.count is a class attribute shared by every instance and reset to 0 by
    # each OcSort constructor (ocsort.py:61,115-116,244): mirrored here.
    _id_count = 0

    def __init__(self, per_class: bool = False, min_conf: float = 0.1, det_thresh: float = 0.2,
                 max_age: int = 30, min_hits: int = 3, asso_threshold: float = 0.3,
                 delta_t: int = 3, asso_func: str = "iou", inertia: float = 0.2,
                 use_byte: bool = False, Q_xy_scaling: float = 0.01,
                 Q_s_scaling: float = 0.0001, track_cap: int = 256, det_cap: int = 256):
        super().__init__(max_age=max_age, per_class=per_class, asso_func=asso_func)
        self.min_conf = min_conf
        self.max_age = max_age
        self.min_hits = min_hits
        self.asso_threshold = asso_threshold
        self.frame_count = 0
        self.det_thresh = det_thresh
        self.delta_t = delta_t
        self.inertia = inertia
        self.use_byte = use_byte
        self.Q_xy_scaling = Q_xy_scaling
        self.Q_s_scaling = Q_s_scaling
        OcSort._id_count = 0
        # per_class: class c is engine sequence c (OCSort's state is all in the swapped
        # active_tracks, so classes are isolated trackers; basetracker.py:155-201)
        self.engine = OcsortEngine(
            n_seq=self.nr_classes if per_class else 1, track_cap=track_cap, det_cap=det_cap,
            params=OcsortParams(min_conf=min_conf, det_thresh=det_thresh, max_age=max_age,
                                min_hits=min_hits, asso_threshold=asso_threshold,
                                delta_t=delta_t, inertia=inertia, use_byte=use_byte,
                                Q_xy_scaling=Q_xy_scaling, Q_s_scaling=Q_s_scaling,
                                asso_func=asso_func if asso_func in KINDS else "iou"))
        self._engine_ids = 0
        self._frame_latched = False
        self._cap = CapacityGuard()

    @BaseTracker.setup_decorator
    @BaseTracker.per_class_decorator
    def update(self, dets: np.ndarray, img: np.ndarray, embs: np.ndarray = None) -> np.ndarray:
        self.check_inputs(dets, img)
        if not self._frame_latched and self._first_frame_processed:
            # the engine's asso_func / centroid frame size follow BaseTracker's first-frame latch
            for q in range(self.engine.n_seq):
                self.engine.set_frame_size(q, self.w, self.h)
            self._frame_latched = True
        self.frame_count += 1
        d = np.asarray(dets).reshape(-1, 6)
        if self.per_class:  # class c runs as sequence c: its births are at most its detections
            cls = d[:, 5].astype(np.float32)
            ok = (cls >= 0) & (cls < self.nr_classes) & (cls == np.floor(cls))
            per = np.bincount(cls[ok].astype(np.int64), minlength=self.nr_classes)
            self.engine = self._cap.fit(self.engine, {c: int(k) for c, k in enumerate(per) if k},
                                        d.shape[0])
        else:
            self.engine = self._cap.fit(self.engine, {0: d.shape[0]}, d.shape[0])
        if self.per_class:  # one launch over the class sequences, ids renumbered class-globally
            out, OcSort._id_count = self.engine.update_classes_host(0, self.nr_classes, dets,
                                                                    OcSort._id_count)
            return out
        if self._engine_ids != OcSort._id_count:
            self.engine.set_id_count(0, OcSort._id_count)
        out = self.engine.update_host(0, dets)
        self._engine_ids = OcSort._id_count = self.engine.counters(0)["id_count"]
        return out if out.shape[0] else np.array([])

    @property
    def active_tracks(self):
        """Track list snapshot: ids and XYSR Kalman state (x [7], P [7, 7]) per track (per_class:
        the list of the class that ran last, as the reference's swap leaves it)."""
        return self._seq_tracks(self.nr_classes - 1 if self.per_class else 0)

    def _seq_tracks(self, q):
        snap = self.engine.tracks(q)
        return [{"id": int(i), "x": x, "P": p} for i, x, p in zip(snap["id"], snap["x"], snap["P"])]

    def _class_active_lists(self):
        # class c is engine sequence c
        return [self._seq_tracks(c) for c in range(self.nr_classes)]
