"""Drop-in BaseTracker: the reference's plugin contract (trackers/basetracker.py:12-226) with the
per-frame numerics delegated to the MI355X engine.

Kept byte-compatible with the reference: ``update(dets, img, embs=None)`` → ``np.ndarray`` rows
``[x1, y1, x2, y2, id, conf, cls, det_ind]``; the same input unwrapping (``.data``/memoryview →
float32, basetracker.py:122-128 — which rounds every det to float32, including for plain numpy
arrays since they expose ``.data``), the same AssertionErrors (check_inputs, :203-226), the same
empty-input handling (:162-163) and the first-frame latch of image size.
"""
from __future__ import annotations

import numpy as np


def _with_index(dets: np.ndarray) -> np.ndarray:
    """dets with the detection-index column the reference appends before its CMC call
    (botsort.py:169, boosttrack.py:239)."""
    d = np.asarray(dets)
    # an empty frame may arrive 1-D (np.array([])); normalised like class_warps does
    d = d.reshape(-1, d.shape[-1]) if d.size and d.ndim else np.empty((0, 6))
    return np.hstack([d, np.arange(len(d)).reshape(-1, 1)])


def _reshape_warp(w) -> np.ndarray:
    return np.asarray(w, np.float64).reshape(2, 3)


def class_warps(cmc, img, dets: np.ndarray, nr_classes: int, conv=_reshape_warp) -> np.ndarray:
    """The warps of one frame's class calls under per_class=True: the reference calls
    ``cmc.apply(img, class_dets)`` once per class id (basetracker.py:175-189 ->
    botsort.py:218 / boosttrack.py:243-246), class_dets = dets[dets[:, 5] == c]
    (get_class_dets_n_embs, basetracker.py:83-106).  Returns [nr_classes, 2, 3]."""
    d = np.asarray(dets)
    d = d.reshape(-1, 6) if d.size else np.empty((0, 6))
    out = np.empty((int(nr_classes), 2, 3), np.float64)
    for c in range(int(nr_classes)):
        out[c] = conv(cmc.apply(img, _with_index(d[d[:, 5] == c])))
    return out


def _pow2(n: int) -> int:
    return 1 << max(0, int(n) - 1).bit_length()


class CapacityGuard:
    """Grows a drop-in's engine before a frame could overflow it.  The reference's track and
    detection lists are unbounded (bytetrack.py:272-346, sort/tracker.py:118-181); the engines
    have fixed slot arenas, so before each frame the drop-in checks that every sequence's slots
    in use plus the frame's detections (an upper bound on its births) fit, and otherwise moves
    the tracker state into an engine with twice the capacity (``engine.grown``, a device copy).
    The slots in use are tracked as an upper bound (+ detections per frame) and re-read from
    the engine only when that bound reaches the capacity."""

    def __init__(self):
        self.ub = {}
        self.t_max = None  # track_cap the engine could not grow past (its LDS / solver limit)

    def fit(self, eng, dets_per_seq: dict, n_frame: int):
        T, D = eng.track_cap, eng.det_cap
        need = T
        for q, n in dets_per_seq.items():
            if self.ub.get(q) is None or self.ub[q] + n > T:
                self.ub[q] = eng.slots_used(q)
            need = max(need, self.ub[q] + n)
        t2 = T if need <= T else max(2 * T, _pow2(need))
        if self.t_max is not None:
            t2 = min(t2, self.t_max)
        d2 = D if n_frame <= D else max(2 * D, _pow2(n_frame))
        while (t2, d2) != (T, D):
            try:
                eng = eng.grown(t2, d2)
                break
            except ValueError:  # past the engine's limits: the births bound is loose, so go on
                if t2 <= T:      # at the current slots (the engine still raises on a real overflow)
                    raise
                self.t_max = t2 = max(T, t2 // 2)
        for q, n in dets_per_seq.items():
            self.ub[q] += n
        return eng


class TrackView:
    """Read-only host view of one engine track (what ``active_tracks`` entries expose)."""

    __slots__ = ("id", "state", "is_activated", "frame_id", "start_frame", "mean", "covariance",
                 "_box_fn")

    def __init__(self, tid, state, act, fid, sf, mean, cov, box_fn):
        self.id, self.state, self.is_activated = int(tid), int(state), bool(act)
        self.frame_id, self.start_frame = int(fid), int(sf)
        self.mean, self.covariance, self._box_fn = mean, cov, box_fn

    @property
    def end_frame(self):
        return self.frame_id

    @property
    def xyxy(self):
        return self._box_fn(self.mean)

    def __repr__(self):
        return f"TrackView(id={self.id}, state={self.state}, activated={self.is_activated})"


class BaseTracker:
    def __init__(self, det_thresh: float = 0.3, max_age: int = 30, min_hits: int = 3,
                 iou_threshold: float = 0.3, max_obs: int = 50, nr_classes: int = 80,
                 per_class: bool = False, asso_func: str = "iou", is_obb: bool = False):
        self.det_thresh = det_thresh
        self.max_age = max_age
        self.max_obs = max_obs
        self.min_hits = min_hits
        self.per_class = per_class
        self.nr_classes = nr_classes
        self.iou_threshold = iou_threshold
        self.last_emb_size = None
        self.asso_func_name = asso_func + "_obb" if is_obb else asso_func
        self.is_obb = is_obb
        self.frame_count = 0
        self._first_frame_processed = False
        self._first_dets_processed = False
        if self.max_age >= self.max_obs:
            self.max_obs = self.max_age + 5

    @property
    def per_class_active_tracks(self):
        """basetracker.py:52-60,181-192: with per_class, {class id: the active list that class's
        last update left}; None otherwise.  Read from the engine (``_class_active_lists``)."""
        if not self.per_class:
            return None
        return dict(enumerate(self._class_active_lists()))

    def _class_active_lists(self) -> list:
        return [[] for _ in range(self.nr_classes)]

    # -------------------------------------------------------------------- reference decorators
    @staticmethod
    def setup_decorator(method):
        def wrapper(self, *args, **kwargs):
            dets = args[0]
            img = args[1] if len(args) > 1 else kwargs.get("img")
            if hasattr(dets, "data"):
                dets = dets.data
            if isinstance(dets, memoryview):
                dets = np.array(dets, dtype=np.float32)
            if not self._first_dets_processed and dets is not None:
                if dets.ndim == 2 and dets.shape[1] == 6:
                    self.is_obb = False
                    self._first_dets_processed = True
                elif dets.ndim == 2 and dets.shape[1] == 7:
                    self.is_obb = True
                    self._first_dets_processed = True
            if not self._first_frame_processed and img is not None:
                self.h, self.w = img.shape[0:2]
                # basetracker.py:140-147: the association function is chosen here, so an
                # unknown asso_func raises ValueError on the first update
                from ..iou import AssociationFunction

                self.asso_func = AssociationFunction(
                    w=self.w, h=self.h, asso_mode=self.asso_func_name).asso_func
                self._first_frame_processed = True
            rest = args[2:]
            if "embs" in kwargs:
                rest = (kwargs.pop("embs"),)
            kwargs.pop("img", None)
            return method(self, dets, img, *rest, **kwargs)

        return wrapper

    @staticmethod
    def per_class_decorator(update_method):
        """basetracker.py:155-201.  With per_class=True the reference calls the update once per
        class id 0..nr_classes-1 on that class's detections, swapping only ``active_tracks``;
        here the whole per-class frame is one native call (``*_update_classes_host``) that
        restates that loop on the device, so the wrapper only normalises empty input and checks
        the detection/embedding pairing the class split asserts (basetracker.py:95-98)."""

        def wrapper(self, dets, img, embs=None):
            if dets is None or len(dets) == 0:
                dets = np.empty((0, 6))
            if self.per_class and embs is not None and dets.size:
                assert dets.shape[0] == embs.shape[0], (
                    "Detections and embeddings must have the same number of elements when both "
                    "are provided")
            return update_method(self, dets=dets, img=img, embs=embs)

        return wrapper

    def check_inputs(self, dets, img, embs=None):
        assert isinstance(dets, np.ndarray), (
            f"Unsupported 'dets' input format '{type(dets)}', valid format is np.ndarray")
        assert isinstance(img, np.ndarray), (
            f"Unsupported 'img_numpy' input format '{type(img)}', valid format is np.ndarray")
        assert len(dets.shape) == 2, "Unsupported 'dets' dimensions, valid number of dimensions is two"
        if embs is not None:
            assert dets.shape[0] == embs.shape[0], "Missmatch between detections and embeddings sizes"
        if self.is_obb:
            assert dets.shape[1] == 7, "Unsupported 'dets' 2nd dimension lenght, valid lenghts is 6 (cx,cy,w,h,angle,conf,cls)"
        else:
            assert dets.shape[1] == 6, "Unsupported 'dets' 2nd dimension lenght, valid lenghts is 6 (x1,y1,x2,y2,conf,cls)"

    def update(self, dets: np.ndarray, img: np.ndarray, embs: np.ndarray = None) -> np.ndarray:
        raise NotImplementedError

    # ------------------------------------------------------------------------ engine helpers
    @staticmethod
    def _views(snap, box_fn):
        return [TrackView(snap["id"][k], snap["state"][k], snap["is_activated"][k],
                          snap["frame_id"][k], snap["start_frame"][k], snap["mean"][k],
                          snap["covariance"][k], box_fn)
                for k in range(snap["id"].shape[0])]

    def _track_views(self, engine, box_fn):
        snap = engine.tracks(0)
        views = self._views(snap, box_fn)
        return views[: snap["n_active"]], views[snap["n_active"]:]

    def _class_track_views(self, engine, box_fn):
        """ByteTrack / BoT-SORT per_class: every class's active list (parked or current)."""
        if engine is None:
            return [[] for _ in range(self.nr_classes)]
        return [self._views(snap, box_fn) for snap in engine.class_tracks(0, self.nr_classes)]
