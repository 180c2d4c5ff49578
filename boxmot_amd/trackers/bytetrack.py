"""ByteTrack on the MI355X engine — drop-in for boxmot.trackers.bytetrack.bytetrack.ByteTrack
(reference trackers/bytetrack/bytetrack.py:119-302).  Same constructor, same ``update``
contract and output rows; the whole frame (KF predict/update, IoU + fuse_score costs, the three
lapx-semantics assignments, list bookkeeping) runs as one HIP kernel launch.
"""
from __future__ import annotations

import numpy as np

from ..engine import Engine, EngineParams
from .basetracker import BaseTracker, CapacityGuard


def _xyah_box(mean):
    r = mean[:4].copy()
    r[2] *= r[3]
    return np.array([r[0] - r[2] / 2, r[1] - r[3] / 2, r[0] + r[2] / 2, r[1] + r[3] / 2])


class ByteTrack(BaseTracker):
    # The reference's id counter is process-global and never reset by ByteTrack
    # (bytetrack/basetrack.py:16,37-40): every instance continues the same sequence.
    _id_count = 0

    def __init__(self, min_conf: float = 0.1, track_thresh: float = 0.45,
                 match_thresh: float = 0.8, track_buffer: int = 25, frame_rate: int = 30,
                 per_class: bool = False, track_cap: int = 1024, det_cap: int = 384):
        super().__init__(per_class=bool(per_class))
        self.min_conf = min_conf
        self.track_thresh = track_thresh
        self.match_thresh = match_thresh
        self.det_thresh = track_thresh
        self.track_buffer = track_buffer
        self.buffer_size = int(frame_rate / 30.0 * track_buffer)
        self.max_time_lost = self.buffer_size
        self.frame_id = 0
        self.engine = Engine("bytetrack", n_seq=1, track_cap=track_cap, det_cap=det_cap,
                             params=EngineParams(min_conf=min_conf, track_thresh=track_thresh,
                                                 match_thresh=match_thresh,
                                                 track_buffer=track_buffer,
                                                 frame_rate=frame_rate))
        self._engine_ids = 0
        self._cap = CapacityGuard()

    @staticmethod
    def clear_count():
        ByteTrack._id_count = 0

    @BaseTracker.setup_decorator
    @BaseTracker.per_class_decorator
    def update(self, dets: np.ndarray, img: np.ndarray = None, embs: np.ndarray = None) -> np.ndarray:
        self.check_inputs(dets, img)
        if self._engine_ids != ByteTrack._id_count:
            self.engine.set_id_count(0, ByteTrack._id_count)
        self.frame_count += 1
        n = int(np.asarray(dets).reshape(-1, 6).shape[0])
        self.engine = self._cap.fit(self.engine, {0: n}, n)
        if self.per_class:  # one update per class id, lost list shared (basetracker.py:155-201)
            out = self.engine.update_classes_host(0, dets, n_classes=self.nr_classes)
        else:
            out = self.engine.update_host(0, dets)
        self._engine_ids = ByteTrack._id_count = self.engine.counters(0)["id_count"]
        if self.per_class:  # np.vstack of the classes' rows, else np.empty((0, 8))
            return out
        # the reference returns np.asarray([]) (shape (0,)) when nothing is output
        return out if out.shape[0] else np.asarray([])

    @property
    def active_tracks(self):
        return self._track_views(self.engine, _xyah_box)[0]

    def _class_active_lists(self):
        return self._class_track_views(self.engine, _xyah_box)

    @property
    def lost_stracks(self):
        return self._track_views(self.engine, _xyah_box)[1]
